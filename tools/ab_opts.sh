#!/bin/bash
# Interleaved A/B of bench.py option sets on one kernel library (dev tool, under gpurun), e.g. an
# rt_upload_options field:   tools/ab_opts.sh ROUNDS "bench args" "opts A" "opts B" ...
# Each result is appended to gpurun_out/ab_opts_raw.txt as it arrives, then the medians are printed.
R=$1; ARGS=$2; shift 2
RAW=gpurun_out/ab_opts_raw.txt
mkdir -p gpurun_out
: > $RAW
for r in $(seq 1 $R); do
  for o in "$@"; do
    v=$(timeout -k 10 300 python bench.py $ARGS $o --no-cpu-baseline 2>/dev/null | python -c "import json,sys; print(json.load(sys.stdin)['value'])")
    echo "${o// /_}|$v" | tee -a $RAW >&2
  done
done
python -c "
import collections, statistics
d = collections.defaultdict(list)
for line in open('$RAW'):
    k, v = line.strip().rsplit('|', 1); d[k].append(float(v))
for k, v in d.items():
    print(f'{statistics.median(v):9.1f}  {min(v):9.1f} {max(v):9.1f}  {k or \"(default)\"}')
"
