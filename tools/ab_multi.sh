#!/bin/bash
# Interleaved A/B over whole environment settings with bench.py (dev tool, under gpurun).
# usage: tools/ab_multi.sh ROUNDS "bench args" "VAR=a VAR2=b" "VAR=c" ...
# Results are appended to gpurun_out/ab_raw.txt as they arrive (see tools/ab.sh).
R=$1; ARGS=$2; shift 2
RAW=gpurun_out/ab_raw.txt
mkdir -p gpurun_out
: > $RAW
for r in $(seq 1 $R); do
  for x in "$@"; do
    v=$(env $x timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline 2>/dev/null | python -c "import json,sys; print(json.load(sys.stdin)['value'])")
    echo "${x// /,} $v" | tee -a $RAW >&2
  done
done
python -c "
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open('$RAW'):
    k, v = line.split(); d[k].append(float(v))
for k, v in d.items():
    print(f'{statistics.median(v):9.1f}  {min(v):9.1f} {max(v):9.1f}  {k}')
"
