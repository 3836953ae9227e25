#!/bin/bash
# Interleaved A/B of kernel library variants with bench.py (dev tool, under gpurun).
# usage: tools/ab.sh ROUNDS "bench args" lib1 lib2 ...
# Each result is appended to gpurun_out/ab_raw.txt as it arrives (gpurun kills a command
# that writes nothing for 180 s), then the medians are printed.
R=$1; ARGS=$2; shift 2
RAW=gpurun_out/ab_raw.txt
mkdir -p gpurun_out
: > $RAW
for r in $(seq 1 $R); do
  for l in "$@"; do
    v=$(RTAMD_HIP_LIB=$l timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline 2>/dev/null | python -c "import json,sys; print(json.load(sys.stdin)['value'])")
    echo "$l $v" | tee -a $RAW >&2
  done
done
python -c "
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open('$RAW'):
    k, v = line.split(); d[k].append(float(v))
for k, v in d.items():
    print(f'{statistics.median(v):9.1f}  {min(v):9.1f} {max(v):9.1f}  {k.split(\"/\")[-1]}')
"
