#!/bin/bash
# Interleaved A/B of kernel library variants with bench.py (dev tool, under gpurun).
# usage: tools/ab.sh ROUNDS "bench args" lib1 lib2 ...
R=$1; ARGS=$2; shift 2
for r in $(seq 1 $R); do
  for l in "$@"; do
    v=$(RTAMD_HIP_LIB=$l timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline 2>/dev/null | python -c "import json,sys; print(json.load(sys.stdin)['value'])")
    echo "$l $v"
  done
done | python -c "
import sys, collections, statistics
d = collections.defaultdict(list)
for line in sys.stdin:
    k, v = line.split(); d[k].append(float(v))
for k, v in d.items():
    print(f'{statistics.median(v):9.1f}  {min(v):9.1f} {max(v):9.1f}  {k.split(\"/\")[-1]}')
"
