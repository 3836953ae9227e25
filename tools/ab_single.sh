#!/bin/bash
# Interleaved A/B of kernel library variants on bench.py's one-frame records (dev tool, under gpurun):
# the default-order record and the natural-order record, kernel ms (HIP events) and ms per frame.
# usage: tools/ab_single.sh ROUNDS "bench args" lib1 lib2 ...
R=$1; ARGS=$2; shift 2
RAW=gpurun_out/ab_single_raw.txt
mkdir -p gpurun_out
: > $RAW
for r in $(seq 1 $R); do
  for l in "$@"; do
    v=$(RTAMD_HIP_LIB=$l timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline 2>/dev/null | python -c "
import json,sys; d=json.load(sys.stdin); s=d['single_frame']; n=s['natural_order']
print(d['value'], s['kernel_ms_avg'], s['ms_per_frame'], n['kernel_ms_avg'], n['ms_per_frame'])")
    echo "$l $v" | tee -a $RAW >&2
  done
done
python -c "
import sys, collections, statistics
d = collections.defaultdict(list)
for line in open('$RAW'):
    k, *v = line.split(); d[k].append([float(x) for x in v])
print('   batched  ord_kern  ord_frame  nat_kern  nat_frame  (medians)')
for k, v in d.items():
    m = [statistics.median(c) for c in zip(*v)]
    print(f'{m[0]:10.1f} {m[1]:9.4f} {m[2]:10.4f} {m[3]:9.4f} {m[4]:10.4f}  {k.split(\"/\")[-1]}')
"
