#!/bin/bash
# Interleaved A/B of kernel libraries on the bench's one-frame records (serial and 3 in flight) and
# the batched value (dev tool, under gpurun).   usage: tools/pipe_halfgrid_ab.sh ROUNDS lib1 lib2 ...
R=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for l in "$@"; do
    RTAMD_HIP_LIB=$l timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tree-record off 2>/dev/null \
      | python -c "import json,sys;d=json.load(sys.stdin);s=d['single_frame'];print('$(basename $l)',d['value'],s['ms_per_frame'],s['pipelined']['ms_per_frame'])" || exit 1
  done
done
