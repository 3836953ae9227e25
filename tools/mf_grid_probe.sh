#!/bin/bash
# Multi-frame launches in flight on two streams with half grids (rt_upload_options.blocks_per_cu = 2)
# against one 20-frame launch, interleaved rounds (dev tool, under gpurun).
set -e
mkdir -p gpurun_out/r05zzc
for r in 1 2 3; do
for m in "base20|--steps 20" "f10s2b2|--steps 20 --frames 10 --streams 2 --opt blocks_per_cu=2" "f5s2b2|--steps 20 --frames 5 --streams 2 --opt blocks_per_cu=2" "f20s2b2|--steps 40 --frames 20 --streams 2 --opt blocks_per_cu=2" "base40|--steps 40 --frames 20"; do
  tag=${m%%|*}; args=${m#*|}
  timeout -k 10 200 python -u bench.py --warmup 20 --no-cpu-baseline --tree-record off --single-frames 0 $args > gpurun_out/r05zzc/$tag.$r.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/r05zzc/$tag.$r.json'));print('$tag',d['value'],d['ms_per_step'],d['kernel_ms_per_frame'])"
done; done
