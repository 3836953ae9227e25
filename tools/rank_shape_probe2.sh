#!/bin/bash
# The N = 8 per-rank launch shape on one GPU (frames of 1920 x 136), 20 frames cut into launches of
# F frames with S in flight (dev tool, under gpurun).
set -e
mkdir -p gpurun_out/r05zzg
for r in 1 2 3; do
for m in "f10s2|--frames 10 --streams 2" "f5s2|--frames 5 --streams 2" "f5s3|--frames 5 --streams 3" "f4s3|--frames 4 --streams 3" "f20s1|--frames 20 --streams 1"; do
  tag=${m%%|*}; args=${m#*|}
  timeout -k 10 200 python -u bench.py --height 136 --steps 20 --warmup 20 --no-cpu-baseline --tree-record off --single-frames 0 $args > gpurun_out/r05zzg/$tag.$r.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/r05zzg/$tag.$r.json'));print('$tag',d['value'],d['ms_per_step'],d['kernel_ms_per_frame'])"
done; done
