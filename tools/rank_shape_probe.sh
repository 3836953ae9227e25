#!/bin/bash
# The N = 8 per-rank launch shape on one GPU: 10 frames of 1920 x 136 (an eighth of 1080 rows) per
# launch, two launches in flight on two streams, whole vs half grids, against one stream
# (dev tool, under gpurun).
set -e
mkdir -p gpurun_out/r05zzf
for r in 1 2 3; do
for m in "s2full|--streams 2" "s2half|--streams 2 --opt blocks_per_cu=2" "s1full|--streams 1"; do
  tag=${m%%|*}; args=${m#*|}
  timeout -k 10 200 python -u bench.py --height 136 --frames 10 --steps 20 --warmup 20 --no-cpu-baseline --tree-record off --single-frames 0 $args > gpurun_out/r05zzf/$tag.$r.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/r05zzf/$tag.$r.json'));print('$tag',d['value'],d['ms_per_step'],d['kernel_ms_per_frame'])"
done; done
