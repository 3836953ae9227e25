#!/bin/bash
# single_frame.pipelined under smaller persistent grids (rt_upload_options.blocks_per_cu)
# and pipeline depths, interleaved rounds (dev tool, under gpurun).
set -e
mkdir -p gpurun_out/r05zzb
for r in 1 2; do
for m in "p3|--pipeline 3" "p3b3|--pipeline 3 --opt blocks_per_cu=3" "p3b2|--pipeline 3 --opt blocks_per_cu=2" "p2b2|--pipeline 2 --opt blocks_per_cu=2" "p4b1|--pipeline 4 --opt blocks_per_cu=1"; do
  tag=${m%%|*}; args=${m#*|}
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --tree-record off $args > gpurun_out/r05zzb/$tag.$r.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/r05zzb/$tag.$r.json'));s=d['single_frame'];print('$tag',d['value'],s['ms_per_frame'],s['pipelined']['ms_per_frame'])"
done; done
