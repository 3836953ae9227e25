#!/bin/bash
# Two 10-frame launches on two streams after one warm-up launch (the N > 1 bench shape on one GPU),
# bench.py at HEAD vs the working tree's bench.py (dev tool, under gpurun).
set -e
mkdir -p gpurun_out/r05zy
for r in 1 2; do
for b in bench_head.py bench.py; do
  timeout -k 10 200 python -u $b --frames 10 --streams 2 --steps 20 --warmup 10 --no-cpu-baseline --tree-record off --single-frames 0 > gpurun_out/r05zy/$b.$r.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/r05zy/$b.$r.json'));print('$b',d['value'],d['ms_per_step'],d['kernel_ms_per_frame'])"
done; done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_gpu.py > gpurun_out/r05zy/test_bench.txt 2>&1
