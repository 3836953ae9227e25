#!/bin/bash
# bench.py over frames-per-launch x launches-in-flight (dev tool, under gpurun)
set -o pipefail
for cfg in "1 1" "2 1" "4 1" "8 1" "4 2" "8 2" "1 4"; do
  set -- $cfg
  v=$(timeout -k 10 200 python bench.py --steps 64 --warmup 8 --frames $1 --streams $2 --no-cpu-baseline 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])") || exit 1
  echo "frames=$1 streams=$2 -> $v"
done
