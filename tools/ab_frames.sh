#!/bin/bash
RAW=gpurun_out/ab_frames.txt; : > $RAW
for r in 1 2 3; do for f in 64 128; do
  v=$(timeout -k 10 200 python bench.py --frames $f --steps 256 --warmup 128 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['roofline']['kernel_ms_avg'])")
  echo "F=$f $v" | tee -a $RAW
done; done
