#!/bin/bash
# Re-measures the non-default configurations for DESIGN.md §5/§8 (dev tool, under gpurun):
# N-GPU striping emulated on one GPU, configs 3/4 (+1 M random triangles), config 5 shard.
set -e -o pipefail
O=gpurun_out/configs_probe.txt
: > $O
timeout -k 10 300 python tools/shard_probe.py | tee -a $O
timeout -k 10 300 python tools/perf_probe.py office:3840x2160:4 random_tris:1920x1080:1:10000000 | tee -a $O
timeout -k 10 300 python tools/perf_probe.py random_tris:1920x1080:1:1000000 | tee -a $O
timeout -k 10 300 python tools/config5_probe.py | tee -a $O
