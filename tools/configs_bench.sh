#!/bin/bash
# One bench.py line per BASELINE.json config, each with its cpu_baseline (the reference-CPU-semantics
# oracle on the box's host cores; configs 3-5 on a 1/16-row sample, frame time extrapolated) -- dev
# tool, under gpurun:   bash tools/configs_bench.sh TAG
#   C1 spheres_proxy 640x480 1 spp (GPU with the analytic primitives; the CPU path is the config)
#   C2 office_proxy 1920x1080 1 spp (the headline workload)
#   C3 office_proxy 3840x2160 16 spp
#   C4 10 M random triangles 1920x1080 1 spp
#   C5 office_proxy 7680x4320 64 spp on ONE GPU (the whole frame; a rank's eighth at N = 8 is that / 8)
# Output: gpurun_out/configs_TAG/c{1..5}.json; python tools/configs_summary.py collects them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}
O=gpurun_out/configs_$TAG
mkdir -p $O
run() {   # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "config $n failed"; exit 1; }
  echo "config $n done"
}
run c1 300 --scene spheres --width 640 --height 480 --cpu-seconds 10
run c2 300 --cpu-seconds 12
run c3 300 --width 3840 --height 2160 --spp 4 --steps 8 --warmup 2 --single-frames 0 --cpu-seconds 12
run c4 400 --scene random_tris --tris 10000000 --cpu-seconds 12
run c5 400 --width 7680 --height 4320 --spp 8 --steps 2 --warmup 1 --single-frames 0 --cpu-seconds 12
