#!/bin/bash
# Round-end records at HEAD (under gpurun): configs 1-5 with CPU baselines, then config 4 profiled
# (kernel stats + PMC passes, committed calibration) -- dev tool.   bash tools/gpu_final2.sh TAG [suite]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}
mkdir -p gpurun_out
if [ "$2" = "suite" ]; then
  bash tools/gpu_r03.sh $TAG || { echo "gpu suite failed"; exit 1; }
  echo "gpu suite done"
fi
bash tools/configs_bench.sh $TAG || exit 1
CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh ${TAG}_rt10m --scene random_tris --tris 10000000 \
  || { echo "profile failed"; exit 1; }
