#!/bin/bash
# End-of-round GPU records (under gpurun) -- dev tool:
#   bash tools/gpu_final.sh TAG [suite] [configs] [profile]
#   suite:   the GPU suite + smoke()
#   configs: one bench line per BASELINE config with its CPU baseline (tools/configs_bench.sh)
#   profile: the driver-shape bench profiled (kernel stats + PMC passes, committed calibration)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; shift
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    suite)
      bash tools/gpu_suite.sh $TAG || { echo "gpu suite failed"; exit 1; }
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
      echo "suite + smoke done" ;;
    configs)
      bash tools/configs_bench.sh $TAG || exit 1 ;;
    profile)
      CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh ${TAG}_drv --gpus 1 --steps 20 --warmup 5 \
        || { echo "profile failed"; exit 1; }
      echo "profile done" ;;
  esac
done
