#!/bin/bash
# End-of-round GPU check (under gpurun): the GPU suite, smoke(), then the driver-shape bench
# profiled (rocprofv3 kernel stats + PMC passes, committed calibration) -- dev tool.
#   bash tools/gpu_final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}
mkdir -p gpurun_out
bash tools/gpu_r03.sh $TAG || { echo "gpu suite failed"; exit 1; }
echo "gpu suite done"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
echo "smoke done"
CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh ${TAG}_drv --gpus 1 --steps 20 --warmup 5 \
  || { echo "profile failed"; exit 1; }
