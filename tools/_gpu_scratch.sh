set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu_r03.sh r03p || exit $?
CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh r03p_drv --steps 20 --warmup 5 || exit $?
CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh r03p || exit $?
echo done
