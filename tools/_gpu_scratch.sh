set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/order_probe.py 20 20 > $O/r03l_order.txt 2>&1 || exit $?
bash tools/gpu_r03.sh r03l || exit $?
echo done
