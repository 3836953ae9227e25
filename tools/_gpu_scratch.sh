set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
T=r03n
timeout -k 10 300 python -u tools/order_probe.py 20 20 > $O/${T}_order.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/${T}_office.json 2> $O/${T}_office.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/${T}_drv.json 2> $O/${T}_drv.err || exit $?
echo done
