set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
T=r03o
timeout -k 10 300 python -u tools/order_probe.py 20 20 > $O/${T}_order.txt 2>&1 || exit $?
B="python -u bench.py --no-cpu-baseline"
timeout -k 10 300 $B > $O/${T}_office.json 2> $O/${T}_office.err || exit $?
for v in base d8 d16; do
  L=my-raytracer_amd/lib/librt_hip.so; [ $v != base ] && L=my-raytracer_amd/lib/variants/librt_hip_$v.so
  RTAMD_HIP_LIB=$L timeout -k 10 300 $B --scene random_tris --tris 10000000 > $O/${T}_rt10m_$v.json 2> $O/${T}_rt10m_$v.err || exit $?
done
bash tools/gpu_r03.sh ${T} || exit $?
echo done
