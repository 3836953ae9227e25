set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
T=r03j
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/${T}_parity.txt 2>&1 || exit $?
B="python -u bench.py --no-cpu-baseline"
for v in share noshare s16 s32 s64; do
  L=my-raytracer_amd/lib/librt_hip.so; [ $v != share ] && L=my-raytracer_amd/lib/variants/librt_hip_$v.so
  RTAMD_HIP_LIB=$L timeout -k 10 300 $B > $O/${T}_office_$v.json 2> $O/${T}_office_$v.err || exit $?
  RTAMD_HIP_LIB=$L timeout -k 10 300 $B --steps 20 --warmup 5 > $O/${T}_drv_$v.json 2> $O/${T}_drv_$v.err || exit $?
  RTAMD_HIP_LIB=$L timeout -k 10 300 $B --scene random_tris --tris 10000000 > $O/${T}_rt10m_$v.json 2> $O/${T}_rt10m_$v.err || exit $?
done
echo done
