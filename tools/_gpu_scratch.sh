set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
T=r03q
bash tools/gpu_r03.sh ${T} || exit $?
B="python -u bench.py --no-cpu-baseline"
for v in new prev new prev; do
  L=my-raytracer_amd/lib/librt_hip.so; [ $v != new ] && L=my-raytracer_amd/lib/variants/librt_hip_$v.so
  RTAMD_HIP_LIB=$L timeout -k 10 300 $B >> $O/${T}_office_$v.jsonl 2> $O/${T}_office_$v.err || exit $?
  RTAMD_HIP_LIB=$L timeout -k 10 300 $B --steps 20 --warmup 5 >> $O/${T}_drv_$v.jsonl 2> $O/${T}_drv_$v.err || exit $?
done
echo done
