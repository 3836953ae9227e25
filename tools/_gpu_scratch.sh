set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
V=my-raytracer_amd/lib/variants
RTAMD_HIP_LIB=$V/librt_hip_prev.so timeout -k 10 300 python -u tools/bitcmp.py $O/bc_base.npz > $O/bc_base.txt 2>&1 || { tail $O/bc_base.txt; exit 1; }
RTAMD_HIP_LIB=$V/librt_hip_ab.so timeout -k 10 300 python -u tools/bitcmp.py $O/bc_all.npz > $O/bc_all.txt 2>&1 || { tail $O/bc_all.txt; exit 1; }
python tools/bitcmp_diff.py $O/bc_base.npz $O/bc_all.npz | tee $O/bc_diff6.txt
rm -f $O/bc_base.npz $O/bc_all.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/ab_gpu_tests.txt 2>&1 || { tail -40 $O/ab_gpu_tests.txt; exit 1; }
tail -1 $O/ab_gpu_tests.txt
bash tools/ab_single.sh 3 "" $V/librt_hip_prev.so $V/librt_hip_ab.so > $O/ab_ab_office.txt || exit 1
cat $O/ab_ab_office.txt
bash tools/ab.sh 2 "--scene random_tris --tris 10000000 --single-frames 0" $V/librt_hip_prev.so $V/librt_hip_ab.so > $O/ab_ab_rt10m.txt || exit 1
cat $O/ab_ab_rt10m.txt
