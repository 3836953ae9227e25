set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
V=my-raytracer_amd/lib/variants
RTAMD_HIP_LIB=$V/librt_hip_f0.so timeout -k 10 300 python -u tools/bitcmp.py $O/bc_base.npz > $O/bc_base.txt 2>&1 || { tail $O/bc_base.txt; exit 1; }
RTAMD_HIP_LIB=$V/librt_hip_f2.so timeout -k 10 300 python -u tools/bitcmp.py $O/bc_all.npz > $O/bc_all.txt 2>&1 || { tail $O/bc_all.txt; exit 1; }
python tools/bitcmp_diff.py $O/bc_base.npz $O/bc_all.npz | tee $O/bc_diff3.txt
rm -f $O/bc_base.npz $O/bc_all.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/fo_gpu_tests.txt 2>&1 || { tail -40 $O/fo_gpu_tests.txt; exit 1; }
tail -1 $O/fo_gpu_tests.txt
bash tools/ab_single.sh 3 "" $V/librt_hip_f0.so $V/librt_hip_f1.so $V/librt_hip_f2.so > $O/ab_fo_office.txt || exit 1
cat $O/ab_fo_office.txt
bash tools/ab.sh 2 "--width 3840 --height 2160 --spp 4 --steps 8 --warmup 2 --single-frames 0" $V/librt_hip_f0.so $V/librt_hip_f2.so > $O/ab_fo_c3.txt || exit 1
cat $O/ab_fo_c3.txt
