set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
V=my-raytracer_amd/lib/variants
RTAMD_HIP_LIB=$V/librt_hip_r0.so timeout -k 10 300 python -u tools/bitcmp.py $O/bc_r0.npz > $O/bc_r0.txt 2>&1 || { tail $O/bc_r0.txt; exit 1; }
RTAMD_HIP_LIB=$V/librt_hip_r1.so timeout -k 10 300 python -u tools/bitcmp.py $O/bc_r1.npz > $O/bc_r1.txt 2>&1 || { tail $O/bc_r1.txt; exit 1; }
python tools/bitcmp_diff.py $O/bc_r0.npz $O/bc_r1.npz | tee $O/bc_diff.txt
rm -f $O/bc_r0.npz $O/bc_r1.npz
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/rc_gpu_tests.txt 2>&1 || { tail -40 $O/rc_gpu_tests.txt; exit 1; }
tail -1 $O/rc_gpu_tests.txt
bash tools/ab_single.sh 3 "" $V/librt_hip_r0.so $V/librt_hip_r1.so > $O/ab_rc_office.txt || exit 1
cat $O/ab_rc_office.txt
bash tools/ab.sh 2 "--scene random_tris --tris 10000000 --single-frames 0" $V/librt_hip_r0.so $V/librt_hip_r1.so > $O/ab_rc_rt10m.txt || exit 1
cat $O/ab_rc_rt10m.txt
