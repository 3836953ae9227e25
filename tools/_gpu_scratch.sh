set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
V=my-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/m3_gpu_tests.txt 2>&1 || { tail -40 $O/m3_gpu_tests.txt; exit 1; }
tail -1 $O/m3_gpu_tests.txt
bash tools/ab.sh 3 "" $V/librt_hip_m0.so $V/librt_hip_m1.so > $O/ab_m3_office.txt || exit 1
cat $O/ab_m3_office.txt
bash tools/ab.sh 2 "--scene random_tris --tris 10000000 --single-frames 0" $V/librt_hip_m0.so $V/librt_hip_m1.so > $O/ab_m3_rt10m.txt || exit 1
cat $O/ab_m3_rt10m.txt
