set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
V=my-raytracer_amd/lib/variants
RTAMD_HIP_LIB=$V/librt_hip_lv32.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "config4 or stack_ring or suspend_resume or fuzz_scene_matches" > $O/lv_gpu_tests.txt 2>&1 || { tail -40 $O/lv_gpu_tests.txt; exit 1; }
tail -1 $O/lv_gpu_tests.txt
bash tools/ab_single.sh 2 "--scene random_tris --tris 10000000 --single-frames 8" $V/librt_hip_lv0.so $V/librt_hip_lv16.so $V/librt_hip_lv32.so $V/librt_hip_lv48.so > $O/ab_lv_rt10m.txt || exit 1
cat $O/ab_lv_rt10m.txt
