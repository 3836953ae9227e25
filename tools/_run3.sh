set -o pipefail
export TMPDIR=/tmp
L=my-raytracer_amd/lib/variants
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo TESTS FAILED; grep -E "^FAILED|Error|assert" gpurun_out/gpu_tests.txt | head -20; tail -5 gpurun_out/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/gpu_tests.txt
timeout -k 10 600 python -u tools/ab_frame.py 3 $L/librt_hip_base.so $L/librt_hip_helper.so > gpurun_out/ab.txt 2>&1; tail -2 gpurun_out/ab.txt
