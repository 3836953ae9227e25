set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error|error" gpurun_out/gpu_tests.txt | head -20; tail -5 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
