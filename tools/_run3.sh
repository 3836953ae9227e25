set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_gpu.py -m gpu -x -q -k "adaptive" --timeout 280 --timeout-method thread > gpurun_out/gpu_tests.txt 2>&1 || { echo TESTS FAILED; grep -E "^FAILED|Error|assert" gpurun_out/gpu_tests.txt | head -20; tail -5 gpurun_out/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/gpu_tests.txt
timeout -k 10 300 python -u tools/adapt_probe.py 2>&1 | grep -v amdgpu.ids | grep "it3"
timeout -k 10 300 python bench.py --adaptive --steps 128 --warmup 32 --no-cpu-baseline > gpurun_out/badapt.json 2>gpurun_out/badapt.err || { tail -20 gpurun_out/badapt.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/badapt.json')); print(d['value'], d['ms_per_step'], d['config']['adaptive_pass'], d['roofline']['kernel_ms_avg'])"
