set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python bench.py --adaptive --no-cpu-baseline > $O/bench_adaptive.json 2> $O/bench_adaptive.err && cut -c1-200 $O/bench_adaptive.json &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "adaptive" > $O/t_adapt.txt 2>&1 && tail -1 $O/t_adapt.txt
