set -e
mkdir -p gpurun_out/r05zx
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_bench_gpu.py -k contract > gpurun_out/r05zx/test_bench.txt 2>&1
for p in 2 3 4 6; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --tree-record off --pipeline $p > gpurun_out/r05zx/pipe$p.json 2> gpurun_out/r05zx/pipe$p.err
  python -c "import json;d=json.load(open('gpurun_out/r05zx/pipe$p.json'));s=d['single_frame'];print($p,d['value'],s['ms_per_frame'],s['natural_order']['ms_per_frame'],s['pipelined'])"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05zx/bench_driver.json 2> gpurun_out/r05zx/bench_driver.err
