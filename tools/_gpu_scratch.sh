set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/final_gpu_tests.txt 2>&1 || { tail -40 $O/final_gpu_tests.txt; exit 1; }
tail -1 $O/final_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/final_smoke.txt 2>&1 || { tail $O/final_smoke.txt; exit 1; }
tail -1 $O/final_smoke.txt
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/final_bench_drv.json 2> $O/final_bench_drv.err || exit 1
python -c "import json; d=json.loads(open('$O/final_bench_drv.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['valu_roof']['frac'], d['cpu_baseline']['value'])"
