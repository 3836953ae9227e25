set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r02s_gpu_tests.txt 2>&1 && tail -1 $O/r02s_gpu_tests.txt &&
CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh r02s > $O/prof_r02s.out 2>&1 && tail -1 $O/prof_r02s.out &&
CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh r02s_rt10m --scene random_tris --tris 10000000 --steps 20 --warmup 5 > $O/prof_r02s_rt10m.out 2>&1 && tail -1 $O/prof_r02s_rt10m.out &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_r02s.json 2> $O/bench_driver_r02s.err && cat $O/bench_driver_r02s.json | cut -c1-200
