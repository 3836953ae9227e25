set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r02u_gpu_tests.txt 2>&1 && tail -1 $O/r02u_gpu_tests.txt &&
CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh r02u > $O/prof_r02u.out 2>&1 && tail -1 $O/prof_r02u.out &&
CALIB=profiles/r02/hbm_calib.json bash tools/profile_round.sh r02u_rt10m --scene random_tris --tris 10000000 --steps 64 --warmup 16 > $O/prof_r02u_rt10m.out 2>&1 && tail -1 $O/prof_r02u_rt10m.out &&
timeout -k 10 400 python bench.py > $O/bench_default_r02u.json 2> $O/bench_default_r02u.err && cut -c1-120 $O/bench_default_r02u.json &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_r02u.json 2> $O/bench_driver_r02u.err && cut -c1-120 $O/bench_driver_r02u.json &&
timeout -k 10 300 python bench.py --width 3840 --height 2160 --spp 4 --steps 16 --warmup 4 --no-cpu-baseline > $O/cfg3_r02u.json 2>/dev/null &&
timeout -k 10 400 python bench.py --width 7680 --height 4320 --spp 8 --steps 3 --warmup 1 --single-frames 0 --no-cpu-baseline > $O/cfg5_r02u.json 2>/dev/null &&
timeout -k 10 300 python bench.py --adaptive --no-cpu-baseline > $O/adapt_r02u.json 2>/dev/null && echo configs ok
