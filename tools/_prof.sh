set -e -o pipefail
export CALIB=profiles/r02/hbm_calib.json
bash tools/profile_round.sh r02r
timeout -k 10 300 python bench.py > gpurun_out/bench_r02r_full.json 2> gpurun_out/bench_r02r_full.err
