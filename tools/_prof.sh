set -e -o pipefail
export CALIB=profiles/r02/hbm_calib.json
bash tools/profile_round.sh r02q
bash tools/profile_round.sh r02q_rt10m --scene random_tris --tris 10000000 --steps 64 --warmup 32 --single-frames 4
