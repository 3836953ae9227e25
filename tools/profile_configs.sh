#!/bin/bash
# rocprofv3 kernel stats + PMC summaries for every BASELINE config's bench workload (dev tool,
# under gpurun), so each config line's roofline.traffic comes from its own counters:
#   bash tools/profile_configs.sh TAG [c1 c2 c3 c4 c5]
# The bench arguments match tools/configs_bench.sh (the workload key must be the same).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; shift
CS=${*:-c1 c2 c3 c4 c5}
export CALIB=profiles/r02/hbm_calib.json
for c in $CS; do
  case $c in
    c1) A="--scene spheres --width 640 --height 480" ;;
    c2) A="" ;;
    c3) A="--width 3840 --height 2160 --spp 4 --steps 8 --warmup 2 --single-frames 0" ;;
    c4) A="--scene random_tris --tris 10000000" ;;
    c5) A="--width 7680 --height 4320 --spp 8 --steps 2 --warmup 1 --single-frames 0" ;;
  esac
  bash tools/profile_round.sh ${TAG}_$c $A || { echo "profile $c failed"; exit 1; }
done
