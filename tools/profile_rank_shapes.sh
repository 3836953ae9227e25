#!/bin/bash
# rocprofv3 summaries of the N-GPU rank shapes on one GPU (dev tool, under gpurun): bench.py
# --rank-shape N renders exactly rank 0's launches of an N-GPU run, so the committed summary (its
# workload_key carries n_gpus = N) gives the N > 1 bench lines their roofline (bench.py
# pmc_per_frame).  The driver's command shape: --steps 20 --warmup 5 (gather: 10 frames per launch,
# two in flight).   usage: bash tools/profile_rank_shapes.sh TAG [N ...]
# FRAMES=20: the peer assembly's shape instead (all 20 frames in one launch), tags TAG_nN_f20 -- the
# same profiling round, so an N-GPU line picks the summary of its own frames per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; shift
NS=${*:-2 4 8}
export CALIB=profiles/r02/hbm_calib.json
export PASSES="fetch write td sq sqa valu"
for n in $NS; do
  if [ -n "$FRAMES" ]; then T=${TAG}_n${n}_f$FRAMES; X="--frames $FRAMES"; else T=${TAG}_n$n; X=""; fi
  bash tools/profile_round.sh $T --rank-shape $n --steps 20 --warmup 5 --single-frames 0 $X \
    || { echo "profile n=$n failed"; exit 1; }
done
