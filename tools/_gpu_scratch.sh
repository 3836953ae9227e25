set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r03.sh r03f && \
timeout -k 10 200 python -u tools/repro_pathstate.py b64st-b128ld > gpurun_out/r03f_repro.txt 2>&1 && \
bash tools/pmc_quick.sh r03f --steps 256 --warmup 128
