#!/bin/bash
# GPU check (under gpurun): the GPU suite, then an optional bench line -- dev tool.
#   bash tools/gpu_suite.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 \
  > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || exit $?
if [ "$#" -gt 0 ]; then
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
fi
