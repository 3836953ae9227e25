#!/bin/bash
# One gpurun call of several steps (dev tool): the GPU suite first, then the named measurement
# steps, each under its own time limit; a step that times out, aborts or faults ends the call
# (exit >= 124), a failing test does not.
#   bash tools/gpu_call.sh TAG "pytest args" [step-command ...]
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:?tag}; PT=$2; shift 2
mkdir -p gpurun_out
if [ -n "$PT" ]; then
  # (PT is shell words: -k "a or b" keeps its quotes)
  eval "timeout -k 10 720 python -u -m pytest -v --timeout 200 --timeout-method thread $PT" > gpurun_out/${TAG}_gpu_tests.txt 2>&1
  rc=$?
  tail -3 gpurun_out/${TAG}_gpu_tests.txt
  if [ $rc -ge 124 ] || [ $rc -eq 2 ] || [ $rc -gt 5 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
fi
for step in "$@"; do
  echo "== $step"
  bash -c "$step"
  rc=$?
  if [ $rc -ne 0 ]; then echo "step ended with $rc: stopping"; exit $rc; fi
done
echo "call $TAG done"
