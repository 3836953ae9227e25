#!/bin/bash
# Quick HBM-bytes check of a bench workload (dev tool, under gpurun): the bench line, then one
# FETCH_SIZE and one WRITE_SIZE pass (separate runs), summarised per frame with the committed
# calibration.   usage: tools/pmc_quick.sh TAG [bench args...]
set -e -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline $*"
timeout -k 10 300 $B > $O/bench_$TAG.json 2> $O/bench_$TAG.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_${TAG}_fetch -o run -- $B > $O/pmc_${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_${TAG}_write -o run -- $B > $O/pmc_${TAG}_write.log 2>&1
python tools/pmc_summary.py $O/pmc_$TAG.json --bench $O/bench_$TAG.json --calib profiles/r02/hbm_calib.json $O/pmc_${TAG}_fetch $O/pmc_${TAG}_write
echo "pmc $TAG done"
