#!/bin/bash
# Steady-state PMC (frames in flight) for the production kernel (dev tool, run under gpurun).
set -e -o pipefail
TAG=${1:?tag}
O=gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 12 --warmup 2 --no-cpu-baseline"
pass() {
  local name=$1; shift
  timeout -k 10 150 rocprofv3 --pmc "$@" --output-format csv -d $O/pmcs_${TAG}_$name -o run -- $B > $O/pmcs_${TAG}_$name.log 2>&1
}
pass lat VmemLatency
pass memstall MemUnitStalled
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS
pass sq3 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS
pass td TD_TD_BUSY_sum GRBM_GUI_ACTIVE
pass ta TA_BUSY_avr
pass tcc TCC_HIT_sum TCC_MISS_sum
pass tcplat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
python tools/pmc_summary.py $O/pmcs_$TAG.json $O/pmcs_${TAG}_*/
echo "steady $TAG done"
