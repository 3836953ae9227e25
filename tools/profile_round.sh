#!/bin/bash
# Profiles bench.py on the GPU box (dev tool, run under gpurun):
#   bench line, rocprofv3 --kernel-trace --stats, then separate --pmc passes.
# usage: tools/profile_round.sh TAG      (outputs under gpurun_out/prof_TAG*)
set -e -o pipefail
TAG=${1:?tag}
O=gpurun_out
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline"        # default launch shape (64 frames per launch)
S="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --frames 1"   # one frame per launch
timeout -k 10 300 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err
timeout -k 10 300 python bench.py --steps 32 --warmup 8 --frames 1 --no-cpu-baseline > $O/bench_${TAG}_serial.json 2>> $O/bench_$TAG.err
# kernel trace of the bench's own default command (frames in flight) and of serial frames
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python bench.py --no-cpu-baseline > $O/prof_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_serial -o run -- $S > $O/prof_${TAG}_serial.log 2>&1
pass() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d $O/pmc_${TAG}_$name -o run -- $B > $O/pmc_${TAG}_$name.log 2>&1
}
# one block per pass, few counters each (a pass that over-subscribes a block aborts)
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass ta TA_BUSY_avr GRBM_GUI_ACTIVE
pass taaddr TA_ADDR_STALLED_BY_TC_CYCLES_sum
pass tadata TA_DATA_STALLED_BY_TC_CYCLES_sum
pass tcp1 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
pass tcp2 TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
pass tcc TCC_HIT_sum TCC_MISS_sum
pass td TD_TD_BUSY_sum
pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES
pass sq2 SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
PMC_CMD="$B" PMC_FRAMES=128 python tools/pmc_summary.py $O/pmc_$TAG.json $O/pmc_${TAG}_*/
echo "profile $TAG done"
