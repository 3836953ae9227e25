#!/bin/bash
# Profiles bench.py on the GPU box (dev tool, run under gpurun):
#   the bench line, rocprofv3 --kernel-trace --stats of the same command, separate --pmc
#   passes (one block per pass), the FETCH_SIZE/WRITE_SIZE calibration (tools/hbm_calib.bin),
#   and the per-frame PMC summary bench.py reads for roofline.traffic.
# usage: tools/profile_round.sh TAG [bench args...]      (outputs under gpurun_out/prof_TAG*)
set -e -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --tree-record off $*"
timeout -k 10 300 $B > $O/bench_$TAG.json 2> $O/bench_$TAG.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- $B > $O/prof_$TAG.log 2>&1
# the traced run prints its own bench line: compare per-shape kernel durations with its HIP events
grep '^{' $O/prof_$TAG.log | tail -1 > $O/prof_${TAG}_bench.json
python tools/trace_summary.py $O/trace_$TAG.json $O/prof_$TAG $O/prof_${TAG}_bench.json > /dev/null
# PASSES (optional): the pass names to run (default all); the summary takes the passes that ran
PASSES=${PASSES:-fetch write td ta tcc tcp sq sqa valu}
pass() {
  local name=$1; shift
  case " $PASSES " in *" $name "*) ;; *) return 0 ;; esac
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $O/pmc_${TAG}_$name -o run -- $B > $O/pmc_${TAG}_$name.log 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass td TD_TD_BUSY_sum GRBM_GUI_ACTIVE
pass ta TA_BUSY_avr
pass tcc TCC_HIT_sum TCC_MISS_sum
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU
# where a wave's cycles go (bench.py wave_cycles) and the VALU mix
pass sqa SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM
pass valu SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32
# FETCH_SIZE/WRITE_SIZE access-width calibration: the committed one (CALIB=...), else measured here
CAL=${CALIB:-$O/hbm_calib.json}
if [ ! -f $CAL ]; then
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_fetch -o run -- ./tools/hbm_calib.bin > $O/calib_fetch.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib_write -o run -- ./tools/hbm_calib.bin > $O/calib_write.log 2>&1
  python tools/calib_summary.py $CAL $O/calib_fetch $O/calib_write > /dev/null
fi
# (the passes of this tag only: a glob pmc_${TAG}_*/ would also take those of a tag that extends it)
python tools/pmc_summary.py $O/pmc_$TAG.json --bench $O/bench_$TAG.json --calib $CAL \
  $(for p in $PASSES; do echo $O/pmc_${TAG}_$p; done)
echo "profile $TAG done"
