set -o pipefail
export TMPDIR=/tmp
L=my-raytracer_amd/lib/variants
O=gpurun_out
B="python bench.py --no-cpu-baseline --steps 128 --warmup 16"
timeout -k 10 600 python -u tools/ab_frame.py 3 $L/librt_hip_deep.so $L/librt_hip_nop16.so $L/librt_hip_valu16.so > $O/ab_sens.txt 2>&1 && tail -3 $O/ab_sens.txt &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU --output-format csv -d $O/pmc_mix_a -o run -- $B > $O/pmc_mix_a.log 2>&1 && echo A ok &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 --output-format csv -d $O/pmc_mix_b -o run -- $B > $O/pmc_mix_b.log 2>&1 && echo B ok &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_LDS --output-format csv -d $O/pmc_mix_c -o run -- $B > $O/pmc_mix_c.log 2>&1 && echo C ok
