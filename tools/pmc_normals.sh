#!/bin/bash
# SQ counters of the normals kernel (separate passes, kernel-trace only).
set -u
OUT=gpurun_out/pmc_normals; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/prep_only.py 65 2 > $OUT/plain.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_BRANCH" \
           "SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex normals --output-format csv -d $OUT/p$i -o run -- python3 tools/prep_only.py 65 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
cat $OUT/plain.log
