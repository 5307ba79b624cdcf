#!/bin/bash
# PMC comparison of the lcq GEMM and hipBLASLt on one shape (separate passes, each bounded).
set -o pipefail
OUT=${OUT:-gpurun_out/gemm_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${ARGS:-"--m 65536 --n 4096 --k 4096 --iters 10"}
SETS=${SETS:-all}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 scripts/gemm_one.py $ARGS > $OUT/kt.log 2>&1 || exit 1
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 scripts/gemm_one.py $ARGS > $OUT/pmc$i.log 2>&1 || exit 1
done
