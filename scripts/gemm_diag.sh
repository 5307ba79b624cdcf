#!/bin/bash
# gemm_diag.py plain, then one PMC pass (wait / busy / clock counters) over the same run.
set -o pipefail
OUT=${OUT:-gpurun_out/gemm_diag}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/gemm_diag.py > $OUT/time.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 scripts/gemm_diag.py --rounds 1 --iters 3 > $OUT/pmc.log 2>&1 || exit 1
