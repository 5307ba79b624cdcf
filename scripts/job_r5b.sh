# round 5, call 2: projection-GEMM stall / clock counters (one SQ pass + the kernel trace) on the
# AWQ gate-sized shape, and the AWQ / GPTQ per-leg kernel stats of the current code
set -o pipefail
OUT=gpurun_out/r5b
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--m 65536 --n 14336 --k 4096 --iters 10 --only lcq"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gemm_kt -o run \
  -- python3 scripts/gemm_one.py $ARGS > $OUT/gemm_kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv \
  -d $OUT/gemm_pmc1 -o run -- python3 scripts/gemm_one.py $ARGS > $OUT/gemm_pmc1.log 2>&1 || exit 1
for leg in awq gptq; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$leg -o run \
    -- python3 bench.py --algo $leg --no-cpu-baseline > $OUT/kt_$leg.log 2>&1 || exit 1
done
