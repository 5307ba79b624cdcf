# Hessian SYRK counters: LDS conflicts / MFMA busy / waits, and L2 hits, at IC 4096 and 14336
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hessprof
mkdir -p $O
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
for ic in 4096 14336; do
  timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv -d $O/p3_$ic -o run -- python3 scripts/hessian_rate.py --n 65536 --ics $ic --rounds 1 --iters 1 > $O/p3_$ic.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2_$ic -o run -- python3 scripts/hessian_rate.py --n 65536 --ics $ic --rounds 1 --iters 1 > $O/p2_$ic.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$ic -o run -- python3 scripts/hessian_rate.py --n 262144 --ics $ic --rounds 1 --iters 3 > $O/kt_$ic.log 2>&1 || exit 1
done
