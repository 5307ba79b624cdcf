# round 5, call 5: PMC of the projection GEMM (lcq k_gemm16b, the ping-pong probe and
# hipBLASLt through F.linear) at the o_proj shape 65536 x 4096 x 4096
set -o pipefail
O=gpurun_out/r5e
mkdir -p $O
export TMPDIR=/tmp
PP=scripts/_lib/liblcq_pp.so
ARGS="--m 65536 --n 4096 --k 4096 --iters 20"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum"
for who in lcq torch; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$who -o run \
    -- python3 scripts/gemm_one.py $ARGS --only $who > $O/kt_$who.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/p1_$who -o run \
    -- python3 scripts/gemm_one.py $ARGS --only $who > $O/p1_$who.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $O/p2_$who -o run \
    -- python3 scripts/gemm_one.py $ARGS --only $who > $O/p2_$who.log 2>&1 || exit 1
done
LCQ_LIB_PATH=$PP timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_pp -o run \
  -- python3 scripts/gemm_one.py $ARGS --only lcq > $O/kt_pp.log 2>&1 || exit 1
LCQ_LIB_PATH=$PP timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/p1_pp -o run \
  -- python3 scripts/gemm_one.py $ARGS --only lcq > $O/p1_pp.log 2>&1 || exit 1
