# round 5, call 7: the persistent cross-tile-prefetch GEMM (probe liblcq_s.so) and the
# three-barrier one (liblcq_h.so): tests, digests, rates, o_proj-shape PMC
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
S=scripts/_lib/liblcq_s.so
H=scripts/_lib/liblcq_h.so
LCQ_LIB_PATH=$S timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 120 \
  --timeout-method thread > $O/gemm_tests_s.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python3 -u scripts/gemm_pp_check.py > $O/digest_b.txt 2>&1 || exit 1
LCQ_LIB_PATH=$S timeout -k 10 300 python3 -u scripts/gemm_pp_check.py > $O/digest_s.txt 2>&1 || exit 1
LCQ_LIB_PATH=$S timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_s.txt 2>&1 || exit 1
LCQ_LIB_PATH=$H timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_h.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_b.txt 2>&1 || exit 1
export TMPDIR=/tmp
ARGS="--m 65536 --n 4096 --k 4096 --iters 20 --only lcq"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
LCQ_LIB_PATH=$S timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_s -o run \
  -- python3 scripts/gemm_one.py $ARGS > $O/kt_s.log 2>&1 || exit 1
LCQ_LIB_PATH=$S timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/p1_s -o run \
  -- python3 scripts/gemm_one.py $ARGS > $O/p1_s.log 2>&1 || exit 1
