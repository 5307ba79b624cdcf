# round 5, call 4: the 8-wave ping-pong projection GEMM (probe library liblcq_pp.so) against
# the product k_gemm16b -- GEMM tests on both, bit-identity digests, rates at the AWQ shapes
set -o pipefail
O=gpurun_out/r5d
mkdir -p $O
PP=scripts/_lib/liblcq_pp.so
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $O/gemm_tests.log 2>&1 || exit 1
LCQ_LIB_PATH=$PP timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -q --timeout 120 \
  --timeout-method thread > $O/gemm_tests_pp.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python3 -u scripts/gemm_pp_check.py > $O/digest_b.txt 2>&1 || exit 1
LCQ_LIB_PATH=$PP timeout -k 10 300 python3 -u scripts/gemm_pp_check.py > $O/digest_pp.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_b.txt 2>&1 || exit 1
LCQ_LIB_PATH=$PP timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_pp.txt 2>&1 || exit 1
export TMPDIR=/tmp
ARGS="--m 65536 --n 14336 --k 4096 --iters 10 --only lcq"
LCQ_LIB_PATH=$PP timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gemm_kt_pp -o run \
  -- python3 scripts/gemm_one.py $ARGS > $O/gemm_kt_pp.log 2>&1 || exit 1
LCQ_LIB_PATH=$PP timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv \
  -d $O/gemm_pmc1_pp -o run -- python3 scripts/gemm_one.py $ARGS > $O/gemm_pmc1_pp.log 2>&1 || exit 1
