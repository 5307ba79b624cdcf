# round 5, call 3: the restructured tile (load overlapped with S1(0), X streamed out per panel)
# -- its tests, stage timing (IEEE and hardware sqrt / rcp), the GPU suite on the product
# library and on the fast-rsqrt probe library, the streaming memory probe and the bench line
set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "chol or inverse_cholesky or static_plugin" > $O/chol_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2.so > $O/chol_tile_prof2.txt 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2_fast.so > $O/chol_tile_prof2_fast.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/stream_mem_probe.py > $O/stream_mem_probe.txt 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 5 \
  > $O/gputest_full.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
LCQ_LIB_PATH=scripts/_lib/liblcq_fastrsq.so timeout -k 10 800 python -u -m pytest tests -m gpu -q \
  --timeout 300 --timeout-method thread --maxfail 5 -k "gptq or chol or pipeline" > $O/gputest_fastrsq.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || exit 1
export TMPDIR=/tmp
ARGS="--m 65536 --n 14336 --k 4096 --iters 10 --only lcq"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gemm_kt -o run \
  -- python3 scripts/gemm_one.py $ARGS > $O/gemm_kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv \
  -d $O/gemm_pmc1 -o run -- python3 scripts/gemm_one.py $ARGS > $O/gemm_pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_INSTS_MFMA SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum --output-format csv \
  -d $O/gemm_pmc2 -o run -- python3 scripts/gemm_one.py $ARGS > $O/gemm_pmc2.log 2>&1 || exit 1
