# round 5, call 1 (again): tile tests + stage timing probe + the fast-rsqrt probe library's
# accuracy, the streaming memory probe, the full GPU suite and the default bench line
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "chol or inverse_cholesky or static_plugin" > gpurun_out/r5a/chol_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py > gpurun_out/r5a/chol_tile_prof2.txt 2>&1 || exit 1
LCQ_LIB_PATH=scripts/_lib/liblcq_fastrsq.so timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -q \
  --timeout 120 --timeout-method thread -k "chol or static_plugin" > gpurun_out/r5a/chol_tests_fastrsq.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 200 python3 -u scripts/chain_breakdown.py > gpurun_out/r5a/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/stream_mem_probe.py > gpurun_out/r5a/stream_mem_probe.txt 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 5 \
  > gpurun_out/r5a/gputest_full.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5a/bench_default.log 2>&1 || exit 1
