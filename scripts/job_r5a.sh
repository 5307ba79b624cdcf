# round 5, call 1: the new diagonal-tile Cholesky kernel and the row-split chain first, then the
# full GPU suite, the chain breakdown and the default bench line (with the sampled GFX clock)
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "chol or inverse_cholesky or gather_rc or gemm_f32_rows" > gpurun_out/r5a/chol_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/chain_breakdown.py > gpurun_out/r5a/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5a/gputest_full.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5a/bench_default.log 2>&1 || exit 1
