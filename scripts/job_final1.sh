# round-end call 1: full GPU suite, FP8 plan sweep, Cholesky chain probe
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_full.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/fp8_gemm_rate.py > gpurun_out/fp8_gemm_rate.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/chol_chain_rate.py > gpurun_out/chol_chain_rate.txt 2>&1 || exit 1
