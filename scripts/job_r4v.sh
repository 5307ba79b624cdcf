# fp32 recursion / trailing GEMMs: XCD-aware tile order (tiled and stream-K); tests, chain and
# column-loop rates, GPTQ bench leg
set -o pipefail
OUT=gpurun_out/r4v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_gptq_gpu.py tests/test_multirank_gpu.py -q -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chol_chain_rate.py > $OUT/chol_chain_rate.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/column_loop_rate.py > $OUT/column_loop_rate.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > $OUT/bench_gptq.log 2>&1 || exit 1
