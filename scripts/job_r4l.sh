# fp8: software-pipelined K-block accumulate (tests + per-projection rates + single-shape
# rates); chain with / without stream-K (2-stage ring); GPTQ bench
set -o pipefail
OUT=gpurun_out/r4l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/fp8test.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/fp8_grouped_rate.py > $OUT/fp8_grouped_rate.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/fp8_gemm_rate.py > $OUT/fp8_gemm_rate.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chol_chain_rate.py > $OUT/chol_chain_rate.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > $OUT/bench_gptq.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --no-cpu-baseline > $OUT/bench_fp8.log 2>&1 || exit 1
