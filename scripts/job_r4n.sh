# GPTQ trailing update on the LDS-DMA fp32 GEMM (A k-major): GPTQ + multirank tests, column
# loop probe, GPTQ bench leg
set -o pipefail
OUT=gpurun_out/r4n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gptq_gpu.py tests/test_multirank_gpu.py tests/test_pipeline_golden_gpu.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/column_loop_rate.py > $OUT/column_loop.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > $OUT/bench_gptq.log 2>&1 || exit 1
