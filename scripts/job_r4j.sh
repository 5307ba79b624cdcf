# grouped fp8 (gather, two sets, combine), pipelined GPTQ near updates, token-sharded static
# act qparams; fp32 GEMM ring / occupancy probe; fp8 + gptq bench legs
set -o pipefail
OUT=gpurun_out/r4j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/fp8test.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gptq_gpu.py tests/test_multirank_gpu.py -q -x --timeout 300 --timeout-method thread > $OUT/gptqtest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/f32_variants.py run > $OUT/f32_variants.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --no-cpu-baseline > $OUT/bench_fp8.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > $OUT/bench_gptq.log 2>&1 || exit 1
