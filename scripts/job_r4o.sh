# diagonal tile kernel with 4-column panels: GPTQ tests, chain rate, GPTQ bench
set -o pipefail
OUT=gpurun_out/r4o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gptq_gpu.py tests/test_pipeline_golden_gpu.py -q -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chol_chain_rate.py > $OUT/chol_chain_rate.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chain_breakdown.py > $OUT/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > $OUT/bench_gptq.log 2>&1 || exit 1
