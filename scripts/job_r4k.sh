# grouped fp8 pair mode tests; column-loop probe (host vs device, near pipeline, superblock);
# chain breakdown with the 2-stage fp32 GEMM ring; GPTQ + fp8 bench legs
set -o pipefail
OUT=gpurun_out/r4k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/fp8test.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/column_loop_rate.py > $OUT/column_loop.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chain_breakdown.py > $OUT/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > $OUT/bench_gptq.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --no-cpu-baseline > $OUT/bench_fp8.log 2>&1 || exit 1
