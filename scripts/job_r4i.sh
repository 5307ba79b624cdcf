# grouped fp8 GEMM: its tests, then the fp8 bench leg
set -o pipefail
OUT=gpurun_out/r4i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/fp8test.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --no-cpu-baseline > $OUT/bench_fp8.log 2>&1 || exit 1
