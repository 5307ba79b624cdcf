# fp8 body reverted (rates + tests); packed-U GPTQ block kernel (GPTQ tests); fp8 deploy leg
# host profile; GPTQ and fp8 bench legs
set -o pipefail
OUT=gpurun_out/r4m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_gptq_gpu.py -q -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/fp8_gemm_rate.py > $OUT/fp8_gemm_rate.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/fp8_grouped_rate.py > $OUT/fp8_grouped_rate.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u -m cProfile -o $OUT/fp8.prof bench.py --algo fp8 --no-cpu-baseline > $OUT/bench_fp8.log 2>&1 || exit 1
python3 scripts/prof_top.py $OUT/fp8.prof 40 > $OUT/fp8_prof.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > $OUT/bench_gptq.log 2>&1 || exit 1
