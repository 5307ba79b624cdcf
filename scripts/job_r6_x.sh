# round 6 (x): k_auto_clip_tw automatic: auto-clip tests, prefetch depth two chunks (product) vs
# three (probe LCQ_PROBE_TW_DEEP), and the AWQ bench leg
set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_awq_gpu.py -v --timeout 120 --timeout-method thread -x > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/clip_rate.py > $O/clip_rate_product.txt 2>&1 || exit 1
LCQ_LIB_PATH=scripts/_lib/liblcq_twdeep.so timeout -k 10 300 python -u scripts/clip_rate.py > $O/clip_rate_deep.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py --algo awq --no-cpu-baseline > $O/bench_awq.log 2>&1 || exit 1
