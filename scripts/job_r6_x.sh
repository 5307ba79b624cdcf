# round 6 (x): k_auto_clip_tw prefetch depth: two chunks (product) vs three (probe LCQ_PROBE_TW_DEEP)
set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 300 python -u scripts/clip_rate.py > $O/clip_rate_product.txt 2>&1 || exit 1
LCQ_LIB_PATH=scripts/_lib/liblcq_twdeep.so timeout -k 10 300 python -u scripts/clip_rate.py > $O/clip_rate_deep.txt 2>&1 || exit 1
