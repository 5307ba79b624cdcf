# round 6 (sb): lcq_scale_bcast with 8 rows in flight per thread (probe LCQ_PROBE_SB_STEP=8) vs 4
set -o pipefail
O=gpurun_out/r6sb
mkdir -p $O
timeout -k 10 120 python -u scripts/scale_rate.py > $O/product.txt 2>&1 || exit 1
LCQ_LIB_PATH=scripts/_lib/liblcq_sb8.so timeout -k 10 120 python -u scripts/scale_rate.py > $O/sb8.txt 2>&1 || exit 1
