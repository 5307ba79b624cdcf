# round 5, call 18: the dynamically claimed persistent GEMM (probe liblcq_d.so) vs the product
set -o pipefail
O=gpurun_out/r5r
mkdir -p $O
D=scripts/_lib/liblcq_d.so
timeout -k 10 300 python3 -u scripts/gemm_pp_check.py > $O/digest_p.txt 2>&1 || exit 1
LCQ_LIB_PATH=$D timeout -k 10 300 python3 -u scripts/gemm_pp_check.py > $O/digest_d.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_p_$r.txt 2>&1 || exit 1
  LCQ_LIB_PATH=$D timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_d_$r.txt 2>&1 || exit 1
done
