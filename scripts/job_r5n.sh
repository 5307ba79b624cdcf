# round 5, call 14: MFMA issue order inside the k_gemm16h k half (probe liblcq_nout.so, B-
# fragment-major) against the product order; digests + rates, alternating processes
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
N=scripts/_lib/liblcq_nout.so
timeout -k 10 300 python3 -u scripts/gemm_pp_check.py > $O/digest_p.txt 2>&1 || exit 1
LCQ_LIB_PATH=$N timeout -k 10 300 python3 -u scripts/gemm_pp_check.py > $O/digest_n.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_p_$r.txt 2>&1 || exit 1
  LCQ_LIB_PATH=$N timeout -k 10 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/rate_n_$r.txt 2>&1 || exit 1
done
