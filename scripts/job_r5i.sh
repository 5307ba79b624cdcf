# round 5, call 9: Hessian schedule A/B repeated (product / three-barrier probe, alternating
# processes), the chain rate, and the default bench line with the k_gemm16h product GEMM
set -o pipefail
O=gpurun_out/r5i
mkdir -p $O
SX=scripts/_lib/liblcq_sx3.so
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/hessian_grouped_rate.py > $O/rate_b_$r.txt 2>&1 || exit 1
  LCQ_LIB_PATH=$SX timeout -k 10 300 python3 -u scripts/hessian_grouped_rate.py > $O/rate_sx3_$r.txt 2>&1 || exit 1
done
timeout -k 10 300 python3 -u scripts/chol_chain_rate.py > $O/chain_rate.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || exit 1
