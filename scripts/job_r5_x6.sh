# round 5: fp32 chain products on split-plane bf16 MFMA (lcq_gemm_f32x6): tests, chain rate,
# per-product breakdown
set -o pipefail
O=gpurun_out/r5x6d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gptq_gpu.py -k "f32x6 or x6 or inverse_cholesky or gemm_f32 or trailing or column_loop or block" -v --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chol_chain_rate.py > $O/chain_rate.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chain_breakdown.py > $O/breakdown.txt 2>&1 || exit 1
