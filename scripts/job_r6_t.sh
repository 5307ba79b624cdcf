# round 6 (t): small chain products on k_gemm_f32_small (32 x 32 tiles from registers):
# GPTQ tests (fp32 GEMM vs torch, inverse Cholesky vs fp64, goldens, BASELINE-shape parity,
# sharded chains), chain breakdown and rates, the GPTQ bench leg
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gptq_gpu.py tests/test_gptq_shapes_gpu.py tests/test_multirank_gpu.py tests/test_pipeline_golden_gpu.py tests/test_l70b_gpu.py -v -s --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python -u scripts/chain_breakdown.py > $O/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/chol_chain_rate.py > $O/chain_rate.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py --algo gptq --no-cpu-baseline > $O/bench_gptq.log 2>&1 || exit 1
