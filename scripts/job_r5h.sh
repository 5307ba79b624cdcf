# round 5, call 8: the three-barrier Hessian schedule (probe liblcq_sx3.so): Hessian tests,
# bit-identity digests against the product schedule, grouped-Hessian rates; the product GEMM
# (k_gemm16h) through the AWQ / GEMM GPU tests
set -o pipefail
O=gpurun_out/r5h
mkdir -p $O
SX=scripts/_lib/liblcq_sx3.so
LCQ_LIB_PATH=$SX timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py tests/test_l70b_gpu.py -q \
  --timeout 120 --timeout-method thread -k "hessian" > $O/hess_tests_sx3.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python3 -u scripts/hessian_digest.py > $O/digest_b.txt 2>&1 || exit 1
LCQ_LIB_PATH=$SX timeout -k 10 300 python3 -u scripts/hessian_digest.py > $O/digest_sx3.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/hessian_grouped_rate.py > $O/rate_b.txt 2>&1 || exit 1
LCQ_LIB_PATH=$SX timeout -k 10 300 python3 -u scripts/hessian_grouped_rate.py > $O/rate_sx3.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_awq_gpu.py tests/test_pipeline_gpu.py tests/test_pipeline_golden_gpu.py -q \
  --timeout 300 --timeout-method thread > $O/awq_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
