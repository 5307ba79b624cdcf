# fp32 recursion GEMM: parity (both kernels) + rates at the recursion's shapes; GPTQ core tests
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -k "gemm_f32 or chol or hessian_prepare or inverse" -q --timeout 120 --timeout-method thread > gpurun_out/f32gemm_test.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
for sh in "7168 1792 1792 1" "1792 1792 1792 1" "7168 3584 3584 0" "3584 7168 3584 1" "4096 4096 4096 1" "1024 1024 1024 1" "2048 1024 1024 0"; do
  timeout -k 10 60 python3 scripts/f32_gemm_one.py $sh 10 >> gpurun_out/f32_gemm_rate.txt 2>&1 || exit 1
done
