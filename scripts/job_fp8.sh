mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp8_test.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/fp8_gemm_rate.py > gpurun_out/fp8_rate.log 2>&1 || exit 1
LCQ_FP8_GEMM=1 timeout -k 10 300 python -u scripts/fp8_gemm_rate.py > gpurun_out/fp8_rate_old.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_l70b_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sub_test2.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_rate.py --variants="-,LCQ_GEMM_KERNEL=a" --rounds 5 > gpurun_out/gemm_rate_wide.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/hessian_rate.py > gpurun_out/hessian_rate.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/clip_ab.py > gpurun_out/clip_ab.log 2>&1 || exit 1
