mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_awq_gpu.py -x -q --timeout 120 --timeout-method thread -k "scale" > gpurun_out/scale_test.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/scale_ab.py > gpurun_out/scale_ab.log 2>&1 || exit 1
OUT=gpurun_out/gemm_diag_b bash scripts/gemm_diag.sh || exit 1
LCQ_FP8_GEMM=2 timeout -k 10 300 python -u scripts/fp8_gemm_rate.py > gpurun_out/fp8_rate_new_forced.log 2>&1 || exit 1
