# FP8 GEMM parity + MFMA precision probe + rate (tile plans of fp8_gemm.hip)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -k "gemm or fp8_linear" -q --timeout 120 --timeout-method thread > gpurun_out/fp8gemm_test.log 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc   # test failures (1) go on to the probes; crashes / timeouts stop here
timeout -k 10 120 python -u scripts/fp8_mfma_precision.py > gpurun_out/fp8_mfma_precision.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/fp8_gemm_rate.py > gpurun_out/fp8_gemm_rate.txt 2>&1 || exit 1
