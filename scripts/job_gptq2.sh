# GPTQ in-block kernel + scale broadcast (div_exact) parity, then the GPTQ bench leg
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gptq_gpu.py tests/test_awq_gpu.py tests/test_pipeline_golden_gpu.py tests/test_fp8_algos_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/gptq2_test.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --algo gptq --no-cpu-baseline > gpurun_out/bench_gptq.log 2>&1 || exit 1
