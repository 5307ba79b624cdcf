# round 4: residual-fused GEMM epilogue, register-resident rmsnorm, FP8 size-class requant
mkdir -p gpurun_out/r4f
ok() { rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_forward_fused_gpu.py tests/test_fp8_gpu.py tests/test_pipeline_golden_gpu.py tests/test_models_gpu.py tests/test_residency_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4f/tests.log 2>&1; ok
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > gpurun_out/r4f/bench_gptq.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --steps 5 > gpurun_out/r4f/bench_fp8.log 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo awq --no-cpu-baseline --steps 5 > gpurun_out/r4f/bench_awq.log 2>&1 || exit 1
