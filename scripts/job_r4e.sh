# round 4: stream-K fp32 GEMM -- tests, chain breakdown and rates, GPTQ + FP8 legs
mkdir -p gpurun_out/r4e
ok() { rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gptq_gpu.py tests/test_pipeline_golden_gpu.py -k "gemm_f32 or cholesky or gptq" -v --timeout 200 --timeout-method thread > gpurun_out/r4e/tests.log 2>&1; ok
timeout -k 10 300 python -u scripts/chain_breakdown.py > gpurun_out/r4e/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/chol_chain_rate.py > gpurun_out/r4e/chol_chain_rate.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > gpurun_out/r4e/bench_gptq.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --steps 5 > gpurun_out/r4e/bench_fp8.log 2>&1 || exit 1
