# GPTQ: core GPU tests + chain rate + the GPTQ bench leg with per-kernel stats
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gptq_gpu.py tests/test_multirank_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/gptq_test.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/chol_chain_rate.py > gpurun_out/chol_chain_rate.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --algo gptq --no-cpu-baseline > gpurun_out/bench_gptq.log 2>&1 || exit 1
