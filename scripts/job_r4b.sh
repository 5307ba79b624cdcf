# round 4: new residency / shard_units GPU tests first, then the full GPU suite
mkdir -p gpurun_out/r4b
timeout -k 10 600 python -u -m pytest tests/test_residency_gpu.py tests/test_l70b_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4b/residency.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4b/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --steps 5 > gpurun_out/r4b/bench_fp8.log 2>&1 || exit 1
