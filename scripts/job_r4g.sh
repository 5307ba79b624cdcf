# round 4: overlapped AWQ clip (bit-identity + headline), FP8 deploy leg
mkdir -p gpurun_out/r4g
ok() { rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_awq_gpu.py tests/test_multirank_gpu.py tests/test_clip_v2_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4g/tests.log 2>&1; ok
timeout -k 10 400 python3 -u bench.py --algo awq --no-cpu-baseline --steps 10 > gpurun_out/r4g/bench_awq.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --steps 5 > gpurun_out/r4g/bench_fp8.log 2>&1 || exit 1
