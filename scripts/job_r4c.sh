# round 4: residency + GPTQ (fused gather, one-launch grouped Hessian) tests, chain breakdown,
# GPTQ and FP8 bench legs. A test assertion (pytest rc 1) does not stop the job; a crash,
# abort or time limit does.
mkdir -p gpurun_out/r4c
ok() { rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_residency_gpu.py tests/test_gptq_gpu.py tests/test_multirank_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4c/tests.log 2>&1; ok
timeout -k 10 300 python -u scripts/chain_breakdown.py > gpurun_out/r4c/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > gpurun_out/r4c/bench_gptq.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --algo fp8 --steps 5 > gpurun_out/r4c/bench_fp8.log 2>&1 || exit 1
