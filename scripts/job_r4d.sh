# round 4: XCD-interleaved grouped SYRK -- correctness, rate vs the per-group form, GPTQ leg
mkdir -p gpurun_out/r4d
ok() { rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -k "hessian or grouped or gather" -v --timeout 200 --timeout-method thread > gpurun_out/r4d/tests.log 2>&1; ok
timeout -k 10 300 python -u scripts/hessian_grouped_rate.py > gpurun_out/r4d/hess_rate.txt 2>&1 || exit 1
for gns in 1 2 3 4; do
  LCQ_SYRK_GNS=$gns timeout -k 10 300 python -u scripts/hessian_grouped_rate.py > gpurun_out/r4d/hess_rate_gns$gns.txt 2>&1 || exit 1
done
timeout -k 10 400 python3 -u bench.py --algo gptq --no-cpu-baseline > gpurun_out/r4d/bench_gptq.log 2>&1 || exit 1
