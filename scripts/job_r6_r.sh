# round 6 (r): left-looking near updates in lcq_gptq_block: bit identity against the trailing
# launches, the GPTQ GPU tests (goldens, T2, sharded), the BASELINE-shape parity, column-loop
# rates, the GPTQ bench leg
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gptq_left_looking_gpu.py tests/test_gptq_gpu.py tests/test_gptq_shapes_gpu.py tests/test_multirank_gpu.py tests/test_pipeline_golden_gpu.py -v --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python -u scripts/column_loop_rate.py > $O/column_loop_rate.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py --algo gptq --no-cpu-baseline > $O/bench_gptq.log 2>&1 || exit 1
