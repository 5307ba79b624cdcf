# round 6 (j): streamed residency with pinned reuse + ahead allocation: residency tests, the
# 32-block streamed GPTQ probe; the BASELINE-shape GPTQ parity numbers (-s)
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_residency_gpu.py -v --timeout 300 \
  --timeout-method thread > $O/residency_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 600 python -u scripts/stream_gptq_probe.py 32 > $O/stream_probe32.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gptq_shapes_gpu.py -v -s --timeout 500 \
  --timeout-method thread > $O/gptq_shapes.log 2>&1
exit 0
