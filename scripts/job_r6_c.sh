# round 6 (c): token-lane auto-clip -- bit identity vs k_auto_clip and the reference fixtures,
# rate at the Llama-3-8B shapes; the BASELINE-shape GPTQ parity with its restated criteria
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_awq_gpu.py -k "auto_clip" -v --timeout 120 \
  --timeout-method thread > $O/clip_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python -u scripts/clip_rate.py > $O/clip_rate.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gptq_shapes_gpu.py -v -s --timeout 500 \
  --timeout-method thread > $O/gptq_shapes.log 2>&1
exit 0
