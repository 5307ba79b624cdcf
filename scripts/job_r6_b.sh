# round 6 (b): BASELINE-shape GPTQ parity with the decomposed criteria, and the FP8 deploy
# per-layer host time at 3 / 20 layers after the gc.freeze fix
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gptq_shapes_gpu.py -v -s --timeout 500 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 600 python -u scripts/fp8_layers_probe.py 3 20 > $O/fp8_probe.log 2>&1 || exit 1
