# round 6, first call: the new BASELINE-shape GPTQ parity test, the x6 row-split test, smoke,
# and the FP8 deploy leg's per-layer host time at 3 and 20 layers
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gptq_shapes_gpu.py tests/test_multirank_gpu.py \
  -k "baseline_shape or chain_row_split" -v -s --timeout 600 --timeout-method thread \
  > $O/tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/fp8_layers_probe.py 3 20 > $O/fp8_probe.log 2>&1 || exit 1
