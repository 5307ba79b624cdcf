# round 6 (n): streamed fake-quant deploy from the FakeQuantLinear memos (no HBM pass):
# residency tests (bit identity, 7 modules per block built on the host), 32-block probe
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_residency_gpu.py tests/test_pipeline_golden_gpu.py -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 600 python -u scripts/stream_gptq_probe.py 32 noprof > $O/stream_probe32.txt 2>&1 || exit 1
