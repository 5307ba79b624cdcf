# round 6 (l): streamed residency with host-copy recycling, ahead allocation and the dropped
# FakeQuantLinear.tmp_weight cache: residency tests (bit identity), 32-block streamed GPTQ
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_residency_gpu.py -v --timeout 300 \
  --timeout-method thread > $O/residency_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 600 python -u scripts/stream_gptq_probe.py 32 noprof > $O/stream_probe32.txt 2>&1 || exit 1
