# round 6 (d): token-lane auto-clip with pipelined scalar loads: bit identity and rate
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_awq_gpu.py -k "auto_clip" -v --timeout 120 \
  --timeout-method thread > $O/clip_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python -u scripts/clip_rate.py > $O/clip_rate.txt 2>&1 || exit 1
