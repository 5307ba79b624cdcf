# round 6 (v): auto-clip token-lane kernel with LDS-staged candidates (k_auto_clip_tw, variant 3):
# bit-identity against k_auto_clip, then the rate at the Llama-3-8B shapes
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_awq_gpu.py -k "scalar_operand or auto_clip" -v --timeout 120 --timeout-method thread -x > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/clip_rate.py > $O/clip_rate.txt 2>&1 || exit 1
