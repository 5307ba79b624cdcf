# round 6 (y): k_auto_clip_tw with the accumulation on v_dot2_f32_bf16 (variant 4) vs the
# packed form (variant 3): bit identity and rates
set -o pipefail
O=gpurun_out/r6y2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_awq_gpu.py -k "scalar_operand" -v --timeout 120 --timeout-method thread -x > $O/tests.log 2>&1
timeout -k 10 300 python -u scripts/clip_rate.py > $O/clip_rate.txt 2>&1 || exit 1
