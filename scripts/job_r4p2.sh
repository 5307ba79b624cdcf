# attention: 2 heads per 8-wave workgroup (probe build) vs the product build; product tests
set -o pipefail
OUT=gpurun_out/r4p2
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_attention_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/tests_attn.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/attn_hpw_probe.py run > $OUT/hpw.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/attn_rate.py > $OUT/attn_rate.txt 2>&1 || exit 1
