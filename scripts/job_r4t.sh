# attention: O held transposed (lane-local rescale / normalise, 8-byte epilogue LDS writes)
set -o pipefail
OUT=gpurun_out/r4t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -q -x -s --timeout 120 --timeout-method thread > $OUT/tests_attn.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/attn_rate.py > $OUT/attn_rate.txt 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_pipeline_golden_gpu.py tests/test_awq_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
