# attention: XCD-aware work order (the workgroups sharing a K/V head on one XCD); tests, rate,
# FETCH and SQ counters at the AWQ shape (B 128, H 32, KV 8, S 512)
set -o pipefail
OUT=gpurun_out/r4u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -q -x -s --timeout 120 --timeout-method thread > $OUT/tests_attn.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/attn_rate.py > $OUT/attn_rate.txt 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 scripts/attn_rate.py 512 > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- python3 scripts/attn_rate.py 512 > $OUT/pmc_sq.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_pipeline_golden_gpu.py tests/test_awq_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
