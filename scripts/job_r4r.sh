# per-group auto-clip: weights kept in registers across passes; clip parity tests, clip and
# attention rates, clip SQ / FETCH counters
set -o pipefail
OUT=gpurun_out/r4r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_awq_gpu.py tests/test_clip_v2_gpu.py tests/test_fp8_algos_gpu.py tests/test_pipeline_golden_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/clip_rate.py > $OUT/clip_rate.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/attn_rate.py > $OUT/attn_rate.txt 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 scripts/clip_rate.py > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $OUT/pmc_sq -o run -- python3 scripts/clip_rate.py > $OUT/pmc_sq.log 2>&1 || exit 1
