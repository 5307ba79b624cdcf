# combine ordering change: fp8 GPU tests
set -o pipefail
OUT=gpurun_out/r4q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
