# attention tests incl. the odd workgroup-count cases
set -o pipefail
mkdir -p gpurun_out/r4w
timeout -k 10 200 python -u -m pytest tests/test_attention_gpu.py -q -x -s --timeout 120 --timeout-method thread > gpurun_out/r4w/tests_attn.log 2>&1
