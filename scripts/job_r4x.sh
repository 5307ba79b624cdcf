# final library sanity: smoke + attention / AWQ / models tests
set -o pipefail
mkdir -p gpurun_out/r4x
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4x/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_awq_gpu.py tests/test_models_gpu.py tests/test_gptq_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r4x/tests.log 2>&1
