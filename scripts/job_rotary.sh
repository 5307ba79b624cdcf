# rotary table without the K=1 vendor GEMM: pipeline / model parity, then the GPTQ leg's
# kernel trace checked for Cijk_* kernels
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_pipeline_golden_gpu.py tests/test_models_gpu.py tests/test_pipeline_gpu.py tests/test_forward_fused_gpu.py -q -x --timeout 250 --timeout-method thread > gpurun_out/rotary_test.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_gptq_final -o run -- python3 bench.py --algo gptq --no-cpu-baseline > gpurun_out/kt_gptq_final.log 2>&1 || exit 1
