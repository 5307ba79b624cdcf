# round 5: x / s with the bf16 rounding on the conversion instruction (k_scale_bcast): AWQ
# tests and the AWQ leg's kernel trace
set -o pipefail
O=gpurun_out/r5scale
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_awq_gpu.py -q --timeout 300 --timeout-method thread -x > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --algo awq --no-cpu-baseline --no-e2e --no-l70b > $O/bench.log 2>&1 || exit 1
