# round 5, call 15: the rotary GEMM epilogue (lcq_gemm_rope) -- GEMM / attention / AWQ /
# pipeline / model tests, then the AWQ and GPTQ legs of the bench
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 5 \
  -k "gemm or attention or awq or pipeline or models or llama or residency or multirank" > $O/tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 900 python3 -u bench.py --algo both --no-e2e --no-l70b --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
