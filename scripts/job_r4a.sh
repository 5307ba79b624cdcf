# round 4 first check: full GPU suite on the env-switch-free package, then the default bench line
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/gputest.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py --no-e2e > gpurun_out/r4a/bench.log 2>&1 || exit 1
