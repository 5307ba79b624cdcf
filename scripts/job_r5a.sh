# round 5, call 1: full GPU suite on the round's first changes, then the default bench line
# (now with the sampled GFX clock) and the chain breakdown (baseline for the tile kernel work)
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5a/gputest_full.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > gpurun_out/r5a/bench_default.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/chain_breakdown.py > gpurun_out/r5a/chain_breakdown.txt 2>&1 || exit 1
