# full GPU suite, then the round profile (default bench line + per-leg kernel-trace stats)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_full.log 2>&1 || exit 1
TAG=${TAG:-r2s3} bash scripts/profile_round.sh A || exit 1
