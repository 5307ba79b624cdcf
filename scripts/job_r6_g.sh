# round 6 (g): state after the container restore -- full GPU suite, smoke, auto-clip rate
# (row-lane / token-lane / lane-pair), default bench line
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 5 \
  > $O/gputest_full.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/clip_rate.py > $O/clip_rate.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || exit 1
