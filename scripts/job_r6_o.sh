# round 6 (o): full GPU suite, smoke, default bench line after the streaming changes
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 5 \
  > $O/gputest_full.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || exit 1
