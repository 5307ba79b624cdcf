# round 6 (final): the full GPU suite, smoke and the driver bench command (--steps 20 --warmup 5)
# on the final code (k_auto_clip_tw automatic, left-looking column loop, small chain products)
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 5 \
  > $O/gputest_full.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_steps20.log 2>&1 || exit 1
