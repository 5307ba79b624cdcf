# round-4 final (after the clip / attention changes), part 1: full GPU suite, default bench line
set -o pipefail
OUT=gpurun_out/r4y
mkdir -p $OUT
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1; ok
timeout -k 10 600 python3 -u bench.py > $OUT/bench_default.log 2>&1 || exit 1
