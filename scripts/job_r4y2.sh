# round-4 final (after the clip / attention changes), part 2: per-leg kernel stats, streamed-residency copy/compute trace, PMC HBM
# traffic per leg (separate FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md HBM section)
set -o pipefail
OUT=gpurun_out/r4y
mkdir -p $OUT
export TMPDIR=/tmp
for leg in awq gptq fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$leg -o run \
    -- python3 bench.py --algo $leg --no-cpu-baseline > $OUT/kt_$leg.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/stream -o run \
  -- python3 scripts/stream_e2e.py 4 > $OUT/stream.log 2>&1 || exit 1
python3 scripts/copy_overlap.py $OUT/stream > $OUT/stream_overlap.txt 2>&1 || exit 1
for leg in awq gptq fp8; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${leg}_$c -o run \
      -- python3 bench.py --algo $leg --no-cpu-baseline --steps 1 --warmup 0 --gptq-steps 1 \
      > $OUT/pmc_${leg}_$c.log 2>&1 || exit 1
  done
  python3 scripts/pmc_summary.py $OUT/pmc_${leg}_FETCH_SIZE/run_counter_collection.csv \
    $OUT/pmc_${leg}_WRITE_SIZE/run_counter_collection.csv $OUT/pmc_traffic_$leg.json \
    > $OUT/pmc_traffic_$leg.txt 2>&1 || exit 1
done
