# fp8 leg with the calibration forward over all 32 routed experts of the rank: bench line,
# kernel stats, PMC traffic
set -o pipefail
OUT=gpurun_out/r4p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --algo fp8 --no-cpu-baseline > $OUT/bench_fp8.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_fp8 -o run \
  -- python3 bench.py --algo fp8 --no-cpu-baseline > $OUT/kt_fp8.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_fp8_$c -o run \
    -- python3 bench.py --algo fp8 --no-cpu-baseline --steps 1 --warmup 0 \
    > $OUT/pmc_fp8_$c.log 2>&1 || exit 1
done
python3 scripts/pmc_summary.py $OUT/pmc_fp8_FETCH_SIZE/run_counter_collection.csv \
  $OUT/pmc_fp8_WRITE_SIZE/run_counter_collection.csv $OUT/pmc_traffic_fp8.json \
  > $OUT/pmc_traffic_fp8.txt 2>&1 || exit 1
