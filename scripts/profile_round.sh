#!/bin/bash
# Round profiling on the GPU box (run via gpurun from the repo root). Stage A: default bench
# line + rocprofv3 kernel-trace stats per leg. Stage B: PMC HBM traffic (separate FETCH_SIZE /
# WRITE_SIZE passes per leg, MI355X_MICROARCH.md HBM section), summarised per launch.
set -o pipefail
TAG=${TAG:-r2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
stage=${1:-A}
if [ "$stage" = A ]; then
  timeout -k 10 600 python3 -u bench.py > $OUT/bench_default.log 2>&1 || exit 1
  for leg in awq gptq fp8; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$leg -o run \
      -- python3 bench.py --algo $leg --no-cpu-baseline > $OUT/kt_$leg.log 2>&1 || exit 1
  done
else
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
fi
