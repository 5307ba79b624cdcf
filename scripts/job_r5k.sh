# round 5, call 11: kernel trace of the GPTQ bench leg (graph chains) for the idle-gap analysis
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run \
  -- python3 -u bench.py --algo gptq --no-cpu-baseline --no-e2e --no-l70b --gptq-steps 2 > $O/bench.log 2>&1 || exit 1
