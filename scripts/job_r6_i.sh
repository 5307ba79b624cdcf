# round 6 (i): where the streamed GPTQ run's extra time goes: fresh pinned allocation cost,
# and the 32-block streamed run with the streamer's host-time counters
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 300 python -u scripts/pinned_alloc_probe.py > $O/pinned_alloc.txt 2>&1 || exit 1
timeout -k 10 600 python -u scripts/stream_gptq_probe.py 32 > $O/stream_probe32.txt 2>&1 || exit 1
