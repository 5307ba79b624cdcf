# rehearsal of the driver's N > 1 bench path on one GPU: bench.py --gpus 2 starts its own two
# ranks (gloo, both on cuda:0); AWQ headline (shard_blocks ring + packed-shard gather) and
# the GPTQ leg (token shards)
mkdir -p gpurun_out
LCQ_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 2 --warmup 1 --algo both --no-cpu-baseline --no-e2e --gptq-steps 1 > gpurun_out/bench_n2.log 2>&1 || exit 1
