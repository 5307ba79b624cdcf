# round 5, call 10: GPTQ bench leg with the chain as a HIP graph vs eager
set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 900 python3 -u scripts/gptq_ab.py 2 > $O/gptq_ab.txt 2>&1 || exit 1
