# round 5: GPTQ leg A/B, chain products + far column-loop updates on lcq_gemm_f32x6 (X6=1) vs
# fp32 MFMA (X6=0), one box
set -o pipefail
O=gpurun_out/r5x6ab2
mkdir -p $O
A="--algo gptq --no-cpu-baseline --no-e2e --no-l70b --steps 3 --warmup 1"
for i in 1 2; do
timeout -k 10 400 python -u scripts/bench_with.py X6=1 -- $A > $O/on_$i.json 2> $O/on_$i.err || exit 1
timeout -k 10 400 python -u scripts/bench_with.py X6=0 -- $A > $O/off_$i.json 2> $O/off_$i.err || exit 1
done
