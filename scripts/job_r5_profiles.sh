# Round 5: the GPU commands behind profiles/r5_* (run from the repo root through gpurun; build
# the probe libraries first on the CPU side:
#   python scripts/probe_build.py b LCQ_PROBE_GEMM_PP=0          # the r4 GEMM body
#   python scripts/probe_build.py ieee LCQ_PROBE_CHOL_IEEE_RSQ=1  # IEEE sqrt / div in the tile
#   scripts/build_chol_prof.sh                                   # tile stage-stamp libraries
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
O=gpurun_out/r5_profiles
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; timeout -k 10 "$t" "$@" || exit 1; }
# r5_gemm_variants.md / r5_gemm_rate_{b,h}.txt: product (k_gemm16h) vs r4 body, digests + rates
step 300 python3 -u scripts/gemm_pp_check.py > $O/gemm_digest_h.txt 2>&1
LCQ_LIB_PATH=scripts/_lib/liblcq_b.so step 300 python3 -u scripts/gemm_pp_check.py > $O/gemm_digest_b.txt 2>&1
step 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/gemm_rate_h.txt 2>&1
LCQ_LIB_PATH=scripts/_lib/liblcq_b.so step 300 python3 -u scripts/gemm_rate.py --rounds 3 > $O/gemm_rate_b.txt 2>&1
# the o_proj-shape PMC of the product GEMM and of hipBLASLt (r5_gemm_variants.md table)
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for who in lcq torch; do
  timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $O/gemm_p1_$who -o run \
    -- python3 scripts/gemm_one.py --m 65536 --n 4096 --k 4096 --iters 20 --only $who \
    > $O/gemm_p1_$who.log 2>&1 || exit 1
done
# r5_chol_tile_stages{,_ieee}.txt, r5_chain_breakdown.txt, r5_chain_rate.txt
step 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2.so > $O/chol_tile_stages.txt 2>&1
step 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2_ieee.so > $O/chol_tile_stages_ieee.txt 2>&1
step 200 python3 -u scripts/chain_breakdown.py > $O/chain_breakdown.txt 2>&1
step 300 python3 -u scripts/chol_chain_rate.py > $O/chain_rate.txt 2>&1
# r5_hessian_schedule_ab.txt: grouped / per-group Hessian rates (product schedule choice)
step 300 python3 -u scripts/hessian_grouped_rate.py > $O/hessian_rate.txt 2>&1
step 300 python3 -u scripts/hessian_digest.py > $O/hessian_digest.txt 2>&1
# r5_gptq_graph_ab.txt and r5_gptq_block_gaps.txt (python3 scripts/trace_gaps.py on the trace)
step 900 python3 -u scripts/gptq_ab.py 2 > $O/gptq_graph_ab.txt 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/gptq_kt -o run \
  -- python3 -u bench.py --algo gptq --no-cpu-baseline --no-e2e --no-l70b --gptq-steps 2 \
  > $O/gptq_kt.log 2>&1 || exit 1
