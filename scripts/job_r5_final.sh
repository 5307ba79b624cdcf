# round 5, final (3): the full GPU suite, smoke, the default bench line and the per-leg
# kernel-trace stats on the final code (chain products and far GPTQ updates on split-plane bf16 MFMA, lcq_gemm_f32x6)
set -o pipefail
O=gpurun_out/r5final5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 5 \
  > $O/gputest_full.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
TAG=r5e timeout -k 10 1500 bash scripts/profile_round.sh A || exit 1
