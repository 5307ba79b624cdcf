# round 6 (q): two-barrier K-tile schedule probe (ktile16e, probe build pp4) vs the product:
# rates (two alternating rounds), digests of every GEMM entry point, cycles / waits at o_proj
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python -u scripts/gemm_rate.py --rounds 3 --iters 10 > $O/rate_default_$r.txt 2>&1 || exit 1
  LCQ_LIB_PATH=scripts/_lib/liblcq_pp4.so timeout -k 10 300 python -u scripts/gemm_rate.py --rounds 3 --iters 10 > $O/rate_pp4_$r.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u scripts/gemm_pp_check.py > $O/digest_default.txt 2>&1 || exit 1
LCQ_LIB_PATH=scripts/_lib/liblcq_pp4.so timeout -k 10 300 python -u scripts/gemm_pp_check.py > $O/digest_pp4.txt 2>&1 || exit 1
export LCQ_LIB_PATH=scripts/_lib/liblcq_pp4.so
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/g_pp4 -o run -- python3 scripts/gemm_one.py --only lcq --iters 10 > $O/g_pp4.log 2>&1 || exit 1
