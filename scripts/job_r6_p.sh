# round 6 (p): FETCH / WRITE / clock of hipBLASLt's kernel vs k_gemm16h at the o_proj and down
# shapes (is hipBLASLt's edge in its tile order's L2 locality?)
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp
for shp in "4096 4096" "4096 14336"; do
  set -- $shp; tag=n$1k$2
  for who in lcq torch; do
    timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_${who}_$tag -o run -- python3 scripts/gemm_one.py --n $1 --k $2 --only $who --iters 10 > $O/f_${who}_$tag.log 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/g_${who}_$tag -o run -- python3 scripts/gemm_one.py --n $1 --k $2 --only $who --iters 10 > $O/g_${who}_$tag.log 2>&1 || exit 1
    timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${who}_$tag -o run -- python3 scripts/gemm_one.py --n $1 --k $2 --only $who --iters 10 > $O/kt_${who}_$tag.log 2>&1 || exit 1
  done
done
# and the 3-deep B ring (k_gemm16t, probe build pp3): rates against the product and hipBLASLt,
# bit identity of every GEMM entry point
timeout -k 10 300 python -u scripts/gemm_rate.py --rounds 3 --iters 10 > $O/rate_default.txt 2>&1 || exit 1
LCQ_LIB_PATH=scripts/_lib/liblcq_pp3.so timeout -k 10 300 python -u scripts/gemm_rate.py --rounds 3 --iters 10 > $O/rate_pp3.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_pp_check.py > $O/digest_default.txt 2>&1 || exit 1
LCQ_LIB_PATH=scripts/_lib/liblcq_pp3.so timeout -k 10 300 python -u scripts/gemm_pp_check.py > $O/digest_pp3.txt 2>&1 || exit 1
