# kernel-trace + PMC passes of the FP8 GEMM (DSv3 calibration shapes) and of the fp32 GEMM
# (GPTQ Cholesky recursion shapes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gemmprof
mkdir -p $O
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
for sh in "2048 2048 7168" "2048 7168 7168"; do
  tag=fp8_$(echo $sh | tr ' ' x)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$tag -o run -- python3 scripts/fp8_gemm_one.py $sh 20 > $O/kt_$tag.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p1_$tag -o run -- python3 scripts/fp8_gemm_one.py $sh 3 > $O/p1_$tag.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2_$tag -o run -- python3 scripts/fp8_gemm_one.py $sh 3 > $O/p2_$tag.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $SQ --output-format csv -d $O/p3_$tag -o run -- python3 scripts/fp8_gemm_one.py $sh 3 > $O/p3_$tag.log 2>&1 || exit 1
done
for sh in "7168 1792 1792 1" "1792 1792 1792 1" "7168 3584 3584 0" "4096 4096 4096 1"; do
  tag=f32_$(echo $sh | tr ' ' x)
  timeout -k 10 60 python3 scripts/f32_gemm_one.py $sh 10 > $O/rate_$tag.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $SQ --output-format csv -d $O/p3_$tag -o run -- python3 scripts/f32_gemm_one.py $sh 2 > $O/p3_$tag.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2_$tag -o run -- python3 scripts/f32_gemm_one.py $sh 2 > $O/p2_$tag.log 2>&1 || exit 1
done
