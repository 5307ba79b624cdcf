# round 6 (e): PMC of the token-lane auto-clip vs k_auto_clip at the gate shape
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp
for k in tl pair; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$k -o run -- python3 scripts/clip_one.py $k > $O/kt_$k.log 2>&1 || exit 1
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM" \
             "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc_${k}_$i -o run -- python3 scripts/clip_one.py $k > $O/pmc_${k}_$i.log 2>&1 || exit 1
  done
done
timeout -s KILL 60 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES --output-format csv -d $O/pmc_tl_sqc -o run -- python3 scripts/clip_one.py tl > $O/pmc_tl_sqc.log 2>&1
exit 0
