# round 6 (w): PMC of the LDS-candidate token-lane auto-clip kernel (k_auto_clip_tw) at the
# gate/up shape: VALU issue, waits, LDS instructions, clock; kernel trace split qtable / search
set -o pipefail
O=gpurun_out/r6w
mkdir -p $O
export TMPDIR=/tmp
for k in tw:14336; do
  kind=${k%%:*}; oc=${k##*:}
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $O/pmc_${kind}_1 -o run -- python3 scripts/clip_one.py $kind $oc > $O/pmc_${kind}_1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_${kind}_2 -o run -- python3 scripts/clip_one.py $kind $oc > $O/pmc_${kind}_2.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${kind} -o run -- python3 scripts/clip_one.py $kind $oc > $O/kt_${kind}.log 2>&1 || exit 1
done
