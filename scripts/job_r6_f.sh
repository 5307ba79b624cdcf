# round 6 (f): row-lane auto-clip (tokens as scalar operands): bit identity, rate, PMC
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_awq_gpu.py -k "auto_clip" -v --timeout 120 \
  --timeout-method thread > $O/clip_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 400 python -u scripts/clip_rate.py > $O/clip_rate.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d $O/pmc_rl_1 -o run -- python3 scripts/clip_one.py tl > $O/pmc_rl_1.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_rl_2 -o run -- python3 scripts/clip_one.py tl > $O/pmc_rl_2.log 2>&1
exit 0
