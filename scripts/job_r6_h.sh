# round 6 (h): automatic auto-clip choice (token-lane below 65536 row-groups, lane-pair above):
# bit identity, rates, a PMC pass of both kernels; the streamed-GPTQ probe; the default bench
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_awq_gpu.py -k "auto_clip" -v --timeout 120 \
  --timeout-method thread > $O/clip_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
for k in pair:14336 tl:1024; do
  kind=${k%%:*}; oc=${k##*:}
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $O/pmc_${kind}_1 -o run -- python3 scripts/clip_one.py $kind $oc > $O/pmc_${kind}_1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM --output-format csv -d $O/pmc_${kind}_2 -o run -- python3 scripts/clip_one.py $kind $oc > $O/pmc_${kind}_2.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${kind} -o run -- python3 scripts/clip_one.py $kind $oc > $O/kt_${kind}.log 2>&1 || exit 1
done
timeout -k 10 600 python -u scripts/stream_gptq_probe.py 8 > $O/stream_probe.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > $O/bench_default.log 2>&1 || exit 1
