# round 6 (m): streamed residency with the host-copy pool fixed (exclusivity check), residency
# tests and the 32-block streamed GPTQ probe; the GEMM chunk-shape probe (LCQ_PROBE_GEMM_CM:
# tile rows per 32-tile XCD chunk) -- rates at the AWQ shapes and FETCH at the o_proj shape
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_residency_gpu.py -v --timeout 300 \
  --timeout-method thread > $O/residency_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 600 python -u scripts/stream_gptq_probe.py 32 noprof > $O/stream_probe32.txt 2>&1 || exit 1
for v in default cm2 cm8 cm16; do
  if [ $v = default ]; then L=""; else L="LCQ_LIB_PATH=scripts/_lib/liblcq_$v.so"; fi
  env $L timeout -k 10 300 python -u scripts/gemm_rate.py --rounds 3 --iters 10 > $O/rate_$v.txt 2>&1 || exit 1
done
for v in default cm2 cm8 cm16; do
  if [ $v = default ]; then unset LCQ_LIB_PATH; else export LCQ_LIB_PATH=scripts/_lib/liblcq_$v.so; fi
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o run -- python3 scripts/gemm_one.py --only lcq --iters 10 > $O/pmc_$v.log 2>&1 || exit 1
done
unset LCQ_LIB_PATH
exit 0
