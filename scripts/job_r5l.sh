# round 5, call 12: the tile kernel with scalar-loaded S3 job rows and X rows stored by wave 0
# -- its tests (product and fast-rsqrt probe libraries), stage timing, chain breakdown
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "chol or inverse_cholesky or static_plugin" > $O/chol_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2.so > $O/chol_tile_prof2.txt 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2_fast.so > $O/chol_tile_prof2_fast.txt 2>&1 || exit 1
LCQ_LIB_PATH=scripts/_lib/liblcq_fastrsq.so timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -q \
  --timeout 120 --timeout-method thread -k "chol or inverse_cholesky or static_plugin" > $O/chol_tests_fast.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
timeout -k 10 200 python3 -u scripts/chain_breakdown.py > $O/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chol_chain_rate.py > $O/chain_rate.txt 2>&1 || exit 1
