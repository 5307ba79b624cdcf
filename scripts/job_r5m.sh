# round 5, call 13: the tile kernel with X rows stored after S3 from registers, hardware
# sqrt / rcp as the product (IEEE probe library beside it): tests, stage timing, chain rates,
# and the GPTQ tests on both libraries
set -o pipefail
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "chol or inverse_cholesky or static_plugin" > $O/chol_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2.so > $O/chol_tile_prof2.txt 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2_ieee.so > $O/chol_tile_prof2_ieee.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/chain_breakdown.py > $O/chain_breakdown.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chol_chain_rate.py > $O/chain_rate.txt 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --maxfail 5 \
  -k "gptq or chol or pipeline or multirank or l70b" > $O/gptq_tests.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
LCQ_LIB_PATH=scripts/_lib/liblcq_ieee.so timeout -k 10 800 python -u -m pytest tests -m gpu -q \
  --timeout 300 --timeout-method thread --maxfail 5 -k "gptq or chol" > $O/gptq_tests_ieee.log 2>&1
rc=$?; if [ $rc -ge 124 ]; then exit 1; fi
