# round 5, call 16: tile kernel with the S2 chains of waves 1-3 interleaved -- tests, stages
set -o pipefail
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gptq_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "chol or inverse_cholesky or static_plugin" > $O/chol_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2.so > $O/chol_tile_prof2.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/chol_chain_rate.py > $O/chain_rate.txt 2>&1 || exit 1
