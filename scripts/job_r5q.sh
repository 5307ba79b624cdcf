# round 5, call 17: finer stage stamps of the tile's S2 on wave 1
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 120 python3 -u scripts/chol_tile_prof2.py libchol_prof2.so > $O/chol_tile_prof2.txt 2>&1 || exit 1
