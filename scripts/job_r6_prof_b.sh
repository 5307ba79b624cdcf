# round 6 final profiles (B): PMC FETCH_SIZE / WRITE_SIZE passes per leg (separate runs)
set -o pipefail
TAG=r6 timeout -k 10 1100 bash scripts/profile_round.sh B || exit 1
