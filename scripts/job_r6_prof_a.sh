# round 6 final profiles (A): the default bench line + rocprofv3 kernel-trace stats per leg
set -o pipefail
TAG=r6 timeout -k 10 1100 bash scripts/profile_round.sh A || exit 1
