# round 6 final profiles: the default bench line and per-leg rocprofv3 kernel-trace stats
set -o pipefail
TAG=r6f timeout -k 10 1100 bash scripts/profile_round.sh A || exit 1
