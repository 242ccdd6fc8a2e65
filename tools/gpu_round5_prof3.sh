set -o pipefail
BENCH_ARGS="--config 4" PASSES=lite bash tools/profile.sh r05c4 || exit 11
