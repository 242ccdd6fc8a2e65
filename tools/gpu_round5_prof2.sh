set -o pipefail
bash tools/profile.sh r05c2_iso iso "gmapdp::gg_kernel<1, false>" || exit 12
BENCH_ARGS="--config 1" PASSES=lite bash tools/profile.sh r05c1 || exit 13
