set -o pipefail
PASSES=lite bash tools/profile.sh r05simd simd || exit 11
