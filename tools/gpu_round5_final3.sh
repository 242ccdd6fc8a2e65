set -o pipefail
bash tools/profile.sh r05c2b || exit 11
