set -o pipefail
bash tools/profile.sh r05c2 || exit 11
