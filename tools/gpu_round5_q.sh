set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 200 python -u tools/oi_timing.py 10000 > $O/oi_timing.json 2> $O/oi_timing.err || exit 11
