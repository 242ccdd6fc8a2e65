set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 200 python -u tools/oi_timing.py 10000 > $O/oi_timing.json 2> $O/oi_timing.err || exit 11
timeout -k 10 200 python -u tools/oi_timing.py gg > $O/gg_timing.json 2> $O/gg_timing.err || exit 12
