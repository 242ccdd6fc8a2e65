set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/oi_timing.py 10000 > $O/oi_timing.json 2> $O/oi_timing.err || exit 11
