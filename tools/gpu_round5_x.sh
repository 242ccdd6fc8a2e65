set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 14
