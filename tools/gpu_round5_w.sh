set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
GMAPDP_BENCH_SIDES=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_s1.json 2> $O/bench_s1.err || exit 14
