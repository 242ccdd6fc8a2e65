set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_p0.json 2> $O/bench_p0.err || exit 14
GMAPDP_BENCH_S2_PRIORITY=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_p1.json 2> $O/bench_p1.err || exit 15
