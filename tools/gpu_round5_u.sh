set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
GMAPDP_BENCH_S2_PRIORITY=2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_p2.json 2> $O/bench_p2.err || exit 14
GMAPDP_S2B_LDS=20480 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_l20.json 2> $O/bench_l20.err || exit 15
