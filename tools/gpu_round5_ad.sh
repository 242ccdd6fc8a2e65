set -o pipefail
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_pipe.json 2> $O/bench_pipe.err || exit 11
GMAPDP_BENCH_PIPELINE=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_nopipe.json 2> $O/bench_nopipe.err || exit 12
