set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
GPU_MAX_HW_QUEUES=8 GMAPDP_BENCH_SIDES=3 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_s3q8.json 2> $O/bench_s3q8.err || exit 14
GPU_MAX_HW_QUEUES=8 GMAPDP_BENCH_SIDES=2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_s2q8.json 2> $O/bench_s2q8.err || exit 15
