set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
GMAPDP_LIB=$PWD/gmap-2024_amd/lib_qt/libgmapdp.so timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_qt.json 2> $O/bench_qt.err || exit 13
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 14
