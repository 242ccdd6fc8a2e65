set -o pipefail
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 11
timeout -k 10 400 python -u bench.py --config 1 --steps 10 --warmup 2 > $O/bench_c1.json 2> $O/bench_c1.err || exit 12
timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err || exit 13
timeout -k 10 400 python -u bench.py --simd --steps 10 --warmup 2 > $O/bench_simd.json 2> $O/bench_simd.err || exit 14
