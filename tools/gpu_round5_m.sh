set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export GMAPDP_BENCH_WORKERS=1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 11
f=$(find $O/trace -name '*kernel_trace.csv' | head -n 1)
python3 tools/timeline.py $f 1 4 > $O/timeline.json || exit 12
