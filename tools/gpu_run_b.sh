mkdir -p gpurun_out/r03_b
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/oi_timing.py gg > gpurun_out/r03_b/gg_phases.json 2> gpurun_out/r03_b/gg_phases.err; echo "gg rc=$?"
timeout -k 10 500 python -u bench.py --config 4 --steps 8 --warmup 2 --batches 4 --no-cpu-baseline > gpurun_out/r03_b/bench_c4.json 2> gpurun_out/r03_b/bench_c4.err || exit $?
timeout -k 10 400 python -u bench.py --simd --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_b/bench_simd.json 2> gpurun_out/r03_b/bench_simd.err
