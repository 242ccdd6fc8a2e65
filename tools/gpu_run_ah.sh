mkdir -p gpurun_out/r03_ah
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/gg_bench.py --variants lib_base,gg_kernel,lib_base,gg_kernel --reps 5 > gpurun_out/r03_ah/gg_bench.json 2> gpurun_out/r03_ah/gg_bench.err; echo "gg rc=$?"; cat gpurun_out/r03_ah/gg_bench.err | cut -c1-200
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_genome_gap.py tests/test_gpu_latency_mode.py tests/test_gpu_shim.py tests/test_gpu_bench_workload.py tests/test_gpu_simd.py > gpurun_out/r03_ah/tests.txt 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r03_ah/tests.txt
