set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_stage2_plan.py tests/test_gpu_stage2.py tests/test_gpu_genome_gap.py tests/test_gpu_maxent.py > gpurun_out/t1.log 2>&1 || exit 11
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 12
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_bench_workload.py -k "configs2" > gpurun_out/t2.log 2>&1 || exit 13
