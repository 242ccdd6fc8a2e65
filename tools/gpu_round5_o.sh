set -o pipefail
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_oligo.py tests/test_gpu_stage2.py tests/test_gpu_stage2_plan.py > $O/t1.log 2>&1 || exit 11
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_gpu_bench_workload.py -k "configs2_stage2" > $O/t2.log 2>&1 || exit 12
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 14
