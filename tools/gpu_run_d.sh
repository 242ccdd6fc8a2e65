mkdir -p gpurun_out/r03_d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_latency_mode.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r03_d/latency_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_d/latency_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/gg_bench.py > gpurun_out/r03_d/gg_bench.json 2> gpurun_out/r03_d/gg_bench.err; echo "gg rc=$?"; tail -5 gpurun_out/r03_d/gg_bench.err
