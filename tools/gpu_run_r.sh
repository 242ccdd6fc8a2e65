mkdir -p gpurun_out/r03_r
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dp_rows.py tests/test_gpu_single_gap.py tests/test_gpu_end_gap.py tests/test_gpu_latency_mode.py tests/test_gpu_shim.py > gpurun_out/r03_r/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r03_r/tests.txt
[ $rc -eq 0 ] || exit $rc
S="GMAPDP_SHIM_SPIN=1,GMAPDP_SHIM_LONG_DISPATCHERS=1,GMAPDP_SHIM_STAGE2_DISPATCHERS=1,GPU_MAX_HW_QUEUES=4"
timeout -k 10 600 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512,1024 --trace gpurun_out/r03_r \
  --configs "s211:GMAPDP_SHIM_DISPATCHERS=2,$S" \
  > gpurun_out/r03_r/e2e.json 2> gpurun_out/r03_r/e2e.err; echo "e2e rc=$?"; tail -3 gpurun_out/r03_r/e2e.err | cut -c1-300
