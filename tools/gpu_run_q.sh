mkdir -p gpurun_out/r03_q
export TMPDIR=/tmp
S="GMAPDP_SHIM_SPIN=1,GMAPDP_SHIM_LONG_DISPATCHERS=1,GMAPDP_SHIM_STAGE2_DISPATCHERS=1,GPU_MAX_HW_QUEUES=4"
timeout -k 10 600 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 1024 --skip-cpu --trace gpurun_out/r03_q \
  --configs "s211:GMAPDP_SHIM_DISPATCHERS=2,$S" \
  > gpurun_out/r03_q/e2e.json 2> gpurun_out/r03_q/e2e.err; echo "e2e rc=$?"; tail -3 gpurun_out/r03_q/e2e.err | cut -c1-300
