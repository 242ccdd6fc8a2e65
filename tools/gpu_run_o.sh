mkdir -p gpurun_out/r03_o
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512 --trace gpurun_out/r03_o \
  --configs "cur:;spin:GMAPDP_SHIM_SPIN=1;small_spin:GMAPDP_SHIM_SPIN=1,GMAPDP_SHIM_DISPATCHERS=2,GMAPDP_SHIM_LONG_DISPATCHERS=1,GMAPDP_SHIM_STAGE2_DISPATCHERS=1,GPU_MAX_HW_QUEUES=4;small_block:GMAPDP_SHIM_DISPATCHERS=2,GMAPDP_SHIM_LONG_DISPATCHERS=1,GMAPDP_SHIM_STAGE2_DISPATCHERS=1,GPU_MAX_HW_QUEUES=4" \
  > gpurun_out/r03_o/e2e.json 2> gpurun_out/r03_o/e2e.err; echo "e2e rc=$?"; tail -8 gpurun_out/r03_o/e2e.err
