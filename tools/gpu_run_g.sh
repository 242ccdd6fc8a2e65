mkdir -p gpurun_out/r03_g
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/e2e_timing.py --reads 1000 --threads 16 --gpu-threads 256 --trace gpurun_out/r03_g > gpurun_out/r03_g/e2e.json 2> gpurun_out/r03_g/e2e.err; echo "e2e rc=$?"; tail -3 gpurun_out/r03_g/e2e.err
