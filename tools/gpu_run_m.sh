mkdir -p gpurun_out/r03_m
timeout -k 10 300 python -u tools/sync_cpu.py > gpurun_out/r03_m/sync_cpu.json 2> gpurun_out/r03_m/sync_cpu.err; echo "rc=$?"; cat gpurun_out/r03_m/sync_cpu.json
