mkdir -p gpurun_out/r03_s
export TMPDIR=/tmp
S="GMAPDP_SHIM_SPIN=1"
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512 --skip-cpu --trace gpurun_out/r03_s \
  --configs "s121:$S,GMAPDP_SHIM_DISPATCHERS=1,GMAPDP_SHIM_LONG_DISPATCHERS=2,GMAPDP_SHIM_STAGE2_DISPATCHERS=1,GPU_MAX_HW_QUEUES=4;s112:$S,GMAPDP_SHIM_DISPATCHERS=1,GMAPDP_SHIM_LONG_DISPATCHERS=1,GMAPDP_SHIM_STAGE2_DISPATCHERS=2,GPU_MAX_HW_QUEUES=4;s212:$S,GMAPDP_SHIM_DISPATCHERS=2,GMAPDP_SHIM_LONG_DISPATCHERS=1,GMAPDP_SHIM_STAGE2_DISPATCHERS=2,GPU_MAX_HW_QUEUES=5;s213:$S,GMAPDP_SHIM_DISPATCHERS=2,GMAPDP_SHIM_LONG_DISPATCHERS=1,GMAPDP_SHIM_STAGE2_DISPATCHERS=3,GPU_MAX_HW_QUEUES=6;s212q4:$S,GMAPDP_SHIM_DISPATCHERS=2,GMAPDP_SHIM_LONG_DISPATCHERS=1,GMAPDP_SHIM_STAGE2_DISPATCHERS=2,GPU_MAX_HW_QUEUES=4" \
  > gpurun_out/r03_s/e2e.json 2> gpurun_out/r03_s/e2e.err; echo "e2e rc=$?"
python -c "
import json
for l in open('gpurun_out/r03_s/e2e.err'):
    if l.startswith('{'):
        r=json.loads(l); print(r['config'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
"
