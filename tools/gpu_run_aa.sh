mkdir -p gpurun_out/r03_aa
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512 --skip-cpu --trace gpurun_out/r03_aa \
  --configs "d212:;s213q6:GMAPDP_SHIM_STAGE2_DISPATCHERS=3,GPU_MAX_HW_QUEUES=6;s214q7:GMAPDP_SHIM_STAGE2_DISPATCHERS=4,GPU_MAX_HW_QUEUES=7;s313q7:GMAPDP_SHIM_DISPATCHERS=3,GMAPDP_SHIM_STAGE2_DISPATCHERS=3,GPU_MAX_HW_QUEUES=7;s214q4:GMAPDP_SHIM_STAGE2_DISPATCHERS=4" \
  > gpurun_out/r03_aa/e2e.json 2> gpurun_out/r03_aa/e2e.err; echo "e2e rc=$?"
python -c "
import json
for l in open('gpurun_out/r03_aa/e2e.err'):
    if l.startswith('{'):
        r=json.loads(l); print(r['config'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
print(json.load(open('gpurun_out/r03_aa/e2e.json'))['outputs_identical'])
"
