mkdir -p gpurun_out/r03_t
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512,1024 --skip-cpu --trace gpurun_out/r03_t \
  --configs "oq2:;oq0:GMAPDP_SHIM_OLIGO_QUEUE=0" \
  > gpurun_out/r03_t/e2e.json 2> gpurun_out/r03_t/e2e.err; echo "e2e rc=$?"
python -c "
import json
for l in open('gpurun_out/r03_t/e2e.err'):
    if l.startswith('{'):
        r=json.loads(l); print(r['config'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
"
