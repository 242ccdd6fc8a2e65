mkdir -p gpurun_out/r03_u
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512 --skip-cpu --trace gpurun_out/r03_u \
  --configs "spin:;poll20:GMAPDP_SHIM_POLL=1;poll50:GMAPDP_SHIM_POLL=1,GMAPDP_POLL_US=50;poll10:GMAPDP_SHIM_POLL=1,GMAPDP_POLL_US=10;poll20_1024:GMAPDP_SHIM_POLL=1,GMAPDP_SHIM_DISPATCHERS=2" \
  > gpurun_out/r03_u/e2e.json 2> gpurun_out/r03_u/e2e.err; echo "e2e rc=$?"
python -c "
import json
for l in open('gpurun_out/r03_u/e2e.err'):
    if l.startswith('{'):
        r=json.loads(l); print(r['config'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
"
