mkdir -p gpurun_out/r03_z
export TMPDIR=/tmp
P="GMAPDP_SHIM_POLL=1,GMAPDP_POLL_US=10"
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512 --skip-cpu --trace gpurun_out/r03_z \
  --configs "legacy4:$P,GMAPDP_S2_LEGACY=1,GMAPDP_S2_SCRATCH_MULT=4;legacy16:$P,GMAPDP_S2_LEGACY=1;exact4:$P,GMAPDP_S2_EXACT=1,GMAPDP_S2_SCRATCH_MULT=4;bounded:$P;legacy4b:$P,GMAPDP_S2_LEGACY=1,GMAPDP_S2_SCRATCH_MULT=4" \
  > gpurun_out/r03_z/e2e.json 2> gpurun_out/r03_z/e2e.err; echo "e2e rc=$?"
python -c "
import json
for l in open('gpurun_out/r03_z/e2e.err'):
    if l.startswith('{'):
        r=json.loads(l); print(r['config'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
print(json.load(open('gpurun_out/r03_z/e2e.json'))['outputs_identical'])
"
