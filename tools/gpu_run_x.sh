mkdir -p gpurun_out/r03_x
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stage2.py tests/test_gpu_shim.py > gpurun_out/r03_x/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_x/tests.txt
[ $rc -eq 0 ] || exit $rc
P="GMAPDP_SHIM_POLL=1,GMAPDP_POLL_US=10"
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512 --skip-cpu --trace gpurun_out/r03_x \
  --configs "d212:$P;s213q6:$P,GMAPDP_SHIM_STAGE2_DISPATCHERS=3,GPU_MAX_HW_QUEUES=6;s214q7:$P,GMAPDP_SHIM_STAGE2_DISPATCHERS=4,GPU_MAX_HW_QUEUES=7;s215q8:$P,GMAPDP_SHIM_STAGE2_DISPATCHERS=5,GPU_MAX_HW_QUEUES=8;s214q4:$P,GMAPDP_SHIM_STAGE2_DISPATCHERS=4" \
  > gpurun_out/r03_x/e2e.json 2> gpurun_out/r03_x/e2e.err; echo "e2e rc=$?"
python -c "
import json
for l in open('gpurun_out/r03_x/e2e.err'):
    if l.startswith('{'):
        r=json.loads(l); print(r['config'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
print(json.load(open('gpurun_out/r03_x/e2e.json'))['outputs_identical'])
"
