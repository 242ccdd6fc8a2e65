mkdir -p gpurun_out/r03_w
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_shim.py tests/test_gmap_e2e.py tests/test_gpu_microexon.py > gpurun_out/r03_w/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r03_w/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512 --trace gpurun_out/r03_w \
  --configs "spin:;poll10:GMAPDP_SHIM_POLL=1,GMAPDP_POLL_US=10" \
  > gpurun_out/r03_w/e2e.json 2> gpurun_out/r03_w/e2e.err; echo "e2e rc=$?"
python -c "
import json
for l in open('gpurun_out/r03_w/e2e.err'):
    if l.startswith('{'):
        r=json.loads(l); print(r['config'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
print(json.load(open('gpurun_out/r03_w/e2e.json'))['outputs_identical'])
"
