mkdir -p gpurun_out/r03_ae
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/e2e_timing.py --reads 30000 --threads 16 --gpu-threads 1536,2048 --skip-cpu > gpurun_out/r03_ae/e2e.json 2> gpurun_out/r03_ae/e2e.err; echo "e2e rc=$?"
python -c "
import json
d=json.load(open('gpurun_out/r03_ae/e2e.json'))
for r in d['runs']: print(r['program'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
print('identical', d['outputs_identical'])
"
