mkdir -p gpurun_out/r03_af
export TMPDIR=/tmp
for cfg in "base:" "latmode:GMAPDP_LATENCY_BATCH=100000000"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_af/bench_$name.json 2> gpurun_out/r03_af/bench_$name.err || exit 1
  python -c "
import json
t=open('gpurun_out/r03_af/bench_$name.json').read().strip().splitlines()
d=json.loads([l for l in t if l.startswith('{')][-1])
print('$name', round(d['value']), round(d['ms_per_step'],2), d['step_split_ms'], d['roofline']['kernel'], round(d['roofline']['kernel_ms_per_launch'],3))
"
done
