# Full round check on one MI355X: GPU tests, smoke, the bench line, GMAP end to end, rocprof.
# bash tools/gpu_run_full.sh TAG
TAG=${1:-r03_full}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gputest.txt 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gputest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 2
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench_progress.txt || exit 3
tail -c 600 $O/bench.json; echo
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512,1024 --trace $O > $O/e2e.json 2> $O/e2e.err || exit 4
python -c "
import json
d=json.load(open('$O/e2e.json'))
for r in d['runs']: print(r['program'], r['threads'], round(r['reads_per_s'],1), round(r['cpu_cores_busy'],1))
print('identical', d['outputs_identical'])
"
