# Round check on one MI355X: the GPU suite, smoke, the bench line and the rocprof / PMC profile of it.
# bash tools/gpu_run_final.sh TAG
TAG=${1:-r03_final3}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.txt 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gputest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench_progress.txt || exit 3
tail -c 400 $O/bench.json; echo
timeout -k 10 900 bash tools/profile.sh $TAG > $O/profile.txt 2>&1 || exit 4
echo profiled
