#!/bin/bash
# One GPU-box session: the -m gpu suite, smoke, and the bench (default configs[2] line), each step under
# its own time limit; a test failure (pytest rc 1) does not stop the later steps, anything else (a fault,
# an abort, a time limit) ends the session.  Usage: bash tools/gpu_check.sh <tag> [pytest -k expr] [bench args]
TAG=${1:-check}
KEXPR=${2:-}
BENCHARGS=${3:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$KEXPR" > $OUT/gputest.txt 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gputest.txt 2>&1
fi
rc=$?; echo "gputest rc=$rc"; tail -3 $OUT/gputest.txt; ok $rc || exit $rc
if [ "$KEXPR" = "none" ]; then exit 0; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.txt; ok $rc || exit $rc
timeout -k 10 500 python -u bench.py $BENCHARGS > $OUT/bench.json 2> $OUT/bench_progress.txt
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench_progress.txt; exit $rc
