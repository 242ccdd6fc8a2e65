mkdir -p gpurun_out/r03_e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "e2e or shim or latency" > gpurun_out/r03_e/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_e/tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/e2e_timing.py --reads 1000 --threads 16 --gpu-threads 64,256,512 --dispatchers 3 > gpurun_out/r03_e/e2e.json 2> gpurun_out/r03_e/e2e.err; echo "e2e rc=$?"; tail -5 gpurun_out/r03_e/e2e.err
