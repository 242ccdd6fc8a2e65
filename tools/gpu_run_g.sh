mkdir -p gpurun_out/r03_k
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "gmap_e2e or shim or latency" > gpurun_out/r03_k/tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03_k/tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u tools/e2e_timing.py --reads 10000 --threads 16 --gpu-threads 512,1024 --trace gpurun_out/r03_k > gpurun_out/r03_k/e2e.json 2> gpurun_out/r03_k/e2e.err; echo "e2e rc=$?"; tail -4 gpurun_out/r03_k/e2e.err
