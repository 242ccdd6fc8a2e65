mkdir -p gpurun_out/r03_ab
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/oi_timing.py s2 > gpurun_out/r03_ab/s2_timing.json 2> gpurun_out/r03_ab/s2_timing.err; echo "s2 rc=$?"
timeout -k 10 300 python -u tools/latency.py 50 > gpurun_out/r03_ab/latency.json 2> gpurun_out/r03_ab/latency.err; echo "lat rc=$?"
cat gpurun_out/r03_ab/s2_timing.json gpurun_out/r03_ab/latency.json
