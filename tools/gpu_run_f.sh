mkdir -p gpurun_out/r03_f
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/latency.py 100 > gpurun_out/r03_f/latency.json 2> gpurun_out/r03_f/latency.err; echo "lat rc=$?"; tail -1 gpurun_out/r03_f/latency.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_f/prof -o lat -- python3 tools/latency.py 20 > gpurun_out/r03_f/prof.log 2>&1; echo "prof rc=$?"
