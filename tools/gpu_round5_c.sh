set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/oi_timing.py s2 10000 > gpurun_out/s2_timing.json 2> gpurun_out/s2_timing.err || exit 11
