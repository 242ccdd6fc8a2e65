set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/oi_timing.py s2 10000 > gpurun_out/s2_timing.json 2> gpurun_out/s2_timing.err || exit 11
timeout -k 10 200 python -u tools/oi_timing.py 10000 > gpurun_out/oi_timing.json 2> gpurun_out/oi_timing.err || exit 12
timeout -k 10 900 bash tools/profile.sh r05a > gpurun_out/prof_r05a.log 2>&1 || exit 13
