set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gg_tests.log 2>&1
run() { timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/gg_$1.json 2> gpurun_out/gg_$1.err; }
for t in 65536 16384 12288 8192 0; do GMAPDP_GG_LDS_DIRS_MAX=$t run e$t; done
