set -e
mkdir -p gpurun_out
for t in 0 1024 2048 3072 4096 5120; do
  GMAPDP_DPX_LDS_DIRS_MAX=$t timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/gd_$t.json 2> gpurun_out/gd_$t.err
done
