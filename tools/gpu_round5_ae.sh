set -o pipefail
O=gpurun_out/r05ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_oligo.py tests/test_gpu_stage2_plan.py > $O/t1.log 2>&1 || exit 11
for V in default wpe7 wpe8; do
  L=$PWD/gmap-2024_amd/lib/libgmapdp.so
  [ $V != default ] && L=$PWD/gmap-2024_amd/lib_$V/libgmapdp.so
  GMAPDP_LIB=$L timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_$V.json 2> $O/bench_$V.err || exit 12
done
