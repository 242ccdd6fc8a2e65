#!/bin/bash
# Round 5's GPU measurements, reproducible on a gpurun box (one step per call; each bounded by its own
# timeout, the steps chained so that a failure ends the call):
#   bash tools/gpu_round5.sh tests     -- the GPU suite and smoke            -> gpurun_out/r05/
#   bash tools/gpu_round5.sh bench     -- the bench lines of configs[2], [1], [4] and --simd -> gpurun_out/r05/
#   bash tools/gpu_round5.sh prof c2   -- tools/profile.sh on one workload (c2 | c1 | c4 | simd | iso)
#   bash tools/gpu_round5.sh e2e       -- GMAP end to end on the indexed chr22-length genome (needs
#                                         e2e_pack/ from tools/e2e_index.py, which .gpurunignore skips:
#                                         take it off that list for the call)
#   bash tools/gpu_round5.sh sweep B   -- s2b per-call profile of bench block B's slowest calls (timing build)
# Summaries: python3 tools/pmc_summary.py [--iso] gpurun_out/prof_<tag> profiles/<tag>
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
case "$1" in
  tests)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 11
    timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
    ;;
  bench)
    timeout -k 10 500 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 11
    timeout -k 10 400 python -u bench.py --config 1 --steps 10 --warmup 2 > $O/bench_c1.json 2> $O/bench_c1.err || exit 12
    timeout -k 10 400 python -u bench.py --config 4 --steps 10 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err || exit 13
    timeout -k 10 400 python -u bench.py --simd --steps 10 --warmup 2 > $O/bench_simd.json 2> $O/bench_simd.err || exit 14
    ;;
  prof)
    case "$2" in
      c2) bash tools/profile.sh r05c2 || exit 11 ;;
      c1) BENCH_ARGS="--config 1" PASSES=lite bash tools/profile.sh r05c1 || exit 11 ;;
      c4) BENCH_ARGS="--config 4" PASSES=lite bash tools/profile.sh r05c4 || exit 11 ;;
      simd) PASSES=lite bash tools/profile.sh r05simd simd || exit 11 ;;
      iso) bash tools/profile.sh r05c2_iso iso "gmapdp::gg_kernel<1, false>" || exit 11 ;;
      *) echo "prof: c2 | c1 | c4 | simd | iso"; exit 2 ;;
    esac
    ;;
  e2e)
    mkdir -p e2e_idx
    tar xzf e2e_pack/db.tgz -C e2e_idx && gunzip -c e2e_pack/r.fa.gz > e2e_idx/r.fa && cp e2e_pack/meta.json e2e_idx/ || exit 10
    timeout -k 10 1000 python -u tools/e2e_timing.py --index e2e_idx --reads 30000 --threads 16 --gpu-threads 2048 > $O/e2e_30k_d_nosimd.json 2> $O/e2e_30k_d_nosimd.err || exit 11
    timeout -k 10 600 python -u tools/e2e_timing.py --index e2e_idx --reads 30000 --build avx2 --threads 16 --gpu-threads 4096 > $O/e2e_30k_d_avx2.json 2> $O/e2e_30k_d_avx2.err || exit 12
    ;;
  sweep)
    B=${2:-1}
    timeout -k 10 300 python -u tools/s2_slow.py $B $O/slow_b$B.npz > $O/slow_b$B.json 2> $O/slow_b$B.err || exit 11
    ;;
  *)
    echo "usage: bash tools/gpu_round5.sh tests | bench | prof <c2|c1|c4|simd|iso> | e2e | sweep <block>"
    exit 2
    ;;
esac
echo done
