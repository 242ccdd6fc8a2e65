#!/bin/bash
# One GPU-box session (gpurun -- 'bash tools/gpu_session.sh <tag> <steps...>'): each step under its own time
# limit, the session ends at the first failure.  Outputs under gpurun_out/<tag>/.
#   tests          the whole -m gpu suite
#   tests:<k>      the -m gpu tests matching -k <k>
#   bench:<lib>    bench.py --steps 20 --no-cpu-baseline with gmap-2024_amd/<lib>/libgmapdp.so
#   bx:<tag>:<args>  bench.py --steps 10 --no-cpu-baseline <args> -> bx_<tag>.json
#   benchfull      bench.py as the driver runs it (CPU baseline included)
#   simd:<lib>     bench.py --simd;  c4:<lib>  bench.py --config 4
#   iso:<kernel>   tools/profile.sh <tag>_iso iso <kernel>  (the dominant kernel's launches alone)
#   prof           tools/profile.sh <tag>  (kernel stats + PMC passes of the bench step)
#   smoke          __graft_entry__.smoke()
#   e2e:<b>:<n>[:<gpu threads>[:<configs>]]  tools/e2e_timing.py --build <b> --reads <n> (gmap -t 16 vs the
#                  drop-in at -t 512 or the given list; configs as e2e_timing.py --configs)
#   isot:<lib>     bench.py --iso-kernel $ISO_KERNEL (default gg_kernel<1, false>) with <lib>: HIP-event time per launch
#   s2timing       tools/oi_timing.py s2 (the GMAPDP_OI_TIMING build: stage-2 sweep phases and counts)
#   e2eidx:<b>:<n>[:<gpu threads>]  gmap -d over tools/e2e_index.py's index (e2e_pack/, unpacked on the box;
#                  take ./e2e_pack off .gpurunignore for that call): unmodified vs drop-in
set -o pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
for S in "$@"; do
  echo "[session] $S $(date +%T)"
  case "$S" in
    tests) timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gputest.txt 2>&1 || exit 11 ;;
    tests:*) timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "${S#tests:}" tests > $O/gputest_k.txt 2>&1 || exit 12 ;;
    bench:*) L=${S#bench:}; GMAPDP_LIB=$PWD/gmap-2024_amd/$L/libgmapdp.so timeout -k 10 400 python bench.py --steps 20 --no-cpu-baseline > $O/bench_$L.json 2> $O/bench_$L.err || exit 13 ;;
    bp:*) L=${S#bp:}; GMAPDP_BENCH_S2_PRIORITY=1 GMAPDP_LIB=$PWD/gmap-2024_amd/$L/libgmapdp.so timeout -k 10 400 python bench.py --steps 20 --no-cpu-baseline > $O/bp_$L.json 2> $O/bp_$L.err || exit 27 ;;
    simd:*) L=${S#simd:}; GMAPDP_LIB=$PWD/gmap-2024_amd/$L/libgmapdp.so timeout -k 10 400 python bench.py --steps 20 --simd --no-cpu-baseline > $O/simd_$L.json 2> $O/simd_$L.err || exit 14 ;;
    c4:*) L=${S#c4:}; GMAPDP_LIB=$PWD/gmap-2024_amd/$L/libgmapdp.so timeout -k 10 600 python bench.py --steps 10 --config 4 --no-cpu-baseline > $O/c4_$L.json 2> $O/c4_$L.err || exit 15 ;;
    bx:*) X=${S#bx:}; T=${X%%:*}; A=${X#*:}; timeout -k 10 600 python bench.py --steps 10 --no-cpu-baseline $A > $O/bx_$T.json 2> $O/bx_$T.err || exit 23 ;;
    benchfull) timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || exit 16 ;;
    iso:*) bash tools/profile.sh ${TAG}_iso iso "${S#iso:}" > $O/prof_iso.txt 2>&1 || exit 17 ;;
    prof) bash tools/profile.sh $TAG > $O/prof.txt 2>&1 || exit 18 ;;
    profs2) bash tools/profile_s2.sh ${TAG}_s2 > $O/profs2.txt 2>&1 || exit 30 ;;
    profsimd) bash tools/profile.sh ${TAG}_simd simd > $O/profsimd.txt 2>&1 || exit 28 ;;
    isosimd:*) bash tools/profile.sh ${TAG}_isosimd isosimd "${S#isosimd:}" > $O/prof_isosimd.txt 2>&1 || exit 29 ;;
    e2e:*) IFS=: read -r _ B N T C <<< "$S"; timeout -k 10 900 python tools/e2e_timing.py --build $B --reads $N --threads 16 --gpu-threads ${T:-512} ${C:+--configs "$C"} > $O/e2e_${B}_$N.json 2> $O/e2e_${B}_$N.err || exit 20 ;;
    isot:*) L=${S#isot:}; GMAPDP_LIB=$PWD/gmap-2024_amd/$L/libgmapdp.so timeout -k 10 300 python bench.py --iso-kernel "${ISO_KERNEL:-gmapdp::gg_kernel<1, false>}" --iso-reps ${ISO_REPS:-3} > $O/isot_$L.json 2> $O/isot_$L.err || exit 22 ;;
    oitiming) timeout -k 10 300 python tools/oi_timing.py 5000 > $O/oitiming.json 2> $O/oitiming.err || exit 24 ;;
    ggtiming) timeout -k 10 300 python tools/oi_timing.py gg 10000 > $O/ggtiming.json 2> $O/ggtiming.err || exit 33 ;;
    e2eprof:*) IFS=: read -r _ B N T <<< "$S"; timeout -k 10 900 python tools/e2e_timing.py --build $B --reads $N --threads 16 --gpu-threads ${T:-2048} --prof $O/prof_$N > $O/e2eprof_${B}_$N.json 2> $O/e2eprof_${B}_$N.err || exit 26 ;;
    e2ecpu:*) IFS=: read -r _ B N T <<< "$S"; timeout -k 10 900 python tools/e2e_timing.py --build $B --reads $N --threads 16 --gpu-threads ${T:-2048} --thread-cpu > $O/e2ecpu_${B}_$N.json 2> $O/e2ecpu_${B}_$N.err || exit 25 ;;
    s2timing) timeout -k 10 300 python tools/oi_timing.py s2 5000 > $O/s2timing.json 2> $O/s2timing.err || exit 21 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 19 ;;
    e2eidx:*) IFS=: read -r _ B N T <<< "$S"; mkdir -p e2e_idx && { [ -f e2e_idx/meta.json ] || { tar xzf e2e_pack/db.tgz -C e2e_idx && gunzip -c e2e_pack/r.fa.gz > e2e_idx/r.fa && cp e2e_pack/meta.json e2e_idx/; }; } || exit 31
      timeout -k 10 900 python -u tools/e2e_timing.py --index e2e_idx --build $B --reads $N --threads 16 --gpu-threads ${T:-2048} > $O/e2eidx_${B}_$N.json 2> $O/e2eidx_${B}_$N.err || exit 32 ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "[session] ok $(date +%T)"
