#!/bin/bash
# Profiling recipe run on the GPU box (see DESIGN.md "Measurement").
# Usage: bash tools/profile.sh <tag>                 -- the bench step (kernel stats + PMC passes)
#        bash tools/profile.sh <tag> iso <kernel>    -- one kernel's launch classes run alone
#                                                      (bench.py --iso-kernel: what the line's roofline times)
#        bash tools/profile.sh <tag> simd            -- the --simd step (gmap.avx2 semantics)
#        bash tools/profile.sh <tag> isosimd <kernel> -- as iso, in the --simd step
#        BENCH_ARGS="--config 4" bash tools/profile.sh <tag>  -- another workload (recorded in workload.txt)
# Summarise with: python3 tools/pmc_summary.py [--iso] gpurun_out/prof_<tag> profiles/<tag>
set -o pipefail
TAG=${1:-r1}
MODE=${2:-step}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# one process, no forked generator workers (a forked worker ending under rocprofv3 --pmc hung the pass)
export GMAPDP_BENCH_WORKERS=1
SIMD=()
if [ "$MODE" = simd ] || [ "$MODE" = isosimd ]; then SIMD=(--simd); fi
# further bench.py arguments (the workload: --config 4, --mix appb, ...) and the workload id bench.py
# matches committed summaries by (bench.py workload_id)
read -r -a EXTRA <<< "${BENCH_ARGS:-}"
SIMD+=("${EXTRA[@]}")
python3 - "${SIMD[@]}" > $OUT/workload.txt <<'PY'
import sys
a = sys.argv[1:]
cfg = a[a.index("--config") + 1] if "--config" in a else "2"
mix = a[a.index("--mix") + 1] if "--mix" in a else "d"
print("c%s%s%s" % (cfg, "-appb" if mix == "appb" else "", "-simd" if "--simd" in a else ""))
PY
echo "${SIMD[@]}" > $OUT/bench_args.txt
if [ "$MODE" = iso ] || [ "$MODE" = isosimd ]; then
  KERNEL=$3
  BENCH=(python3 bench.py --iso-kernel "$KERNEL" --iso-reps 3 "${SIMD[@]}")
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- "${BENCH[@]}" > $OUT/iso_bench.json 2> $OUT/stats.log || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- "${BENCH[@]}" > $OUT/fetch.log 2>&1 || exit 2
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- "${BENCH[@]}" > $OUT/write.log 2>&1 || exit 3
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- "${BENCH[@]}" > $OUT/sq.log 2>&1 || exit 4
  echo done
  exit 0
fi
BENCH=(python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "${SIMD[@]}")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- "${BENCH[@]}" > $OUT/stats.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- "${BENCH[@]}" > $OUT/fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- "${BENCH[@]}" > $OUT/write.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- "${BENCH[@]}" > $OUT/sq.log 2>&1 || exit 4
if [ "${PASSES:-full}" != lite ]; then  # PASSES=lite: no second SQ pass (the wait/issue counters)
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/sq2 -o run -- "${BENCH[@]}" > $OUT/sq2.log 2>&1 || exit 5
fi
echo done
