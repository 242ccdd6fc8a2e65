#!/bin/bash
# rocprofv3 passes over the stage-2 kernels run alone (seeding + chaining, tools/s2_run.py) on the GPU box:
# kernel stats, SQ counters, FETCH_SIZE and WRITE_SIZE.
# Usage: bash tools/profile_s2.sh <tag>
set -o pipefail
TAG=${1:-s2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
RUN="python3 tools/s2_run.py 5000"  # (the batch API sizes its arenas by bounds: 5 000 calls on 214-kb windows fit)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $RUN > $OUT/stats.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- $RUN > $OUT/sq.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_SMEM --output-format csv -d $OUT/sq2 -o run -- $RUN > $OUT/sq2.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $RUN > $OUT/fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $RUN > $OUT/write.log 2>&1 || exit 5
echo done
