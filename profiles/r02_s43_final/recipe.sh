#!/bin/bash
# run on the GPU box at commit 89344c4 (tools/profile.sh stats pass only; the PMC passes of the same
# gg_kernel (the roofline kernel, unchanged since) are profiles/r02_s42_pmc; since then s2b's entry
# test changed (38be309) and bench.py's stream assignment (678f27d))
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python bench.py > gpurun_out/s43/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02_s43/stats -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
