mkdir -p gpurun_out/r03_l /tmp/e2e_l
export TMPDIR=/tmp
python tools/e2e_inputs.py /tmp/e2e_l 10000 || exit 1
cd /tmp/e2e_l
timeout -k 10 300 python -u $GRAFT_REPO_ROOT/tools/thread_cpu.py -- $GRAFT_REPO_ROOT/oracle/_ref/gmap_gpu_nosimd -t 512 -O -g g.fa -f samse --no-sam-headers r.fa > $GRAFT_REPO_ROOT/gpurun_out/r03_l/threads_gpu.json; echo "gpu rc=$?"
timeout -k 10 300 python -u $GRAFT_REPO_ROOT/tools/thread_cpu.py -- $GRAFT_REPO_ROOT/oracle/_ref/gmap_nosimd -t 16 -O -g g.fa -f samse --no-sam-headers r.fa > $GRAFT_REPO_ROOT/gpurun_out/r03_l/threads_cpu.json; echo "cpu rc=$?"
