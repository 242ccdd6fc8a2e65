mkdir -p gpurun_out/r03_n /tmp/e2e_n
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/sync_cpu.py > gpurun_out/r03_n/sync_cpu.json 2> gpurun_out/r03_n/sync_cpu.err || exit 1
python tools/e2e_inputs.py /tmp/e2e_n 10000 || exit 1
cd /tmp/e2e_n
timeout -k 10 300 python -u $GRAFT_REPO_ROOT/tools/thread_cpu.py -- $GRAFT_REPO_ROOT/oracle/_ref/gmap_gpu_nosimd -t 512 -O -g g.fa -f samse --no-sam-headers r.fa > $GRAFT_REPO_ROOT/gpurun_out/r03_n/threads_gpu.json || exit 1
cat $GRAFT_REPO_ROOT/gpurun_out/r03_n/sync_cpu.json
