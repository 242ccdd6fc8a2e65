mkdir -p gpurun_out/r03_v /tmp/e2e_v
export TMPDIR=/tmp
python tools/e2e_inputs.py /tmp/e2e_v 10000 || exit 1
cd /tmp/e2e_v
export GMAPDP_SHIM_POLL=1 GMAPDP_POLL_US=10 GMAPDP_SHIM_STATS=1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_v -o run -- $GRAFT_REPO_ROOT/oracle/_ref/gmap_gpu_nosimd -t 512 -O -g g.fa -f samse --no-sam-headers r.fa > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/r03_v/gmap.err; echo "rc=$?"
tail -3 $GRAFT_REPO_ROOT/gpurun_out/r03_v/gmap.err
find /tmp/prof_v /tmp/e2e_v -type f | head -20; find /tmp/prof_v /tmp/e2e_v -name "*stats*" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/r03_v/ \; ; ls $GRAFT_REPO_ROOT/gpurun_out/r03_v/
