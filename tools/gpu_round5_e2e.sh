set -o pipefail
O=gpurun_out/r05e2e
mkdir -p $O e2e_idx
tar xzf e2e_pack/db.tgz -C e2e_idx && gunzip -c e2e_pack/r.fa.gz > e2e_idx/r.fa && cp e2e_pack/meta.json e2e_idx/ || exit 10
timeout -k 10 900 python -u tools/e2e_timing.py --index e2e_idx --reads 30000 --threads 16 --gpu-threads 2048 --skip-cpu --configs 'h24:GMAPDP_SHIM_FIBER_HOSTS=24;h32:GMAPDP_SHIM_FIBER_HOSTS=32;h24s3l2:GMAPDP_SHIM_FIBER_HOSTS=24,GMAPDP_SHIM_STAGE2_DISPATCHERS=3,GMAPDP_SHIM_LONG_DISPATCHERS=2;h32s3l2:GMAPDP_SHIM_FIBER_HOSTS=32,GMAPDP_SHIM_STAGE2_DISPATCHERS=3,GMAPDP_SHIM_LONG_DISPATCHERS=2;h48s3l2:GMAPDP_SHIM_FIBER_HOSTS=48,GMAPDP_SHIM_STAGE2_DISPATCHERS=3,GMAPDP_SHIM_LONG_DISPATCHERS=2' > $O/e2e_sweep2.json 2> $O/e2e_sweep2.err || exit 11
