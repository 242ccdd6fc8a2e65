set -o pipefail
O=gpurun_out/r05e2e
mkdir -p $O e2e_idx
tar xzf e2e_pack/db.tgz -C e2e_idx && gunzip -c e2e_pack/r.fa.gz > e2e_idx/r.fa && cp e2e_pack/meta.json e2e_idx/ || exit 10
timeout -k 10 600 python -u tools/e2e_timing.py --index e2e_idx --reads 30000 --threads 16 --gpu-threads 4096,8192 --skip-cpu > $O/e2e_30k_d_nosimd_t.json 2> $O/e2e_30k_d_nosimd_t.err || exit 11
timeout -k 10 600 python -u tools/e2e_timing.py --index e2e_idx --reads 30000 --build avx2 --threads 16 --gpu-threads 4096 > $O/e2e_30k_d_avx2.json 2> $O/e2e_30k_d_avx2.err || exit 12
