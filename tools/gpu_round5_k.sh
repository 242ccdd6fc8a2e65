set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
for P in 0 64 256 1024; do
  GMAPDP_S2B_PRIO=$P timeout -k 10 200 python bench.py --iso-kernel gmapdp::s2b_kernel --iso-reps 2 > $O/iso_s2b_$P.json 2> $O/iso_s2b_$P.err || exit 14
done
