set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
GMAPDP_LIB=$PWD/gmap-2024_amd/lib_wpe5/libgmapdp.so timeout -k 10 200 python bench.py --iso-kernel gmapdp::s2b_kernel --iso-reps 2 > $O/iso_s2b_wpe5.json 2> $O/iso_wpe5.err || exit 13
timeout -k 10 200 python bench.py --iso-kernel gmapdp::s2b_kernel --iso-reps 2 > $O/iso_s2b.json 2> $O/iso.err || exit 14
