set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
for B in 1 4; do
  timeout -k 10 300 python -u tools/s2_slow.py $B $O/slow_b$B.npz > $O/slow_b$B.json 2> $O/slow_b$B.err || exit 11
done
