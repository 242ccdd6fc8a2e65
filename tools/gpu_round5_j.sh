set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 300 python -u tools/s2_call_profile.py 1 3636 2849 6207 100 > $O/prof_b1.jsonl 2> $O/prof_b1.err || exit 13
