set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u tools/s2_call_profile.py 1 3636 2849 6207 5843 100 200 > $O/prof_b1.jsonl 2> $O/prof_b1.err || exit 11
timeout -k 10 300 python -u tools/s2_call_profile.py 4 3154 6305 100 > $O/prof_b4.jsonl 2> $O/prof_b4.err || exit 12
