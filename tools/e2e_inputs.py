"""Write the end-to-end timing inputs (tests/golden/make_e2e.py's synthetic segment and N spliced reads)
to a directory: g.fa, r.fa.   python tools/e2e_inputs.py DIR N"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import make_e2e as M  # noqa: E402

d, n = sys.argv[1], int(sys.argv[2])
os.makedirs(d, exist_ok=True)
genome = list(M.synth_genome())
reads = [M.synth_read(genome, i) for i in range(n)]
M.write_fasta(os.path.join(d, "g.fa"), [("synseg", "".join(genome))])
M.write_fasta(os.path.join(d, "r.fa"), reads)
