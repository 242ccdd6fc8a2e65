"""Inputs for GMAP end to end on an indexed genome (`gmap -d`, the mix the headline bench restates):
a chr22-length synthetic genome indexed by the reference's own `gmap_build` / `gmapindex` (compiled here by
`make -C oracle -f ref.mk index_tools`), and seeded synthetic 2-kb spliced reads drawn from it.

Run in the development container (the index build needs the reference tree's util/ scripts):

    python tools/e2e_index.py [--out e2e_idx] [--length 50818468] [--reads 30000]

Writes <out>/db/<name>/ (the index, k = 15, gmap_build's default; the suffix-array files dropped: gmap
does not read them), <out>/r.fa (the reads) and <out>/meta.json.  `tools/e2e_timing.py --index <out>` then
runs both programs on the GPU box with `-D <out>/db -d <name>`.  The reads follow tests/golden/make_e2e.py's
generator (5 exons x 400 nt, introns 80-20 000 nt log-uniform, GT...AG planted, 2 % substitutions, half
reverse-complemented) on the larger genome."""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
REFTREE = "/root/reference"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "e2e_idx"))
    ap.add_argument("--name", default="chr22s")
    ap.add_argument("--length", type=int, default=50818468)  # GRCh38 chr22
    ap.add_argument("--reads", type=int, default=30000)
    ap.add_argument("--seed", type=int, default=22)
    a = ap.parse_args()
    import make_e2e as M
    t0 = time.time()
    rng = np.random.default_rng(a.seed)
    genome = list(np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, a.length)].tobytes().decode())
    reads = [M.synth_read(genome, i, seed=a.seed) for i in range(a.reads)]  # plants GT...AG in `genome`
    os.makedirs(a.out, exist_ok=True)
    M.write_fasta(os.path.join(a.out, "r.fa"), reads)
    bindir = os.path.join(ROOT, "oracle", "_ref", "bin")
    db = os.path.join(a.out, "db")
    if os.path.isdir(db):
        shutil.rmtree(db)
    with tempfile.TemporaryDirectory() as tmp:
        fa = os.path.join(tmp, "g.fa")
        M.write_fasta(fa, [(a.name, "".join(genome))])
        del genome
        tbin = os.path.join(tmp, "bin")
        os.makedirs(tbin)
        for t in ("gmapindex", "iit_store"):
            shutil.copy(os.path.join(bindir, t), tbin)
        for t in ("fa_coords", "gmap_process"):
            os.symlink(os.path.join(REFTREE, "util", t), os.path.join(tbin, t))
        subprocess.run(["perl", os.path.join(REFTREE, "util", "gmap_build"), "-B", tbin, "-D", db, "-d", a.name, fa],
                       check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    d = os.path.join(db, a.name)
    for f in os.listdir(d):  # suffix arrays / localdb: gsnap's, not read by gmap
        if f.startswith(a.name + ".sa") or f.startswith(a.name + ".sarray"):
            os.remove(os.path.join(d, f))
    size = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d) if os.path.isfile(os.path.join(d, f)))
    meta = {"name": a.name, "length": a.length, "reads": a.reads, "seed": a.seed, "index_bytes": size,
            "build_s": round(time.time() - t0, 1)}
    json.dump(meta, open(os.path.join(a.out, "meta.json"), "w"))
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
