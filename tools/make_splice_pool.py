"""Generate the bench workload's splice-site contexts (gmap-2024_amd/gmapdp/splice_contexts.txt).

WORKLOAD INFRASTRUCTURE (run here, where the oracle is built; the output is committed data).  The bench plants
a donor context (x-3 .. x+5, x = first intron base) and an acceptor context (y-19 .. y+3, y = last intron
base) at every genome-gap intron so that MaxEnt, evaluated on the device in the step, finds strong sites as it
does at real introns.  One fixed context at ~4 M sites made its 8-mers ~1 per 750 nt of the genome and
doubled the stage-2 seeding hits of reads that cross them; a pool of distinct contexts keeps every 8-mer's
frequency near the i.i.d. background.  Every context here scores >= 0.9 with the oracle's MaxEnt restatement
(oracle/maxent_oracle.c, pinned to maxent_hr.c by tests/test_maxent.py):
  donor: all 4^7 9-mers with GT at x, x+1;  acceptor: 23-mers with AG at y-1, y, a pyrimidine-rich tract
  (80 % C/T) before it and random bases after, seeded.

    python tools/make_splice_pool.py
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dpbind import Oracle  # noqa: E402

OUT = os.path.join(ROOT, "gmap-2024_amd", "gmapdp", "splice_contexts.txt")
NACC = 4096


def scores(orc, rng, cands, model, off):
    sp = 60
    parts, bases = [], []
    pos = 0
    for c in cands:
        parts.append("".join(rng.choice("ACGT") for _ in range(sp)))
        pos += sp
        bases.append(pos)
        parts.append(c)
        pos += len(c)
    parts.append("A" * 100)
    orc.set_genome("".join(parts).encode())
    return [orc.maxent(model, b + off, 0) for b in bases]


def main():
    orc = Oracle()
    rng = random.Random(2024)
    acgt = "ACGT"
    donors = []
    for k in range(4 ** 7):
        s = [acgt[(k >> (2 * i)) & 3] for i in range(7)]
        donors.append("".join(s[:3]) + "GT" + "".join(s[3:]))
    ds = scores(orc, rng, donors, 0, 3)
    donors = sorted(d for d, p in zip(donors, ds) if p >= 0.9)
    accs, seen = [], set()
    while len(accs) < NACC:
        batch = []
        while len(batch) < 2048:
            s = "".join(rng.choice("CT") if rng.random() < 0.8 else rng.choice("AG") for _ in range(18))
            s += "AG" + "".join(rng.choice(acgt) for _ in range(3))
            if s not in seen:
                seen.add(s)
                batch.append(s)
        for a, p in zip(batch, scores(orc, rng, batch, 1, 20)):
            if p >= 0.9 and len(accs) < NACC:
                accs.append(a)
    with open(OUT, "w") as f:
        f.write("# bench splice contexts (tools/make_splice_pool.py): D <donor x-3..x+5> / A <acceptor y-19..y+3>, "
                "MaxEnt >= 0.9 each\n")
        for d in donors:
            f.write("D %s\n" % d)
        for a in accs:
            f.write("A %s\n" % a)
    print("donors %d acceptors %d -> %s" % (len(donors), len(accs), OUT))


if __name__ == "__main__":
    main()
