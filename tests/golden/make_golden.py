"""Generate the committed golden vectors for Dynprog_single_gap.

Run in the development container (needs /root/reference, built into
oracle/_ref/ by `make -C oracle ref`):

    python tests/golden/make_golden.py

Inputs are seeded GMAP-shaped sub-problems (tests/dpbind.py); expected
outputs come from the REFERENCE's own compiled objects (nosimd build: the
Dynprog_standard path; avx2 build: the SIMD path), called through
oracle/refharness.c.  The output file holds data only: the genome, the
problem parameters, the query bytes and the reference's outputs.
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from dpbind import (Ref, call_single, edge_single_gap_problem, random_genome,  # noqa: E402
                    single_gap_problem)

PARAMS = ["rlength", "glength", "roffset", "goffset", "chroffset", "chrhigh", "watsonp", "genestrand",
          "jump_late_p", "extraband", "widebandp", "dynprogindex"]
PAIR_DT = np.dtype([("querypos", "<i4"), ("genomepos", "<i4"), ("queryjump", "<i4"), ("genomejump", "<i4"),
                    ("dynprogindex", "<i4"), ("cdna", "S1"), ("comp", "S1"), ("genome", "S1"), ("genomealt", "S1"),
                    ("gapp", "<i4")])


def problems(seed=2024, n_typical=1200, n_edge=400, genome_len=20000):
    rng = random.Random(seed)
    g = random_genome(rng, genome_len)
    probs = [single_gap_problem(rng, g) for _ in range(n_typical)]
    probs += [edge_single_gap_problem(rng, g) for _ in range(n_edge)]
    return g, probs


def pack(g, probs, outputs):
    par = np.array([[p[k] for k in PARAMS] for p in probs], dtype=np.int64)
    defect = np.array([p["defect_rate"] for p in probs], dtype=np.float64)
    qlen = np.array([len(p["q"]) for p in probs], dtype=np.int32)
    qbuf = np.frombuffer(b"".join(p["q"] for p in probs), dtype=np.uint8)
    qucbuf = np.frombuffer(b"".join(p["quc"] for p in probs), dtype=np.uint8)
    d = dict(genome=np.frombuffer(g, dtype=np.uint8), params=par, param_names=np.array(PARAMS), defect=defect,
             qlen=qlen, qbuf=qbuf, qucbuf=qucbuf)
    for tag, outs in outputs.items():
        scal = np.array([o[0] for o in outs], dtype=np.int32)
        npairs = np.array([-1 if o[1] is None else len(o[1]) for o in outs], dtype=np.int32)
        flat = [pr for o in outs if o[1] is not None for pr in o[1]]
        pairs = np.array(flat, dtype=PAIR_DT)
        d[tag + "_scalars"] = scal
        d[tag + "_npairs"] = npairs
        d[tag + "_pairs"] = pairs
    return d


def load(path):
    """Inverse of pack: (genome bytes, [problem dicts], {tag: [(scalars, pairs-or-None)]})."""
    z = np.load(path, allow_pickle=False)
    names = [str(x) for x in z["param_names"]]
    qoff = np.concatenate([[0], np.cumsum(z["qlen"])])
    qb, qub = z["qbuf"].tobytes(), z["qucbuf"].tobytes()
    probs = []
    for i, row in enumerate(z["params"]):
        p = {k: int(v) for k, v in zip(names, row)}
        p["defect_rate"] = float(z["defect"][i])
        p["q"] = qb[qoff[i]:qoff[i + 1]]
        p["quc"] = qub[qoff[i]:qoff[i + 1]]
        probs.append(p)
    outs = {}
    for key in z.files:
        if key.endswith("_scalars"):
            tag = key[:-len("_scalars")]
            scal, npairs, pairs = z[tag + "_scalars"], z[tag + "_npairs"], z[tag + "_pairs"]
            res, pos = [], 0
            for i in range(len(scal)):
                n = int(npairs[i])
                if n < 0:
                    res.append((tuple(int(x) for x in scal[i]), None))
                    continue
                seg = pairs[pos:pos + n]
                pos += n
                res.append((tuple(int(x) for x in scal[i]),
                            [(int(r["querypos"]), int(r["genomepos"]), int(r["queryjump"]), int(r["genomejump"]),
                              int(r["dynprogindex"]), bytes(r["cdna"]) or b"\0", bytes(r["comp"]) or b"\0",
                              bytes(r["genome"]) or b"\0", bytes(r["genomealt"]) or b"\0", int(r["gapp"]))
                             for r in seg]))
            outs[tag] = res
    return z["genome"].tobytes(), probs, outs


def main():
    g, probs = problems()
    outputs = {}
    for variant in ("nosimd",):  # avx2 (SIMD semantics): see DESIGN.md, aborts on some edge shapes
        ref = Ref(variant)
        ref.set_genome(g)
        outputs["ref_" + variant] = [call_single(ref, p) for p in probs]
    out = os.path.join(HERE, "single_gap_golden.npz")
    np.savez_compressed(out, **pack(g, probs, outputs))
    print("wrote %s: %d problems" % (out, len(probs)))


if __name__ == "__main__":
    main()
