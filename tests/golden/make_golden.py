"""Generate the committed golden vectors for the Dynprog_* entry points.

Run in the development container (needs /root/reference, built into
oracle/_ref/ by `make -C oracle ref`):

    python tests/golden/make_golden.py

Inputs are seeded GMAP-shaped sub-problems (tests/dpbind.py); expected
outputs come from the REFERENCE's own compiled objects (nosimd build: the
Dynprog_standard path), called through oracle/refharness.c.  Each output
file holds data only: the genome, the problem parameters, the query bytes
and the reference's outputs.

  single_gap_golden.npz  Dynprog_single_gap   (dynprog_single.c:429)
  end_gap_golden.npz     Dynprog_end5_gap / Dynprog_end3_gap (dynprog_end.c:1294/1924)
  genome_gap_golden.npz  Dynprog_genome_gap   (dynprog_genome.c:3288), with the reference's
                         MaxEnt splice probabilities (Maxent_hr_*_prob) at every entry the
                         engine reads; halfp problems come from the --enable-alloca nosimd
                         build (the default heap build dereferences a freed array there)
  cdna_gap_golden.npz, simd_cdna_gap_golden.npz
                         Dynprog_cdna_gap (dynprog_cdna.c:787) from the nosimd and AVX2 objects
  simd_{single,end,genome}_gap_golden.npz
                         the same entry points as the SIMD builds compute them (gmap.avx2:
                         Dynprog_simd_8/16, the _upper/_lower triangles, bridge_intron_gap_*_ud),
                         from the reference's AVX2 objects called on zeroed Dynprog_T arenas, on
                         problems inside the domain where that build is defined (see
                         simd_domain below); halfp genome gaps from the --enable-alloca AVX2 build
  stage2_golden.npz      Stage2_compute (stage2.c:6325): seeding, chaining, convert_to_nucleotides,
                         filter_unique (python tests/golden/make_golden.py stage2)
  splicejunction_golden.npz
                         Dynprog_end5_splicejunction / Dynprog_end3_splicejunction (dynprog_end.c:1653/2249),
                         the known-splice end fills Splicetrie_solve_end5/end3 issue with -s
                         (python tests/golden/make_golden.py splicejunction)
  oligo_golden.npz       stage-2 seeding: Oligoindex_hr_tally + Oligoindex_get_mappings
                         (oligoindex_hr.c:33849/34127) as Stage2_compute runs them for GMAP
                         (python tests/golden/make_golden.py oligo)
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from dpbind import (GG_FLAG_HALF, Oracle, Ref, call_end, call_single, cdna_gap_problem,  # noqa: E402
                    edge_single_gap_problem, end_gap_problem, genome_gap_problem, oligo_problem,
                    random_genome, single_gap_problem, splice_probs)

SINGLE_PARAMS = ["rlength", "glength", "roffset", "goffset", "chroffset", "chrhigh", "watsonp", "genestrand",
                 "jump_late_p", "extraband", "widebandp", "dynprogindex"]
END_PARAMS = ["end3p", "rlength", "glength", "roffset", "goffset", "chroffset", "chrhigh", "watsonp",
              "genestrand", "jump_late_p", "extraband", "endalign", "require_pos_score_p", "dynprogindex"]
CDNA_PARAMS = ["qposL", "qposR", "rlengthL", "rlengthR", "glength", "roffsetL", "rev_roffsetR", "goffset",
               "chroffset", "chrhigh", "watsonp", "genestrand", "jump_late_p", "extraband", "dynprogindex"]
GENOME_PARAMS = ["rlength", "glengthL", "glengthR", "roffset", "goffsetL", "rev_goffsetR", "chroffset", "chrhigh",
                 "cdna_direction", "flags", "genestrand", "extraband", "maxpeelback", "dynprogindex"]
PAIR_DT = np.dtype([("querypos", "<i4"), ("genomepos", "<i4"), ("queryjump", "<i4"), ("genomejump", "<i4"),
                    ("dynprogindex", "<i4"), ("cdna", "S1"), ("comp", "S1"), ("genome", "S1"), ("genomealt", "S1"),
                    ("gapp", "<i4")])


def single_problems(seed=2024, n_typical=1200, n_edge=400, genome_len=20000):
    rng = random.Random(seed)
    g = random_genome(rng, genome_len)
    probs = [single_gap_problem(rng, g) for _ in range(n_typical)]
    probs += [edge_single_gap_problem(rng, g) for _ in range(n_edge)]
    return g, probs


def end_problems(seed=2025, n_typical=1200, n_edge=400, genome_len=20000):
    rng = random.Random(seed)
    g = random_genome(rng, genome_len)
    probs = [end_gap_problem(rng, g) for _ in range(n_typical)]
    probs += [end_gap_problem(rng, g, edge=True) for _ in range(n_edge)]
    return g, probs


def genome_problems(seed=2026, n_typical=1200, n_edge=400, genome_len=60000):
    rng = random.Random(seed)
    g = bytearray(random_genome(rng, genome_len))
    probs = [genome_gap_problem(rng, g) for _ in range(n_typical)]
    probs += [genome_gap_problem(rng, g, edge=True) for _ in range(n_edge)]
    return bytes(g), probs


def cdna_problems(seed=2027, n_typical=1000, n_edge=300, genome_len=30000):
    rng = random.Random(seed)
    g = random_genome(rng, genome_len)
    probs = [cdna_gap_problem(rng, g) for _ in range(n_typical)]
    probs += [cdna_gap_problem(rng, g, edge=True) for _ in range(n_edge)]
    return g, probs


def call_cdna(impl, p):
    return impl.cdna_gap(p)


def main_cdna():
    """Dynprog_cdna_gap goldens of both builds (the same problems; halfp does not apply)."""
    g, probs = cdna_problems()
    for name, variant in (("cdna_gap_golden.npz", "nosimd"), ("simd_cdna_gap_golden.npz", "avx2")):
        ref = Ref(variant)
        ref.set_genome(g)
        outputs = {"ref_" + variant: [call_cdna(ref, p) for p in probs]}
        out = os.path.join(HERE, name)
        np.savez_compressed(out, **pack(g, probs, outputs, CDNA_PARAMS))
        print("wrote %s: %d problems" % (out, len(probs)))


def pack(g, probs, outputs, names):
    par = np.array([[p[k] for k in names] for p in probs], dtype=np.int64)
    defect = np.array([p["defect_rate"] for p in probs], dtype=np.float64)
    qlen = np.array([len(p["q"]) for p in probs], dtype=np.int32)
    qbuf = np.frombuffer(b"".join(p["q"] for p in probs) or b"\0", dtype=np.uint8)
    qucbuf = np.frombuffer(b"".join(p["quc"] for p in probs) or b"\0", dtype=np.uint8)
    d = dict(genome=np.frombuffer(g, dtype=np.uint8), params=par, param_names=np.array(names), defect=defect,
             qlen=qlen, qbuf=qbuf, qucbuf=qucbuf)
    if "probsL" in probs[0]:
        d["splice_probs"] = np.array([x for p in probs for x in list(p["probsL"]) + list(p["probsR"])],
                                     dtype=np.float64)
    for tag, outs in outputs.items():
        nint = sum(1 for x in outs[0][0] if isinstance(x, int))
        if nint < len(outs[0][0]):
            d[tag + "_dscalars"] = np.array([o[0][nint:] for o in outs], dtype=np.float64)
        scal = np.array([o[0][:nint] for o in outs], dtype=np.int32)
        npairs = np.array([-1 if o[1] is None else len(o[1]) for o in outs], dtype=np.int32)
        flat = [pr for o in outs if o[1] is not None for pr in o[1]]
        d[tag + "_scalars"] = scal
        d[tag + "_npairs"] = npairs
        d[tag + "_pairs"] = np.array(flat, dtype=PAIR_DT)
    return d


def load(path):
    """Inverse of pack: (genome bytes, [problem dicts], {tag: [(scalars, pairs-or-None)]})."""
    z = dict(np.load(path, allow_pickle=False))  # NpzFile re-reads an array on every subscript
    names = [str(x) for x in z["param_names"]]
    qoff = np.concatenate([[0], np.cumsum(z["qlen"])])
    qb, qub = z["qbuf"].tobytes(), z["qucbuf"].tobytes()
    probs = []
    poff = 0
    for i, row in enumerate(z["params"]):
        p = {k: int(v) for k, v in zip(names, row)}
        p["defect_rate"] = float(z["defect"][i])
        p["q"] = qb[qoff[i]:qoff[i + 1]]
        p["quc"] = qub[qoff[i]:qoff[i + 1]]
        if "splice_probs" in z:
            gl, gr = max(0, p["glengthL"]), max(0, p["glengthR"])
            p["probsL"] = [float(x) for x in z["splice_probs"][poff:poff + gl]]
            p["probsR"] = [float(x) for x in z["splice_probs"][poff + gl:poff + gl + gr]]
            poff += gl + gr
        probs.append(p)
    outs = {}
    for key in z:
        if key.endswith("_scalars"):
            tag = key[:-len("_scalars")]
            scal, npairs, pairs = z[tag + "_scalars"], z[tag + "_npairs"], z[tag + "_pairs"]
            dscal = z[tag + "_dscalars"] if (tag + "_dscalars") in z else None
            res, pos = [], 0
            for i in range(len(scal)):
                n = int(npairs[i])
                sc = tuple(int(x) for x in scal[i]) + (() if dscal is None else tuple(float(x) for x in dscal[i]))
                if n < 0:
                    res.append((sc, None))
                    continue
                seg = pairs[pos:pos + n]
                pos += n
                res.append((sc,
                            [(int(r["querypos"]), int(r["genomepos"]), int(r["queryjump"]), int(r["genomejump"]),
                              int(r["dynprogindex"]), bytes(r["cdna"]) or b"\0", bytes(r["comp"]) or b"\0",
                              bytes(r["genome"]) or b"\0", bytes(r["genomealt"]) or b"\0", int(r["gapp"]))
                             for r in seg]))
            outs[tag] = res
    return z["genome"].tobytes(), probs, outs


def simd_domain(kind, p):
    """Problems on which the AVX2 build is defined: single gaps whose band reaches the corner
    (otherwise Dynprog_traceback_8/16 aborts with "Bad dir", dynprog_simd.c:9278), end gaps with
    rlength <= glength + 1 (otherwise the lower-triangle scans read columns filled from
    uninitialised pair scores), genome gaps with glengthL, glengthR > rlength (as for nosimd)."""
    if kind == "single":
        return p["widebandp"] or abs(p["rlength"] - p["glength"]) <= p["extraband"]
    if kind == "end":
        return p["endalign"] == 2 or p["rlength"] <= p["glength"] + 1
    return p["rlength"] <= 1 or (p["glengthL"] > p["rlength"] and p["glengthR"] > p["rlength"])


def main_simd():
    for name, maker, call, names, kind, seed in (
            ("simd_single_gap_golden.npz", single_problems, call_single, SINGLE_PARAMS, "single", 3024),
            ("simd_end_gap_golden.npz", end_problems, call_end, END_PARAMS, "end", 3025)):
        g, probs = maker(seed=seed)
        probs = [p for p in probs if simd_domain(kind, p)]
        ref = Ref("avx2")
        ref.set_genome(g)
        outputs = {"ref_avx2": [call(ref, p) for p in probs]}
        out = os.path.join(HERE, name)
        np.savez_compressed(out, **pack(g, probs, outputs, names))
        print("wrote %s: %d problems" % (out, len(probs)))
    g, probs = genome_problems(seed=3026)
    probs = [p for p in probs if simd_domain("genome", p)]
    ref, refa, orc = Ref("avx2"), Ref("avx2a"), Oracle()
    for r in (ref, refa, orc):
        r.set_genome(g)
    for p in probs:
        p["probsL"], p["probsR"] = splice_probs(ref, orc, p)
    outputs = {"ref_avx2": [(refa if p["flags"] & GG_FLAG_HALF else ref).genome_gap(p) for p in probs]}
    out = os.path.join(HERE, "simd_genome_gap_golden.npz")
    np.savez_compressed(out, **pack(g, probs, outputs, GENOME_PARAMS))
    print("wrote %s: %d problems" % (out, len(probs)))


def main():
    # nosimd goldens (the SIMD build's are main_simd)
    for name, maker, call, names in (("single_gap_golden.npz", single_problems, call_single, SINGLE_PARAMS),
                                     ("end_gap_golden.npz", end_problems, call_end, END_PARAMS)):
        g, probs = maker()
        ref = Ref("nosimd")
        ref.set_genome(g)
        outputs = {"ref_nosimd": [call(ref, p) for p in probs]}
        out = os.path.join(HERE, name)
        np.savez_compressed(out, **pack(g, probs, outputs, names))
        print("wrote %s: %d problems" % (out, len(probs)))
    g, probs = genome_problems()
    ref, refa, orc = Ref("nosimd"), Ref("nosimda"), Oracle()
    for r in (ref, refa, orc):
        r.set_genome(g)
    for p in probs:
        p["probsL"], p["probsR"] = splice_probs(ref, orc, p)
    outputs = {"ref_nosimd": [(refa if p["flags"] & GG_FLAG_HALF else ref).genome_gap(p) for p in probs]}
    out = os.path.join(HERE, "genome_gap_golden.npz")
    np.savez_compressed(out, **pack(g, probs, outputs, GENOME_PARAMS))
    print("wrote %s: %d problems" % (out, len(probs)))


OLIGO_PARAMS = ["chrstart", "chrend", "chroffset", "chrhigh", "plusp", "minor"]


def oligo_problems(seed=2028, n_typical=300, n_edge=100, genome_len=200000):
    rng = random.Random(seed)
    g = bytearray(random_genome(rng, genome_len))
    g[90000:91500] = b"A" * 1500  # an A-rich stretch: 8-mer counts past 256 (Count_T wraps)
    g = bytes(g)
    probs = [oligo_problem(rng, g) for _ in range(n_typical)]
    probs += [oligo_problem(rng, g, edge=True) for _ in range(n_edge)]
    return g, probs


def main_oligo():
    g, probs = oligo_problems()
    ref = Ref("nosimd")
    ref.set_genome(g)
    outs = [ref.oligo_mappings(p) for p in probs]
    assert all(len(o) == 4 for o in outs)
    d = dict(genome=np.frombuffer(g, dtype=np.uint8),
             params=np.array([[p[k] for k in OLIGO_PARAMS] for p in probs], dtype=np.int64),
             param_names=np.array(OLIGO_PARAMS), qlen=np.array([len(p["quc"]) for p in probs], dtype=np.int32),
             qucbuf=np.frombuffer(b"".join(p["quc"] for p in probs), dtype=np.uint8),
             scalars=np.array([o[0] for o in outs], dtype=np.int32),
             npositions=np.array([x for o in outs for x in o[1]], dtype=np.int32),
             npos_total=np.array([len(o[2]) for o in outs], dtype=np.int32),
             positions=np.array([x for o in outs for x in o[2]], dtype=np.uint32),
             diags=np.array([x for o in outs for d_ in o[3] for x in d_], dtype=np.int32))
    out = os.path.join(HERE, "oligo_golden.npz")
    np.savez_compressed(out, **d)
    print("wrote %s: %d problems" % (out, len(probs)))


def load_oligo(path):
    """(genome bytes, [problem dicts], [(scalars, npositions, positions, diagonals)])."""
    z = dict(np.load(path, allow_pickle=False))
    names = [str(x) for x in z["param_names"]]
    qoff = np.concatenate([[0], np.cumsum(z["qlen"])])
    poff = np.concatenate([[0], np.cumsum(z["npos_total"])])
    qub = z["qucbuf"].tobytes()
    probs, outs, doff = [], [], 0
    for i, row in enumerate(z["params"]):
        p = {k: int(v) for k, v in zip(names, row)}
        p["quc"] = qub[qoff[i]:qoff[i + 1]]
        probs.append(p)
        sc = tuple(int(x) for x in z["scalars"][i])
        nd = sc[3]
        dg = [tuple(int(x) for x in z["diags"][doff + 4 * k:doff + 4 * k + 4]) for k in range(nd)]
        doff += 4 * nd
        outs.append((sc, [int(x) for x in z["npositions"][qoff[i]:qoff[i + 1]]],
                     [int(x) for x in z["positions"][poff[i]:poff[i + 1]]], dg))
    return z["genome"].tobytes(), probs, outs


STAGE2_PARAMS = ["chrstart", "chrend", "chroffset", "chrhigh", "plusp", "splicingp", "maxintronlen"]


def stage2_problems(seed=2029, n_typical=240, n_edge=60, genome_len=300000):
    from dpbind import repeat_genome, stage2_problem
    rng = random.Random(seed)
    g = repeat_genome(rng, genome_len)
    probs = [stage2_problem(rng, g) for _ in range(n_typical)]
    probs += [stage2_problem(rng, g, edge=True) for _ in range(n_edge)]
    return g, probs


def main_stage2():
    g, probs = stage2_problems()
    ref = Ref("nosimd")
    ref.set_genome(g)
    outs = [ref.stage2_compute(p) for p in probs]
    assert all(o[0] != "err" for o in outs)
    flat = [pr for o in outs for path in o[1] for pr in path]
    d = dict(genome=np.frombuffer(g, dtype=np.uint8),
             params=np.array([[p[k] for k in STAGE2_PARAMS] for p in probs], dtype=np.int64),
             param_names=np.array(STAGE2_PARAMS), qlen=np.array([len(p["quc"]) for p in probs], dtype=np.int32),
             qbuf=np.frombuffer(b"".join(p["q"] for p in probs), dtype=np.uint8),
             nresults=np.array([o[0] for o in outs], dtype=np.int32),
             path_npairs=np.array([len(path) for o in outs for path in o[1]], dtype=np.int32),
             pairs_int=np.array([pr[:5] + (pr[9],) for pr in flat], dtype=np.int32).reshape(-1, 6),
             pairs_chr=np.array([[ord(c) for c in pr[5:9]] for pr in flat], dtype=np.uint8).reshape(-1, 4))
    out = os.path.join(HERE, "stage2_golden.npz")
    np.savez_compressed(out, **d)
    print("wrote %s: %d problems, %d results, %d pair records" % (out, len(probs), len(d["path_npairs"]), len(flat)))


def load_stage2(path):
    """(genome bytes, [problem dicts], [(nresults, [pair-key lists])])."""
    z = dict(np.load(path, allow_pickle=False))  # NpzFile re-reads an array on every subscript
    names = [str(x) for x in z["param_names"]]
    qoff = np.concatenate([[0], np.cumsum(z["qlen"])])
    qb = z["qbuf"].tobytes()
    z["pairs_int"] = z["pairs_int"].tolist()
    z["pairs_chr"] = z["pairs_chr"].tolist()
    probs, outs, pi, ri = [], [], 0, 0
    for i, row in enumerate(z["params"]):
        p = {k: int(v) for k, v in zip(names, row)}
        p["q"] = qb[qoff[i]:qoff[i + 1]]
        p["quc"] = p["q"].upper()
        probs.append(p)
        paths = []
        for _ in range(int(z["nresults"][i])):
            n = int(z["path_npairs"][ri])
            ri += 1
            paths.append([tuple(int(x) for x in z["pairs_int"][pi + j][:5])
                          + tuple(bytes([int(c)]) for c in z["pairs_chr"][pi + j])
                          + (int(z["pairs_int"][pi + j][5]),) for j in range(n)])
            pi += n
        outs.append((int(z["nresults"][i]), paths))
    return z["genome"].tobytes(), probs, outs


ME_PARAMS = ["rlength", "roffset", "goffsetL", "rev_goffsetR", "cdna_direction", "chroffset", "chrhigh", "watsonp",
             "genestrand", "dynprogindex"]


def microexon_problems(seed=2030, n=600, genome_len=1500000):
    from dpbind import microexon_problem
    rng = random.Random(seed)
    g = bytearray(random_genome(rng, genome_len))
    at = [100]
    probs = [microexon_problem(rng, g, edge=(i % 4 == 0), at=at) for i in range(n)]
    return bytes(g), probs


def main_microexon():
    """Dynprog_microexon_int: the reference's outputs, and per problem the candidate list (the oracle's,
    in the reference's loop order) with the reference's own MaxEnt probabilities at its splice sites."""
    from dpbind import Oracle, microexon_probs
    g, probs = microexon_problems()
    ref, orc = Ref("nosimd"), Oracle()
    ref.set_genome(g)
    orc.set_genome(g)
    outs = [ref.microexon_int(p) for p in probs]
    cands = [orc.microexon_candidates(p) or [] for p in probs]
    cprobs = [microexon_probs(ref, c, p["chroffset"]) for c, p in zip(cands, probs)]
    assert all(orc.microexon_int(p, cp) == o for p, cp, o in zip(probs, cprobs, outs))
    flat = [pr for o in outs for pr in (o[2] or [])]
    d = dict(genome=np.frombuffer(g, dtype=np.uint8),
             params=np.array([[p[k] for k in ME_PARAMS] for p in probs], dtype=np.int64),
             param_names=np.array(ME_PARAMS), qbuf=np.frombuffer(b"".join(p["q"] for p in probs), dtype=np.uint8),
             scalars=np.array([o[0] for o in outs], dtype=np.int32),
             dscalars=np.array([o[1] for o in outs], dtype=np.float64),
             npairs=np.array([-1 if o[2] is None else len(o[2]) for o in outs], dtype=np.int32),
             ncands=np.array([len(c) for c in cands], dtype=np.int32),
             cands=np.array([list(x) for c in cands for x in c], dtype=np.int64).reshape(-1, 8),
             cand_probs=np.array([x for cp in cprobs for x in cp], dtype=np.float64),
             pairs_int=np.array([pr[:5] + (pr[9],) for pr in flat], dtype=np.int32).reshape(-1, 6),
             pairs_chr=np.array([[ord(c) for c in pr[5:9]] for pr in flat], dtype=np.uint8).reshape(-1, 4))
    out = os.path.join(HERE, "microexon_golden.npz")
    np.savez_compressed(out, **d)
    print("wrote %s: %d problems, %d found, %d candidates" % (out, len(probs), sum(o[2] is not None for o in outs),
                                                             len(d["cands"])))


def load_microexon(path):
    """(genome bytes, [problem dicts], [candidate lists], [flat candidate probabilities],
    [((dpi, microintrontype), (prob2, prob3), pairs-or-None)])."""
    z = dict(np.load(path, allow_pickle=False))
    names = [str(x) for x in z["param_names"]]
    qoff = np.concatenate([[0], np.cumsum(z["params"][:, names.index("rlength")])])
    qb = z["qbuf"].tobytes()
    pint, pchr, cands_all = z["pairs_int"].tolist(), z["pairs_chr"].tolist(), z["cands"].tolist()
    cp_all = z["cand_probs"].tolist()
    probs, cands, cprobs, outs, pi, ci = [], [], [], [], 0, 0
    for i, row in enumerate(z["params"]):
        p = {k: int(v) for k, v in zip(names, row)}
        p["q"] = qb[qoff[i]:qoff[i + 1]]
        p["quc"] = p["q"].upper()
        probs.append(p)
        k = int(z["ncands"][i])
        cands.append([tuple(int(x) for x in c) for c in cands_all[ci:ci + k]])
        cprobs.append(cp_all[2 * ci:2 * (ci + k)])
        ci += k
        n = int(z["npairs"][i])
        pairs = None
        if n >= 0:
            pairs = [tuple(int(x) for x in pint[pi + j][:5]) + tuple(bytes([int(c)]) for c in pchr[pi + j])
                     + (int(pint[pi + j][5]),) for j in range(n)]
            pi += n
        outs.append((tuple(int(x) for x in z["scalars"][i]), tuple(float(x) for x in z["dscalars"][i]), pairs))
    return z["genome"].tobytes(), probs, cands, cprobs, outs


SJ_PARAMS = ["end3p", "rlength", "glength", "roffset", "goffset_anchor", "goffset_far", "genestrand", "jump_late_p",
             "extraband", "contlength", "dynprogindex"]


def splicejunction_problems(seed=2031, n_typical=1200, n_edge=400, genome_len=60000):
    from dpbind import splicejunction_problem
    rng = random.Random(seed)
    g = random_genome(rng, genome_len)
    probs = [splicejunction_problem(rng, g) for _ in range(n_typical)]
    probs += [splicejunction_problem(rng, g, edge=True) for _ in range(n_edge)]
    return g, probs


def main_splicejunction():
    g, probs = splicejunction_problems()
    ref = Ref("nosimd")
    ref.set_genome(g)
    outputs = {"ref_nosimd": [ref.end_splicejunction(p) for p in probs]}
    d = pack(g, probs, outputs, SJ_PARAMS)
    d["jlen"] = np.array([len(p["j"]) for p in probs], dtype=np.int32)
    d["jbuf"] = np.frombuffer(b"".join(p["j"] for p in probs), dtype=np.uint8)
    out = os.path.join(HERE, "splicejunction_golden.npz")
    np.savez_compressed(out, **d)
    print("wrote %s: %d problems, %d NULL" % (out, len(probs), sum(o[1] is None for o in outputs["ref_nosimd"])))


def load_splicejunction(path):
    g, probs, outs = load(path)
    z = np.load(path, allow_pickle=False)
    joff = np.concatenate([[0], np.cumsum(z["jlen"])])
    jb = z["jbuf"].tobytes()
    for i, p in enumerate(probs):
        p["j"] = jb[joff[i]:joff[i + 1]]
    return g, probs, outs


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "simd":
        main_simd()
    elif len(sys.argv) > 1 and sys.argv[1] == "cdna":
        main_cdna()
    elif len(sys.argv) > 1 and sys.argv[1] == "oligo":
        main_oligo()
    elif len(sys.argv) > 1 and sys.argv[1] == "stage2":
        main_stage2()
    elif len(sys.argv) > 1 and sys.argv[1] == "microexon":
        main_microexon()
    elif len(sys.argv) > 1 and sys.argv[1] == "splicejunction":
        main_splicejunction()
    else:
        main()
