"""Spot check of bench.py's own workload against the oracle (VERDICT r2 "the bench's outputs are never
checked"): the sub-problems of a bench read block -- generated exactly as bench.py generates them
(gmapdp.workload: packed genome, the stream's planted intron sites, block seeds) at the bench's real
universal coordinates -- run on the engine with the whole genome resident in HBM, and a 1 % sample of
every family (Dynprog_single_gap, _end5/3_gap, _genome_gap, _microexon_int, Stage2_compute) is compared
bit-exactly with the oracle run on the problem's chromosome alone (chroffset 0; outputs are
chromosome-relative, so only the addresses the kernels compute differ, as in test_gpu_large_coords.py).
The splice-site probabilities are GMAP's MaxEnt models as the bench computes them: on the device at the
universal coordinates (gmapdp.DEVICE), against the oracle's restatement on the chromosome alone -- so the
device MaxEnt is pinned past 2^31 (GRCh38) and past 2^32 (wheat) too.

configs[2]: block 0 of the default bench stream (GRCh38 layout, 3.09 Gnt, 10 000 reads, 8 blocks planted).
configs[4]: a 2 000-read block of the Iso-Seq stream on the 17-Gnt wheat layout (coordinates past 2^32),
sampled on its three smallest chromosomes."""
import random

import numpy as np
import pytest

import gmapdp
from gmapdp import workload as W
from dpbind import Oracle, call_end, call_single, microexon_probs, oracle_splice_probs

pytestmark = pytest.mark.gpu
TAIL = 8192


def _sample(n, frac, rng, allowed=None):
    idx = np.arange(n) if allowed is None else np.nonzero(allowed)[0]
    k = max(1, int(round(frac * n)))
    return np.sort(rng.choice(idx, size=min(k, len(idx)), replace=False)) if len(idx) else idx


def _run(layout, shape, reads, nblocks, chroms=None, frac=0.01):
    genome = W.PackedGenome(layout.total, seed=38)
    W.plant_stream(genome, layout, reads, range(nblocks), shape)
    d = W.make_blocks(genome, layout, reads, [0], shape=shape, sprob=False)[0]
    eng = gmapdp.Engine(0)
    eng.set_genome(blocks=genome.blocks, length=genome.length)
    rng = np.random.default_rng(77)
    allow = None
    if chroms is not None:
        offs = set(int(layout.offsets[layout.names.index(c)]) for c in chroms)
        allow = lambda arr: np.isin(arr["chroffset"].astype(np.int64), list(offs))  # noqa: E731
    q = d["q"].tobytes()
    sp, ep, gp, mp, op = d["single"], d["end"], d["genome"], d["microexon"], d["oligo"]
    pick = {"single": _sample(len(sp), frac, rng, allow and allow(sp)),
            "end": _sample(len(ep), frac, rng, allow and allow(ep)),
            "genome": _sample(len(gp), frac, rng, allow and allow(gp)),
            "microexon": _sample(len(mp), frac, rng, allow and allow(mp)),
            "oligo": _sample(len(op), frac, rng, allow and allow(op))}

    def single_call(p):
        o, r = int(p["qoff"]), int(p["rlength"])
        f = int(p["flags"])
        return dict(q=q[o:o + r], quc=q[o:o + r], rlength=r, glength=int(p["glength"]), roffset=int(p["roffset"]),
                    goffset=int(p["goffset"]), chroffset=int(p["chroffset"]), chrhigh=int(p["chrhigh"]),
                    watsonp=f & 1, genestrand=int(p["genestrand"]), jump_late_p=(f >> 1) & 1,
                    extraband=int(p["extraband"]), widebandp=(f >> 2) & 1, defect_rate=float(p["defect_rate"]),
                    dynprogindex=int(p["dynprogindex"]))

    def end_call(p):
        c = single_call(p)
        del c["widebandp"]
        c.update(end3p=int(p["end3p"]), endalign=int(p["endalign"]), require_pos_score_p=int(p["require_pos_score_p"]))
        return c

    def genome_call(p):
        o, r = int(p["qoff"]), int(p["rlength"])
        c = {k: int(p[k]) for k in ("rlength", "glengthL", "glengthR", "roffset", "goffsetL", "rev_goffsetR",
                                    "chroffset", "chrhigh", "flags", "cdna_direction", "genestrand", "extraband",
                                    "maxpeelback", "dynprogindex")}
        c.update(q=q[o:o + r], quc=q[o:o + r], defect_rate=float(p["defect_rate"]))
        return c

    def mx_call(p):
        o, r = int(p["qoff"]), int(p["rlength"])
        c = {k: int(p[k]) for k in ("rlength", "roffset", "goffsetL", "rev_goffsetR", "cdna_direction", "chroffset",
                                    "chrhigh", "watsonp", "genestrand", "dynprogindex")}
        c.update(q=q[o:o + r], quc=q[o:o + r])
        return c

    def s2_call(p):
        o, n = int(p["qoff"]), int(p["querylength"])
        s = d["oq"][o:o + n].tobytes()
        return dict(q=s, quc=s, chrstart=int(p["chrstart"]), chrend=int(p["chrend"]), chroffset=int(p["chroffset"]),
                    chrhigh=int(p["chrhigh"]), plusp=int(p["plusp"]), splicingp=1, maxintronlen=500000)

    calls = {"single": [single_call(sp[i]) for i in pick["single"]], "end": [end_call(ep[i]) for i in pick["end"]],
             "genome": [genome_call(gp[i]) for i in pick["genome"]], "microexon": [mx_call(mp[i]) for i in pick["microexon"]],
             "oligo": [s2_call(op[i]) for i in pick["oligo"]]}
    # the engine, at universal coordinates (MaxEnt on the device)
    got = {"single": eng.single_gap_batch(calls["single"]), "end": eng.end_gap_batch(calls["end"]),
           "genome": eng.genome_gap_batch(calls["genome"], gmapdp.DEVICE),
           "microexon": eng.microexon_batch(calls["microexon"], gmapdp.DEVICE),
           "oligo": eng.stage2_batch(calls["oligo"])}
    eng.close()
    # the oracle, chromosome by chromosome
    orc = Oracle()
    bad = {k: [] for k in calls}
    byc = {}
    for fam, lst in calls.items():
        for k, c in enumerate(lst):
            byc.setdefault((c["chroffset"], c["chrhigh"]), []).append((fam, k))
    for (cho, chh), items in sorted(byc.items()):
        orc.set_genome(genome.ascii(cho, min(genome.length, chh + TAIL)))
        for fam, k in items:
            c = dict(calls[fam][k], chroffset=0, chrhigh=chh - cho)
            if fam == "single":
                exp = call_single(orc, c)
            elif fam == "end":
                exp = call_end(orc, c)
            elif fam == "genome":
                exp = orc.genome_gap(c, *oracle_splice_probs(orc, c))
            elif fam == "microexon":
                cands = orc.microexon_candidates(c) or []
                exp = orc.microexon_int(c, microexon_probs(orc, cands, 0))
            else:
                exp = orc.stage2_compute(c)
            if got[fam][k] != exp:
                bad[fam].append(int(pick[fam][k]))
    sizes = {k: len(v) for k, v in calls.items()}
    assert not any(bad.values()), "bench-workload problems differ from the oracle: %s of %s" % (
        {k: v[:8] for k, v in bad.items() if v}, sizes)
    return sizes, got


def test_gpu_bench_configs2_block_sample():
    sizes, got = _run(W.Layout(W.GRCH38), W.CDNA2K, 10000, 8)
    assert sizes["single"] > 2000 and sizes["genome"] > 4000 and sizes["oligo"] >= 150
    assert sum(1 for r in got["oligo"] if r[0] > 0) > 0.9 * sizes["oligo"]     # the reads chain


def test_gpu_bench_configs4_block_sample():
    lay = W.Layout(W.WHEAT17)
    small = [lay.names[i] for i in np.argsort(lay.lens)[:3]]
    sizes, got = _run(lay, W.ISOSEQ5K, 2000, 1, chroms=small, frac=0.05)
    assert sizes["oligo"] >= 5 and sizes["genome"] > 100
    assert sum(1 for r in got["oligo"] if r[0] > 0) > 0.8 * sizes["oligo"]
