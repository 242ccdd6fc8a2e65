"""GPU parity of the engine's device MaxEnt: Maxent_hr_*_prob on the device
(gmapdp_maxent_sites, csrc/me_device.h) and its uses -- the genome gaps' probability arena computed in the
batch (splice_probs = NULL), the microexon choice with the candidates' sites evaluated in the finish kernel
(cand_probs = NULL) and the one-round-trip whole microexon call (gmapdp_mixed whole section).

Bar: doubles bit-identical to the oracle restatement (pinned to the reference's own functions on the CPU,
tests/test_maxent.py) at every position of a test genome, both strands' models; every genome-gap and
microexon output equal to the reference objects' (which evaluate their own MaxEnt) and to the oracle fed
the oracle's MaxEnt.
"""
import random

import numpy as np
import pytest

import gmapdp
from dpbind import (GG_FLAG_HALF, Oracle, Ref, genome_gap_problem, microexon_probs, microexon_problem,
                    oracle_splice_probs, random_genome, ref_available)
from test_maxent import site_genome

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0)
    yield e
    e.close()


def test_gpu_maxent_sites_bit_identical_everywhere(engine):
    g = site_genome()
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    n = len(g) + 8
    pos = np.tile(np.arange(n, dtype=np.uint64), 4)
    models = np.repeat(np.arange(4, dtype=np.uint8), n)
    for chroffset in (0, 7000):
        got = engine.maxent_sites(pos, models, chroffset)
        exp = np.array([orc.maxent(int(m), int(p), chroffset) for p, m in zip(pos, models)])
        bad = np.nonzero(got.view(np.uint64) != exp.view(np.uint64))[0]
        assert len(bad) == 0, (chroffset, bad[:5], got[bad[:5]], exp[bad[:5]])
        assert (got > 0.9).sum() > 100
    if ref_available("nosimd"):
        ref = Ref("nosimd")
        ref.set_genome(g)
        sel = np.arange(0, len(pos), 7)
        got = engine.maxent_sites(pos[sel], models[sel], 0)
        exp = np.array([ref.maxent(int(m), int(p), 0) for p, m in zip(pos[sel], models[sel])])
        assert np.array_equal(got.view(np.uint64), exp.view(np.uint64))


def _gg_problems(seed, n=2000, size=80000):
    rng = random.Random(seed)
    g = bytearray(random_genome(rng, size))
    probs = [genome_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(n)]
    return bytes(g), probs


def _first_diff(got, exp):
    for i, (a, b) in enumerate(zip(got, exp)):
        if a != b:
            return i, a, b
    return None


def test_gpu_genome_gap_device_maxent_matches_oracle(engine):
    g, probs = _gg_problems(811)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    got = engine.genome_gap_batch(probs, gmapdp.DEVICE)
    exp = [orc.genome_gap(p, *oracle_splice_probs(orc, p)) for p in probs]
    assert _first_diff(got, exp) is None, _first_diff(got, exp)
    assert sum(1 for o in got if o[1]) > 500


@pytest.mark.skipif(not ref_available("nosimda"), reason="reference objects did not travel")
def test_gpu_genome_gap_device_maxent_matches_reference_objects(engine):
    """The reference's Dynprog_genome_gap evaluates Maxent_hr_*_prob itself: no probability crosses over."""
    g, probs = _gg_problems(79)
    engine.set_genome(g)
    ref, refa = Ref("nosimd"), Ref("nosimda")
    for r in (ref, refa):
        r.set_genome(g)
    got = engine.genome_gap_batch(probs, gmapdp.DEVICE)
    exp = [(refa if p["flags"] & GG_FLAG_HALF else ref).genome_gap(p) for p in probs]
    assert _first_diff(got, exp) is None, _first_diff(got, exp)


def test_gpu_genome_gap_device_maxent_simd(engine):
    g, probs = _gg_problems(812, n=800)
    probs = [p for p in probs if p["rlength"] <= 1 or (p["glengthL"] > p["rlength"] and p["glengthR"] > p["rlength"])]
    for p in probs:
        p["simd"] = True
    engine.set_genome(g)
    orc = Oracle(simd=True)
    orc.set_genome(g)
    got = engine.genome_gap_batch(probs, gmapdp.DEVICE)
    exp = [orc.genome_gap(p, *oracle_splice_probs(orc, p)) for p in probs]
    assert _first_diff(got, exp) is None, _first_diff(got, exp)


def _mx_problems(seed, n=800):
    rng = random.Random(seed)
    g = bytearray(random_genome(rng, 3000000))
    at = [100]
    probs = [microexon_problem(rng, g, edge=(i % 4 == 0), at=at) for i in range(n)]
    return bytes(g), probs


@pytest.mark.parametrize("whole", [False, True])
def test_gpu_microexon_device_maxent(engine, whole):
    g, probs = _mx_problems(9600 + whole)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    got = engine.microexon_whole_batch(probs) if whole else engine.microexon_batch(probs, gmapdp.DEVICE)
    exp = [orc.microexon_int(p, microexon_probs(orc, orc.microexon_candidates(p), p["chroffset"])) for p in probs]
    for i, (a, b) in enumerate(zip(got, exp)):
        assert a == b, (i, a[:2], b[:2])
    assert sum(o[2] is not None for o in got) > 200
    if ref_available("nosimd"):
        ref = Ref("nosimd")
        ref.set_genome(g)
        assert got == [ref.microexon_int(p) for p in probs]


def test_gpu_microexon_whole_calls_past_the_candidate_pool(engine):
    """Whole calls with more candidates than a search keeps in LDS (test_gpu_microexon_many_candidates'
    construction, ~3 000 candidates each) next to ordinary ones: rerun inside the batch, same answers."""
    rng = random.Random(9600)
    tile = b"AGACGGT"
    body = bytearray(b"GT" + tile * 3000 + b"AG")
    gg = bytearray(random_genome(rng, 100000))
    start = 2000
    gg[start:start + 5] = b"ACGTA"
    gg[start + 5:start + 5 + len(body)] = body
    end = start + 5 + len(body)
    gg[end:end + 6] = b"TTGCAC"
    at = [end + 2000]
    others = [microexon_problem(rng, gg, at=at) for _ in range(20)]
    gg = bytes(gg)
    q = b"ACGTA" + b"ACG" + b"TTGCAC"
    big = dict(q=q, quc=q, rlength=len(q), roffset=100, goffsetL=start - 1000, rev_goffsetR=end + 5 - 1000,
               cdna_direction=1, chroffset=1000, chrhigh=len(gg) - 1000, watsonp=1, genestrand=0, dynprogindex=3)
    probs = [big] + others + [big]
    engine.set_genome(gg)
    orc = Oracle()
    orc.set_genome(gg)
    assert len(orc.microexon_candidates(big)) > 256
    got = engine.microexon_whole_batch(probs)
    exp = [orc.microexon_int(p, microexon_probs(orc, orc.microexon_candidates(p), p["chroffset"])) for p in probs]
    assert got == exp
