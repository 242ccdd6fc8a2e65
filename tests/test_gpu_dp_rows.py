"""Single and end gaps whose band is much wider than the query (a short query across a long genomic
gap: the stage-3 single gaps over ~2000-nt gaps that GMAP issues for every spliced read).  The engine
fills these with lanes over the query's rows (dpr_kernel, fill_rows in dp_device.h) instead of band
offsets; the results must stay bit-exact against the oracle (and the reference objects where built)."""
import random

import pytest

import gmapdp
from dpbind import (Oracle, Ref, call_end, call_single, end_gap_problem, mutate, random_genome, ref_available,
                    revcomp)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0)
    yield e
    e.close()


def pick_r(w):
    r = 1
    while r * 64 < w:
        r <<= 1
    return r


def wide_single(rng, g):
    """query = the two ends of a long genome segment (an intron-like gap in between), mutated, or a
    random short query; row counts around the 64-row word boundaries"""
    glength = rng.randint(300, 2000)
    watsonp = rng.random() < 0.6
    goffset = rng.randint(1, len(g) - glength - 2)
    seg = g[goffset:goffset + glength] if watsonp else revcomp(g[len(g) - goffset - glength + 1:len(g) - goffset + 1])
    want = rng.choice([1, 2, 5, 20, 40, 63, 64, 65, 100, 127, 128, 129, 200, 255, 256, 300, 450, 640])
    want = min(want, glength // 2, 660)
    mode = rng.random()
    if mode < 0.15:
        q = bytes(rng.choice(b"ACGT") for _ in range(max(1, want)))
        quc = q
    else:
        a = rng.randint(0, want)
        piece = seg[:a] + seg[glength - (want - a):] if want - a > 0 else seg[:a]
        q, quc = mutate(rng, piece or seg[:1], sub=rng.choice([0.0, 0.02, 0.08]), indel=rng.choice([0.0, 0.02]))
        q, quc = (q or b"A")[:660], (quc or b"A")[:660]
    return dict(q=q, quc=quc, rlength=len(q), glength=glength, roffset=rng.randint(0, 3000), goffset=goffset,
                chroffset=0, chrhigh=len(g), watsonp=int(watsonp), genestrand=0, jump_late_p=rng.randint(0, 1),
                extraband=rng.choice([0, 3, 6, 6, 14, 40]), widebandp=int(rng.random() < 0.9),
                defect_rate=rng.choice([0.001, 0.005, 0.02, 0.05]), dynprogindex=rng.choice([1, 5, -1, -7]))


def wide_end(rng, g):
    p = end_gap_problem(rng, g)
    L = rng.choice([1, 3, 10, 40, 63, 64, 65, 120, 130, 250])
    p["glength"] = rng.randint(max(L + 100, 300), 2000)
    if p["end3p"]:
        p["goffset"] = rng.randint(1, len(g) - p["glength"] - 2)
    else:
        p["goffset"] = rng.randint(p["glength"] + 1, len(g) - 2)
    q = (p["q"] * (L // max(1, len(p["q"])) + 1))[:L] if p["q"] else b"A" * L
    p.update(q=q, quc=q.upper(), rlength=len(q))
    return p


def _check(got, exp, probs):
    for i, (a, b) in enumerate(zip(got, exp)):
        assert a == b, "problem %d (%s): gpu %s vs expected %s" % (
            i, {k: v for k, v in probs[i].items() if k not in ("q", "quc")}, a, b)


@pytest.mark.parametrize("seed", [1, 2])
def test_wide_single_gaps_vs_oracle(engine, seed):
    rng = random.Random(4400 + seed)
    g = random_genome(rng, 80000)
    probs = [wide_single(rng, g) for _ in range(1500)]
    rows = sum(1 for p in probs if p["widebandp"] and
               pick_r(p["rlength"] + 1) < pick_r(abs(p["glength"] - p["rlength"]) + 2 * p["extraband"] + 1))
    assert rows > len(probs) // 2  # most of the set takes the row layout
    engine.set_genome(g)
    got = engine.single_gap_batch(probs)
    small = [x for i in range(0, len(probs), 100) for x in engine.single_gap_batch(probs[i:i + 100])]
    assert small == got  # latency-mode planning gives the same answers
    orc = Oracle()
    orc.set_genome(g)
    _check(got, [call_single(orc, p) for p in probs], probs)


def test_wide_end_gaps_vs_oracle(engine):
    rng = random.Random(4500)
    g = random_genome(rng, 80000)
    probs = [wide_end(rng, g) for _ in range(1500)]
    engine.set_genome(g)
    got = engine.end_gap_batch(probs)
    orc = Oracle()
    orc.set_genome(g)
    _check(got, [call_end(orc, p) for p in probs], probs)


@pytest.mark.skipif(not ref_available(), reason="reference objects not built")
def test_wide_single_gaps_vs_reference(engine):
    rng = random.Random(4600)
    g = random_genome(rng, 80000)
    probs = [wide_single(rng, g) for _ in range(400)]
    engine.set_genome(g)
    got = engine.single_gap_batch(probs)
    ref = Ref()
    ref.set_genome(g)
    _check(got, [call_single(ref, p) for p in probs], probs)
