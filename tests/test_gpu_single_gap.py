"""GPU parity tests: the HIP engine (libgmapdp.so through its C ABI) against
the oracle restatement and the reference's golden vectors.  Bar: bit-exact
pairs, scores, counters and dynprogindex (integer/byte work)."""
import os
import random

import numpy as np
import pytest

import gmapdp
from dpbind import (Oracle, Ref, call_single, edge_single_gap_problem, random_genome, ref_available,
                    single_gap_problem)

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(HERE, "golden", "single_gap_golden.npz"))


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0)
    yield e
    e.close()


def _first_diff(got, exp):
    for i, (a, b) in enumerate(zip(got, exp)):
        if a != b:
            return i, a, b
    return None


def test_gpu_matches_reference_golden(engine):
    g, probs, outs = _golden()
    engine.set_genome(g)
    got = engine.single_gap_batch(probs)
    d = _first_diff(got, outs["ref_nosimd"])
    assert d is None, "problem %d: gpu %s vs ref %s" % (d[0], d[1][0], d[2][0])


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_matches_oracle_random(engine, seed):
    rng = random.Random(1000 + seed)
    g = random_genome(rng, 60000)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs = [single_gap_problem(rng, g) if i % 5 else edge_single_gap_problem(rng, g) for i in range(6000)]
    got = engine.single_gap_batch(probs)
    exp = [call_single(orc, p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs oracle %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc")}, d[1], d[2])


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects did not travel")
def test_gpu_matches_reference_objects(engine):
    rng = random.Random(77)
    g = random_genome(rng, 40000)
    engine.set_genome(g)
    ref = Ref("nosimd")
    ref.set_genome(g)
    probs = [single_gap_problem(rng, g) if i % 3 else edge_single_gap_problem(rng, g) for i in range(3000)]
    got = engine.single_gap_batch(probs)
    exp = [call_single(ref, p) for p in probs]
    assert _first_diff(got, exp) is None


def test_gpu_size_guard_and_empty(engine):
    rng = random.Random(3)
    g = random_genome(rng, 5000)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    base = single_gap_problem(rng, g)
    probs = []
    for rl, gl in [(0, 10), (10, 0), (661, 700), (100, 2001), (660, 2000), (1, 1)]:
        p = dict(base)
        q = bytes(rng.choice(b"ACGT") for _ in range(max(rl, 1)))
        p.update(q=q, quc=q, rlength=rl, glength=gl, goffset=100, watsonp=1, dynprogindex=-3)
        probs.append(p)
    got = engine.single_gap_batch(probs)
    exp = [call_single(orc, p) for p in probs]
    assert got == exp
    assert engine.single_gap_batch([]) == []


def test_gpu_deterministic_and_self_consistent_at_scale(engine):
    """Size-independent properties at bench scale: repeat runs are identical,
    counters agree with the emitted pairs, and a random sample matches the oracle."""
    rng = random.Random(11)
    g = random_genome(rng, 400000)
    engine.set_genome(g)
    probs = [single_gap_problem(rng, g) for _ in range(40000)]
    a = engine.single_gap_batch(probs)
    b = engine.single_gap_batch(probs)
    assert a == b
    for (scal, pairs) in a:
        if pairs is None:
            continue
        nm = sum(1 for x in pairs if x[9] == 0 and x[6] in (b"*", b":"))
        nmm = sum(1 for x in pairs if x[9] == 0 and x[6] == b" ")
        assert nm <= scal[2] and nmm <= scal[3]
    orc = Oracle()
    orc.set_genome(g)
    for i in rng.sample(range(len(probs)), 1500):
        assert a[i] == call_single(orc, probs[i]), i


def _stage3_band_problem(rng, g):
    """stage3.c:9070-9077: Dynprog_single_gap with extraband_single = |queryjump - genomejump|
    (widebandp), so the band runs to ~3 x glength -- wider than the matrix (seen on real reads:
    a 1,400-nt genome jump over a short query gap)."""
    p = edge_single_gap_problem(rng, g)
    glength = rng.choice([rng.randint(900, 2000), rng.randint(40, 900)])
    rlength = rng.choice([rng.randint(1, 60), rng.randint(1, 660)])
    goffset = rng.randint(1, len(g) - glength - 1)
    seg = g[goffset:goffset + glength]
    a = rng.randint(0, max(0, glength - rlength))
    q = bytes(seg[a:a + rlength]) if rng.random() < 0.7 else bytes(rng.choice(b"ACGT") for _ in range(rlength))
    q = (q + b"A" * rlength)[:rlength]
    if rng.random() < 0.3:  # swap: query gap longer than the genome gap
        glength, q = max(1, rlength // 3), q
    p.update(q=q, quc=q, rlength=len(q), glength=glength, goffset=goffset, watsonp=1, widebandp=1,
             extraband=max(3, abs(len(q) - glength)))
    return p


def test_gpu_stage3_band_wider_than_matrix(engine):
    """Bands far past the matrix edges (found by the end-to-end run: band > 4096 cells) give the
    same cells as the clamped band: engine vs oracle, and vs the reference objects when present."""
    rng = random.Random(4242)
    g = random_genome(rng, 60000)
    engine.set_genome(g)
    probs = [_stage3_band_problem(rng, g) for _ in range(600)]
    assert max(abs(p["rlength"] - p["glength"]) * 3 + 1 for p in probs) > 4096
    got = engine.single_gap_batch(probs)
    orc = Oracle()
    orc.set_genome(g)
    d = _first_diff(got, [call_single(orc, p) for p in probs])
    assert d is None, "problem %d: gpu %s vs oracle %s" % d
    if ref_available("nosimd"):
        ref = Ref("nosimd")
        ref.set_genome(g)
        assert _first_diff(got, [call_single(ref, p) for p in probs[:200]]) is None
