"""GPU parity tests for Dynprog_end5_splicejunction / Dynprog_end3_splicejunction (SURVEY §8a a13;
dynprog_end.c:1653/2249), bit-exact against the reference's golden fixture, the oracle restatement
and -- where they travelled -- the reference objects themselves."""
import os
import random

import pytest

import gmapdp
from dpbind import Oracle, Ref, random_genome, ref_available, splicejunction_problem

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load_splicejunction(os.path.join(HERE, "golden", "splicejunction_golden.npz"))


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


def _desc(p):
    return {k: v for k, v in p.items() if k not in ("q", "quc", "j")}


def test_gpu_splicejunction_matches_reference_golden(engine):
    g, probs, outs = _golden()
    got = engine.end_splicejunction_batch(probs)
    assert len(got) == len(probs) == 1600
    d = _first_diff(got, outs["ref_nosimd"])
    assert d is None, "problem %d (%s): gpu %s vs ref %s" % (d[0], _desc(probs[d[0]]), d[1], d[2])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_splicejunction_matches_oracle_random(engine, seed):
    rng = random.Random(5150 + seed)
    g = random_genome(rng, 200000)
    orc = Oracle()
    orc.set_genome(g)
    probs = [splicejunction_problem(rng, g, edge=(i % 6 == 0)) for i in range(4000)]
    got = engine.end_splicejunction_batch(probs)
    exp = [orc.end_splicejunction(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs oracle %s" % (d[0], _desc(probs[d[0]]), d[1], d[2])
    # every branch of the path was exercised: NULL by the size guard, NULL by a negative endpoint,
    # lists with the known gap holder inside and at either end
    kinds = set()
    for s, pairs in got:
        if pairs is None:
            kinds.add("guard" if s[2] == -100 else "negative")
        else:
            kinds.add("pairs")
            assert pairs[s[7]][0] == -1 and pairs[s[7]][9] == 1
    assert kinds == {"guard", "negative", "pairs"}


def test_gpu_splicejunction_wide_bands_and_long_junctions(engine):
    """Junctions up to 2000 nt against short and long read ends: bands wider than 64 lanes (R up to 32)
    and direction planes in the global scratch."""
    rng = random.Random(77)
    g = random_genome(rng, 300000)
    orc = Oracle()
    orc.set_genome(g)
    probs = []
    while len(probs) < 400:
        p = splicejunction_problem(rng, g)
        if p["glength"] < 300:
            continue
        probs.append(p)
    for p in probs[:40]:  # maximum sizes
        p["glength"] = 2000
        p["j"] = (p["j"] * (2000 // max(1, len(p["j"])) + 1))[:2000]
    got = engine.end_splicejunction_batch(probs)
    exp = [orc.end_splicejunction(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs oracle %s" % (d[0], _desc(probs[d[0]]), d[1], d[2])


def test_gpu_splicejunction_empty_batch(engine):
    assert engine.end_splicejunction_batch([]) == []


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects did not travel")
def test_gpu_splicejunction_matches_reference_objects(engine):
    rng = random.Random(9090)
    g = random_genome(rng, 200000)
    ref = Ref("nosimd")
    ref.set_genome(g)
    probs = [splicejunction_problem(rng, g, edge=(i % 5 == 0)) for i in range(2000)]
    got = engine.end_splicejunction_batch(probs)
    exp = [ref.end_splicejunction(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs ref %s" % (d[0], _desc(probs[d[0]]), d[1], d[2])


@pytest.mark.skipif(not ref_available("avx2"), reason="reference objects did not travel")
def test_gpu_splicejunction_simd_matches_reference_objects(engine):
    """The SIMD builds' Dynprog_end5/3_splicejunction (usj_kernel: the 8/16-bit triangles,
    find_best_endpoint_to_queryend_indels_8/16, traceback_local_8/16_upper/_lower) against the AVX2
    objects, inside the domain Splicetrie calls them in (glength >= rlength - 1)."""
    rng = random.Random(9393)
    g = random_genome(rng, 200000)
    ref = Ref("avx2")
    ref.set_genome(g)
    probs = []
    while len(probs) < 2500:
        p = splicejunction_problem(rng, g, edge=(len(probs) % 5 == 0))
        if p["rlength"] <= p["glength"] + 1:
            p["simd"] = True
            probs.append(p)
    got = engine.end_splicejunction_batch(probs)
    exp = [ref.end_splicejunction(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs ref %s" % (d[0], _desc(probs[d[0]]), d[1], d[2])
    assert sum(1 for s, pairs in exp if pairs is not None) > 500
