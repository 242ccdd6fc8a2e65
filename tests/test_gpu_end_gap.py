"""GPU parity tests for Dynprog_end5_gap / Dynprog_end3_gap (bit-exact)."""
import os
import random

import pytest

import gmapdp
from dpbind import Oracle, Ref, call_end, end_gap_problem, random_genome, ref_available

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(HERE, "golden", "end_gap_golden.npz"))


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


def test_gpu_end_gap_matches_reference_golden(engine):
    g, probs, outs = _golden()
    engine.set_genome(g)
    got = engine.end_gap_batch(probs)
    d = _first_diff(got, outs["ref_nosimd"])
    assert d is None, "problem %d (%s): gpu %s vs ref %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc")}, d[1], d[2])


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_end_gap_matches_oracle_random(engine, seed):
    rng = random.Random(2000 + seed)
    g = random_genome(rng, 60000)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs = [end_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(6000)]
    got = engine.end_gap_batch(probs)
    exp = [call_end(orc, p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs oracle %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc")}, d[1], d[2])


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects did not travel")
def test_gpu_end_gap_matches_reference_objects(engine):
    rng = random.Random(78)
    g = random_genome(rng, 40000)
    engine.set_genome(g)
    ref = Ref("nosimd")
    ref.set_genome(g)
    probs = [end_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(3000)]
    got = engine.end_gap_batch(probs)
    exp = [call_end(ref, p) for p in probs]
    assert _first_diff(got, exp) is None
