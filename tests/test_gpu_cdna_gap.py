"""GPU parity tests for Dynprog_cdna_gap (dynprog_cdna.c:787), both builds: cg_kernel (nosimd:
Dynprog_standard fills + bridge_cdna_gap) and uxc_kernel (SIMD: the upper/lower triangles +
bridge_cdna_gap_8/16_ud).  Bar: bit-exact pairs (including the 9 x 9 SHORTGAP block and the gap
holder with its queryjump), traceback score, incompletep and dynprogindex -- against the goldens
from the reference's own objects, the oracle restatement, and the reference objects directly."""
import os
import random

import pytest

import gmapdp
from dpbind import Oracle, Ref, cdna_gap_problem, random_genome, ref_available

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden(name):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(HERE, "golden", name))


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


def _msg(probs, d, what):
    return "problem %d (%s): gpu %s vs %s %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc")}, d[1], what, d[2])


def _simd(probs, on):
    for p in probs:
        p["simd"] = bool(on)
    return probs


@pytest.mark.parametrize("simd", [0, 1])
def test_gpu_cdna_gap_matches_reference_golden(engine, simd):
    name, tag = ("simd_cdna_gap_golden.npz", "ref_avx2") if simd else ("cdna_gap_golden.npz", "ref_nosimd")
    g, probs, outs = _golden(name)
    engine.set_genome(g)
    got = engine.cdna_gap_batch(_simd(probs, simd))
    d = _first_diff(got, outs[tag])
    assert d is None, _msg(probs, d, tag)
    # the SHORTGAP-block exit and the gap-holder exit are both exercised
    assert sum(1 for s, pr in got if pr and any(x[6] == b"~" for x in pr)) > 10
    assert sum(1 for s, pr in got if s[2] == 1) > 1000


@pytest.mark.parametrize("simd", [0, 1])
def test_gpu_cdna_gap_matches_oracle_random(engine, simd):
    rng = random.Random(6100 + simd)
    g = random_genome(rng, 60000)
    engine.set_genome(g)
    orc = Oracle(simd=bool(simd))
    orc.set_genome(g)
    probs = _simd([cdna_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(1500)], simd)
    got = engine.cdna_gap_batch(probs)
    exp = [orc.cdna_gap(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")


@pytest.mark.skipif(not ref_available("avx2"), reason="reference objects did not travel")
@pytest.mark.parametrize("variant", ["nosimd", "avx2"])
def test_gpu_cdna_gap_matches_reference_objects(engine, variant):
    rng = random.Random(6200 + (variant == "avx2"))
    g = random_genome(rng, 40000)
    engine.set_genome(g)
    ref = Ref(variant)
    ref.set_genome(g)
    probs = _simd([cdna_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(600)], variant == "avx2")
    got = engine.cdna_gap_batch(probs)
    exp = [ref.cdna_gap(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "ref " + variant)


def test_gpu_cdna_gap_domain_check_and_empty(engine):
    """rlengthL != rlengthR (or < glength) is outside the reference's defined domain: rejected."""
    rng = random.Random(7)
    g = random_genome(rng, 20000)
    engine.set_genome(g)
    assert engine.cdna_gap_batch([]) == []
    p = cdna_gap_problem(rng, g)
    p["rlengthR"] -= 1
    with pytest.raises(gmapdp.GmapdpError):
        engine.cdna_gap_batch([p])
