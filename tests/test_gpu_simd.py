"""GPU parity of the SIMD-build semantics (GMAPDP_SIMD): the Dynprog_* entry points as
gmap.avx2 computes them -- single gaps with Dynprog_simd_8/16 + Dynprog_traceback_8/16, end
and genome gaps with the Dynprog_simd_8/16_upper/_lower triangles, their endpoint scans,
bridge_intron_gap_*_ud and the upper/lower tracebacks (dynprog_simd.c, dynprog_end.c,
dynprog_genome.c) -- against the AVX2 goldens, the oracle's restatement and the reference's
own AVX2 objects.  The reference is called on freshly zeroed Dynprog_T arenas (its SIMD
fills read cells the call never writes; see DESIGN.md "Parity").  Bar:
bit-exact pairs, scores, counters and dynprogindex."""
import random

import pytest

import gmapdp
import os

from dpbind import (GG_FLAG_HALF, Oracle, Ref, call_end, call_single, edge_single_gap_problem, end_gap_problem,
                    genome_gap_problem, random_genome, ref_available, single_gap_problem, splice_probs)

HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.gpu

USE8P = {0: 41, 1: 63, 2: 127}  # use8p_size by mismatch type (dynprog.c:1022-1025)


def _mtype(d):
    return 0 if d < 0.003 else (1 if d < 0.014 else 2)


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0)
    yield e
    e.close()


def _problems(rng, g, n):
    out = []
    for i in range(n):
        p = single_gap_problem(rng, g) if i % 5 else edge_single_gap_problem(rng, g)
        p["simd"] = True
        out.append(p)
    return out


def _first_diff(got, exp):
    for i, (a, b) in enumerate(zip(got, exp)):
        if a != b:
            return i, a, b
    return None


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_simd_single_matches_oracle(engine, seed):
    rng = random.Random(4000 + seed)
    g = random_genome(rng, 60000)
    engine.set_genome(g)
    orc = Oracle(simd=True)
    orc.set_genome(g)
    probs = _problems(rng, g, 5000)
    n8 = sum(1 for p in probs if p["rlength"] < USE8P[_mtype(p["defect_rate"])]
             and p["glength"] < USE8P[_mtype(p["defect_rate"])])
    assert n8 > 500 and len(probs) - n8 > 500  # both fill widths exercised
    got = engine.single_gap_batch(probs)
    exp = [call_single(orc, p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs oracle %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc")}, d[1][0], d[2][0])


@pytest.mark.skipif(not ref_available("avx2"), reason="reference objects did not travel")
def test_gpu_simd_single_matches_reference_avx2(engine):
    rng = random.Random(4100)
    g = random_genome(rng, 40000)
    engine.set_genome(g)
    ref = Ref("avx2")
    ref.set_genome(g)
    probs = _problems(rng, g, 2500)
    got = engine.single_gap_batch(probs)
    exp = [call_single(ref, p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d: gpu %s vs reference avx2 %s" % (d[0], d[1][0], d[2][0])


def _golden(name):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(HERE, "golden", name))


def _simd(probs):
    for p in probs:
        p["simd"] = True
    return probs


def _in_domain_end(p):
    return p["endalign"] == 2 or p["rlength"] <= p["glength"] + 1


def test_gpu_simd_goldens(engine):
    """All three entry points against the goldens generated from the reference's AVX2 objects."""
    g, probs, outs = _golden("simd_single_gap_golden.npz")
    engine.set_genome(g)
    d = _first_diff(engine.single_gap_batch(_simd(probs)), outs["ref_avx2"])
    assert d is None, "single gap %d: gpu %s vs ref %s" % (d[0], d[1][0], d[2][0])
    g, probs, outs = _golden("simd_end_gap_golden.npz")
    engine.set_genome(g)
    d = _first_diff(engine.end_gap_batch(_simd(probs)), outs["ref_avx2"])
    assert d is None, "end gap %d (%s): gpu %s vs ref %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc")}, d[1], d[2])
    g, probs, outs = _golden("simd_genome_gap_golden.npz")
    engine.set_genome(g)
    got = engine.genome_gap_batch(_simd(probs), [(p["probsL"], p["probsR"]) for p in probs])
    d = _first_diff(got, outs["ref_avx2"])
    assert d is None, "genome gap %d (%s): gpu %s vs ref %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc", "probsL", "probsR")}, d[1], d[2])


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_simd_end_gaps_match_oracle(engine, seed):
    rng = random.Random(4300 + seed)
    g = random_genome(rng, 60000)
    engine.set_genome(g)
    orc = Oracle(simd=True)
    orc.set_genome(g)
    probs = _simd([p for p in (end_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(6000)) if _in_domain_end(p)])
    n8 = sum(1 for p in probs if p["endalign"] != 2 and 0 < p["rlength"] and (p["rlength"] < 24 or p["glength"] < 24))
    assert n8 > 300 and len(probs) - n8 > 1000  # both fill widths
    got = engine.end_gap_batch(probs)
    exp = [call_end(orc, p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs oracle %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc")}, d[1], d[2])


@pytest.mark.skipif(not ref_available("avx2"), reason="reference objects did not travel")
def test_gpu_simd_end_gaps_match_reference_avx2(engine):
    rng = random.Random(4400)
    g = random_genome(rng, 40000)
    engine.set_genome(g)
    ref = Ref("avx2")
    ref.set_genome(g)
    probs = _simd([p for p in (end_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(2500)) if _in_domain_end(p)])
    d = _first_diff(engine.end_gap_batch(probs), [call_end(ref, p) for p in probs])
    assert d is None, "problem %d: gpu %s vs reference avx2 %s" % (d[0], d[1], d[2])


def _synthetic_probs(rng, p):
    """Coarse probabilities with many exact ties, to stress the (score, prob, scan order) rule."""
    vals = [0.0, 0.25, 0.5, 0.5, 0.9, 0.95, 1.0]
    return ([rng.choice(vals) for _ in range(max(0, p["glengthL"]))],
            [rng.choice(vals) for _ in range(max(0, p["glengthR"]))])


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_simd_genome_gaps_match_oracle(engine, seed):
    rng = random.Random(4500 + seed)
    g = bytearray(random_genome(rng, 120000))
    probs = _simd([genome_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(4000)])
    g = bytes(g)
    engine.set_genome(g)
    orc = Oracle(simd=True)
    orc.set_genome(g)
    sp = [_synthetic_probs(rng, p) for p in probs]
    got = engine.genome_gap_batch(probs, sp)
    exp = [orc.genome_gap(p, lp, rp) for p, (lp, rp) in zip(probs, sp)]
    d = _first_diff(got, exp)
    assert d is None, "problem %d (%s): gpu %s vs oracle %s" % (
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc")}, d[1], d[2])


@pytest.mark.skipif(not ref_available("avx2a"), reason="reference objects did not travel")
def test_gpu_simd_genome_gaps_match_reference_avx2(engine):
    rng = random.Random(4600)
    g = bytearray(random_genome(rng, 80000))
    probs = _simd([genome_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(1500)])
    g = bytes(g)
    engine.set_genome(g)
    ref, refa, orc = Ref("avx2"), Ref("avx2a"), Oracle()
    for r in (ref, refa, orc):
        r.set_genome(g)
    sp = [splice_probs(ref, orc, p) for p in probs]
    got = engine.genome_gap_batch(probs, sp)
    exp = [(refa if p["flags"] & GG_FLAG_HALF else ref).genome_gap(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d: gpu %s vs reference avx2 %s" % (d[0], d[1], d[2])


def test_gpu_simd_end_gap_domain_check(engine):
    """rlength > glength + 1: the reference's lower-triangle scan reads uninitialised scores -- rejected."""
    rng = random.Random(4200)
    g = random_genome(rng, 20000)
    engine.set_genome(g)
    p = dict(end3p=1, q=b"ACGTACGTACGT", quc=b"ACGTACGTACGT", qpos=0, rlength=12, glength=8, roffset=0, goffset=100,
             chroffset=0, chrhigh=20000, watsonp=1, genestrand=0, jump_late_p=0, extraband=3, defect_rate=0.01,
             endalign=0, require_pos_score_p=0, dynprogindex=1, simd=True)
    with pytest.raises(gmapdp.GmapdpError):
        engine.end_gap_batch([p])
