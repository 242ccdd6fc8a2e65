"""GPU parity of the SIMD-build semantics (GMAPDP_SIMD): Dynprog_single_gap as
gmap.avx2 computes it (Dynprog_simd_8 / Dynprog_simd_16 + Dynprog_traceback_8/16,
dynprog_simd.c), against the oracle's restatement and the reference's own AVX2
objects.  The reference is called on freshly zeroed Dynprog_T arenas (its SIMD
fills read cells the call never writes; see DESIGN.md "Parity").  Bar:
bit-exact pairs, scores, counters and dynprogindex."""
import random

import pytest

import gmapdp
from dpbind import (Oracle, Ref, call_single, edge_single_gap_problem, random_genome, ref_available,
                    single_gap_problem)

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


def test_gpu_simd_refuses_end_and_genome_gaps(engine):
    rng = random.Random(4200)
    g = random_genome(rng, 20000)
    engine.set_genome(g)
    p = dict(end3p=1, q=b"ACGTACGT", quc=b"ACGTACGT", qpos=0, rlength=8, glength=12, roffset=0, goffset=100,
             chroffset=0, chrhigh=20000, watsonp=1, genestrand=0, jump_late_p=0, extraband=3, defect_rate=0.01,
             endalign=0, require_pos_score_p=0, dynprogindex=1, simd=True)
    with pytest.raises(Exception):
        engine.end_gap_batch([p])
