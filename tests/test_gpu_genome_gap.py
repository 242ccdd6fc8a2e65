"""GPU parity tests for Dynprog_genome_gap (bit-exact, including the double
splice-probability tie-breaks of bridge_intron_gap_site_level)."""
import os
import random

import pytest

import gmapdp
from dpbind import (GG_FLAG_HALF, Oracle, Ref, genome_gap_problem, random_genome, ref_available, splice_probs)

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(HERE, "golden", "genome_gap_golden.npz"))


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
        d[0], {k: v for k, v in probs[d[0]].items() if k not in ("q", "quc", "probsL", "probsR")}, d[1], what, d[2])


def test_gpu_genome_gap_matches_reference_golden(engine):
    g, probs, outs = _golden()
    engine.set_genome(g)
    got = engine.genome_gap_batch(probs, [(p["probsL"], p["probsR"]) for p in probs])
    d = _first_diff(got, outs["ref_nosimd"])
    assert d is None, _msg(probs, d, "ref")


def _synthetic_probs(rng, p):
    """Coarse probabilities with many exact ties, to stress the (score, prob, scan order) rule."""
    vals = [0.0, 0.25, 0.5, 0.5, 0.9, 0.95, 1.0]
    return ([rng.choice(vals) for _ in range(max(0, p["glengthL"]))],
            [rng.choice(vals) for _ in range(max(0, p["glengthR"]))])


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_genome_gap_matches_oracle_random(engine, seed):
    rng = random.Random(3000 + seed)
    g = bytearray(random_genome(rng, 120000))
    probs = [genome_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(5000)]
    g = bytes(g)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    sp = [_synthetic_probs(rng, p) for p in probs]
    got = engine.genome_gap_batch(probs, sp)
    exp = [orc.genome_gap(p, lp, rp) for p, (lp, rp) in zip(probs, sp)]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")


@pytest.mark.parametrize("lds_dirs", ["0", "163840"])
def test_gpu_genome_gap_direction_planes_global_and_lds(engine, monkeypatch, lds_dirs):
    """Both placements of the fills' direction planes: L2-resident scratch (4 x 64-bit ballots per column)
    and LDS (GMAPDP_GG_LDS_DIRS_MAX: one-word bands packed to 16 + 4 nhigh bytes per column, PackedDirs),
    with bands of every packed width class (W <= 32, <= 40, <= 48, <= 64) and wider ones."""
    monkeypatch.setenv("GMAPDP_GG_LDS_DIRS_MAX", lds_dirs)
    rng = random.Random(3100)
    g = bytearray(random_genome(rng, 120000))
    probs = []
    for i in range(2400):
        p = genome_gap_problem(rng, g, edge=(i % 5 == 0))
        if i % 3 == 0:  # vary the band: extraband 2..30 (W = |g - r| + 2 extraband + 1)
            p["extraband"] = rng.randint(2, 30)
        probs.append(p)
    g = bytes(g)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    sp = [_synthetic_probs(rng, p) for p in probs]
    got = engine.genome_gap_batch(probs, sp)
    exp = [orc.genome_gap(p, lp, rp) for p, (lp, rp) in zip(probs, sp)]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")


@pytest.mark.skipif(not ref_available("nosimda"), reason="reference objects did not travel")
def test_gpu_genome_gap_matches_reference_objects(engine):
    rng = random.Random(79)
    g = bytearray(random_genome(rng, 80000))
    probs = [genome_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(2000)]
    g = bytes(g)
    engine.set_genome(g)
    ref, refa, orc = Ref("nosimd"), Ref("nosimda"), Oracle()
    for r in (ref, refa, orc):
        r.set_genome(g)
    sp = [splice_probs(ref, orc, p) for p in probs]
    got = engine.genome_gap_batch(probs, sp)
    exp = [(refa if p["flags"] & GG_FLAG_HALF else ref).genome_gap(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "ref")


def test_gpu_genome_gap_domain_check(engine):
    """glength <= rlength is outside the reference's defined domain: rejected, not guessed."""
    rng = random.Random(5)
    g = bytearray(random_genome(rng, 20000))
    p = genome_gap_problem(rng, g)
    p["glengthL"] = p["rlength"]
    engine.set_genome(bytes(g))
    with pytest.raises(gmapdp.GmapdpError):
        engine.genome_gap_batch([p], [([0.0] * p["glengthL"], [0.0] * p["glengthR"])])


def test_gpu_genome_gap_every_packed_band_class(engine):
    """Band widths from narrow (W <= 40, <= 48, <= 64) to wide
    (gg_kernel), with glength - rlength from 1 to 12: engine vs oracle."""
    rng = random.Random(4711)
    g = bytearray(random_genome(rng, 150000))
    probs = []
    for i in range(3000):
        p = genome_gap_problem(rng, g, edge=(i % 7 == 0))
        if p["rlength"] >= 2:
            d = rng.choice([1, 2, 4, 8, 12])
            p["glengthL"] = p["rlength"] + d
            p["glengthR"] = p["rlength"] + rng.choice([1, 2, 4, 8, 12])
            p["extraband"] = rng.choice([0, 1, 3, 8, 14, 16, 18, 19, 20, 22, 24, 26, 27, 28, 30, 34])
        probs.append(p)
    g = bytes(g)
    W = [2 * p["extraband"] + max(p["glengthL"], p["glengthR"]) - p["rlength"] + 1 for p in probs if p["rlength"] >= 2]
    for lo, hi in ((1, 40), (41, 48), (49, 64), (65, 200)):
        assert sum(lo <= w <= hi for w in W) > 50, (lo, hi)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    sp = [_synthetic_probs(rng, p) for p in probs]
    got = engine.genome_gap_batch(probs, sp)
    exp = [orc.genome_gap(p, lp, rp) for p, (lp, rp) in zip(probs, sp)]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")



@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_genome_gap_known_sites_match_oracle(engine, seed):
    """Known splice sites (gmap -s, GMAPDP_KNOWN_SITES): probability 1.0 at a known site in the bridge and
    in genome_gap_simple's probability test, KNOWN_SPLICESITE_REWARD in genome_gap_simple's score and
    candidate test (dynprog_genome.c:2577-2652, 3118-3119, 339-372); calls without flags in the same batch
    stay as they were."""
    from dpbind import random_known_flags
    rng = random.Random(7100 + seed)
    g = bytearray(random_genome(rng, 120000))
    probs = [genome_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(3000)]
    for p in probs[::2]:
        p["defect_rate"] = 0.001  # genome_gap_simple runs first (:3479)
    g = bytes(g)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    sp = [_synthetic_probs(rng, p) for p in probs]
    known = [None if i % 7 == 0 else random_known_flags(rng, p, density=rng.choice([0.01, 0.05, 0.2]))
             for i, p in enumerate(probs)]
    got = engine.genome_gap_batch_known(probs, sp, known)
    exp = [orc.genome_gap_known(p, lp, rp, k) for p, (lp, rp), k in zip(probs, sp, known)]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")
    # the flags changed results (rewarded simple-path splices, bridges on known sites)
    plain = [orc.genome_gap(p, lp, rp) for p, (lp, rp) in zip(probs, sp)]
    assert sum(1 for a, b in zip(exp, plain) if a != b) > 50


def test_gpu_genome_gap_known_sites_simd_match_oracle(engine):
    """Known splice sites in the SIMD builds' genome gap (uxg_kernel): the same flags, the SIMD bridge."""
    from dpbind import random_known_flags
    rng = random.Random(7300)
    g = bytearray(random_genome(rng, 120000))
    probs = [genome_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(1500)]
    for i, p in enumerate(probs):
        p["simd"] = True
        if i % 2:
            p["defect_rate"] = 0.001
    g = bytes(g)
    engine.set_genome(g)
    orc = Oracle(simd=True)
    orc.set_genome(g)
    sp = [_synthetic_probs(rng, p) for p in probs]
    known = [None if i % 7 == 0 else random_known_flags(rng, p, density=rng.choice([0.01, 0.05, 0.2]))
             for i, p in enumerate(probs)]
    got = engine.genome_gap_batch_known(probs, sp, known)
    exp = [orc.genome_gap_known(p, lp, rp, k) for p, (lp, rp), k in zip(probs, sp, known)]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")
