"""GPU parity tests for stage-2 seeding: oi_kernel's Oligoindex_hr_tally +
Oligoindex_get_mappings (oligoindex_hr.c:33849/34127, as Stage2_compute runs them for GMAP) against
the goldens from the reference's own objects, the oracle restatement (oracle/stage2_oracle.c) and
the reference objects directly.  Bar: bit-exact npositions, mapping lists (order included),
totalpositions, maxnconsecutive, oned_matrix_p and the diagonals list."""
import os
import random

import pytest

import gmapdp
from dpbind import Oracle, Ref, oligo_problem, random_genome, ref_available

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load_oligo(os.path.join(HERE, "golden", "oligo_golden.npz"))


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
    i, a, b = d
    p = {k: v for k, v in probs[i].items() if k != "quc"}
    if len(a) == 4 and len(b) == 4:
        parts = [k for k, x, y in zip(("scalars", "npositions", "positions", "diagonals"), a, b) if x != y]
        return "problem %d (%s, qlen %d): %s differ; gpu %s vs %s %s" % (i, p, len(probs[i]["quc"]), parts, a[0],
                                                                          what, b[0])
    return "problem %d (%s): gpu %s vs %s %s" % (i, p, a[:1], what, b[:1])


def test_gpu_oligo_matches_reference_golden(engine):
    g, probs, exp = _golden()
    engine.set_genome(g)
    got = engine.oligo_mappings_batch(probs)
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "ref")


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_oligo_matches_oracle_random(engine, seed):
    rng = random.Random(8100 + seed)
    g = bytearray(random_genome(rng, 400000))
    g[200000:202500] = b"A" * 2500  # 8-mer counts past Count_T's 255
    g = bytes(g)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs = [oligo_problem(rng, g, edge=(i % 5 == 0)) for i in range(600)]
    got = engine.oligo_mappings_batch(probs)
    exp = [orc.oligo_mappings(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects did not travel")
def test_gpu_oligo_matches_reference_objects(engine):
    rng = random.Random(8200)
    g = random_genome(rng, 200000)
    engine.set_genome(g)
    ref = Ref("nosimd")
    ref.set_genome(g)
    probs = [oligo_problem(rng, g, edge=(i % 4 == 0)) for i in range(300)]
    got = engine.oligo_mappings_batch(probs)
    d = _first_diff(got, [ref.oligo_mappings(p) for p in probs])
    assert d is None, _msg(probs, d, "ref")


def test_gpu_oligo_domain_check(engine):
    """querylength <= 8 leaves the reference's inquery table stale: rejected, not guessed."""
    rng = random.Random(9)
    g = random_genome(rng, 20000)
    engine.set_genome(g)
    p = dict(quc=b"ACGTACGT", chrstart=100, chrend=5000, chroffset=0, chrhigh=20000, plusp=1, minor=0)
    with pytest.raises(gmapdp.GmapdpError):
        engine.oligo_mappings_batch([p])


def test_gpu_oligo_batch_refuses_shared_query_slices(engine):
    """the host-array API writes npositions / mappings per problem at its query slice and makes
    the mappings absolute per problem; two problems on overlapping slices are refused (GMAPDP_EINVAL)."""
    rng = random.Random(10)
    g = random_genome(rng, 20000)
    engine.set_genome(g)
    q = bytes(g[3000:3400])
    p = dict(quc=q, chrstart=100, chrend=8000, chroffset=0, chrhigh=20000, plusp=1, minor=0)
    probs, qucbuf = gmapdp.Engine.build_oligo_batch([p, p])
    probs[1]["qoff"] = 200  # overlaps problem 0's [0, 400)
    with pytest.raises(gmapdp.GmapdpError):
        engine.oligo_mappings_batch_raw(probs, qucbuf + bytes(200))
    probs[1]["qoff"] = 400  # disjoint again: accepted
    engine.oligo_mappings_batch_raw(probs, qucbuf)


def _repeat_genome(rng, n):
    """A genome with tandem copies of short units: queries drawn over them put many diagonals past
    suffnconsecutive, which exercises the order of the good list."""
    g = bytearray(random_genome(rng, n))
    for start in range(5000, n - 20000, 25000):
        unit = bytes(g[start:start + rng.randint(40, 400)])
        pos = start
        for _ in range(rng.randint(3, 12)):
            g[pos:pos + len(unit)] = unit
            pos += len(unit) + rng.randint(0, 30)
    return bytes(g)


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_oligo_repeats_match_oracle(engine, seed):
    rng = random.Random(8300 + seed)
    g = _repeat_genome(rng, 300000)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs = [oligo_problem(rng, g, edge=(i % 7 == 0)) for i in range(400)]
    got = engine.oligo_mappings_batch(probs)
    exp = [orc.oligo_mappings(p) for p in probs]
    assert max(len(e[3]) for e in exp) > 3  # the test is only worth it with many good diagonals
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")


def test_gpu_oligo_pool_overflow_falls_back(engine, monkeypatch):
    """oi_build_kernel's fallbacks: the table image and the candidates kept out of LDS (GMAPDP_OI_LDS_TABLE 0:
    scattered table stores, every event through the global pool; 512: tables past 512 entries and
    candidate lists past 256 take the global paths, the rest stay in LDS), and a small event pool (the
    problems that no longer fit run the sequential walk); same results every way."""
    rng = random.Random(8400)
    g = _repeat_genome(rng, 200000)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs = [oligo_problem(rng, g) for i in range(200)]
    exp = [orc.oligo_mappings(p) for p in probs]
    for lds in ("0", "512", None):
        if lds is None:
            monkeypatch.delenv("GMAPDP_OI_LDS_TABLE", raising=False)
        else:
            monkeypatch.setenv("GMAPDP_OI_LDS_TABLE", lds)
        for slots in ("0", "20000", None):
            if slots is None:
                monkeypatch.delenv("GMAPDP_OLIGO_POOL_SLOTS", raising=False)
            else:
                monkeypatch.setenv("GMAPDP_OLIGO_POOL_SLOTS", slots)
            d = _first_diff(engine.oligo_mappings_batch(probs), exp)
            assert d is None, _msg(probs, d, "oracle (LDS table %s, pool %s)" % (lds, slots))


def test_gpu_oligo_wide_windows_match_oracle(engine):
    """Windows of 65 536 or more 8-mer starts take the 32-bit-counter build of oi_kernel; with a
    poly-A stretch some counts wrap Count_T many times over."""
    rng = random.Random(8500)
    g = bytearray(random_genome(rng, 400000))
    g[250000:252000] = b"A" * 2000
    g = bytes(g)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs = []
    for i in range(40):
        p = oligo_problem(rng, g, edge=(i % 5 == 0))
        span = rng.randint(65536, 180000)
        p["chrstart"] = max(0, min(p["chrstart"], len(g) - 2000 - span))
        p["chrend"] = p["chrstart"] + span
        if i % 3 == 0:
            p["quc"] = b"A" * rng.randint(9, 300) + p["quc"]
        probs.append(p)
    got = engine.oligo_mappings_batch(probs)
    exp = [orc.oligo_mappings(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")


def test_gpu_oligo_event_key_formats(engine):
    """oi_map_kernel's three event-key formats against the oracle: 32-bit (diagi << 12 | t) for queries of
    <= 4 096 8-mer positions on windows below 2^20 (the bench's shape, covered above too), 64-bit with q and
    t for longer queries or windows of 2^20 and more, 64-bit with q alone past 2^16 query positions (a
    repetitive query: few distinct 8-mers).  Records carry querypos values recovered from t in the 32-bit
    format (binary search over cum_nohits), from the key otherwise."""
    rng = random.Random(8600)
    g = _repeat_genome(rng, 1400000)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs = []
    for i in range(24):
        p = oligo_problem(rng, g, edge=(i % 5 == 0))
        kind = i % 3
        if kind == 0:  # a long query: 4 097+ positions
            extra = bytes(g[p["chrstart"]:p["chrstart"] + 4200 + rng.randint(0, 1500)])
            p["quc"] = extra + p["quc"]
        elif kind == 1:  # a window past 2^20
            span = rng.randint((1 << 20) + 10, (1 << 20) + 200000)
            p["chrstart"] = max(0, min(p["chrstart"], len(g) - 2000 - span))
            p["chrend"] = p["chrstart"] + span
        else:  # past 2^16 query positions: a short unit repeated
            unit = bytes(p["quc"][:rng.randint(300, 900)])
            p["quc"] = unit * (66000 // len(unit) + 1)
        probs.append(p)
    got = engine.oligo_mappings_batch(probs)
    exp = [orc.oligo_mappings(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, _msg(probs, d, "oracle")
