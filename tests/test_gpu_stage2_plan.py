"""The device-resident Stage2_compute plan (gmapdp_stage2_plan_*: what bench.py times) against the oracle
at the edges of its seeding layout (stage2.c:6325, oligoindex_hr.c:33849 tally,
:34127 get_mappings):

  * windows of 2^16 8-mer starts or more, whose hit lists straddle 2^16: the plan's sizing run measures
    each call's hit list and moves the calls below 2^16 hits to the 16-bit seeding counters
    (gmapdp_engine.cpp oligo_plan_relayout); the calls at or above it stay 32-bit;
  * a plan run on another query than the one it was sized on: a call that needs more hit-list, table or
    diagonal room than the measured layout gave it reports overflow (status -2) and writes nothing past
    its slices, while the other calls stay exact.

Outputs are compared bit for bit (results, every kept path's pair records) with orc_stage2_batch."""
import numpy as np
import pytest

import gmapdp
from dpbind import Oracle, oracle_stage2_batch, stage2_mismatches

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def _genome(rng, n):
    return ACGT[rng.integers(0, 4, n)]


def _repeat_calls(seed=5, reps=(52000, 58000, 61000, 62800, 63400, 64000, 64600, 66000, 70000, 0)):
    """One 2-Mnt chromosome; per call a 76-kb window holding a tandem repeat stretch of `rep` nt and the
    read's locus, and a 2-kb read: 1 800 nt of the locus (2 % substitutions) + 200 nt of the repeat unit.
    Every position of the stretch is a hit (its 8-mers are the read's), so the hit list is ~rep plus the
    window's random matches (~2 300)."""
    rng = np.random.default_rng(seed)
    g = _genome(rng, 2_000_000)
    calls = []
    at = 20_000
    for k, rep in enumerate(reps):
        W = 76_000
        unit = _genome(rng, 7 + k % 5)                          # primitive with high probability
        start = at
        g[start + 2000:start + 2000 + rep] = np.resize(unit, rep)  # the stretch
        loc = start + 2000 + rep + 1000                          # the read's locus after it
        read = g[loc:loc + 1800].copy()
        sub = rng.random(1800) < 0.02
        read[sub] = ACGT[rng.integers(0, 4, int(sub.sum()))]
        read = np.concatenate([read, np.resize(unit, 200)])
        unit2 = _genome(rng, 9)                                  # a second stretch the read does not hold
        g[loc + 2400:loc + 10400] = np.resize(unit2, 8000)
        wend = max(start + W, loc + 10400)
        calls.append(dict(quc=read.tobytes(), chrstart=start, chrend=wend, chroffset=0, chrhigh=len(g) - 1,
                          plusp=1, splicingp=1, maxintronlen=500000, unit2=np.resize(unit2, 200).tobytes()))
        at = wend + 5000
    for c in list(calls):  # the minus strand of every window too
        calls.append(dict(c, plusp=0))
    return g.tobytes(), calls


def _nhits(g, c):
    """The seeding's hit-list length of a call: window 8-mer starts (oligoindex_hr.c count_positions_fwd /
    _rev: [chrstart, chrend - 8], the minus strand one further) whose 8-mer (minus: reverse complement) is
    one of the read's."""
    q = c["quc"]
    kset = {q[i:i + 8] for i in range(len(q) - 7)}
    plus = c["plusp"]
    lo, hi = c["chrstart"], c["chrend"] - 8 + (0 if plus else 1)
    comp = bytes.maketrans(b"ACGT", b"TGCA")
    n = 0
    for p in range(lo, hi + 1):
        k = g[p:p + 8]
        n += (k if plus else k.translate(comp)[::-1]) in kset
    return n


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0)
    yield e
    e.close()


def test_gpu_stage2_plan_16bit_demotion_edge(engine):
    g, calls = _repeat_calls()
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs, qb, qub = gmapdp.Engine.build_stage2_batch(calls)
    exp = oracle_stage2_batch(orc, probs, qb, qub)
    assert np.all(exp[0][:, 0] >= 0)
    res, paths, pairs, (n16, n32) = engine.stage2_plan_raw(probs, qb, qub)
    bad = stage2_mismatches(res, paths, pairs, exp)
    assert not bad, bad[:8]
    # the re-layout's rule: 16-bit counters exactly for the calls whose measured hit list is below 2^16
    nh = [_nhits(g, c) for c in calls]
    assert (n16, n32) == (sum(h < 65536 for h in nh), sum(h >= 65536 for h in nh)), (n16, n32, nh)
    assert n32 >= 3 and any(60000 < h < 65536 for h in nh), nh  # both classes, and calls at the edge
    # the synchronous API on the same calls (32-bit counters everywhere: windows of 2^16 starts or more)
    res2, paths2, pairs2 = engine.stage2_batch_raw(probs, qb, qub)
    assert not stage2_mismatches(res2, paths2, pairs2, exp)
    assert (res["status"] == 2).sum() >= len(calls) // 2


def test_gpu_stage2_plan_other_query_reports_overflow(engine):
    """A plan sized on query arena A, run on arena B of the same layout where three calls' reads start with
    200 nt of their window's second repeat unit (8 000 more hits than A's measured hit lists): those three
    report status -2; every other call equals the oracle on B."""
    g, calls = _repeat_calls(seed=9, reps=(20000, 30000, 40000, 50000, 0, 0))
    engine.set_genome(g)
    probs, qb, qub = gmapdp.Engine.build_stage2_batch(calls)
    qa = bytearray(qub)
    grow = [0, 2, 3]
    for k in grow:
        o = int(probs[k]["qoff"])
        qa[o:o + 200] = calls[k]["unit2"]
    qb2 = bytes(qa)
    orc = Oracle()
    orc.set_genome(g)
    exp = oracle_stage2_batch(orc, probs, qb2, qb2)
    res, paths, pairs, _ = engine.stage2_plan_raw(probs, qub, qub, run_qbuf=qb2, run_qucbuf=qb2)
    assert [int(res[k]["status"]) for k in grow] == [-2] * len(grow)
    keep = [i for i in range(len(calls)) if i not in grow]
    bad = stage2_mismatches(res[keep], paths, pairs, exp, index=keep)
    assert not bad, bad[:8]


def test_gpu_stage2_plan_other_query_more_distinct_8mers(engine):
    """a plan sized on reads whose first 1 400 nt are a 9-nt tandem unit (under 1 024 distinct
    8-mers: the smallest LDS bucket), run on the ordinary reads of the same windows (~1 990 distinct 8-mers,
    more than the bucket holds): those calls report status -2 (the seeding kernel checks the distinct
    8-mers against its bucket before writing any per-8-mer counter), the unchanged calls equal the oracle."""
    g, calls = _repeat_calls(seed=11, reps=(0, 0, 0, 0))
    engine.set_genome(g)
    probs, qb, qub = gmapdp.Engine.build_stage2_batch(calls)
    rng = np.random.default_rng(3)
    qa = bytearray(qub)
    shrink = [0, 3, 5]
    for k in shrink:
        o = int(probs[k]["qoff"])
        qa[o:o + 1400] = np.resize(_genome(rng, 9), 1400).tobytes()
    qa = bytes(qa)
    orc = Oracle()
    orc.set_genome(g)
    exp = oracle_stage2_batch(orc, probs, qub, qub)
    res, paths, pairs, _ = engine.stage2_plan_raw(probs, qa, qa, run_qbuf=qub, run_qucbuf=qub)
    assert [int(res[k]["status"]) for k in shrink] == [-2] * len(shrink)
    keep = [i for i in range(len(calls)) if i not in shrink]
    bad = stage2_mismatches(res[keep], paths, pairs, exp, index=keep)
    assert not bad, bad[:8]


def test_gpu_stage2_plan_sizing_pool_overflow(engine, monkeypatch):
    """A stage-2 plan's sizing run keeps no sequential-walk region; a call that exhausts its chunk's event pool
    there (forced here with GMAPDP_OLIGO_POOL_SLOTS) reports overflow in the sizing run only: the re-layout
    gives it the diagonal arena's upper bound and chaining scratch sized from it, the plan's own runs have an
    exact pool, and every call equals the oracle."""
    g, calls = _repeat_calls(seed=13, reps=(20000, 0, 30000, 0))
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs, qb, qub = gmapdp.Engine.build_stage2_batch(calls)
    exp = oracle_stage2_batch(orc, probs, qb, qub)
    monkeypatch.setenv("GMAPDP_OLIGO_POOL_SLOTS", "30000")
    res, paths, pairs, _ = engine.stage2_plan_raw(probs, qb, qub)
    assert np.all(res["status"] >= 0), res["status"]
    bad = stage2_mismatches(res, paths, pairs, exp)
    assert not bad, bad[:8]
