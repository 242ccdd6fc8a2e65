"""GPU parity tests for Dynprog_microexon_int (dynprog_single.c:900): mx_search_kernel's
candidate lists (the reference's loop order) and mx_finish_kernel's choice and pairs, against the golden
from the reference's own objects, the oracle restatement (oracle/microexon_oracle.c) and the reference
objects directly.  MaxEnt probabilities are the host's (Maxent_hr_*_prob through the reference harness,
or the golden's stored values).  Bar: bit-exact candidates, dynprogindex, microintrontype, the two float
probabilities and every pair record (gap holders' comp and genomejump included)."""
import os
import random

import pytest

import gmapdp
from dpbind import Oracle, Ref, microexon_probs, microexon_problem, random_genome, ref_available

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0)
    yield e
    e.close()


def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load_microexon(os.path.join(HERE, "golden", "microexon_golden.npz"))


def _check(got, exp, probs, what):
    for i, (a, b) in enumerate(zip(got, exp)):
        if a != b:
            p = {k: v for k, v in probs[i].items() if k not in ("q", "quc")}
            raise AssertionError("problem %d (%s): gpu %s %s vs %s %s %s" % (i, p, a[:2], (a[2] or [])[:4], what,
                                                                            b[:2], (b[2] or [])[:4]))


def test_gpu_microexon_matches_reference_golden(engine):
    g, probs, cands, cprobs, exp = _golden()
    engine.set_genome(g)
    got_c = engine.microexon_candidates(probs)
    bad = [i for i, (a, b) in enumerate(zip(got_c, cands)) if (a or []) != b]
    assert not bad, "candidate lists differ: %s" % bad[:10]
    table = {}
    for c, cp in zip(cands, cprobs):
        for k, x in enumerate(c):
            table[(x[5], x[4])] = cp[2 * k]
            table[(x[7], x[6])] = cp[2 * k + 1]
    got = engine.microexon_batch(probs, lambda m, pos, chroffset: table[(m, pos)])
    _check(got, exp, probs, "ref")


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects did not travel")
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_microexon_matches_oracle_and_reference(engine, seed):
    rng = random.Random(9500 + seed)
    g = bytearray(random_genome(rng, 3000000))
    at = [100]
    probs = [microexon_problem(rng, g, edge=(i % 4 == 0), at=at) for i in range(1000)]
    g = bytes(g)
    engine.set_genome(g)
    ref, orc = Ref("nosimd"), Oracle()
    ref.set_genome(g)
    orc.set_genome(g)
    got_c = engine.microexon_candidates(probs)
    exp_c = [orc.microexon_candidates(p) for p in probs]
    bad = [i for i, (a, b) in enumerate(zip(got_c, exp_c)) if a != b]
    assert not bad, "candidate lists differ from the oracle: %s" % bad[:10]
    got = engine.microexon_batch(probs, ref.maxent)
    _check(got, [orc.microexon_int(p, microexon_probs(ref, c, p["chroffset"])) for p, c in zip(probs, exp_c)],
           probs, "oracle")
    _check(got, [ref.microexon_int(p) for p in probs], probs, "ref")
    assert sum(o[2] is not None for o in got) > 300


def test_gpu_microexon_many_candidates(engine):
    """A microexon of low complexity in long introns of its own repeats: hundreds of candidates per call,
    more than the kernel holds in LDS, so the rerun into a region of its own is taken."""
    rng = random.Random(9600)
    orc = Oracle()
    # a synthetic call: the query's middle piece is "AGACG" around tiles "AG ACG GT" repeated
    tile = b"AGACGGT"
    body = bytearray(b"GT" + tile * 3000 + b"AG")
    gg = bytearray(random_genome(rng, 100000))
    start = 2000
    gg[start:start + 5] = b"ACGTA"
    gg[start + 5:start + 5 + len(body)] = body
    end = start + 5 + len(body)
    gg[end:end + 6] = b"TTGCAC"
    gg = bytes(gg)
    q = b"ACGTA" + b"ACG" + b"TTGCAC"
    call = dict(q=q, quc=q, rlength=len(q), roffset=100, goffsetL=start - 1000, rev_goffsetR=end + 5 - 1000,
                cdna_direction=1, chroffset=1000, chrhigh=len(gg) - 1000, watsonp=1, genestrand=0, dynprogindex=3)
    engine.set_genome(gg)
    orc.set_genome(gg)
    exp = orc.microexon_candidates(call)
    assert len(exp) > 256
    assert engine.microexon_candidates([call, call]) == [exp, exp]


def test_gpu_microexon_empty_and_direction0(engine):
    rng = random.Random(9700)
    g = random_genome(rng, 20000)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    call = dict(q=b"ACGTACGTAC", quc=b"ACGTACGTAC", rlength=10, roffset=0, goffsetL=100, rev_goffsetR=900,
                cdna_direction=0, chroffset=1000, chrhigh=19000, watsonp=1, genestrand=0, dynprogindex=1)
    got = engine.microexon_batch([call], lambda m, pos, c: 0.5)
    assert got == [orc.microexon_int(call, [])] == [((1, 0), (0.0, 0.0), None)]
    assert engine.microexon_batch([], lambda m, pos, c: 0.5) == []


def test_gpu_microexon_plan_matches_batch(engine):
    """The device-resident plan (bench.py's path: fixed candidate regions, caller-owned device outputs)
    gives the synchronous API's results and pairs."""
    import ctypes as C
    import numpy as np
    rng = random.Random(9800)
    g = bytearray(random_genome(rng, 1500000))
    at = [100]
    probs = [microexon_problem(rng, g, edge=(i % 4 == 0), at=at) for i in range(400)]
    g = bytes(g)
    engine.set_genome(g)
    table = {}

    def maxent(m, pos, chroffset):
        return table.setdefault((m, pos), random.Random(m * 1000003 + pos).random())
    exp = engine.microexon_batch(probs, maxent)
    cands = engine.microexon_candidates(probs)
    mp, qb, qub = engine.build_microexon_batch(probs)
    lib = engine.lib
    plan = C.c_void_p()
    engine._check(lib.gmapdp_microexon_plan_create(engine.h, mp.ctypes.data, len(mp), qb, qub, len(qb),
                                                   C.byref(plan)), "gmapdp_microexon_plan_create")
    try:
        assert lib.gmapdp_microexon_plan_candidates(plan) == sum(len(c or []) for c in cands)
        cp = np.array([maxent(x[m], x[p], 0) for c in cands for x in (c or []) for p, m in ((4, 5), (6, 7))]
                      + [0.0, 0.0])
        hip = C.CDLL("libamdhip64.so")  # test plumbing: device buffers for the plan's caller-owned outputs
        hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        hip.hipFree.argtypes = [C.c_void_p]

        def dbuf(nbytes, src=None):
            ptr = C.c_void_p()
            assert hip.hipMalloc(C.byref(ptr), max(nbytes, 16)) == 0
            if src is not None:
                assert hip.hipMemcpy(ptr, src, nbytes, 1) == 0  # hipMemcpyHostToDevice
            return ptr
        npc = lib.gmapdp_microexon_plan_pair_capacity(plan)
        d_q = dbuf(len(qb), qb)
        d_quc = dbuf(len(qub), qub)
        d_cp = dbuf(cp.nbytes, cp.ctypes.data)
        d_res = dbuf(len(mp) * gmapdp.MICROEXON_RESULT_DTYPE.itemsize)
        d_pairs = dbuf(npc * 16)
        engine._check(lib.gmapdp_microexon_plan_run(engine.h, plan, d_q, d_quc, d_cp, d_res, d_pairs, 3, None),
                      "gmapdp_microexon_plan_run")
        assert hip.hipDeviceSynchronize() == 0  # the plan ran on the engine's own (non-blocking) stream
        res = np.zeros(len(mp), dtype=gmapdp.MICROEXON_RESULT_DTYPE)
        pairs = np.zeros(max(npc, 1), dtype=gmapdp.PAIR_DTYPE)
        assert hip.hipMemcpy(res.ctypes.data, d_res, res.nbytes, 2) == 0  # hipMemcpyDeviceToHost (synchronous)
        assert hip.hipMemcpy(pairs.ctypes.data, d_pairs, npc * 16, 2) == 0
        for b in (d_q, d_quc, d_cp, d_res, d_pairs):
            hip.hipFree(b)
    finally:
        lib.gmapdp_microexon_plan_destroy(plan)
    for i, (p, r, e) in enumerate(zip(probs, res, exp)):
        assert (int(r["dynprogindex"]), int(r["microintrontype"])) == e[0], i
        assert (float(r["bestprob2"]), float(r["bestprob3"])) == e[1], i
        assert int(r["npairs"]) == (-1 if e[2] is None else len(e[2])), i
        if e[2]:
            got = pairs[int(r["pair_offset"]):int(r["pair_offset"]) + int(r["npairs"])]
            assert [int(x["genomepos"]) for x in got] == [x[1] for x in e[2]], i
            assert [bytes(x["comp"]) for x in got] == [x[6] for x in e[2]], i
