"""Plans created back to back before any of them runs (bench.py creates a plan per block up front): the
descriptor upload gmapdp_plan_create_all leaves in flight, the pinned staging buffer the next plan reuses,
the recycled host arrays and the plan threads' pool must give every plan the results it gets when it is
created and run alone.  Single and end gaps of a configs[1]-shaped block on chr22 (two halves of 40 000+
problems each, so both plans take the threaded plan build)."""
import ctypes as C

import numpy as np
import pytest

import gmapdp
from gmapdp import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def chr22_block():
    layout = W.Layout(W.CHR22)
    genome = W.PackedGenome(layout.total, seed=38)
    W.plant_stream(genome, layout, 4000, range(1), W.CDNA2K)
    d = W.make_blocks(genome, layout, 4000, [0], shape=W.CDNA2K, sprob=False)[0]
    return genome, d


def _halves(d):
    sp, ep = d["single"], d["end"]
    hs, he = len(sp) // 2, len(ep) // 2
    return [(sp[:hs].copy(), ep[:he].copy()), (sp[hs:].copy(), ep[he:].copy())]


def _create(eng, sp, ep):
    res = np.zeros(len(sp) + len(ep), dtype=gmapdp.RESULT_DTYPE)
    gres = np.zeros(1, dtype=gmapdp.GENOME_RESULT_DTYPE)
    plan = C.c_void_p()
    eng._check(eng.lib.gmapdp_plan_create_all(eng.h, sp.ctypes.data, len(sp), ep.ctypes.data, len(ep), None, 0,
                                              res.ctypes.data, gres.ctypes.data, C.byref(plan)),
               "gmapdp_plan_create_all")
    return plan, res


def _run(eng, plan, host_res, d_q):
    lib = eng.lib
    hip = gmapdp._hip()
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    ngpu, cap = lib.gmapdp_plan_gpu_problems(plan), lib.gmapdp_plan_pair_capacity(plan)
    d_res, d_pairs = C.c_void_p(), C.c_void_p()
    assert hip.hipMalloc(C.byref(d_res), 32 * max(ngpu, 1)) == 0
    assert hip.hipMalloc(C.byref(d_pairs), 16 * max(cap, 1)) == 0
    try:
        eng._check(lib.gmapdp_plan_run(eng.h, plan, d_q, d_q, d_res, d_pairs, None), "gmapdp_plan_run")
        assert hip.hipDeviceSynchronize() == 0
        dres = np.zeros(max(ngpu, 1), dtype=gmapdp.RESULT_DTYPE)
        pairs = np.zeros(max(cap, 1), dtype=gmapdp.PAIR_DTYPE)
        assert hip.hipMemcpy(dres.ctypes.data, d_res, dres.nbytes, 2) == 0
        assert hip.hipMemcpy(pairs.ctypes.data, d_pairs, pairs.nbytes, 2) == 0
    finally:
        hip.hipFree(d_res)
        hip.hipFree(d_pairs)
    res = host_res.copy()
    di = np.array([lib.gmapdp_plan_dev_index(plan, i) for i in range(len(res))], dtype=np.int64)
    res[di >= 0] = dres[di[di >= 0]]
    # each problem's pair records, in problem order
    recs = [pairs[int(r["pair_offset"]):int(r["pair_offset"]) + max(int(r["npairs"]), 0)].tobytes()
            if di[i] >= 0 else b"" for i, r in enumerate(res)]
    return res, recs


def test_gpu_plans_created_back_to_back(chr22_block):
    genome, d = chr22_block
    parts = _halves(d)
    assert all(len(sp) + len(ep) >= 16384 for sp, ep in parts)
    eng = gmapdp.Engine(0)
    eng.set_genome(blocks=genome.blocks, length=genome.length)
    hip = gmapdp._hip()
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    q = d["q"]
    d_q = C.c_void_p()
    assert hip.hipMalloc(C.byref(d_q), len(q)) == 0
    try:
        assert hip.hipMemcpy(d_q, q.ctypes.data, len(q), 1) == 0
        # each plan alone: created, run, destroyed
        alone = []
        for sp, ep in parts:
            plan, hres = _create(eng, sp, ep)
            try:
                alone.append(_run(eng, plan, hres, d_q))
            finally:
                eng.lib.gmapdp_plan_destroy(plan)
        # both created before either runs, run in reverse order
        made = [_create(eng, sp, ep) for sp, ep in parts]
        try:
            got = [None, None]
            for k in (1, 0):
                got[k] = _run(eng, made[k][0], made[k][1], d_q)
        finally:
            for plan, _ in made:
                eng.lib.gmapdp_plan_destroy(plan)
    finally:
        hip.hipFree(d_q)
        eng.close()
    for k in range(2):
        (ra, pa), (rb, pb) = alone[k], got[k]
        assert np.array_equal(ra.tobytes(), rb.tobytes()), "half %d: results differ" % k
        assert pa == pb, "half %d: pair records differ" % k
        assert (ra["npairs"] > 0).mean() > 0.5
