"""gmapdp_mixed_batch, the GMAP drop-in's one-round-trip dispatcher batch (include/gmapdp.h): single,
end and genome gaps, microexon searches and the finishes of earlier searches over ONE query arena must
give exactly what the separate entry points give (gmapdp_dynprog_batch, gmapdp_microexon_search,
gmapdp_microexon_finish), which the other gpu tests pin against the oracle and the reference objects.
Also: the candidate-pool rerun (a search with more candidates than the kernel's LDS list), the
GMAPDP_ESPACE contract (candidates_needed set, the other sections still filled in), empty batches."""
import random

import numpy as np
import pytest

import gmapdp
from dpbind import end_gap_problem, genome_gap_problem, microexon_problem, random_genome, single_gap_problem

pytestmark = pytest.mark.gpu

ESPACE = -6


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0)
    yield e
    e.close()


def _arena(*sections):
    """Concatenate the sections' query arenas; shift each section's qoff by its base."""
    qs, qus, base = [], [], 0
    for probs, qb, qub, keys in sections:
        for k in keys:
            probs[k] += base
        qs.append(qb)
        qus.append(qub)
        base += len(qb)
    return b"".join(qs), b"".join(qus)


def _fake_maxent(model, pos, chroffset):
    # any deterministic probability works: both paths take the same values as input
    return ((pos * 2654435761 + model * 97) % 1000) / 1000.0


def _workload(rng, nsingle=300, nend=200, ngenome=150, nsearch=200, nfinish=150, many=False):
    g = bytearray(random_genome(rng, 3200000))
    lo = bytearray(g[:1500000])  # the DP problems live in the first 1.5 Mnt, the microexon sites above
    singles = [single_gap_problem(rng, bytes(lo)) for _ in range(nsingle)]
    ends = [end_gap_problem(rng, bytes(lo)) for _ in range(nend)]
    genomes = [genome_gap_problem(rng, lo) for _ in range(ngenome)]
    g[:1500000] = lo
    at = [1500000]  # chromosome positions (the microexon calls' chromosome starts at 1000)
    searches = [microexon_problem(rng, g, edge=(i % 5 == 0), at=at) for i in range(nsearch)]
    finishes = [microexon_problem(rng, g, edge=(i % 5 == 0), at=at) for i in range(nfinish)]
    if many:  # a low-complexity microexon in long introns of its own repeats (> the LDS candidate list)
        tile = b"AGACGGT"
        body = b"GT" + tile * 3000 + b"AG"
        start = 1000 + at[0] + 100
        g[start:start + 5] = b"ACGTA"
        g[start + 5:start + 5 + len(body)] = body
        end = start + 5 + len(body)
        g[end:end + 6] = b"TTGCAC"
        assert end + 6 < len(g) - 1000
        q = b"ACGTA" + b"ACG" + b"TTGCAC"
        searches.append(dict(q=q, quc=q, rlength=len(q), roffset=100, goffsetL=start - 1000,
                             rev_goffsetR=end + 5 - 1000, cdna_direction=1, chroffset=1000, chrhigh=len(g) - 1000,
                             watsonp=1, genestrand=0, dynprogindex=3))
    return bytes(g), singles, ends, genomes, searches, finishes


def _pack(engine, singles, ends, genomes, searches, finishes):
    S = engine.build_single_batch(singles)
    E = engine.build_end_batch(ends)
    G, gq, gqu, nprob = gmapdp.build_genome_batch(genomes)
    XS = engine.build_microexon_batch(searches)
    XF = engine.build_microexon_batch(finishes)
    probs = np.array([_fake_maxent(1, k, 0) for k in range(max(nprob, 1))])[:nprob]
    q, qu = _arena((S[0], S[1], S[2], ["qoff"]), (E[0], E[1], E[2], ["qoff"]), (G, gq, gqu, ["qoff"]),
                   (XS[0], XS[1], XS[2], ["qoff"]), (XF[0], XF[1], XF[2], ["qoff"]))
    return q, qu, S[0], E[0], G, probs, XS[0], XF[0]


def _finish_inputs(engine, XF, q, qu):
    """The finishes' searches, run separately, and the probabilities the host would give them."""
    res, cands = engine.microexon_search_raw(XF, q, qu)
    cp = np.array([_fake_maxent(int(c[m]), int(c[p]), 0) for c in cands for p, m in (("pos2", "model2"),
                                                                                       ("pos3", "model3"))])
    return res, cands, cp


def _separate(engine, q, qu, S, E, G, probs, XS, XF, fres, fcands, fcp):
    lib = engine.lib
    n = len(S) + len(E)
    cap = (lib.gmapdp_single_pair_capacity(S.ctypes.data, len(S)) + lib.gmapdp_end_pair_capacity(E.ctypes.data, len(E))
           + lib.gmapdp_genome_pair_capacity(G.ctypes.data, len(G)))
    results = np.zeros(max(n, 1), dtype=gmapdp.RESULT_DTYPE)
    gresults = np.zeros(max(len(G), 1), dtype=gmapdp.GENOME_RESULT_DTYPE)
    pairs = np.zeros(max(cap, 1), dtype=gmapdp.PAIR_DTYPE)
    sp = np.ascontiguousarray(probs if len(probs) else np.zeros(1))
    rc = lib.gmapdp_dynprog_batch(engine.h, S.ctypes.data, len(S), E.ctypes.data, len(E), G.ctypes.data, len(G), q,
                                  qu, len(q), sp.ctypes.data, len(probs), results.ctypes.data, gresults.ctypes.data,
                                  pairs.ctypes.data, cap)
    engine._check(rc, "gmapdp_dynprog_batch")
    sres, scands = engine.microexon_search_raw(XS, q, qu) if len(XS) else (None, None)
    fout = engine.microexon_finish_raw(XF, q, qu, fcands, fcp, fres) if len(XF) else (None, None)
    return results[:n], gresults[:len(G)], pairs[:cap], sres, scands, fout


def _same(a, b, what):
    bad = [i for i, (x, y) in enumerate(zip(a, b)) if x != y]
    assert not bad and len(a) == len(b), "%s differ at %s (of %d / %d)" % (what, bad[:10], len(a), len(b))


def _used(pairs, r):
    return pairs[int(r["pair_offset"]):int(r["pair_offset"]) + max(0, int(r["npairs"]))].tobytes()


def _dp_lists(res, pairs):
    """Per problem: the result without its pair offset, and its pairs (slots past a call's pairs are
    scratch, and a batch of other sections lays the arena out differently)."""
    return [(tuple(x for k, x in zip(res.dtype.names, r) if k != "pair_offset"), _used(pairs, r)) for r in res]


def _cand_lists(res, cands):
    return [[tuple(c) for c in cands[int(r["cand_offset"]):int(r["cand_offset"]) + int(r["ncandidates"])]]
            for r in res]


def _no_offsets(res):
    return [tuple(x for k, x in zip(res.dtype.names, r) if k != "cand_offset") for r in res]


def _finish_lists(res, pairs):
    return [(tuple(x for k, x in zip(res.dtype.names, r) if k not in ("pair_offset", "cand_offset")),
             pairs[int(r["pair_offset"]):int(r["pair_offset"]) + max(0, int(r["npairs"]))].tobytes()) for r in res]


@pytest.mark.parametrize("seed,many", [(1, False), (2, True)])
def test_mixed_batch_matches_separate_calls(engine, seed, many):
    rng = random.Random(7700 + seed)
    g, singles, ends, genomes, searches, finishes = _workload(rng, many=many)
    engine.set_genome(g)
    q, qu, S, E, G, probs, XS, XF = _pack(engine, singles, ends, genomes, searches, finishes)
    fres, fcands, fcp = _finish_inputs(engine, XF, q, qu)
    rc, got = engine.mixed_batch_raw(q, qu, singles=S, ends=E, genomes=G, splice_probs=probs, searches=XS, finishes=XF,
                                     finish_cands=fcands, finish_probs=fcp, finish_results=fres)
    engine._check(rc, "gmapdp_mixed_batch")
    results, gresults, pairs, sres, scands, (xfres, xfpairs) = _separate(engine, q, qu, S, E, G, probs, XS, XF, fres,
                                                                          fcands, fcp)
    n = len(S) + len(E)
    assert (got["results"][:n] == results).all()  # the same plan: the same arena layout
    assert (got["genome_results"][:len(G)] == gresults).all()
    _same(_dp_lists(got["results"][:n], got["pairs"]), _dp_lists(results, pairs), "single/end gaps")
    _same(_dp_lists(got["genome_results"][:len(G)], got["pairs"]), _dp_lists(gresults, pairs), "genome gaps")
    assert sum(int(r["npairs"]) > 0 for r in results) > n // 4
    # searches: the pool's order depends on the atomics, so compare per call
    _same(_no_offsets(got["search_results"][:len(XS)]), _no_offsets(sres), "search results")
    _same(_cand_lists(got["search_results"][:len(XS)], got["candidates"]), _cand_lists(sres, scands), "candidates")
    assert got["candidates_needed"] >= sum(int(r["ncandidates"]) for r in sres)
    if many:
        assert max(int(r["ncandidates"]) for r in sres) > 256  # the rerun path was taken
    _same(_finish_lists(got["finish_results"][:len(XF)], got["finish_pairs"]), _finish_lists(xfres, xfpairs),
          "finishes")
    assert sum(int(r["npairs"]) > 0 for r in xfres) > len(XF) // 8


def test_mixed_batch_sections_alone_and_empty(engine):
    rng = random.Random(7800)
    g, singles, ends, genomes, searches, finishes = _workload(rng, 40, 30, 20, 30, 20)
    engine.set_genome(g)
    q, qu, S, E, G, probs, XS, XF = _pack(engine, singles, ends, genomes, searches, finishes)
    fres, fcands, fcp = _finish_inputs(engine, XF, q, qu)
    results, gresults, pairs, sres, scands, (xfres, xfpairs) = _separate(engine, q, qu, S, E, G, probs, XS, XF, fres,
                                                                          fcands, fcp)
    rc, got = engine.mixed_batch_raw(q, qu, singles=S)
    assert rc == 0
    _same(_dp_lists(got["results"][:len(S)], got["pairs"]), _dp_lists(results[:len(S)], pairs), "singles")
    rc, got = engine.mixed_batch_raw(q, qu, genomes=G, splice_probs=probs)
    assert rc == 0
    _same(_dp_lists(got["genome_results"][:len(G)], got["pairs"]), _dp_lists(gresults, pairs), "genome gaps")
    rc, got = engine.mixed_batch_raw(q, qu, searches=XS)
    assert rc == 0
    _same(_cand_lists(got["search_results"][:len(XS)], got["candidates"]), _cand_lists(sres, scands), "candidates")
    rc, got = engine.mixed_batch_raw(q, qu, finishes=XF, finish_cands=fcands, finish_probs=fcp, finish_results=fres)
    assert rc == 0
    _same(_finish_lists(got["finish_results"][:len(XF)], got["finish_pairs"]), _finish_lists(xfres, xfpairs),
          "finishes")
    rc, got = engine.mixed_batch_raw(q, qu)
    assert rc == 0


def test_mixed_batch_candidate_espace(engine):
    """candidate_capacity too small: GMAPDP_ESPACE with candidates_needed, the DP sections filled in."""
    rng = random.Random(7900)
    g, singles, ends, genomes, searches, finishes = _workload(rng, 60, 0, 20, 60, 0)
    engine.set_genome(g)
    q, qu, S, E, G, probs, XS, XF = _pack(engine, singles, ends, genomes, searches, finishes)
    results, gresults, pairs, sres, scands, _ = _separate(engine, q, qu, S, E, G, probs, XS, XF, None, None, None)
    total = sum(int(r["ncandidates"]) for r in sres)
    assert total > 1
    rc, got = engine.mixed_batch_raw(q, qu, singles=S, genomes=G, splice_probs=probs, searches=XS,
                                     candidate_capacity=total - 1)
    assert rc == ESPACE
    assert got["candidates_needed"] == total
    _same(_dp_lists(got["results"][:len(S)], got["pairs"]), _dp_lists(results, pairs), "singles")
    _same(_dp_lists(got["genome_results"][:len(G)], got["pairs"]), _dp_lists(gresults, pairs), "genome gaps")
    rc, got = engine.mixed_batch_raw(q, qu, singles=S, searches=XS, candidate_capacity=total)
    assert rc == 0
    _same(_cand_lists(got["search_results"][:len(XS)], got["candidates"]), _cand_lists(sres, scands), "candidates")
