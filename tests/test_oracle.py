"""CPU tests: the oracle (oracle/gmapdp_oracle.c) is pinned to the reference.

1. against the committed golden vectors (generated from the reference's own
   nosimd objects by tests/golden/make_golden.py) -- always runs;
2. against the reference objects themselves on fresh seeded problems --
   runs where oracle/_ref was built (this container, or any box the built
   .so files travelled to).
"""
import ctypes as C
import os
import random

import numpy as np
import pytest

from dpbind import (Oracle, Ref, call_single, edge_single_gap_problem, random_genome, ref_available,
                    single_gap_problem, ORACLE_SO, REF_SO)

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "single_gap_golden.npz")


def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(GOLDEN)


@pytest.fixture(scope="module")
def oracle():
    if not os.path.exists(ORACLE_SO):
        pytest.fail("oracle not built: run __graft_entry__.build() (make -C oracle)")
    return Oracle()


def test_oracle_matches_golden(oracle):
    g, probs, outs = _golden()
    oracle.set_genome(g)
    exp = outs["ref_nosimd"]
    assert len(probs) == len(exp) == 1600
    bad = [i for i, p in enumerate(probs) if call_single(oracle, p) != exp[i]]
    assert bad == [], "oracle differs from reference golden on %d problems (first %s)" % (len(bad), bad[:5])


def test_golden_covers_edge_cases():
    g, probs, outs = _golden()
    exp = outs["ref_nosimd"]
    nulls = sum(1 for s, p in exp if p is None)
    gapholders = sum(1 for s, p in exp if p and any(x[9] == 1 for x in p))
    wide = sum(1 for p in probs if p["widebandp"] and p["extraband"] >= 40)
    longg = sum(1 for p in probs if p["glength"] > 700)
    stars = sum(1 for s, p in exp if p and any(x[7] == b"*" for x in p))
    assert nulls > 0 and gapholders > 20 and wide > 20 and longg > 20 and stars > 0


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects (oracle/_ref) not built here")
def test_oracle_vs_reference_random(oracle):
    ref = Ref("nosimd")
    rng = random.Random(99)
    g = random_genome(rng, 30000)
    ref.set_genome(g)
    oracle.set_genome(g)
    bad = 0
    for i in range(4000):
        p = single_gap_problem(rng, g) if i % 4 else edge_single_gap_problem(rng, g)
        if call_single(ref, p) != call_single(oracle, p):
            bad += 1
    assert bad == 0


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects (oracle/_ref) not built here")
def test_tables_match_reference(oracle):
    ref = Ref("nosimd")
    for t in range(4):
        a = np.zeros(128 * 128, dtype=np.int16)
        b = np.zeros(128 * 128, dtype=np.int16)
        ref.lib.refh_pairdistance(t, a.ctypes.data_as(C.c_void_p))
        oracle.lib.orc_pairdistance(t, b.ctypes.data_as(C.c_void_p))
        assert np.array_equal(a, b), "pairdistance type %d" % t
    a = np.zeros(128 * 128, dtype=np.uint8)
    b = np.zeros(128 * 128, dtype=np.uint8)
    ref.lib.refh_consistent(0, a.ctypes.data_as(C.c_void_p))
    oracle.lib.orc_consistent(0, b.ctypes.data_as(C.c_void_p))
    assert np.array_equal(a, b)


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects (oracle/_ref) not built here")
def test_reference_harness_has_no_unresolved_gmap_symbols():
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", REF_SO["nosimd"]], capture_output=True, text=True).stdout
    und = [l.split()[-1] for l in out.splitlines() if l.strip()]
    und = [s for s in und if not s.startswith("_") and "@" not in s and s not in ("gzgetc",)]
    assert und == [], und


# ---------------------------------------------------------------------------
# Dynprog_end5_gap / Dynprog_end3_gap
# ---------------------------------------------------------------------------
def _golden_end():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(HERE, "golden", "end_gap_golden.npz"))


def test_oracle_end_gap_matches_golden(oracle):
    from dpbind import call_end
    g, probs, outs = _golden_end()
    oracle.set_genome(g)
    exp = outs["ref_nosimd"]
    assert len(probs) == len(exp) == 1600
    bad = [i for i, p in enumerate(probs) if call_end(oracle, p) != exp[i]]
    assert bad == [], "oracle differs from reference end-gap golden on %d problems (first %s)" % (len(bad), bad[:5])


def test_end_golden_covers_every_branch():
    g, probs, outs = _golden_end()
    exp = outs["ref_nosimd"]
    seen = set()
    for p, (s, pairs) in zip(probs, exp):
        seen.add((p["end3p"], p["endalign"], pairs is None))
    for end3p in (0, 1):
        for ea in (0, 1, 2, 3):
            assert (end3p, ea, False) in seen
    assert sum(1 for p in probs if p["rlength"] > 660) > 0          # chopping
    assert sum(1 for p in probs if p["require_pos_score_p"]) > 0


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects (oracle/_ref) not built here")
def test_oracle_end_gap_vs_reference_random(oracle):
    from dpbind import call_end, end_gap_problem
    ref = Ref("nosimd")
    rng = random.Random(4242)
    g = random_genome(rng, 30000)
    ref.set_genome(g)
    oracle.set_genome(g)
    bad = 0
    for i in range(4000):
        p = end_gap_problem(rng, g, edge=(i % 5 == 0))
        if call_end(ref, p) != call_end(oracle, p):
            bad += 1
    assert bad == 0


# ---------------------------------------------------------------------------
# Dynprog_genome_gap
# ---------------------------------------------------------------------------
def _golden_genome():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(HERE, "golden", "genome_gap_golden.npz"))


def test_oracle_genome_gap_matches_golden(oracle):
    g, probs, outs = _golden_genome()
    oracle.set_genome(g)
    exp = outs["ref_nosimd"]
    assert len(probs) == len(exp) == 1600
    bad = [i for i, p in enumerate(probs) if oracle.genome_gap(p, p["probsL"], p["probsR"]) != exp[i]]
    assert bad == [], "oracle differs from reference genome-gap golden on %d problems (first %s)" % (len(bad), bad[:5])


def test_genome_golden_covers_every_branch():
    """The golden set exercises each exit of Dynprog_genome_gap (dynprog_genome.c:3354-3897)."""
    from dpbind import GG_FLAG_FINAL, GG_FLAG_HALF
    g, probs, outs = _golden_genome()
    exp = outs["ref_nosimd"]
    kinds = {"small": 0, "guard": 0, "simple": 0, "bridge_fail": 0, "full": 0, "full_null": 0, "half": 0,
             "full_indels": 0, "gapholder_inside": 0}
    for p, (s, pairs) in zip(probs, exp):
        simple_ok = pairs is not None and s[4] == 0 and s[5] == 0 and \
            any(x[9] == 1 and x[2] == 0 for x in pairs) and p["defect_rate"] < 0.014 and not p["flags"] & GG_FLAG_FINAL
        if p["rlength"] <= 1:
            kinds["small"] += 1
        elif s[1] == -32768:
            kinds["guard"] += 1
        elif s[1] == -100 and s[6] == -2147483648:
            kinds["bridge_fail"] += 1
        elif pairs is None:
            kinds["full_null"] += 1
        elif simple_ok:
            kinds["simple"] += 1
        else:
            kinds["full"] += 1
            if sum(1 for x in pairs if x[9] == 1) > 1:
                kinds["gapholder_inside"] += 1
            if s[4] > 0:
                kinds["full_indels"] += 1
        if p["flags"] & GG_FLAG_HALF and pairs is not None:
            kinds["half"] += 1
    for k in ("small", "guard", "simple", "bridge_fail", "full", "full_null", "half", "full_indels", "gapholder_inside"):
        assert kinds[k] > 0, sorted(kinds.items())


@pytest.mark.skipif(not ref_available("nosimda"), reason="reference objects (oracle/_ref) not built here")
def test_oracle_genome_gap_vs_reference_random(oracle):
    from dpbind import GG_FLAG_HALF, genome_gap_problem, splice_probs
    ref, refa = Ref("nosimd"), Ref("nosimda")
    rng = random.Random(4343)
    g = bytearray(random_genome(rng, 80000))
    probs = [genome_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(2500)]
    for r in (ref, refa, oracle):
        r.set_genome(bytes(g))
    bad = []
    for i, p in enumerate(probs):
        lp, rp = splice_probs(ref, oracle, p)
        exp = (refa if p["flags"] & GG_FLAG_HALF else ref).genome_gap(p)
        if oracle.genome_gap(p, lp, rp) != exp:
            bad.append(i)
    assert bad == []


def test_intron_scores_restate_setup(oracle):
    """intron_score_setup (dynprog_genome.c:144-187): the engine's table equals the oracle's."""
    import gmapdp  # noqa: F401  (table is internal to the engine; compare via the oracle's export)
    out = (C.c_int * (3 * 2 * 64))()
    oracle.lib.orc_intron_scores(out)
    t = np.array(out[:]).reshape(3, 2, 64)
    assert t[0, 0, 0x20] == 14 and t[0, 1, 0x20] == 16 and t[1, 0, 0x04] == 14
    assert t[2, 0, 0x20] == 16 and t[2, 1, 0x04] == 14   # the reference's mixed "either" arrays
    assert t.sum() == (14 + 8 + 4) + (16 + 10 + 8) + (14 + 8 + 4) + (16 + 10 + 8) + (16 + 8 + 4 + 14 + 8 + 4) + \
        (16 + 10 + 8 + 14 + 10 + 8)


@pytest.mark.skipif(not ref_available("avx2"), reason="reference AVX2 objects not built")
def test_oracle_simd_single_gap_matches_reference_avx2():
    """The oracle's restatement of the SIMD build's single gap (Dynprog_simd_8/16 +
    traceback_8/16) against the reference's own AVX2 objects, each call on zeroed arenas."""
    import random as _r
    rng = _r.Random(31)
    g = random_genome(rng, 50000)
    ref = Ref("avx2")
    ref.set_genome(g)
    orc = Oracle(simd=True)
    orc.set_genome(g)
    n8 = 0
    for i in range(2500):
        p = single_gap_problem(rng, g) if i % 4 else edge_single_gap_problem(rng, g)
        u = {0: 41, 1: 63, 2: 127}[0 if p["defect_rate"] < 0.003 else (1 if p["defect_rate"] < 0.014 else 2)]
        n8 += p["rlength"] < u and p["glength"] < u
        a, b = call_single(ref, p), call_single(orc, p)
        assert a == b, (i, {k: v for k, v in p.items() if k not in ("q", "quc")}, a[0], b[0])
    assert n8 > 300


# ---------------------------------------------------------------------------
# SIMD-build semantics (gmap.avx2): goldens from the reference's AVX2 objects
# ---------------------------------------------------------------------------
def _load_golden(name):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(HERE, "golden", name))


def _check_simd_golden(name, call):
    g, probs, outs = _load_golden(name)
    orc = Oracle(simd=True)
    orc.set_genome(g)
    exp = outs["ref_avx2"]
    assert len(probs) == len(exp) > 1000
    bad = [i for i, p in enumerate(probs) if call(orc, p) != exp[i]]
    assert bad == [], "%s: oracle differs on %d problems (first %s)" % (name, len(bad), bad[:5])
    return probs, exp


def test_oracle_simd_goldens():
    """The oracle's SIMD semantics against the AVX2 goldens of all three entry points."""
    from dpbind import call_end
    _check_simd_golden("simd_single_gap_golden.npz", call_single)
    probs, exp = _check_simd_golden("simd_end_gap_golden.npz", call_end)
    # both fill widths, both triangles at the endpoint and every endalign exercised
    u8 = sum(1 for p in probs if p["endalign"] != 2 and p["rlength"] > 0 and (p["rlength"] < 24 or p["glength"] < 24))
    assert u8 > 100 and len(probs) - u8 > 400
    assert {p["endalign"] for p in probs} == {0, 1, 2, 3}
    gp, gexp = _check_simd_golden("simd_genome_gap_golden.npz",
                                  lambda o, p: o.genome_gap(p, p["probsL"], p["probsR"]))
    indel_both_sides = sum(1 for s, pr in gexp if pr and s[5] > 0)
    assert indel_both_sides > 50
    assert sum(1 for p in gp if p["flags"] & 8) > 50  # halfp (from the --enable-alloca AVX2 build)


@pytest.mark.skipif(not ref_available("avx2a"), reason="reference AVX2 objects not built")
def test_oracle_simd_end_and_genome_gaps_vs_reference_avx2():
    """Fresh seeded end and genome gaps: the oracle's triangle fills, endpoint scans, bridge and
    upper/lower tracebacks against the reference's AVX2 objects (zeroed arenas)."""
    from dpbind import call_end, end_gap_problem, genome_gap_problem, splice_probs
    rng = random.Random(77)
    ref, orc = Ref("avx2a"), Oracle(simd=True)
    g = random_genome(rng, 30000)
    ref.set_genome(g)
    orc.set_genome(g)
    n = 0
    for i in range(1500):
        p = end_gap_problem(rng, g, edge=(i % 5 == 0))
        if p["endalign"] != 2 and p["rlength"] > p["glength"] + 1:
            continue
        n += 1
        a, b = call_end(ref, p), call_end(orc, p)
        assert a == b, (i, {k: v for k, v in p.items() if k not in ("q", "quc")}, a[0], b[0])
    assert n > 1200
    gg = bytearray(random_genome(rng, 80000))
    probs = [genome_gap_problem(rng, gg, edge=(i % 5 == 0)) for i in range(700)]
    gg = bytes(gg)
    ref.set_genome(gg)
    orc.set_genome(gg)
    for i, p in enumerate(probs):
        if p["rlength"] > 1 and (p["glengthL"] <= p["rlength"] or p["glengthR"] <= p["rlength"]):
            continue
        lp, rp = splice_probs(ref, orc, p)
        a, b = ref.genome_gap(p), orc.genome_gap(p, lp, rp)
        assert a == b, (i, {k: v for k, v in p.items() if k not in ("q", "quc")}, a[0], b[0])


# ---------------------------------------------------------------------------
# Dynprog_cdna_gap (dynprog_cdna.c:787), both builds
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("simd", [0, 1])
def test_oracle_cdna_gap_matches_golden(simd):
    name, tag = ("simd_cdna_gap_golden.npz", "ref_avx2") if simd else ("cdna_gap_golden.npz", "ref_nosimd")
    g, probs, outs = _load_golden(name)
    orc = Oracle(simd=bool(simd))
    orc.set_genome(g)
    exp = outs[tag]
    assert len(probs) == len(exp) == 1300
    bad = [i for i, p in enumerate(probs) if orc.cdna_gap(p) != exp[i]]
    assert bad == [], "%s: oracle differs on %d problems (first %s)" % (name, len(bad), bad[:5])
    # both the gap-holder and the INSERT_PAIRS (9 x 9 SHORTGAP block) exits, and NULL lists
    assert sum(1 for s, pr in exp if pr and any(x[6] == b"~" for x in pr)) > 10
    assert sum(1 for s, pr in exp if s[2] == 1) > 1000
    assert sum(1 for s, pr in exp if pr is None) > 0


@pytest.mark.skipif(not ref_available("avx2"), reason="reference objects not built")
def test_oracle_cdna_gap_vs_reference_random():
    from dpbind import cdna_gap_problem
    rng = random.Random(91)
    g = random_genome(rng, 30000)
    for variant in ("nosimd", "avx2"):
        ref, orc = Ref(variant), Oracle(simd=(variant == "avx2"))
        ref.set_genome(g)
        orc.set_genome(g)
        for i in range(300):
            p = cdna_gap_problem(rng, g, edge=(i % 4 == 0))
            a, b = ref.cdna_gap(p), orc.cdna_gap(p)
            assert a == b, (variant, i, {k: v for k, v in p.items() if k not in ("q", "quc")}, a[0], b[0])


# ---------------------------------------------------------------------------
# Stage-2 seeding: Oligoindex_hr_tally + Oligoindex_get_mappings (oligoindex_hr.c:33849/34127)
# ---------------------------------------------------------------------------
def _load_oligo_golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load_oligo(os.path.join(HERE, "golden", "oligo_golden.npz"))


def test_oracle_oligo_mappings_match_golden():
    g, probs, exp = _load_oligo_golden()
    orc = Oracle()
    orc.set_genome(g)
    bad = [i for i, p in enumerate(probs) if orc.oligo_mappings(p) != exp[i]]
    assert bad == [], "oracle differs on %d problems (first %s)" % (len(bad), bad[:5])
    # both strands, both oligoindex arrays, windows without diagonals, and 8-mer counts wrapping
    # past Count_T's 255 (the A-rich stretch) are all covered
    assert {p["plusp"] for p in probs} == {0, 1} and {p["minor"] for p in probs} == {0, 1}
    assert any(e[0][3] == 0 for e in exp) and sum(1 for e in exp if e[0][3] > 1) > 50
    assert any(max(e[1]) >= 200 for e in exp if e[1])


@pytest.mark.skipif(not ref_available("avx2"), reason="reference objects not built")
def test_oracle_oligo_mappings_vs_reference_random():
    from dpbind import oligo_problem
    rng = random.Random(92)
    g = bytearray(random_genome(rng, 150000))
    g[70000:71000] = b"A" * 1000
    g = bytes(g)
    orc = Oracle()
    orc.set_genome(g)
    for variant in ("nosimd", "avx2"):
        ref = Ref(variant)
        ref.set_genome(g)
        for i in range(120):
            p = oligo_problem(rng, g, edge=(i % 4 == 0))
            a, b = ref.oligo_mappings(p), orc.oligo_mappings(p)
            assert a == b, (variant, i, {k: v for k, v in p.items() if k != "quc"})


# ---------------------------------------------------------------------------
# Stage2_compute (stage2.c:6325): seeding, Diag_compute_bounds, align_compute_lookback,
# convert_to_nucleotides, Stage2_filter_unique
# ---------------------------------------------------------------------------
def _load_stage2_golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load_stage2(os.path.join(HERE, "golden", "stage2_golden.npz"))


def test_oracle_stage2_compute_matches_golden():
    g, probs, exp = _load_stage2_golden()
    orc = Oracle()
    orc.set_genome(g)
    bad = [i for i, p in enumerate(probs) if orc.stage2_compute(p) != exp[i]]
    assert not bad, "stage-2 problems differing from the golden: %s" % bad[:10]
    # the golden holds the exits and shapes the chaining has: no positions, several kept results,
    # gap holders, both strands, splicing off, short maxintronlen
    assert any(o[0] == 0 for o in exp) and any(o[0] > 1 for o in exp)
    assert any(pr[9] for o in exp for path in o[1] for pr in path)
    assert {p["plusp"] for p in probs} == {0, 1} and {p["splicingp"] for p in probs} == {0, 1}


def test_oracle_stage2_batch_matches_single_calls():
    """orc_stage2_batch (the whole-block checker of tests/test_gpu_bench_workload.py: threads, the engine's
    20-B pair records) gives what orc_stage2_compute gives call by call, on the golden's calls."""
    import numpy as np
    import gmapdp
    from dpbind import oracle_stage2_batch
    g, probs, exp = _load_stage2_golden()
    orc = Oracle()
    orc.set_genome(g)
    pr, qb, qub = gmapdp.Engine.build_stage2_batch(probs)
    scal, paths, pairs, off = oracle_stage2_batch(orc, pr, qb, qub, nthreads=4)
    rec = np.dtype([("q", "<i4"), ("g", "<i4"), ("qj", "<i4"), ("gj", "<i4"), ("c", "S1"), ("m", "S1"), ("x", "S1"),
                    ("a", "S1")])
    pv = pairs[:(len(pairs) // 20) * 20].view(rec)
    for i, (n, lists) in enumerate(exp):
        assert int(scal[i, 0]) == n, i
        for k in range(n):
            o, m = int(off[i]) + int(paths[i, k, 0]), int(paths[i, k, 1])
            got = [(int(x["q"]), int(x["g"]), int(x["qj"]), int(x["gj"]), 0, bytes(x["c"]) or b"\0",
                    bytes(x["m"]) or b"\0", bytes(x["x"]) or b"\0", bytes(x["a"]) or b"\0",
                    1 if x["q"] == -1 and x["g"] == -1 else 0) for x in pv[o:o + m]]
            assert got == lists[k], (i, k)


@pytest.mark.skipif(not ref_available(), reason="reference objects not built")
def test_oracle_stage2_compute_vs_reference_random():
    from dpbind import random_genome, repeat_genome, stage2_problem
    ref, orc = Ref("nosimd"), Oracle()
    for seed in (11, 12):
        rng = random.Random(seed)
        g = repeat_genome(rng, 300000) if seed % 2 else random_genome(rng, 300000)
        ref.set_genome(g)
        orc.set_genome(g)
        for i in range(150):
            p = stage2_problem(rng, g, edge=(i % 5 == 0))
            a, b = ref.stage2_compute(p), orc.stage2_compute(p)
            assert a == b, "seed %d problem %d: reference %s vs oracle %s" % (seed, i, a[0], b[0])


# ---- Dynprog_microexon_int (dynprog_single.c:900) ----

def _load_microexon_golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load_microexon(os.path.join(HERE, "golden", "microexon_golden.npz"))


def test_oracle_microexon_matches_golden():
    g, probs, cands, cprobs, exp = _load_microexon_golden()
    orc = Oracle()
    orc.set_genome(g)
    bad = [i for i, p in enumerate(probs) if (orc.microexon_candidates(p) or []) != cands[i]]
    assert not bad, "candidate lists differing from the golden: %s" % bad[:10]
    bad = [i for i, p in enumerate(probs) if orc.microexon_int(p, cprobs[i]) != exp[i]]
    assert not bad, "microexon problems differing from the golden: %s" % bad[:10]
    # the golden holds every exit: found (both intron directions, both strands), no candidate,
    # cdna_direction 0 (NONINTRON), several candidates (the float tie rule)
    found = [p for p, o in zip(probs, exp) if o[2] is not None]
    assert {p["cdna_direction"] for p in found} == {1, -1} and {p["watsonp"] for p in found} == {0, 1}
    assert any(o[2] is None and p["cdna_direction"] != 0 for p, o in zip(probs, exp))
    assert any(o[0][1] == 0 and p["cdna_direction"] == 0 for p, o in zip(probs, exp))
    assert any(len(c) > 1 for c in cands)


@pytest.mark.skipif(not ref_available(), reason="reference objects not built")
def test_oracle_microexon_vs_reference_random():
    from dpbind import microexon_probs, microexon_problem, random_genome
    ref, orc = Ref("nosimd"), Oracle()
    for seed in (21, 22):
        rng = random.Random(seed)
        g = bytearray(random_genome(rng, 2500000))
        at = [100]
        probs = [microexon_problem(rng, g, edge=(i % 4 == 0), at=at) for i in range(800)]
        g = bytes(g)
        ref.set_genome(g)
        orc.set_genome(g)
        for i, p in enumerate(probs):
            cp = microexon_probs(ref, orc.microexon_candidates(p), p["chroffset"])
            a, b = ref.microexon_int(p), orc.microexon_int(p, cp)
            assert a == b, "seed %d problem %d: reference %s vs oracle %s" % (seed, i, a[:2], b[:2])


# ---------------------------------------------------------------------------
# Dynprog_end5_splicejunction / Dynprog_end3_splicejunction
# ---------------------------------------------------------------------------
def _golden_sj():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load_splicejunction(os.path.join(HERE, "golden", "splicejunction_golden.npz"))


def test_oracle_splicejunction_matches_golden(oracle):
    g, probs, outs = _golden_sj()
    oracle.set_genome(g)
    exp = outs["ref_nosimd"]
    assert len(probs) == len(exp) == 1600
    bad = [i for i, p in enumerate(probs) if oracle.end_splicejunction(p) != exp[i]]
    assert bad == [], "oracle differs from the reference splice-junction golden on %d problems (first %s)" % (
        len(bad), bad[:5])


def test_splicejunction_golden_covers_every_branch():
    g, probs, outs = _golden_sj()
    exp = outs["ref_nosimd"]
    unset = -2147483648
    kinds = set()
    for p, (s, pairs) in zip(probs, exp):
        if pairs is None:
            kinds.add((p["end3p"], "guard" if s[2] == -100 else "negative"))
            assert s[2] == -100 or s[1] == unset  # the reference writes nothing on a negative best score
        else:
            kinds.add((p["end3p"], "pairs"))
            assert 0 <= s[7] < len(pairs) and pairs[s[7]][0] == -1  # the known gap holder
            kinds.add((p["end3p"], "gapholder_only" if len(pairs) == 1 else "both"))
    for end3p in (0, 1):
        for k in ("guard", "negative", "pairs", "both"):
            assert (end3p, k) in kinds, (end3p, k)
    assert any(p["contlength"] == 0 for p in probs) and any(p["contlength"] >= p["rlength"] for p in probs)


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects (oracle/_ref) not built here")
def test_oracle_splicejunction_vs_reference_random(oracle):
    from dpbind import splicejunction_problem
    ref = Ref("nosimd")
    rng = random.Random(4343)
    g = random_genome(rng, 200000)
    ref.set_genome(g)
    oracle.set_genome(g)
    bad = [i for i in range(3000)
           for p in [splicejunction_problem(rng, g, edge=(i % 6 == 0))]
           if ref.end_splicejunction(p) != oracle.end_splicejunction(p)]
    assert bad == []


@pytest.mark.parametrize("simd", [False, True])
def test_oracle_dp_batch_matches_single_calls(simd):
    """orc_dp_batch (the whole-block checker of tests/test_gpu_bench_workload.py: a thread pool over engine
    descriptors, the engine's 16-B pair records, MaxEnt from the oracle's restatement) gives, call by call,
    what the per-call oracle gives (dpbind's call_single / call_end / genome_gap with oracle_splice_probs /
    microexon_int with microexon_probs), for every DP family."""
    import numpy as np
    import gmapdp
    from dpbind import (call_end, call_single, end_gap_problem, genome_gap_problem, microexon_probs,
                        microexon_problem, oracle_dp_batch, oracle_splice_probs, random_genome, single_gap_problem)
    rng = random.Random(606)
    orc = Oracle(simd=simd)
    g = bytearray(random_genome(rng, 400000))
    calls = {"single": [single_gap_problem(rng, bytes(g)) for _ in range(150)],
             "end": [end_gap_problem(rng, bytes(g), edge=(i % 4 == 0)) for i in range(150)]}
    calls["genome"] = [genome_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(120)]
    at = [100]
    calls["microexon"] = [microexon_problem(rng, g, edge=(i % 4 == 0), at=at) for i in range(80)]
    g = bytes(g)
    orc.set_genome(g)
    exp = {"single": [call_single(orc, c) for c in calls["single"]],
           "end": [call_end(orc, c) for c in calls["end"]],
           "genome": [orc.genome_gap(c, *oracle_splice_probs(orc, c)) for c in calls["genome"]],
           "microexon": [orc.microexon_int(c, microexon_probs(orc, orc.microexon_candidates(c) or [], c["chroffset"]))
                         for c in calls["microexon"]]}
    E = gmapdp.Engine
    built = {"single": E.build_single_batch(calls["single"]), "end": E.build_end_batch(calls["end"]),
             "genome": gmapdp.build_genome_batch(calls["genome"])[:3],
             "microexon": E.build_microexon_batch(calls["microexon"])}
    for fam, (probs, qb, qub) in built.items():
        if simd and fam == "microexon":  # one semantics (no SIMD build variant)
            continue
        scal, dscal, pairs, off = oracle_dp_batch(orc, fam, probs, qb, qub, nthreads=4)
        for i, e in enumerate(exp[fam]):
            lst = e[-1]
            n = max(int(scal[i, 0]), -1)  # (-3: a SIMD end gap outside the domain, None per call)
            assert n == (-1 if lst is None else len(lst)), (fam, i)
            if fam == "microexon":
                assert tuple(scal[i, 1:3]) == tuple(e[0]) and tuple(dscal[i]) == tuple(e[1]), (fam, i)
            else:
                k = 6 if fam != "genome" else 10
                assert tuple(int(x) for x in scal[i, 1:1 + k]) == tuple(e[0][:k]), (fam, i)
                if fam == "genome":
                    assert tuple(dscal[i]) == tuple(e[0][10:12]), (fam, i)
            assert scal[i, 15] == 0, (fam, i)
            for k, x in enumerate(lst or []):
                r = pairs[int(off[i]) + k]
                if x[9]:  # gap holder: the genomejump, and the queryjump of the intron's holder
                    assert (int(r["querypos"]), int(r["genomepos"]), int(r["jump"])) == (-1, -1, x[3]), (fam, i, k)
                    if x[2]:
                        assert (int(scal[i, 12]), int(scal[i, 13])) == (k, x[2]), (fam, i, k)
                    if fam == "microexon":
                        assert r["comp"] == x[6], (fam, i, k)
                else:
                    got = (int(r["querypos"]), int(r["genomepos"]), 0, 0, x[4], r["cdna"], r["comp"], r["genome"],
                           r["genomealt"], 0)
                    assert got == x, (fam, i, k)
