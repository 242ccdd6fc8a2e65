"""The GMAP drop-in, end to end: the reference's own objects with Dynprog_single_gap,
Dynprog_end5/3_gap, Dynprog_genome_gap and Dynprog_cdna_gap routed (ld --wrap) through
gmap-2024_amd/shim/gmapdp_gmap_shim.c to the GPU engine, against the same objects unmodified:
the nosimd build (oracle/_ref/librefdp_gpushim.so) and the AVX2 build
(librefdp_gpushim_avx2.so, where the shim passes GMAPDP_SIMD).  Pair_T lists (every field the
call sets) and out-parameters must be identical."""
import random

import pytest

from dpbind import (GG_FLAG_HALF, Ref, call_end, call_single, cdna_gap_problem, edge_single_gap_problem,
                    end_gap_problem, genome_gap_problem, random_genome, ref_available, single_gap_problem)

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (ref_available("gpushim") and ref_available("nosimda")),
                                 reason="reference objects / shim harness did not travel")]


@pytest.fixture(scope="module")
def impls():
    return Ref("nosimd"), Ref("nosimda"), Ref("gpushim")


def test_shim_single_and_end_gaps(impls):
    ref, _, shim = impls
    rng = random.Random(606)
    g = random_genome(rng, 30000)
    ref.set_genome(g)
    shim.set_genome(g)
    bad = []
    for i in range(600):
        p = single_gap_problem(rng, g) if i % 3 else edge_single_gap_problem(rng, g)
        if call_single(shim, p) != call_single(ref, p):
            bad.append(("single", i))
    for i in range(400):
        p = end_gap_problem(rng, g, edge=(i % 4 == 0))
        if call_end(shim, p) != call_end(ref, p):
            bad.append(("end", i))
    assert bad == []


def test_shim_genome_gaps(impls):
    ref, refa, shim = impls
    rng = random.Random(707)
    g = bytearray(random_genome(rng, 60000))
    probs = [genome_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(500)]
    g = bytes(g)
    for r in impls:
        r.set_genome(g)
    bad = [i for i, p in enumerate(probs)
           if shim.genome_gap(p) != (refa if p["flags"] & GG_FLAG_HALF else ref).genome_gap(p)]
    assert bad == []


def test_shim_cdna_gaps(impls):
    ref, _, shim = impls
    rng = random.Random(808)
    g = random_genome(rng, 30000)
    ref.set_genome(g)
    shim.set_genome(g)
    probs = [cdna_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(300)]
    bad = [i for i, p in enumerate(probs) if shim.cdna_gap(p) != ref.cdna_gap(p)]
    assert bad == []


@pytest.mark.skipif(not (ref_available("gpushim_avx2") and ref_available("avx2a")),
                    reason="AVX2 shim harness did not travel")
def test_shim_simd_build_all_entry_points():
    """Inside an AVX2 GMAP build the drop-in reproduces gmap.avx2 (the shim passes GMAPDP_SIMD)."""
    ref, shim = Ref("avx2a"), Ref("gpushim_avx2")
    rng = random.Random(909)
    g = bytearray(random_genome(rng, 60000))
    gprobs = [genome_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(300)]
    g = bytes(g)
    ref.set_genome(g)
    shim.set_genome(g)
    bad = []
    for i in range(400):
        p = single_gap_problem(rng, g) if i % 3 else edge_single_gap_problem(rng, g)
        if call_single(shim, p) != call_single(ref, p):
            bad.append(("single", i))
    for i in range(400):
        p = end_gap_problem(rng, g, edge=(i % 4 == 0))
        if p["endalign"] != 2 and p["rlength"] > p["glength"] + 1:
            continue  # outside the engine's SIMD end-gap domain (the reference reads unset cells)
        if call_end(shim, p) != call_end(ref, p):
            bad.append(("end", i))
    for i, p in enumerate(gprobs):
        if shim.genome_gap(p) != ref.genome_gap(p):
            bad.append(("genome", i))
    for i in range(200):
        p = cdna_gap_problem(rng, g, edge=(i % 4 == 0))
        if shim.cdna_gap(p) != ref.cdna_gap(p):
            bad.append(("cdna", i))
    assert bad == []


def test_shim_stage2_seeding():
    """Stage2_compute's Oligoindex_hr_tally + Oligoindex_get_mappings routed to oi_kernel."""
    from dpbind import oligo_problem
    ref = Ref("nosimd")
    shim = Ref("gpushim")
    rng = random.Random(1010)
    g = bytearray(random_genome(rng, 120000))
    g[60000:61000] = b"A" * 1000
    g = bytes(g)
    ref.set_genome(g)
    shim.set_genome(g)
    probs = [oligo_problem(rng, g, edge=(i % 4 == 0)) for i in range(150)]
    bad = [i for i, p in enumerate(probs) if shim.oligo_mappings(p) != ref.oligo_mappings(p)]
    assert bad == []


@pytest.mark.parametrize("build", ["nosimd", "avx2"])
def test_shim_stage2_compute(build):
    """Stage2_compute itself wrapped (seeding + chaining on oi_kernel / s2a-s2c): the Stage2_T list and
    every middle-path Pair_T equal the unmodified reference objects', in both builds."""
    from dpbind import repeat_genome, stage2_problem
    refv, shimv = ("nosimd", "gpushim") if build == "nosimd" else ("avx2a", "gpushim_avx2")
    if not (ref_available(refv) and ref_available(shimv)):
        pytest.skip("reference objects did not travel")
    ref, shim = Ref(refv), Ref(shimv)
    rng = random.Random(1020)
    g = repeat_genome(rng, 250000)
    ref.set_genome(g)
    shim.set_genome(g)
    probs = [stage2_problem(rng, g, edge=(i % 4 == 0)) for i in range(120)]
    probs = [p for p in probs if len(p["quc"]) > 8]
    bad = [i for i, p in enumerate(probs) if shim.stage2_compute(p) != ref.stage2_compute(p)]
    assert bad == []


@pytest.mark.parametrize("build", ["nosimd", "avx2"])
def test_shim_stage2_compute_8nt_queries(build):
    """Stage2_compute on queries of exactly 8 nt (GMAP makes them for 8-nt reads): the
    reference's tally keeps the previous longer query's 8-mer flags (Oligoindex_set_inquery returns early,
    oligoindex_hr.c:33478), so an 8-mer inside them chains its window positions and one outside them gives
    NULL.  A long query, then 8-nt pieces of it, random 8-mers, a piece with an N and a 7-nt query, on one
    oligoindex: the shim (which keeps the flags per oligoindex) equals the reference call for call."""
    from dpbind import random_genome, stage2_problem
    refv, shimv = ("nosimd", "gpushim") if build == "nosimd" else ("avx2a", "gpushim_avx2")
    if not (ref_available(refv) and ref_available(shimv)):
        pytest.skip("reference objects did not travel")
    ref, shim = Ref(refv), Ref(shimv)
    rng = random.Random(808)
    g = random_genome(rng, 200000)
    ref.set_genome(g)
    shim.set_genome(g)
    seq, nonempty = [], 0
    for _ in range(6):
        p = stage2_problem(rng, g)
        q = p["quc"]
        seq.append(p)
        for k in range(10):
            i = rng.randrange(0, len(q) - 8)
            piece = q[i:i + 8] if k < 6 else bytes(rng.choice(b"ACGT") for _ in range(8))
            if k == 8:
                piece = piece[:3] + b"N" + piece[4:]
            if k == 9:
                piece = piece[:7]
            seq.append(dict(p, q=piece.lower() if k % 2 else piece, quc=piece))
    for i, p in enumerate(seq):
        a, b = ref.stage2_compute(p), shim.stage2_compute(p)
        assert a == b, "call %d (%d nt): reference %s vs shim %s" % (i, len(p["quc"]), a[0], b[0])
        nonempty += len(p["quc"]) == 8 and a[0] > 0
    assert nonempty >= 6  # 8-mers inside the flags that chain


@pytest.mark.parametrize("build", ["nosimd", "avx2"])
def test_shim_microexon_int(build):
    """Dynprog_microexon_int wrapped (mx_search_kernel, the host's MaxEnt, mx_finish_kernel): the list,
    its gap holders' comp and every out-parameter equal the unmodified reference objects'."""
    from dpbind import microexon_problem, random_genome
    refv, shimv = ("nosimd", "gpushim") if build == "nosimd" else ("avx2a", "gpushim_avx2")
    if not (ref_available(refv) and ref_available(shimv)):
        pytest.skip("reference objects did not travel")
    ref, shim = Ref(refv), Ref(shimv)
    rng = random.Random(1030)
    g = bytearray(random_genome(rng, 1500000))
    at = [100]
    probs = [microexon_problem(rng, g, edge=(i % 4 == 0), at=at) for i in range(300)]
    g = bytes(g)
    ref.set_genome(g)
    shim.set_genome(g)
    exp = [ref.microexon_int(p) for p in probs]
    bad = [i for i, p in enumerate(probs) if shim.microexon_int(p) != exp[i]]
    assert bad == []
    assert sum(e[2] is not None for e in exp) > 100


def test_shim_splicejunction(impls):
    """Dynprog_end5/3_splicejunction through the drop-in: the Pair_T lists, the
    known-splice gap holder (knowngapp) and every out-parameter, written or not, as the reference's."""
    from dpbind import splicejunction_problem
    ref, _, shim = impls
    rng = random.Random(5353)
    g = random_genome(rng, 120000)
    ref.set_genome(g)
    shim.set_genome(g)
    bad = [i for i in range(800)
           for p in [splicejunction_problem(rng, g, edge=(i % 5 == 0))]
           if shim.end_splicejunction(p) != ref.end_splicejunction(p)]
    assert bad == []


def test_shim_end_known(impls):
    """Dynprog_end5/3_known through the drop-in: the shim's restatement of the
    known-site orchestration (the straight QUERYEND_NOGAPS end gap, the anchor-site scan, the BEST_LOCAL
    fallback) on the engine, against the reference's own function, over sorted known-site lists
    (no splice tries: the trie walk itself is the reference's Splicetrie_solve_end5/3, whose
    splice-junction calls test_shim_splicejunction pins)."""
    from dpbind import end_known_problem
    ref, _, shim = impls
    rng = random.Random(7171)
    g = random_genome(rng, 60000)
    ref.set_genome(g)
    shim.set_genome(g)
    bad = [i for i in range(600)
           for p in [end_known_problem(rng, g)]
           if shim.end_known(p) != ref.end_known(p)]
    assert bad == []
