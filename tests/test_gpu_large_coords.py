"""GPU parity at universal coordinates past 2^31 and 2^32 (BASELINE configs[2]: GRCh38's 3.1 Gnt;
configs[4]: gmapl, 64-bit Univcoord_T).

GMAP passes every entry point a chromosome as (chroffset, chrhigh) in universal coordinates; the
genome positions a kernel reads are chroffset + goffset (plus strand) or chrhigh - goffset (minus).
Here one 3-Mnt chromosome S is placed at C0 = 2^31 - ~1.5 Mnt inside a 2.15-Gnt genome, and at
2^32 - ~1.5 Mnt inside a 4.3-Gnt genome (poly-A elsewhere), so its reads straddle 2^31 / 2^32.  The property: every result on the big genome equals the
oracle's on S alone (chroffset shifted by C0) -- the outputs are chromosome-relative, so nothing may
change but the addresses the kernels compute.  Covers single, end, genome and cDNA gaps (both
builds' semantics for single gaps), stage-2 seeding and Stage2_compute.
"""
import ctypes as C
import random

import numpy as np
import pytest

import gmapdp
from dpbind import (Oracle, call_end, call_single, cdna_gap_problem, end_gap_problem, genome_gap_problem,
                    microexon_problem, oligo_problem, random_genome, single_gap_problem, stage2_problem)

pytestmark = pytest.mark.gpu

PLACEMENTS = {"2^31": (2 ** 31 - 1_500_000) // 32 * 32, "2^32": (2 ** 32 - 1_500_000) // 32 * 32}
TAIL = 8192  # poly-A after S, also present after S in the oracle's genome


def _shift(p, c0, keys=("chroffset", "chrhigh")):
    q = dict(p)
    for k in keys:
        q[k] = p[k] + c0
    return q


@pytest.fixture(scope="module", params=sorted(PLACEMENTS))
def setup(request):
    C0 = PLACEMENTS[request.param]
    rng = random.Random(2031)
    S = bytearray(random_genome(rng, 3_000_000))
    gg = [genome_gap_problem(rng, S, edge=(i % 6 == 0)) for i in range(600)]  # plants motifs into S
    at = [100]
    mx = [microexon_problem(rng, S, edge=(i % 4 == 0), at=at) for i in range(400)]  # plants microexons
    S = bytes(S)
    small = S + b"A" * TAIL
    total = C0 + len(small)
    big = np.full(total, ord("A"), dtype=np.uint8)
    big[C0:] = np.frombuffer(small, dtype=np.uint8)
    lib = gmapdp.load_library()
    words = np.zeros(lib.gmapdp_genome_words(total), dtype=np.uint32)
    rc = lib.gmapdp_pack_genome(C.cast(big.ctypes.data, C.c_char_p), total, words.ctypes.data)
    assert rc == 0
    del big
    eng = gmapdp.Engine(0)
    eng.set_genome(blocks=words, length=total)
    del words
    orc = Oracle()
    orc.set_genome(small)
    yield dict(rng=rng, S=S, gg=gg, mx=mx, eng=eng, orc=orc, C0=C0)
    eng.close()


def _first_diff(got, exp):
    for i, (a, b) in enumerate(zip(got, exp)):
        if a != b:
            return i, a, b
    return None


def test_large_coords_premise(setup):
    """The test's own premise: S really straddles 2^31 or 2^32 in universal coordinates."""
    c0, n = setup["C0"], len(setup["S"])
    assert c0 < 2 ** 31 < c0 + n or c0 < 2 ** 32 < c0 + n


@pytest.mark.parametrize("simd", [0, 1])
def test_large_coords_single_gap(setup, simd):
    rng, S, eng, orc = setup["rng"], setup["S"], setup["eng"], setup["orc"]
    probs = [dict(single_gap_problem(rng, S, maxlen=2000 if i % 7 == 0 else 400), simd=simd) for i in range(1500)]
    for p in probs:
        p["chrhigh"] = len(S)
    got = eng.single_gap_batch([_shift(p, setup["C0"]) for p in probs])
    orc.simd = simd  # one oracle: the library's genome and semantics switch are process-global
    try:
        exp = [call_single(orc, p) for p in probs]
    finally:
        orc.simd = 0
    d = _first_diff(got, exp)
    assert d is None, "problem %d: %s vs %s" % d


def test_large_coords_end_gap(setup):
    rng, S, eng, orc = setup["rng"], setup["S"], setup["eng"], setup["orc"]
    probs = [end_gap_problem(rng, S, edge=(i % 5 == 0)) for i in range(800)]
    got = eng.end_gap_batch([_shift(p, setup["C0"]) for p in probs])
    exp = [call_end(orc, p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d: %s vs %s" % d


def test_large_coords_genome_gap(setup):
    rng, eng, orc, probs = setup["rng"], setup["eng"], setup["orc"], setup["gg"]
    sp = []
    for p in probs:
        gL, gR = max(0, p["glengthL"]), max(0, p["glengthR"])
        sp.append(([round(rng.random(), 2) for _ in range(gL)], [round(rng.random(), 2) for _ in range(gR)]))
    got = eng.genome_gap_batch([_shift(p, setup["C0"]) for p in probs], sp)
    exp = [orc.genome_gap(p, lp, rp) for p, (lp, rp) in zip(probs, sp)]
    d = _first_diff(got, exp)
    assert d is None, "problem %d: %s vs %s" % d


def test_large_coords_cdna_gap(setup):
    rng, S, eng, orc = setup["rng"], setup["S"], setup["eng"], setup["orc"]
    probs = [cdna_gap_problem(rng, S, edge=(i % 5 == 0)) for i in range(300)]
    got = eng.cdna_gap_batch([_shift(p, setup["C0"]) for p in probs])
    exp = [orc.cdna_gap(p) for p in probs]
    d = _first_diff(got, exp)
    assert d is None, "problem %d: %s vs %s" % d


def test_large_coords_stage2(setup):
    rng, S, eng, orc = setup["rng"], setup["S"], setup["eng"], setup["orc"]
    oprobs = [oligo_problem(rng, S, edge=(i % 5 == 0)) for i in range(200)]
    got = eng.oligo_mappings_batch([_shift(p, setup["C0"]) for p in oprobs])
    exp = [orc.oligo_mappings(p) for p in oprobs]
    d = _first_diff(got, exp)
    assert d is None, "seeding problem %d differs" % d[0]
    sprobs = [stage2_problem(rng, S, edge=(i % 5 == 0)) for i in range(200)]
    got = eng.stage2_batch([_shift(p, setup["C0"]) for p in sprobs])
    exp = [orc.stage2_compute(p) for p in sprobs]
    d = _first_diff(got, exp)
    assert d is None, "Stage2_compute problem %d: %s vs %s" % (d[0], d[1][:1], d[2][:1])


def test_large_coords_microexon(setup):
    """Candidates' splice sites are universal coordinates (shifted by C0); the MaxEnt stand-in is a
    function of the chromosome position, so the choice and the pairs must not change."""
    eng, orc, probs, c0 = setup["eng"], setup["orc"], setup["mx"], setup["C0"]

    def me(model, pos, chroffset):
        return random.Random(model * 1000003 + (pos - chroffset)).random()
    got_c = eng.microexon_candidates([_shift(p, c0) for p in probs])
    exp_c = [orc.microexon_candidates(p) for p in probs]
    sh = [None if c is None else [x[:4] + (x[4] - c0, x[5], x[6] - c0, x[7]) for x in c] for c in got_c]
    assert sh == exp_c
    got = eng.microexon_batch([_shift(p, c0) for p in probs], me)
    exp = [orc.microexon_int(p, [me(x[m], x[q], p["chroffset"]) for x in (c or []) for q, m in ((4, 5), (6, 7))])
           for p, c in zip(probs, exp_c)]
    d = _first_diff(got, exp)
    assert d is None, "problem %d: %s vs %s" % d
    assert sum(o[2] is not None for o in got) > 100
