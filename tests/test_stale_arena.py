"""S-semantics parity as gmap.avx2 really runs.  The SIMD builds' Dynprog_T arenas are
allocated once per worker and never cleared (dynprog.c:686-731), and their fills read cells outside the block
they compute (dynprog_simd.c:3290); the engine, the oracle and the goldens define those cells as zero.  These
CPU tests run every S golden through the reference's AVX2 objects the way a gmap.avx2 worker does -- one
process, golden order, arenas never cleared -- and with every call on arenas filled with a random byte, and
require the goldens' outputs (tools/stale_arena.py; profiles/r04_parity/stale_arena.json records all seven
fill patterns: 0 of 5 846 problems differ).  A control shows the poisoning reaches the outputs where the
reference does read stale cells: end gaps outside the domain stage3.c passes (rlength > glength + 1,
rejected by the engine as GMAPDP_EINVAL) change with the fill byte.
"""
import json
import os
import random
import subprocess
import sys

import pytest

from dpbind import Ref, call_end, end_gap_problem, random_genome, ref_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "stale_arena.py")
GOLDENS = ("simd_single_gap_golden.npz", "simd_end_gap_golden.npz", "simd_genome_gap_golden.npz",
           "simd_cdna_gap_golden.npz")

needs_ref = pytest.mark.skipif(not (ref_available("avx2") and ref_available("avx2a")),
                               reason="reference AVX2 objects not built")


@needs_ref
@pytest.mark.parametrize("golden", GOLDENS)
@pytest.mark.parametrize("mode", ["stale", "random"])
def test_simd_goldens_hold_on_stale_and_poisoned_arenas(golden, mode):
    r = subprocess.run([sys.executable, TOOL, "--child", golden, mode], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["problems"] > 1000
    assert rec["differ"] == 0, rec


@needs_ref
def test_poisoning_reaches_out_of_domain_end_gaps():
    rng = random.Random(5)
    g = random_genome(rng, 30000)
    probs = []
    while len(probs) < 120:
        p = end_gap_problem(rng, g)
        if p["endalign"] != 2 and p["rlength"] > p["glength"] + 1:
            probs.append(p)
    outs = []
    saved = Ref._before_call
    try:
        for b in (0, 127):
            ref = Ref("avx2")
            ref.set_genome(g)
            Ref._before_call = (lambda bb: (lambda self: self.lib.refh_poison_arenas(bb, 3)))(b)
            outs.append([call_end(ref, p) for p in probs])
    finally:
        Ref._before_call = saved
    assert sum(1 for a, c in zip(*outs) if a != c) > 10
