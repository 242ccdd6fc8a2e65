"""MaxEnt splice-site models (Maxent_hr_{donor,acceptor,antidonor,antiacceptor}_prob,
maxent_hr.c:27357-27652) from tools/make_maxent_tables.py's table binary.

CPU: the oracle's restatement (oracle/maxent_oracle.c: one 2-bit window per site, the reference's table
products in the reference's order) equals the reference's own functions bit for bit (doubles compared as
their 64-bit patterns) at every position of a test genome, all four models, with and without a chromosome
offset (the margin tests).  GPU: the engine's device MaxEnt (gmapdp_maxent_sites) equals both, at every
position, and past 2^32 (gmapl coordinates) equals the oracle.
"""
import ctypes as C
import os
import random

import numpy as np
import pytest

from dpbind import ORACLE_SO, Oracle, Ref, random_genome, ref_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLES = os.path.join(ROOT, "gmap-2024_amd", "lib", "maxent_hr_tables.bin")


def _oracle():
    lib = C.CDLL(ORACLE_SO)
    lib.orc_maxent_load.argtypes = [C.c_char_p]
    lib.orc_maxent_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_ulonglong, C.c_int, C.c_void_p]
    lib.orc_set_genome.argtypes = [C.c_char_p, C.c_uint]
    assert lib.orc_maxent_load(TABLES.encode()) == 0
    return lib


def site_genome(n=60000, seed=17):
    """A random genome with N runs and planted consensus splice sites (high probabilities too)."""
    rng = random.Random(seed)
    g = bytearray(random_genome(rng, n, nfrac=0.004))
    for _ in range(n // 300):
        p = rng.randrange(30, n - 40)
        g[p:p + 9] = rng.choice([b"CAGGTAAGT", b"AAGGTGAGT", b"ACTTACCTG"])
        q = rng.randrange(30, n - 40)
        g[q:q + 23] = rng.choice([b"TTTTTTTTTTCCCTTTTCAGGTA", b"CTTACCTGAAAAAAAAAAAAAAA"])
    return bytes(g)


def all_sites(n):
    pos = np.arange(n + 8, dtype=np.uint64)  # a few past the end: the padding words
    return [(m, pos) for m in range(4)]


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects not built")
@pytest.mark.skipif(not os.path.exists(TABLES), reason="maxent tables not generated (tools/make_maxent_tables.py)")
def test_oracle_maxent_equals_reference_everywhere():
    g = site_genome()
    orc = _oracle()
    gbuf = C.create_string_buffer(g, len(g))
    orc.orc_set_genome(gbuf, len(g))
    ref = Ref("nosimd")
    ref.set_genome(g)
    f = ref.lib.refh_maxent_batch
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint, C.c_int, C.c_void_p]
    nhigh = 0
    for chroffset in (0, 7000):
        for m, pos in all_sites(len(g)):
            models = np.full(len(pos), m, dtype=np.int32)
            a = np.zeros(len(pos))
            b = np.zeros(len(pos))
            p32 = pos.astype(np.uint32)
            f(models.ctypes.data, p32.ctypes.data, chroffset, len(pos), a.ctypes.data)
            orc.orc_maxent_batch(models.ctypes.data, pos.ctypes.data, chroffset, len(pos), b.ctypes.data)
            bad = np.nonzero(a.view(np.uint64) != b.view(np.uint64))[0]
            assert len(bad) == 0, (m, chroffset, bad[:5], a[bad[:5]], b[bad[:5]])
            nhigh += int((a > 0.9).sum())
    assert nhigh > 200  # the planted consensus sites score high


def test_maxent_table_binary_layout():
    if not os.path.exists(TABLES):
        pytest.skip("maxent tables not generated")
    raw = open(TABLES, "rb").read()
    assert raw[:8] == b"GMDPMXT1"
    assert len(raw) == 16 + 16 * 40 + 8 * (12 * 16384 + 4 * 16)


def test_bench_splice_pool_is_strong_and_diverse():
    """The bench plants these contexts at its genome-gap introns (workload.splice_pool): every one is a strong
    site under MaxEnt (>= 0.9, the oracle restatement), and they are distinct (no 8-mer is planted millions of
    times, which would inflate stage-2 seeding hits)."""
    import random
    from gmapdp import workload as W
    don, acc = W.splice_pool()
    assert len(don) > 1000 and len(acc) >= 4096
    assert len({d.tobytes() for d in don}) == len(don) and len({a.tobytes() for a in acc}) == len(acc)
    rng = random.Random(3)
    orc = Oracle()
    for ctx, model, off in ((don[::7], 0, 3), (acc[::17], 1, 20)):
        parts, bases, pos = [], [], 0
        for c in ctx:
            filler = bytes(rng.choice(b"ACGT") for _ in range(50))
            parts += [filler, c.tobytes()]
            bases.append(pos + 50)
            pos += 50 + len(c)
        orc.set_genome(b"".join(parts) + b"A" * 64)
        assert min(orc.maxent(model, b + off, 0) for b in bases) >= 0.9
