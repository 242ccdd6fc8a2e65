"""CPU tests of the product library's C ABI (no device compute here)."""
import ctypes as C
import os
import random

import numpy as np
import pytest

import gmapdp
from dpbind import REF_SO, ref_available

HERE = os.path.dirname(os.path.abspath(__file__))


def test_library_exports_every_header_symbol():
    lib = gmapdp.load_library()
    syms = gmapdp.exported_symbols()
    assert "gmapdp_single_gap_batch" in syms and "gmapdp_plan_run" in syms
    missing = [s for s in syms if not hasattr(lib, s)]
    assert missing == []


def read_fasta(path):
    seq = []
    for line in open(path, "rb"):
        if not line.startswith(b">"):
            seq.append(line.strip())
    return b"".join(seq)


def test_pack_genome_matches_gmap_build_golden():
    """tests/setup.genomecomp.ok is gmap_build's .genomecomp for ss.chr17test
    (reference tests/setup1.test.in:15-26)."""
    seq = read_fasta(os.path.join(HERE, "golden", "ss.chr17test.fa"))
    ok = np.fromfile(os.path.join(HERE, "golden", "setup.genomecomp.ok"), dtype="<u4")
    mine = gmapdp.pack_genome(seq)
    nb = (len(seq) + 31) // 32
    assert np.array_equal(mine[:3 * nb], ok[:3 * nb])
    # gmap_build appends one extra {high, low} pair of all-ones (compress-write.c:640-643)
    assert np.all(ok[3 * nb:] == 0xFFFFFFFF) and np.all(mine[3 * nb:] == 0xFFFFFFFF)


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects not built")
def test_pack_genome_matches_reference_compressor():
    lib = C.CDLL(REF_SO["nosimd"])
    rng = random.Random(5)
    for n in [1, 5, 31, 32, 33, 64, 100, 999, 4097]:
        s = bytes(rng.choice(b"ACGTacgtNnXx") if rng.random() < 0.2 else rng.choice(b"ACGT") for _ in range(n))
        ref = np.zeros(gmapdp.load_library().gmapdp_genome_words(n), dtype=np.uint32)
        lib.refh_pack_genome(s, n, ref.ctypes.data_as(C.c_void_p))
        assert np.array_equal(ref, gmapdp.pack_genome(s)), n


def test_compute_bands():
    lib = gmapdp.load_library()
    lb, ub = C.c_int(), C.c_int()
    # Dynprog_compute_bands (dynprog.c:1247)
    for r, g, eb, wide, exp in [(10, 20, 3, 1, (3, 13)), (20, 10, 3, 1, (13, 3)), (20, 10, 3, 0, (3, 3)),
                                (7, 7, 0, 1, (0, 0))]:
        lib.gmapdp_compute_bands(C.byref(lb), C.byref(ub), r, g, eb, wide)
        assert (lb.value, ub.value) == exp


def test_engine_fails_loudly_without_device():
    """No CPU fallback on the product path: without a HIP device the engine refuses to start."""
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("a GPU is present")
    with pytest.raises(gmapdp.GmapdpError):
        gmapdp.Engine(0)


def test_problem_struct_layout():
    assert C.sizeof(gmapdp.SingleProblem) == 72  # 64-bit universal coordinates (gmapdp_coord_t)
    assert C.sizeof(gmapdp.Result) == 32
    assert gmapdp.PAIR_DTYPE.itemsize == 16
    assert gmapdp.PROBLEM_DTYPE.itemsize == 72


def test_genome_struct_layout():
    assert C.sizeof(gmapdp.GenomeProblem) == 96
    assert C.sizeof(gmapdp.GenomeResult) == 72
    assert gmapdp.GENOME_PROBLEM_DTYPE.itemsize == 96
    assert gmapdp.GENOME_RESULT_DTYPE.itemsize == 72


def test_struct_layouts_match_the_c_header(tmp_path):
    """The ctypes mirrors against sizeof/offsetof as a C compiler lays out include/gmapdp.h."""
    import subprocess
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gmapdp.h"\nint main(void) {\n'
                   'printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(gmapdp_single_problem), sizeof(gmapdp_end_problem),\n'
                   '  sizeof(gmapdp_genome_problem), sizeof(gmapdp_genome_result), sizeof(gmapdp_cdna_problem),\n'
                   '  sizeof(gmapdp_cdna_result));\n'
                   'printf("%zu %zu\\n", offsetof(gmapdp_cdna_problem, defect_rate), offsetof(gmapdp_cdna_result, gap_queryjump));\n'
                   'printf("%zu %zu %zu\\n", sizeof(gmapdp_oligo_problem), sizeof(gmapdp_oligo_result), offsetof(gmapdp_oligo_result, diag_offset));\n'
                   'return 0; }\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(os.path.dirname(HERE), "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    sizes = [int(x) for x in out]
    assert sizes[:6] == [C.sizeof(gmapdp.SingleProblem), C.sizeof(gmapdp.EndProblem), C.sizeof(gmapdp.GenomeProblem),
                         C.sizeof(gmapdp.GenomeResult), C.sizeof(gmapdp.CdnaProblem), C.sizeof(gmapdp.CdnaResult)]
    assert sizes[6:8] == [gmapdp.CdnaProblem.defect_rate.offset, gmapdp.CdnaResult.gap_queryjump.offset]
    assert gmapdp.CDNA_PROBLEM_DTYPE.itemsize == sizes[4] and gmapdp.CDNA_RESULT_DTYPE.itemsize == sizes[5]
    assert sizes[8:] == [C.sizeof(gmapdp.OligoProblem), C.sizeof(gmapdp.OligoResult), gmapdp.OligoResult.diag_offset.offset]
    assert gmapdp.OLIGO_PROBLEM_DTYPE.itemsize == sizes[8] and gmapdp.OLIGO_RESULT_DTYPE.itemsize == sizes[9]


def test_mixed_struct_layout_matches_the_c_header(tmp_path):
    """gmapdp_mixed (the drop-in's one-round-trip batch): every field's offset and the size."""
    import subprocess
    names = [f for f, _ in gmapdp.Mixed._fields_]
    src = tmp_path / "mixed.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gmapdp.h"\nint main(void) {\n' +
                   "".join('printf("%%zu\\n", offsetof(gmapdp_mixed, %s));\n' % f for f in names) +
                   'printf("%zu\\n", sizeof(gmapdp_mixed));\nreturn 0; }\n')
    exe = tmp_path / "mixed"
    subprocess.run(["gcc", "-I", os.path.join(os.path.dirname(HERE), "include"), str(src), "-o", str(exe)], check=True)
    out = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert out == [getattr(gmapdp.Mixed, f).offset for f in names] + [C.sizeof(gmapdp.Mixed)]


def test_genome_splice_sites_match_oracle():
    """gmapdp_genome_splice_sites (host-only) lists the same Maxent_hr_*_prob calls as the oracle's
    restatement of dynprog_genome.c:2573-2660."""
    from dpbind import Oracle, genome_gap_problem, random_genome
    rng = random.Random(31)
    g = bytearray(random_genome(rng, 30000))
    calls = [genome_gap_problem(rng, g) for _ in range(200)]
    probs, _, _, m = gmapdp.build_genome_batch(calls)
    pos, mod = gmapdp.genome_splice_sites(probs)
    orc = Oracle()
    for i, p in enumerate(calls):
        sl, sr = orc.splice_sites(p)
        o = int(probs[i]["prob_offset"])
        got = list(zip(pos[o:o + len(sl) + len(sr)].tolist(), mod[o:o + len(sl) + len(sr)].tolist()))
        assert got == sl + sr


def test_expand_pairs_decodes_the_stream_format():
    """gmapdp_expand_pairs (host only, no GPU) on a hand-made stream of pc_kernel.hip's format: a diagonal RUN
    with coded and escaped records, an indel RUN, a RAW gap holder; a truncated stream is refused."""
    import struct
    import numpy as np
    import gmapdp
    run = lambda q, g, dq, dg, n: struct.pack("<BiibbH", 1, q, g, dq, dg, n)  # noqa: E731
    code = lambda c, g, m: bytes([("ACGT".index(c)) | ("ACGT".index(g) << 2) | ("*| :".index(m) << 4)])  # noqa: E731
    s = run(10, 100, 1, 1, 3) + code("A", "A", "*") + code("C", "G", " ") + b"\xff" + b"n- N"
    s += run(13, 103, 1, 0, 2) + b"\xff" + b"A- A" + b"\xff" + b"C- C"
    s += b"\x02" + struct.pack("<iii", -1, -1, 250) + b" > ."
    stream = np.frombuffer(s, dtype=np.uint8)
    out = gmapdp.expand_pairs(stream, [0, len(s)], [6], [2], 8)
    got = [(int(r["querypos"]), int(r["genomepos"]), int(r["jump"]), bytes(r["cdna"] + r["comp"] + r["genome"] +
            r["genomealt"])) for r in out[2:8]]
    assert got == [(10, 100, 0, b"A*AA"), (11, 101, 0, b"C GG"), (12, 102, 0, b"n- N"), (13, 103, 0, b"A- A"),
                   (14, 103, 0, b"C- C"), (-1, -1, 250, b" > .")], got
    with pytest.raises(gmapdp.GmapdpError):
        gmapdp.expand_pairs(stream[:-3], [0, len(s) - 3], [6], [2], 8)


def test_expand_path_pairs_decodes_the_stream_format():
    """gmapdp_expand_path_pairs (host only, no GPU): the same ops over stage 2's 20-B path pairs -- a RUN of
    matches, a 21-B RAW gap holder with both jumps -- two paths, the second at its own pair_offset; a stream
    that ends early is refused."""
    import struct
    import numpy as np
    import gmapdp
    run = lambda q, g, dq, dg, n: struct.pack("<BiibbH", 1, q, g, dq, dg, n)  # noqa: E731
    code = lambda c: bytes(["ACGT".index(c) | ("ACGT".index(c) << 2) | (1 << 4)])  # noqa: E731
    a = run(0, 500, 1, 1, 3) + code("A") + code("C") + code("G")
    a += b"\x02" + struct.pack("<iiii", -1, -1, 7, 130) + b" - ."
    b = run(40, 900, 1, 1, 2) + code("T") + b"\xff" + b"n|N."
    stream = np.frombuffer(a + b, dtype=np.uint8)
    paths = np.zeros(2, dtype=gmapdp.PATH_DTYPE)
    paths["pair_offset"] = [0, 6]
    paths["npairs"] = [4, 2]
    out = gmapdp.expand_path_pairs(stream, [0, len(a), len(a) + len(b)], paths, 8)
    got = [(int(r["querypos"]), int(r["genomepos"]), int(r["queryjump"]), int(r["genomejump"]),
            bytes(r["cdna"] + r["comp"] + r["genome"] + r["genomealt"])) for r in out]
    assert got[:4] == [(0, 500, 0, 0, b"A|AA"), (1, 501, 0, 0, b"C|CC"), (2, 502, 0, 0, b"G|GG"),
                       (-1, -1, 7, 130, b" - .")], got
    assert got[6:8] == [(40, 900, 0, 0, b"T|TT"), (41, 901, 0, 0, b"n|N.")], got
    with pytest.raises(gmapdp.GmapdpError):
        gmapdp.expand_path_pairs(stream[:-2], [0, len(a), len(a) + len(b) - 2], paths, 8)
