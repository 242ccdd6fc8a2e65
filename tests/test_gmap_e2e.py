"""End-to-end: GMAP's own per-read pipeline (gmap.c process_request:4486 -> stage 2 -> stage 3 -> every
Dynprog_* call) through the drop-in shim on the MI355X engine, compared byte-for-byte with the
reference program's outputs.

Binaries (oracle/ref.mk, built from /root/reference/src where it lies; they travel to the GPU box):
  oracle/_ref/gmap_{nosimd,avx2}      the unmodified reference `gmap` (the end-to-end oracle)
  oracle/_ref/gmap_gpu_{nosimd,avx2}  the same objects linked with gmap-2024_amd/shim via ld --wrap and
                                      libgmapdp.so
  oracle/_ref/gmap_large, gmap_gpu_large  gmapl: the nosimd build with LARGE_GENOMES (64-bit
                                      Univcoord_T), unmodified and with the shim (BASELINE configs[4])

Fixtures (tests/golden/, data only):
  align.test.ok       the reference's own golden (tests/align.test.in:9: gmap -A -g ss.chr17test ss.her2)
  cdna2_genetest2_*   `gmap -g genetest2.fa cdna2.fa` (BASELINE configs[0] inputs), both builds
  e2e_{nosimd,avx2}.sam  200 synthetic 2-kb spliced reads vs a 300-kb segment (make_e2e.py), both builds
  e2e_short_*            a read of the same stream whose stage 3 makes 8-nt oligoindex queries
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
GOLD = os.path.join(ROOT, "tests", "golden")
BUILDS = ("nosimd", "avx2")


def _exe(name):
    path = os.path.join(REF, name)
    if not os.path.exists(path):
        pytest.skip("%s not built (make -C oracle ref)" % name)
    return path


def _run(exe, args, env=None, timeout=300):
    e = dict(os.environ)
    if env:
        e.update(env)
    r = subprocess.run([exe] + args, cwd=GOLD, env=e, capture_output=True, timeout=timeout)
    assert r.returncode == 0, "%s %s failed (%d): %s" % (exe, args, r.returncode, r.stderr.decode()[-2000:])
    return r.stdout.decode(), r.stderr.decode()


def _read(name):
    with open(os.path.join(GOLD, name)) as f:
        return f.read()


ALIGN_ARGS = ["-A", "-g", "ss.chr17test.fa", "ss.her2.fa"]
CDNA2_ARGS = ["-g", "genetest2.fa", "cdna2.fa"]
E2E_ARGS = ["-g", "e2e_genome.fa", "-f", "samse", "--no-sam-headers", "e2e_reads.fa"]


def _stats(stderr):
    m = re.search(r"gmapdp shim calls:(.*)", stderr)
    assert m, "shim statistics missing (GMAPDP_SHIM_STATS): " + stderr[-500:]
    return {k: float(v) for k, v in re.findall(r"(\w+)=([\d.]+)", m.group(1))}


# ---- the oracle itself: the reference program reproduces the reference's golden and our fixtures ----

@pytest.mark.parametrize("build", BUILDS)
def test_reference_gmap_reproduces_align_golden(build):
    out, _ = _run(_exe("gmap_" + build), ALIGN_ARGS)
    assert out == _read("align.test.ok")


@pytest.mark.parametrize("build", BUILDS)
def test_reference_gmap_reproduces_fixtures(build):
    exe = _exe("gmap_" + build)
    assert _run(exe, CDNA2_ARGS)[0] == _read("cdna2_genetest2_%s.txt" % build)
    assert _run(exe, E2E_ARGS)[0] == _read("e2e_%s.sam" % build)


def test_fixtures_pin_both_semantics():
    """nosimd and SIMD builds differ on a few reads: both fixtures are needed."""
    a = _read("e2e_nosimd.sam").splitlines()
    b = _read("e2e_avx2.sam").splitlines()
    assert len(a) == len(b) == 200
    ndiff = sum(1 for x, y in zip(a, b) if x != y)
    assert 1 <= ndiff <= 20


# ---- the drop-in on the GPU ----

@pytest.mark.gpu
@pytest.mark.parametrize("build", BUILDS)
def test_gpu_gmap_align_golden(build):
    """tests/align.test.in:9 through the drop-in: byte-identical to the reference's align.test.ok."""
    out, err = _run(_exe("gmap_gpu_" + build), ALIGN_ARGS, env={"GMAPDP_SHIM_STATS": "1"})
    st = _stats(err)
    assert out == _read("align.test.ok")
    # a 100 %-identity mRNA: introns and ends, no single gaps
    assert st["Dynprog_genome_gap"] > 0 and st["Stage2_compute"] > 0, st


@pytest.mark.gpu
@pytest.mark.parametrize("build", BUILDS)
def test_gpu_gmap_cdna2_genetest2(build):
    out, _ = _run(_exe("gmap_gpu_" + build), CDNA2_ARGS)
    assert out == _read("cdna2_genetest2_%s.txt" % build)


@pytest.mark.gpu
@pytest.mark.parametrize("build", BUILDS)
def test_gpu_gmap_synthetic_reads(build):
    """200 spliced 2-kb reads: every SAM record identical to the reference build's; every DP family and
    Stage2_compute (seeding + chaining) and Dynprog_microexon_int ran on the GPU (no GMAPDP_EINVAL domain refusal: the shim aborts on one)."""
    out, err = _run(_exe("gmap_gpu_" + build), E2E_ARGS, env={"GMAPDP_SHIM_STATS": "1"})
    st = _stats(err)
    exp = _read("e2e_%s.sam" % build).splitlines()
    got = out.splitlines()
    bad = [i for i, (x, y) in enumerate(zip(got, exp)) if x != y]
    assert len(got) == len(exp) and not bad, "reads differing: %s" % bad[:10]
    for k in ("Dynprog_single_gap", "Dynprog_genome_gap", "Dynprog_end5_gap", "Dynprog_end3_gap",
              "Stage2_compute", "Dynprog_microexon_int"):
        assert st[k] > 0, st


SHORT_ARGS = ["-g", "e2e_short_genome.fa", "-f", "samse", "--no-sam-headers", "e2e_short_reads.fa"]


@pytest.mark.parametrize("build", BUILDS)
def test_reference_gmap_reproduces_short_oligo_fixture(build):
    assert _run(_exe("gmap_" + build), SHORT_ARGS)[0] == _read("e2e_short_%s.sam" % build)


@pytest.mark.gpu
@pytest.mark.parametrize("build", BUILDS)
def test_gpu_gmap_short_oligoindex_queries(build):
    """A read whose stage 3 queries an oligoindex with 8 nt (make_e2e.SHORT_OLIGO_READS): the reference
    answers from the previous longer query's 8-mer flags (Oligoindex_set_inquery returns early), which
    the shim tracks per oligoindex; the output equals the reference program's."""
    out, err = _run(_exe("gmap_gpu_" + build), SHORT_ARGS, env={"GMAPDP_SHIM_STATS": "1"})
    assert out == _read("e2e_short_%s.sam" % build)
    assert _stats(err)["Oligoindex_get_mappings"] > 0


S8_ARGS = ["-t", "1", "-g", "e2e_genome.fa", "-f", "samse", "--no-sam-headers", "e2e_s8_reads.fa"]


@pytest.mark.parametrize("build", BUILDS)
def test_reference_gmap_reproduces_s8_fixture(build):
    assert _run(_exe("gmap_" + build), S8_ARGS)[0] == _read("e2e_s8_%s.sam" % build)


@pytest.mark.gpu
@pytest.mark.parametrize("build", BUILDS)
def test_gpu_gmap_8nt_reads(build):
    """8-nt reads (make_e2e.py e2e_s8_reads.fa): GMAP calls Stage2_compute on each, against the previous
    longer query's 8-mer flags; the drop-in answers as the reference does (no refusal) and the output is
    the reference program's."""
    out, err = _run(_exe("gmap_gpu_" + build), S8_ARGS, env={"GMAPDP_SHIM_STATS": "1"})
    assert out == _read("e2e_s8_%s.sam" % build)
    assert _stats(err)["Stage2_compute"] >= 2


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [4, 32])
def test_gpu_gmap_worker_threads(threads):
    """GMAP worker threads sharing the engine through the shim's dispatcher (per-thread requests and
    stage-2 tally records, one engine context): output identical to the single-threaded reference,
    and the dispatcher really ran several threads' calls per batch."""
    out, err = _run(_exe("gmap_gpu_nosimd"), ["-t", str(threads), "-O"] + E2E_ARGS,
                    env={"GMAPDP_SHIM_STATS": "1", "GMAPDP_SHIM_DISPATCHERS": "2"})
    assert out == _read("e2e_nosimd.sam")
    st = _stats(err)
    assert st["batches"] > 0 and (threads < 8 or st["mean_batch"] > 1.5), st


@pytest.mark.gpu
def test_gpu_gmap_parts(monkeypatch):
    """configs[3]'s sharding (tools/multi_gmap.py): three GMAP drop-in processes on the one GPU, each with
    the reads --part=i/3 gives it, outputs merged in input order: identical to the single-process
    reference output, and every copy ran its calls on the engine."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import multi_gmap
    monkeypatch.setenv("GMAPDP_SHIM_STATS", "1")
    rc, out, errs, _ = multi_gmap.run(3, 1, [_exe("gmap_gpu_nosimd"), "-t", "8", "-O"] + E2E_ARGS[:-1],
                                      E2E_ARGS[-1], cwd=GOLD)
    assert rc == 0, errs
    assert out == _read("e2e_nosimd.sam")
    for err in errs:
        assert _stats(err)["Dynprog_single_gap"] > 0


# ---- gmapl (LARGE_GENOMES, 64-bit Univcoord_T): the nosimd semantics, the same fixtures ----

def test_reference_gmapl_reproduces_fixtures():
    exe = _exe("gmap_large")
    assert _run(exe, ALIGN_ARGS)[0] == _read("align.test.ok")
    assert _run(exe, CDNA2_ARGS)[0] == _read("cdna2_genetest2_nosimd.txt")
    assert _run(exe, E2E_ARGS)[0] == _read("e2e_nosimd.sam")


@pytest.mark.gpu
def test_gpu_gmapl_end_to_end():
    """The shim compiled with LARGE_GENOMES into gmapl: 64-bit universal coordinates through the whole
    drop-in, output identical to the reference's."""
    exe = _exe("gmap_gpu_large")
    out, err = _run(exe, ALIGN_ARGS, env={"GMAPDP_SHIM_STATS": "1"})
    assert out == _read("align.test.ok")
    assert _run(exe, CDNA2_ARGS)[0] == _read("cdna2_genetest2_nosimd.txt")
    out, err = _run(exe, E2E_ARGS, env={"GMAPDP_SHIM_STATS": "1"})
    assert out == _read("e2e_nosimd.sam")
    st = _stats(err)
    for k in ("Dynprog_single_gap", "Dynprog_genome_gap", "Stage2_compute", "Dynprog_microexon_int"):
        assert st[k] > 0, st


# ---- indexed genome (-d: stage 1, two chromosomes) and known splice sites (-s) ----
# tests/golden/idx (make_index.py): a two-chromosome index built by the reference's gmap_build /
# gmapindex, 160 reads (120 with 10-30-nt terminal exons), the known sites as the reference program
# reports them for the full-length transcripts (iit_store), and the reference program's SAM.
IDX_ARGS = ["-D", "idx/db", "-d", "e2eidx", "-f", "samse", "--no-sam-headers", "idx/sj_reads.fa"]
SITES_ARGS = ["-s", "idx/db/e2eidx/e2eidx.maps/e2esites.iit"] + IDX_ARGS


@pytest.mark.parametrize("build", BUILDS)
def test_reference_gmap_indexed_reproduces_fixtures(build):
    exe = _exe("gmap_" + build)
    assert _run(exe, IDX_ARGS)[0] == _read("idx/d_%s.sam" % build)
    assert _run(exe, SITES_ARGS)[0] == _read("idx/ds_%s.sam" % build)


def test_known_sites_fixture_differs_from_plain():
    """the known sites matter: -s recovers short terminal exons on many reads"""
    a, b = _read("idx/d_nosimd.sam").splitlines(), _read("idx/ds_nosimd.sam").splitlines()
    assert len(a) == len(b) == 160
    assert sum(1 for x, y in zip(a, b) if x != y) >= 20


def _same_sam(out, fixture):
    exp = _read(fixture).splitlines()
    got = out.splitlines()
    bad = [i for i, (x, y) in enumerate(zip(got, exp)) if x != y]
    assert len(got) == len(exp) and not bad, "reads differing: %s" % bad[:10]


@pytest.mark.gpu
@pytest.mark.parametrize("build", BUILDS)
def test_gpu_gmap_indexed_genome(build):
    """`gmap -d` (stage 1 over a two-chromosome index, then stages 2-3) through the drop-in: SAM identical
    to the reference program's."""
    out, err = _run(_exe("gmap_gpu_" + build), IDX_ARGS, env={"GMAPDP_SHIM_STATS": "1"})
    _same_sam(out, "idx/d_%s.sam" % build)
    st = _stats(err)
    assert st["Stage2_compute"] > 0 and st["Dynprog_genome_gap"] > 0, st


@pytest.mark.gpu
@pytest.mark.parametrize("build,threads", [("nosimd", 1), ("nosimd", 16), ("avx2", 1), ("avx2", 16)])
def test_gpu_gmap_known_splice_sites(build, threads):
    """`gmap -d -s`: Dynprog_end5/3_known restated in the shim, the splice-trie walk's
    Dynprog_end5/3_splicejunction calls and the known-site genome gaps on the engine, in both builds'
    semantics; SAM identical to the reference program's."""
    args = SITES_ARGS if threads == 1 else ["-t", str(threads), "-O"] + SITES_ARGS
    out, err = _run(_exe("gmap_gpu_" + build), args, env={"GMAPDP_SHIM_STATS": "1"})
    _same_sam(out, "idx/ds_%s.sam" % build)
    st = _stats(err)
    for k in ("Dynprog_end5_known", "Dynprog_end3_known", "Dynprog_end5_splicejunction",
              "Dynprog_end3_splicejunction", "Dynprog_genome_gap"):
        assert st[k] > 0, st
