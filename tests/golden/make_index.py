"""Generate the indexed-genome end-to-end fixtures (`gmap -d`, and `gmap -d -s` with known splice sites):
a small GMAP genome index built by the reference's own tools, seeded synthetic reads, and the reference
`gmap` program's outputs on them.

Run in the development container after `make -C oracle ref` and `make -C oracle -f ref.mk index_tools`
(oracle/_ref/bin/gmapindex and iit_store are compiled from /root/reference/src; the index is made by the
reference's util/gmap_build perl script, and the splice-site list by the reference program itself):

    python tests/golden/make_index.py

Inputs (restated, seeded): the e2e segment (e2e_genome.fa, 300 kb) with further GT...AG junctions planted
for the new reads, plus ss.chr17test.fa as a second chromosome.  Reads: NSJ transcripts of 4 exons whose
first and last exons are short (10-30 nt: the read ends stage 2 cannot anchor, which stage 3 aligns with
Dynprog_end5/3_known against the known sites, dynprog_end.c:2748/3009), 1 % substitutions, half
reverse-complemented; then the first NOLD reads of e2e_reads.fa.  The known sites are what the reference
program reports for the full-length transcripts (`gmap -f splicesites`), stored with iit_store.

Outputs (data only), under tests/golden/idx/:
  db/e2eidx/...              the genome index (gmap_build -k 12; suffix-array files dropped: gmap does
                             not read them)
  db/e2eidx/e2eidx.maps/e2esites.iit   the known splice sites (iit_store)
  sj_reads.fa                the reads
  d_{nosimd,avx2}.sam        `gmap_<build> -D db -d e2eidx -f samse --no-sam-headers sj_reads.fa`
  ds_{nosimd,avx2}.sam       the same with `-s db/e2eidx/e2eidx.maps/e2esites.iit`
"""
import os
import random
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_e2e import ROOT, REF, revcomp, write_fasta  # noqa: E402

OUT = os.path.join(HERE, "idx")
REFTREE = "/root/reference"
SEED = 4242
NSJ = 120
NOLD = 40
SITES = "db/e2eidx/e2eidx.maps/e2esites.iit"  # relative to tests/golden/idx


def read_fasta(path):
    recs, name, buf = [], None, []
    for line in open(path):
        line = line.strip()
        if line.startswith(">"):
            if name is not None:
                recs.append((name, "".join(buf)))
            name, buf = line[1:].split()[0], []
        elif line:
            buf.append(line)
    if name is not None:
        recs.append((name, "".join(buf)))
    return recs


def transcripts(genome, rng, n):
    """n 4-exon transcripts on `genome` (a list, junctions planted in place): full exon coordinates."""
    out = []
    for _ in range(n):
        introns = [rng.randint(90, 6000) for _ in range(3)]
        span = 4 * 300 + sum(introns)
        start = rng.randrange(2000, len(genome) - span - 2000)
        exons, pos = [], start
        for e in range(4):
            exons.append((pos, pos + 300))
            pos += 300 + (introns[e] if e < 3 else 0)
        for e in range(3):
            a = exons[e][1]
            b = exons[e + 1][0]
            genome[a], genome[a + 1] = "G", "T"
            genome[b - 2], genome[b - 1] = "A", "G"
        out.append(exons)
    return out


def main():
    gmap = os.path.join(REF, "gmap_nosimd")
    bindir = os.path.join(REF, "bin")
    for exe in (gmap, os.path.join(bindir, "gmapindex"), os.path.join(bindir, "iit_store")):
        if not os.path.exists(exe):
            sys.exit("missing %s: build oracle/_ref first" % exe)
    rng = random.Random(SEED)
    seg = list(read_fasta(os.path.join(HERE, "e2e_genome.fa"))[0][1])
    chr17 = read_fasta(os.path.join(HERE, "ss.chr17test.fa"))[0]
    tx = transcripts(seg, rng, NSJ)
    seg = "".join(seg)
    full, reads = [], []
    for i, exons in enumerate(tx):
        exseq = [seg[a:b] for a, b in exons]
        full.append(("t%d" % i, "".join(exseq)))
        l5, l3 = rng.randint(10, 30), rng.randint(10, 30)
        s = list(exseq[0][-l5:] + exseq[1] + exseq[2] + exseq[3][:l3])
        for k in range(len(s)):
            if rng.random() < 0.01:
                s[k] = rng.choice([c for c in "ACGT" if c != s[k]])
        s = "".join(s)
        minus = rng.random() < 0.5
        reads.append(("sj%d_%d_%s" % (i, exons[0][1] - l5 + 1, "-" if minus else "+"), revcomp(s) if minus else s))
    reads += read_fasta(os.path.join(HERE, "e2e_reads.fa"))[:NOLD]

    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    os.makedirs(OUT)
    with tempfile.TemporaryDirectory() as tmp:
        fa = os.path.join(tmp, "two.fa")
        write_fasta(fa, [("synseg", seg), chr17])
        tbin = os.path.join(tmp, "bin")
        os.makedirs(tbin)
        for t in ("gmapindex", "iit_store"):
            shutil.copy(os.path.join(bindir, t), tbin)
        for t in ("fa_coords", "gmap_process"):
            os.symlink(os.path.join(REFTREE, "util", t), os.path.join(tbin, t))
        db = os.path.join(OUT, "db")
        subprocess.run(["perl", os.path.join(REFTREE, "util", "gmap_build"), "-B", tbin, "-D", db, "-d", "e2eidx",
                        "-k", "12", fa], check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        d = os.path.join(db, "e2eidx")
        for f in os.listdir(d):  # suffix arrays / localdb: gsnap's, not read by gmap
            if f.startswith("e2eidx.sa") or f.startswith("e2eidx.sarray"):
                os.remove(os.path.join(d, f))
        tfa = os.path.join(tmp, "full.fa")
        write_fasta(tfa, full)
        sites = subprocess.run([gmap, "-D", db, "-d", "e2eidx", "-f", "splicesites", tfa], check=True,
                               capture_output=True).stdout
        open(os.path.join(OUT, "e2esites.txt"), "wb").write(sites)
        subprocess.run([os.path.join(tbin, "iit_store"), "-o", os.path.join(d, "e2eidx.maps", "e2esites")],
                       input=sites, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    write_fasta(os.path.join(OUT, "sj_reads.fa"), reads)
    base = ["-D", "db", "-d", "e2eidx", "-f", "samse", "--no-sam-headers", "sj_reads.fa"]
    # -s takes the .iit path: a bare name that is not a local file makes gmap.c:6318 call strlen on a NULL
    # user_splicingdir (the reference crashes)
    for build in ("nosimd", "avx2"):
        exe = os.path.join(REF, "gmap_" + build)
        for name, extra in (("d_%s.sam" % build, []), ("ds_%s.sam" % build, ["-s", SITES])):
            with open(os.path.join(OUT, name), "w") as f:
                subprocess.run([exe] + extra + base, stdout=f, stderr=subprocess.DEVNULL, check=True, cwd=OUT)
    a = open(os.path.join(OUT, "d_nosimd.sam")).read().splitlines()
    b = open(os.path.join(OUT, "ds_nosimd.sam")).read().splitlines()
    print("wrote %s: %d reads, %d known-site lines, %d SAM lines differ with -s" % (
        OUT, len(reads), sites.count(b"\n"), sum(1 for x, y in zip(a, b) if x != y)))


if __name__ == "__main__":
    sys.exit(main())
