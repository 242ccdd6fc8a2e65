"""Measure the per-read call mix GMAP's own pipeline makes into the hot path for a read shape
(MEASUREMENT INFRASTRUCTURE: runs the unmodified reference gmap, oracle/_ref/gmap_callmix, whose entry
points are counted by oracle/callmix.c; nothing here is product code).

Both read shapes run the same way -- GMAP in user-segment mode (`-g`, stage 2 + stage 3 over a synthetic
segment holding every read's locus) on the same synthetic genome -- so their ratio is measured under one
method:
  cdna2k : 2-kb cDNA, 5 exons x 400 nt, 2 % substitutions (BASELINE configs[2]; SURVEY App. B's shape)
  isoseq5k: 5-kb Iso-Seq-style, 10 exons x 500 nt, 1 % substitutions + 1 % 1-nt indels (configs[4])
Introns log-uniform [80, 20000] nt with GT..AG planted, half the reads reverse-complemented.

  python tools/callmix.py --reads 200 --out profiles/r03_callmix/callmix.json

--index runs GMAP as it runs in production instead (`-d`: stage 1 over a genome index, then stages 2 and
3): the same segment is indexed by the reference's own gmap_build (util/gmap_build with the gmapindex
compiled by `make -C oracle -f ref.mk index_tools`), and the reads are mapped against it.

  python tools/callmix.py --index --reads 200 --genome 20000000 --out profiles/r04_callmix/callmix_d.json
"""
import argparse
import collections
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GMAP = os.path.join(ROOT, "oracle", "_ref", "gmap_callmix")
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
COMPL = np.zeros(256, dtype=np.uint8)
for a, b in zip(b"ACGT", b"TGCA"):
    COMPL[a] = b
SHAPES = {"cdna2k": dict(exons=5, exlen=400, subs=0.02, indel=0.0),
          "isoseq5k": dict(exons=10, exlen=500, subs=0.01, indel=0.01)}


def make_reads(genome, n, seed, exons, exlen, subs, indel):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        introns = np.exp(rng.uniform(np.log(80), np.log(20000), size=exons - 1)).astype(np.int64)
        span = exons * exlen + int(introns.sum())
        start = int(rng.integers(1000, len(genome) - span - 1000))
        pos, parts = start, []
        for e in range(exons):
            parts.append(genome[pos:pos + exlen].copy())
            if e < exons - 1:
                il = int(introns[e])
                genome[pos + exlen:pos + exlen + 2] = np.frombuffer(b"GT", dtype=np.uint8)
                genome[pos + exlen + il - 2:pos + exlen + il] = np.frombuffer(b"AG", dtype=np.uint8)
                pos += exlen + il
        q = np.concatenate(parts)
        q = np.where(rng.random(len(q)) < subs, ACGT[rng.integers(0, 4, size=len(q))], q).astype(np.uint8)
        if indel > 0:
            u = rng.random(len(q))
            reps = np.where(u < indel / 2, 0, np.where(u < indel, 2, 1))
            q = np.repeat(q, reps)
            ends = np.cumsum(reps) - 1
            ins = ends[reps == 2]
            q[ins] = ACGT[rng.integers(0, 4, size=len(ins))]
        if rng.random() < 0.5:
            q = COMPL[q[::-1]]
        out.append(("r%d_%d" % (i, start + 1), q.tobytes().decode()))
    return out


def write_fasta(path, recs):
    with open(path, "w") as f:
        for name, s in recs:
            f.write(">%s\n" % name)
            for k in range(0, len(s), 60):
                f.write(s[k:k + 60] + "\n")


def summarize(log, nreads):
    kinds = collections.defaultdict(list)
    for line in open(log):
        f = line.split()
        if f:
            kinds[f[0]].append([int(x) for x in f[1:]])
    out = {}
    names = {"S": "single", "E5": "end5", "E3": "end3", "G": "genome", "C": "cdna", "M": "microexon",
             "T": "stage2_compute"}
    for k, name in names.items():
        v = np.array(kinds.get(k, []), dtype=np.int64).reshape(-1, 4 if k in ("S", "E5", "E3") else
                                                                (5 if k in ("G", "T") else (3 if k == "C" else 2)))
        rec = {"calls": int(len(v)), "per_read": len(v) / nreads}
        if len(v):
            rec["rlength_mean"] = float(v[:, 0].mean())
            rec["rlength_p50_p99_max"] = [int(np.percentile(v[:, 0], 50)), int(np.percentile(v[:, 0], 99)),
                                          int(v[:, 0].max())]
            if k in ("S", "E5", "E3", "G"):
                rec["glength_mean"] = float(v[:, 1].mean())
                rec["glength_p50_p99_max"] = [int(np.percentile(v[:, 1], 50)), int(np.percentile(v[:, 1], 99)),
                                              int(v[:, 1].max())]
            if k == "G":
                rec["finalp_frac"] = float(v[:, 4].mean())
            if k == "S":
                rec["length_differs_frac"] = float((v[:, 0] != v[:, 1]).mean())
                rec["abs_length_diff_mean"] = float(np.abs(v[:, 0] - v[:, 1]).mean())
            if k == "T":
                rec["window_mean"] = float(v[:, 1].mean())
                rec["window_p10_p50_p90_max"] = [int(np.percentile(v[:, 1], x)) for x in (10, 50, 90)] + [int(v[:, 1].max())]
                rec["plus_frac"] = float(v[:, 3].mean())
                rec["paths_returned_hist"] = {int(x): int((v[:, 4] == x).sum()) for x in np.unique(v[:, 4])}
        out[name] = rec
    return out


REFTREE = "/root/reference"
BIN = os.path.join(ROOT, "oracle", "_ref", "bin")


def build_index(d, gpath, name):
    """gmap_build (the reference's perl driver with the gmapindex / iit_store compiled from its sources)."""
    tbin = os.path.join(d, "bin_" + name)
    os.makedirs(tbin)
    for t in ("gmapindex", "iit_store"):
        os.symlink(os.path.join(BIN, t), os.path.join(tbin, t))
    for t in ("fa_coords", "gmap_process"):
        os.symlink(os.path.join(REFTREE, "util", t), os.path.join(tbin, t))
    db = os.path.join(d, "db")
    subprocess.run(["perl", os.path.join(REFTREE, "util", "gmap_build"), "-B", tbin, "-D", db, "-d", name, gpath],
                   check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return ["-D", db, "-d", name]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=200)
    ap.add_argument("--genome", type=int, default=2_000_000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--index", action="store_true", help="gmap -d over a gmap_build index (stage 1 included)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    mode = ("indexed-genome mode (-d: stage 1 over a gmap_build index of the segment)" if a.index
            else "user-segment mode (-g)")
    res = {"method": "unmodified reference gmap (nosimd) in %s with the hot-path entry points counted "
                     "(oracle/callmix.c); %d reads per shape on a %d-nt i.i.d. segment" % (mode, a.reads, a.genome),
           "shapes": {}}
    with tempfile.TemporaryDirectory() as d:
        for si, (shape, kw) in enumerate(SHAPES.items()):
            genome = np.random.default_rng(38).integers(0, 4, size=a.genome).astype(np.uint8)
            genome = ACGT[genome]
            reads = make_reads(genome, a.reads, 1000 + si, **kw)
            gpath, rpath, log = (os.path.join(d, "%s_%s" % (shape, x)) for x in ("genome.fa", "reads.fa", "log"))
            write_fasta(gpath, [("seg", genome.tobytes().decode())])
            write_fasta(rpath, reads)
            t0 = time.perf_counter()
            src = build_index(d, gpath, shape) if a.index else ["-g", gpath]
            r = subprocess.run([GMAP] + src + ["-t", str(a.threads), "-f", "samse", "--no-sam-headers", rpath],
                               capture_output=True, text=True, env=dict(os.environ, GMAPDP_CALLMIX_LOG=log))
            if r.returncode != 0:
                raise SystemExit(r.stderr[-2000:])
            mapped = sum(1 for ln in r.stdout.splitlines() if ln and not ln.startswith("@") and
                         int(ln.split("\t")[1]) & 4 == 0)
            s = summarize(log, a.reads)
            s["shape"] = kw
            s["reads_mapped_records"] = mapped
            s["seconds"] = time.perf_counter() - t0
            res["shapes"][shape] = s
    base, iso = res["shapes"]["cdna2k"], res["shapes"]["isoseq5k"]
    res["isoseq_over_cdna_per_read"] = {k: (iso[k]["per_read"] / base[k]["per_read"] if base[k]["per_read"] else None)
                                        for k in base if isinstance(base[k], dict) and "per_read" in base[k]}
    txt = json.dumps(res, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    sys.exit(main())
