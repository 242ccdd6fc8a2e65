"""Synthetic configs[2] workload (BASELINE.json): 2-kb cDNA reads (5 exons x 400 nt, 2 %
substitutions) against a GRCh38-shaped genome, as the stream of calls GMAP's per-read pipeline
makes into the path (SURVEY.md §8d "Synthetic inputs", App. B per-read call counts).

Genome: an i.i.d. uniform ACGT genome laid out as GRCh38's 24 primary chromosomes (3.09 Gnt), so
universal coordinates (chroffset + chrpos) run past 2^31 like the real assembly's; chrpos stays
below 2^28.  Random genomes have no repeats, so stage-2 windows carry fewer spurious hits than real
GRCh38 would (stated wherever numbers are reported).

Per 2-kb read (nosimd instrumentation):
  1 stage-2 seeding call (Oligoindex_hr_tally + Oligoindex_get_mappings, stage2.c:6480-6495)
  43.7 Dynprog_single_gap, 7.1 Dynprog_end5_gap, 6.5 Dynprog_end3_gap, 49.4 Dynprog_genome_gap.
Sub-problem shapes follow the measured size distributions (replay mode); genome gaps
span planted GT-AG introns.  Everything is vectorised numpy and seeded.

configs[4] (gmapl, 5-kb Iso-Seq-style reads, 10 exons, 1 % substitutions + 1 % indels, 17-Gnt wheat
genome): the same generators with the ISOSEQ shape (per-read call mix measured with the reference's own
gmap on reads of that shape, oracle/callmix.c) and the WHEAT17 layout, whose universal
coordinates run past 2^32 (64-bit Univcoord_T, univcoord.h:9-11).  Genomes of that size are generated
directly as packed .genomecomp blocks (PackedGenome): no ASCII copy is ever made.

Read stream and sharding: the stream is cut into blocks of `reads` reads; block b is generated from its
own seeds (reads: 1000 + 7919 b, intron sites: 23 + b), so the stream is the same whatever the world
size, and rank r of N takes the blocks b with b % N == r (GMAP's --part=r/N rule, inbuffer.c:283,
applied per block; gmapdp.shard).  Every rank plants the intron sites of every block of the stream in
block order, so all ranks hold the same genome.
"""
import os

import numpy as np

# GRCh38 primary assembly chromosome lengths (chr1..chr22, chrX, chrY)
GRCH38 = [("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555),
          ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636),
          ("chr9", 138394717), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
          ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
          ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
          ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415)]
CHR22 = [("chr22", 50818468)]

# Wheat (Chinese Spring) 21 chromosomes + unplaced, lengths rounded from IWGSC RefSeq v1.0 and scaled by
# 17 / 14.55 so the genome is the 17 Gnt BASELINE configs[4] names; every chromosome stays below 2^31
# (Chrpos_T), universal coordinates run to 1.7e10 > 2^32 (gmapl).
_WHEAT = [("1A", 594.1), ("1B", 689.9), ("1D", 495.5), ("2A", 780.8), ("2B", 801.3), ("2D", 651.9), ("3A", 750.8),
          ("3B", 830.8), ("3D", 615.6), ("4A", 744.6), ("4B", 673.6), ("4D", 509.9), ("5A", 709.8), ("5B", 713.1),
          ("5D", 566.1), ("6A", 618.1), ("6B", 721.0), ("6D", 473.6), ("7A", 736.7), ("7B", 750.6), ("7D", 638.7),
          ("Un", 481.0)]
WHEAT17 = [("chr" + c, int(round(m * 1e6 * 17e9 / (sum(x for _, x in _WHEAT) * 1e6)))) for c, m in _WHEAT]


class Shape:
    """Read shape and per-read call mix of one BASELINE config."""

    def __init__(self, name, exons, exlen, subs, indel, single, end5, end3, genome, microexon, source,
                 single_indel=0.15, single_dmean=0.0, stage2=1.0, pad=1000):
        self.name, self.exons, self.exlen, self.subs, self.indel = name, exons, exlen, subs, indel
        self.single, self.end5, self.end3, self.genome, self.microexon = single, end5, end3, genome, microexon
        self.source = source
        # Stage2_compute calls per read (above 1: a second call on the same read and nearly the same window,
        # as gmap -d makes for part of its reads) and the genomic window: the locus plus `pad` nt each side
        self.stage2, self.pad = stage2, pad
        # single gaps whose query and genome lengths differ: a fraction, and (single_dmean > 0) the mean of
        # an exponential genome-minus-query excess; otherwise a uniform +-1..3 nt indel
        self.single_indel, self.single_dmean = single_indel, single_dmean

    @property
    def readlength(self):
        return self.exons * self.exlen


# configs[2]: 2-kb cDNA, 5 x 400 nt, 2 % substitutions.  Call mix measured with the reference's own gmap as
# it runs in production (`gmap -d` over a gmap_build index: stage 1, then stages 2 and 3; tools/callmix.py
# --index, profiles/r04_callmix/callmix_d.json): per read 21.1 single gaps (2.5 % with query and genome
# lengths differing, by 80 nt on average), 6.78 end5, 6.38 end3, 49.7 genome gaps, 7.53 microexon calls and
# 1.585 Stage2_compute calls over windows of 205-232 kb (p10-p90): stage 1 extends each gregion by
# EXTRA_LONGEND = 100 kb on both sides (gregion.c:27, 899).
CDNA2K = Shape("cdna2k", 5, 400, 0.02, 0.0, 21.1, 6.78, 6.38, 49.7, 7.53,
               "measured: reference gmap -d on 200 reads of this shape (profiles/r04_callmix/callmix_d.json)",
               single_indel=0.025, single_dmean=80.0, stage2=1.585, pad=98000)
# the same reads with SURVEY App. B's mix (rounds 1-3's headline): one Stage2_compute per read over the
# locus +- 1 kb, 43.7 single, 7.1 end5, 6.5 end3, 49.4 genome, 25.6 microexon calls
CDNA2K_APPB = Shape("cdna2k-appb", 5, 400, 0.02, 0.0, 43.7, 7.1, 6.5, 49.4, 25.6, "SURVEY App. B")
# configs[4]: 5-kb Iso-Seq-style reads, 10 x 500 nt, 1 % substitutions + 1 % indels.  Call mix measured
# with the reference's own gmap on 200 reads of that shape (oracle/callmix.c, tools/callmix.py,
# profiles/r03_callmix/callmix.json): per read 285.1 single gaps (91 % with query and genome lengths
# differing, genome longer by 22 nt on average), 4.66 end5, 4.05 end3, 77.4 genome gaps, 36.95 microexon
# calls; Stage2_compute once per read over the read's gregion, as configs[2]
ISOSEQ5K_G = Shape("isoseq5k-g", 10, 500, 0.01, 0.01, 285.1, 4.66, 4.05, 77.4, 36.95,
                   "measured: reference gmap -g on 200 reads of this shape (profiles/r03_callmix/callmix.json)",
                   single_indel=0.91, single_dmean=22.0)
# the same measured with gmap -d (profiles/r04_callmix/callmix_d.json): 584.5 single gaps (96 % lengths
# differing, by 33 nt), 7.72 end5, 6.79 end3, 148.5 genome gaps, 67.5 microexon calls, 1.69 Stage2_compute
# calls over 217-263-kb windows
ISOSEQ5K = Shape("isoseq5k", 10, 500, 0.01, 0.01, 584.5, 7.72, 6.79, 148.5, 67.5,
                 "measured: reference gmap -d on 200 reads of this shape (profiles/r04_callmix/callmix_d.json)",
                 single_indel=0.96, single_dmean=33.0, stage2=1.69, pad=110000)
SHAPES = {"d": CDNA2K, "appb": CDNA2K_APPB}

SINGLE_PER_READ = CDNA2K.single        # Dynprog_single_gap calls per 2-kb read (gmap -d, nosimd)
END5_PER_READ = CDNA2K.end5            # Dynprog_end5_gap
END3_PER_READ = CDNA2K.end3            # Dynprog_end3_gap
GENOME_PER_READ = CDNA2K.genome        # Dynprog_genome_gap
STAGE2_PER_READ = CDNA2K.stage2        # Stage2_compute calls
MICROEXON_PER_READ = CDNA2K.microexon  # Dynprog_microexon_int

COMPL = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTN", b"TGCAN"):
    COMPL[_a] = _b
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
CODE = np.zeros(256, dtype=np.uint8)
for _k, _c in enumerate(b"ACGT"):
    CODE[_c] = _k
# one packed byte (4 nt, nt j in bits 2j..2j+1) -> 4 ASCII bytes as a little-endian uint32
_LUT4 = np.array([sum(int(ACGT[(x >> (2 * k)) & 3]) << (8 * k) for k in range(4)) for x in range(256)],
                 dtype=np.uint32)


class Layout:
    """Chromosomes laid end to end in universal coordinates (chroffset, chrhigh = chroffset + length)."""

    def __init__(self, chroms):
        self.names = [c for c, _ in chroms]
        self.lens = np.array([n for _, n in chroms], dtype=np.int64)
        self.offsets = np.concatenate([[0], np.cumsum(self.lens)[:-1]]).astype(np.int64)
        self.total = int(self.lens.sum())

    def sample(self, rng, n, margin):
        """n chromosomes drawn by length; returns (chroffset, chrhigh, chrlength) arrays."""
        u = rng.random(n) * self.total
        c = np.searchsorted(np.cumsum(self.lens), u, side="right")
        c = np.minimum(c, len(self.lens) - 1)
        return self.offsets[c], self.offsets[c] + self.lens[c], self.lens[c]


class PackedGenome:
    """An i.i.d. ACGT genome held only as the reference's .genomecomp blocks (3 words per 32 nt: high
    nt 16-31, low nt 0-15, flags; 2 bits per nt A0 C1 G2 T3; the last block's tail and 4 trailing
    words are 'X' padding: gmapdp_pack_genome / Compress_create_blocks_comp).  Indexing with an integer
    array of universal positions returns ASCII bytes; assigning ASCII bytes plants them."""

    def __init__(self, length, seed=38, chunk=1 << 24):
        self.length = int(length)
        nb = (self.length + 31) // 32
        self.blocks = np.empty(3 * nb + 4, dtype=np.uint32)
        v = self.blocks[:3 * nb].reshape(nb, 3)
        rng = np.random.default_rng(seed)
        for a in range(0, nb, chunk):
            b = min(nb, a + chunk)
            raw = rng.integers(0, 1 << 32, size=(b - a, 2), dtype=np.uint32)
            v[a:b, 0] = raw[:, 0]
            v[a:b, 1] = raw[:, 1]
            v[a:b, 2] = 0
        tail = 32 * nb - self.length
        if tail:
            j = np.arange(32 - tail, 32)
            for k in j:
                word = 0 if k >= 16 else 1
                v[nb - 1, word] |= np.uint32(3 << (2 * (k & 15)))
                v[nb - 1, 2] |= np.uint32(1 << int(k))
        self.blocks[3 * nb:] = 0xFFFFFFFF

    def __len__(self):
        return self.length

    def _where(self, idx):
        idx = np.asarray(idx, dtype=np.int64)
        j = (idx & 31).astype(np.uint32)
        w = 3 * (idx >> 5) + 1 - (j >> 4).astype(np.int64)
        return w, (j & 15) << 1

    def __getitem__(self, idx):
        w, sh = self._where(idx)
        return ACGT[(self.blocks[w] >> sh) & 3]

    def __setitem__(self, idx, ch):
        idx = np.asarray(idx, dtype=np.int64).ravel()
        code = CODE[np.broadcast_to(np.asarray(ch, dtype=np.uint8), idx.shape)].astype(np.uint32)
        # one write per position (the last wins, as plain fancy assignment), then read-modify-write
        # per word with ufunc.at so two positions of one word both land
        _, last = np.unique(idx[::-1], return_index=True)
        keep = len(idx) - 1 - last
        idx, code = idx[keep], code[keep]
        w, sh = self._where(idx)
        np.bitwise_and.at(self.blocks, w, ~(np.uint32(3) << sh))
        np.bitwise_or.at(self.blocks, w, code << sh)

    def ascii(self, start, end):
        """bytes of universal positions [start, end) (whole blocks through a byte -> 4-nt table; the
        stream has no flagged positions below `length`)"""
        b0, b1 = start // 32, (end + 31) // 32
        v = self.blocks[3 * b0:3 * b1].reshape(b1 - b0, 3)
        out = np.empty((b1 - b0, 32), dtype=np.uint8)
        out[:, :16] = _LUT4[np.ascontiguousarray(v[:, 1]).view(np.uint8)].view(np.uint8).reshape(-1, 16)
        out[:, 16:] = _LUT4[np.ascontiguousarray(v[:, 0]).view(np.uint8)].view(np.uint8).reshape(-1, 16)
        return out.reshape(-1)[start - 32 * b0:end - 32 * b0].tobytes()


def make_genome(layout, seed=38):
    """i.i.d. ACGT genome of layout.total nt (uint8 ASCII), from 2 random bits per nt."""
    rng = np.random.default_rng(seed)
    n = layout.total
    raw = np.frombuffer(rng.bytes((n + 3) // 4), dtype=np.uint8)
    lut = np.zeros(256, dtype=np.uint32)
    for x in range(256):
        lut[x] = sum(int(ACGT[(x >> (2 * k)) & 3]) << (8 * k) for k in range(4))
    return lut[raw].view(np.uint8)[:n]


def genomic_chars(genome, pos, watson, chroff, chrhigh):
    """get_genomic_nt (dynprog.c) for chromosomal positions in range: plus strand genome[chroffset +
    pos], minus strand the complement of genome[chrhigh - pos]."""
    idx = np.where(watson, chroff + pos, chrhigh - pos)
    ch = genome[idx]
    return np.where(watson, ch, COMPL[ch])


def make_single(genome, layout, n, rng, shape=None):
    """Dynprog_single_gap sub-problems (stage3.c:9081): query slices with 2 % substitutions and
    occasional 1-3 nt indels (or, for shapes with single_dmean, a genome-minus-query excess drawn from an
    exponential), extraband 6, wide band."""
    import gmapdp
    shape = shape or CDNA2K
    g = np.clip(rng.gamma(3.0, 40.0, size=n).astype(np.int64), 1, 640)
    if shape.single_dmean > 0:
        d = -np.rint(rng.exponential(shape.single_dmean, size=n)).astype(np.int64) - 1
        d = np.where(rng.random(n) < shape.single_indel, d, 0)
        d = np.maximum(d, 1 - g)
    else:
        d = np.where(rng.random(n) < shape.single_indel, rng.integers(-3, 4, size=n), 0)
    d = np.where(g + d < 1, 0, d)
    r = np.clip(g + d, 1, 660)
    d = r - g
    watson = rng.random(n) < 0.5
    choff, chrhigh, clen = layout.sample(rng, n, 1000)
    goff = (rng.random(n) * (clen - 1700)).astype(np.int64) + 1
    seg_off = np.concatenate([[0], np.cumsum(g)])
    pid = np.repeat(np.arange(n), g)
    i = np.arange(seg_off[-1]) - seg_off[pid]
    seg = genomic_chars(genome, goff[pid] + i, watson[pid], choff[pid], chrhigh[pid])
    q_off = np.concatenate([[0], np.cumsum(r)])
    qpid = np.repeat(np.arange(n), r)
    j = np.arange(q_off[-1]) - q_off[qpid]
    a = (rng.random(n) * np.maximum(r - np.maximum(d, 0), 1)).astype(np.int64)
    dd, aa = d[qpid], a[qpid]
    src = np.where((dd < 0) & (j >= aa), j - dd, j)                      # deletion: skip -d bases
    ins = (dd > 0) & (j >= aa) & (j < aa + dd)
    src = np.where((dd > 0) & (j >= aa + dd), j - dd, src)               # insertion: shift back
    src = np.clip(src, 0, g[qpid] - 1)
    q = seg[seg_off[qpid] + src]
    rnd = ACGT[rng.integers(0, 4, size=q.size, dtype=np.uint8)]
    q = np.where(ins | (rng.random(q.size) < 0.02), rnd, q).astype(np.uint8)
    probs = np.zeros(n, dtype=gmapdp.PROBLEM_DTYPE)
    probs["qoff"] = q_off[:-1]
    probs["rlength"] = r
    probs["glength"] = g
    probs["roffset"] = rng.integers(0, 1800, size=n)
    probs["goffset"] = goff
    probs["chroffset"] = choff
    probs["chrhigh"] = chrhigh
    probs["flags"] = (watson.astype(np.int32) * gmapdp.WATSON | (rng.random(n) < 0.5) * gmapdp.JUMP_LATE |
                      gmapdp.WIDEBAND)
    probs["genestrand"] = 0
    probs["extraband"] = 6
    probs["defect_rate"] = np.where(rng.random(n) < 0.7, 0.02, 0.01)
    probs["dynprogindex"] = rng.integers(1, 50, size=n) * np.where(rng.random(n) < 0.5, 1, -1)
    return probs, q


def make_end(genome, layout, n5, n3, rng):
    """Dynprog_end5_gap / Dynprog_end3_gap sub-problems: the read end beyond the last anchor
    (lognormal length, median 60 nt), genome = rlength + extramaterial_end (10), mixed endalign."""
    import gmapdp
    n = n5 + n3
    end3 = np.zeros(n, dtype=bool)
    end3[n5:] = True
    L = np.clip(rng.lognormal(np.log(60.0), 1.2, size=n).astype(np.int64), 1, 800)
    g = L + 10
    watson = rng.random(n) < 0.5
    choff, chrhigh, clen = layout.sample(rng, n, 1000)
    # end3: chromosomal positions goffset .. goffset+L-1; end5: rev_goffset-L+1 .. rev_goffset
    goff = np.where(end3, (rng.random(n) * (clen - 1900)).astype(np.int64) + 1,
                    (rng.random(n) * (clen - 1900)).astype(np.int64) + 900)
    first = np.where(end3, goff, goff - L + 1)
    q_off = np.concatenate([[0], np.cumsum(L)])
    qpid = np.repeat(np.arange(n), L)
    j = np.arange(q_off[-1]) - q_off[qpid]
    q = genomic_chars(genome, first[qpid] + j, watson[qpid], choff[qpid], chrhigh[qpid])
    # 2 % substitutions; 15 % of ends carry an unalignable tail (adapter / poly-A) over their far 30 %
    tail = rng.random(n) < 0.15
    far = np.where(end3[qpid], j >= (0.7 * L[qpid]).astype(np.int64), j < (0.3 * L[qpid]).astype(np.int64))
    noise = (rng.random(q.size) < 0.02) | (tail[qpid] & far)
    q = np.where(noise, ACGT[rng.integers(0, 4, size=q.size, dtype=np.uint8)], q).astype(np.uint8)
    probs = np.zeros(n, dtype=gmapdp.END_PROBLEM_DTYPE)
    probs["qoff"] = q_off[:-1]
    probs["rlength"] = L
    probs["glength"] = g
    probs["roffset"] = np.where(end3, rng.integers(1200, 1900, size=n), L - 1 + rng.integers(0, 100, size=n))
    probs["goffset"] = goff
    probs["chroffset"] = choff
    probs["chrhigh"] = chrhigh
    probs["flags"] = watson.astype(np.int32) * gmapdp.WATSON | (rng.random(n) < 0.5) * gmapdp.JUMP_LATE
    probs["genestrand"] = 0
    probs["extraband"] = 6
    probs["end3p"] = end3
    u = rng.random(n)
    probs["endalign"] = np.where(u < 0.5, 1, np.where(u < 0.85, 0, np.where(u < 0.9, 3, 2)))
    probs["require_pos_score_p"] = 0
    probs["dynprogindex"] = rng.integers(1, 50, size=n) * np.where(rng.random(n) < 0.5, 1, -1)
    probs["defect_rate"] = np.where(rng.random(n) < 0.7, 0.02, 0.01)
    return probs, q


def genome_gap_sites(layout, n, site_seed=23):
    """The intron sites of n genome-gap sub-problems (stage3.c:9504-9539), drawn from `site_seed` only
    (rank-independent): a query gap of rlength nt = a exonic nt before a GT..AG intron + b after it;
    goffsetL = first genomic position after the left anchor, rev_goffsetR = last one before the right
    anchor."""
    srng = np.random.default_rng(site_seed)
    r = np.clip(srng.gamma(2.2, 50.0, size=n).astype(np.int64), 2, 600)
    a = (srng.random(n) * (r + 1)).astype(np.int64)
    b = r - a
    intron = srng.integers(60, 5000, size=n)
    watson = srng.random(n) < 0.5
    choff, chrhigh, clen = layout.sample(srng, n, 8000)
    goffL = (srng.random(n) * (clen - 7200)).astype(np.int64) + 100
    revR = goffL + a + intron + b - 1
    don, acc = splice_pool()
    dctx = srng.integers(0, len(don), size=n)
    actx = srng.integers(0, len(acc), size=n)
    return {"dctx": dctx, "actx": actx,
            "r": r, "a": a, "b": b, "watson": watson, "choff": choff, "chrhigh": chrhigh, "goffL": goffL,
            "revR": revR}


# Splice-site contexts planted around every genome-gap intron, so that MaxEnt (evaluated on the device in
# the step) finds strong sites there, as at real introns: a donor context x-3 .. x+5 (x = first intron base)
# and an acceptor context y-19 .. y+3 (y = last intron base), GT..AG included, each site drawing its own from a
# pool of distinct contexts that all score >= 0.9 (splice_contexts.txt, tools/make_splice_pool.py).  One fixed
# context at every site made its 8-mers ~1 per 750 nt of the genome and the stage-2 seeding hits of the reads
# crossing them about doubled; the pool keeps every 8-mer near the i.i.d. background.
_SPLICE_POOL = []


def splice_pool():
    """(donor contexts, acceptor contexts) as uint8 arrays of shape (n, 9) and (n, 23)."""
    if not _SPLICE_POOL:
        d, a = [], []
        for line in open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "splice_contexts.txt")):
            if line.startswith("D "):
                d.append(line.split()[1])
            elif line.startswith("A "):
                a.append(line.split()[1])
        _SPLICE_POOL.extend([np.frombuffer("".join(d).encode(), dtype=np.uint8).reshape(-1, 9),
                             np.frombuffer("".join(a).encode(), dtype=np.uint8).reshape(-1, 23)])
    return _SPLICE_POOL[0], _SPLICE_POOL[1]


def plant_sites(genome, st):
    """Write the splice-site contexts of genome_gap_sites (GT..AG introns) into `genome` (in place)."""
    watson, choff, chrhigh = st["watson"], st["choff"], st["chrhigh"]
    x, y = st["goffL"] + st["a"], st["revR"] - st["b"]   # first / last intron base, strand coordinates
    don, acc = splice_pool()
    dc, ac = don[st["dctx"]], acc[st["actx"]]
    idx, ch = [], []
    ctx = [(x + k - 3, dc[:, k]) for k in range(9)] + [(y + k - 19, ac[:, k]) for k in range(23)]
    for pos, c in ctx:
        idx.append(np.where(watson, choff + pos, chrhigh - pos))
        ch.append(np.where(watson, c, COMPL[c]).astype(np.uint8))
    genome[np.concatenate(idx)] = np.concatenate(ch)


def make_genome_gaps(genome, layout, n, rng, site_seed=23, plant=True, sprob=True):
    """Dynprog_genome_gap sub-problems (stage3.c:9504-9539) over the sites of genome_gap_sites:
    glengthL = glengthR = rlength + 8 (extramaterial_paired), extraband_paired 14.  With `plant`, the
    dinucleotides are planted first (in place; call it before the other sub-problems are cut from the
    genome).  Splice probabilities are synthetic host inputs (0.95 at the planted sites, U[0, 0.3)
    elsewhere): with `sprob` the array, otherwise (length, indices of the 0.95 entries) for a caller
    that draws them where they are used (bench.py: on the device)."""
    import gmapdp
    st = genome_gap_sites(layout, n, site_seed)
    if plant:
        plant_sites(genome, st)
    r, a, b, watson = st["r"], st["a"], st["b"], st["watson"]
    choff, chrhigh, goffL, revR = st["choff"], st["chrhigh"], st["goffL"], st["revR"]
    q_off = np.concatenate([[0], np.cumsum(r)])
    qpid = np.repeat(np.arange(n), r)
    j = np.arange(q_off[-1]) - q_off[qpid]
    src = np.where(j < a[qpid], goffL[qpid] + j, revR[qpid] - b[qpid] + 1 + (j - a[qpid]))
    q = genomic_chars(genome, src, watson[qpid], choff[qpid], chrhigh[qpid])
    q = np.where(rng.random(q.size) < 0.02, ACGT[rng.integers(0, 4, size=q.size, dtype=np.uint8)], q)
    gp = np.zeros(n, dtype=gmapdp.GENOME_PROBLEM_DTYPE)
    gp["qoff"] = q_off[:-1]
    gp["rlength"] = r
    gp["glengthL"] = r + 8
    gp["glengthR"] = r + 8
    gp["roffset"] = rng.integers(0, 1500, size=n)
    gp["goffsetL"] = goffL
    gp["rev_goffsetR"] = revR
    gp["chroffset"] = choff
    gp["chrhigh"] = chrhigh
    gp["flags"] = watson.astype(np.int32) * gmapdp.WATSON | (rng.random(n) < 0.5) * gmapdp.JUMP_LATE
    gp["cdna_direction"] = 1
    gp["extraband"] = 14
    gp["maxpeelback"] = 60
    gp["dynprogindex"] = rng.integers(1, 50, size=n) * np.where(rng.random(n) < 0.5, 1, -1)
    gp["defect_rate"] = np.where(rng.random(n) < 0.7, 0.02, 0.01)
    ent = 2 * (r + 8)
    p_off = np.concatenate([[0], np.cumsum(ent)])
    gp["prob_offset"] = p_off[:-1]
    hi = np.concatenate([p_off[:-1] + a, p_off[:-1] + (r + 8) + b])   # left site cL = a, right site cR = b
    if not sprob:
        return gp, q.astype(np.uint8), (int(p_off[-1]), hi)
    sp = rng.random(int(p_off[-1])) * 0.3
    sp[hi] = 0.95
    return gp, q.astype(np.uint8), sp


def mutate(q, rng, subs, indel):
    """Reads of equal length (rows of q) with `subs` uniform substitutions and `indel` 1-nt indels (half
    deletions, half insertions of a random base) per base.  Returns (flat arena, lengths)."""
    n, L = q.shape
    q = np.where(rng.random(q.shape) < subs, ACGT[rng.integers(0, 4, size=q.shape, dtype=np.uint8)], q)
    if indel <= 0:
        return q.reshape(-1).astype(np.uint8), np.full(n, L, dtype=np.int64)
    u = rng.random(q.shape)
    reps = np.where(u < indel / 2, 0, np.where(u < indel, 2, 1)).astype(np.int64)
    flat = np.repeat(q.reshape(-1), reps.reshape(-1))
    ends = np.cumsum(reps.reshape(-1)) - 1
    ins = ends[reps.reshape(-1) == 2]
    flat[ins] = ACGT[rng.integers(0, 4, size=len(ins), dtype=np.uint8)]
    return flat.astype(np.uint8), reps.sum(axis=1)


def make_stage2(genome, layout, n, rng, exons=5, exlen=400, pad=1000, subs=0.02, indel=0.0, extra=0.0):
    """Stage-2 calls of n reads: `exons` exons x `exlen` nt cut from the genome with log-uniform
    [80, 20000] introns, substitutions and indels, half reverse-complemented (seeded on the minus
    strand), against the window spanning the locus plus `pad` nt each side (the extended gregion); then
    round(extra * n) second calls, on the first reads again over the window moved 9 nt left and 18 nt
    shorter (what gmap -d's second calls on a read look like), each with its own copy of the query.
    Returns (gmapdp_oligo_problem array, upper-case query arena)."""
    import gmapdp
    introns = np.exp(rng.uniform(np.log(80), np.log(20000), size=(n, exons - 1))).astype(np.int64)
    span = exons * exlen + introns.sum(axis=1)
    choff, chrhigh, clen = layout.sample(rng, n, 0)
    start = pad + (rng.random(n) * (clen - span - 2 * pad)).astype(np.int64)
    exstart = np.concatenate([np.zeros((n, 1), dtype=np.int64),
                              np.cumsum(exlen + introns, axis=1)], axis=1) + start[:, None]   # (n, exons)
    j = np.arange(exons * exlen)
    src = choff[:, None] + exstart[:, j // exlen] + j % exlen        # universal coordinates, exon by exon
    flat, L = mutate(genome[src], rng, subs, indel)
    off = np.concatenate([[0], np.cumsum(L)])
    plus = rng.random(n) < 0.5
    qpid = np.repeat(np.arange(n), L)
    k = np.arange(off[-1]) - off[qpid]
    rc = ~plus[qpid]
    q = flat[np.where(rc, off[qpid] + L[qpid] - 1 - k, off[qpid] + k)]
    q = np.where(rc, COMPL[q], q).astype(np.uint8)
    probs = np.zeros(n, dtype=gmapdp.OLIGO_PROBLEM_DTYPE)
    probs["qoff"] = off[:-1]
    probs["querylength"] = L
    probs["chrstart"] = start - pad
    probs["chrend"] = start + span + pad
    probs["chroffset"] = choff
    probs["chrhigh"] = chrhigh
    probs["plusp"] = plus
    probs["minor"] = 0
    m = int(round(extra * n))
    if m > 0:
        dup = probs[:m].copy()
        dup["qoff"] = len(q) + off[:m]
        dup["chrstart"] = np.maximum(dup["chrstart"].astype(np.int64) - 9, 0)
        dup["chrend"] = dup["chrend"].astype(np.int64) - 27
        q = np.concatenate([q, q[:off[m]]])
        probs = np.concatenate([probs, dup])
    return probs, q


def make_microexon(gp, n, rng):
    """Dynprog_microexon_int calls (stage3.c:9664): stage 3 tries a microexon inside a genome gap it
    just bridged (a noncanonical intron or one that scores below the peeled anchors), over the same
    gap: rsequence = the query gap, goffsetL = genomedp5, rev_goffsetR = genomedp3.  So the calls are
    the first n genome-gap sub-problems' gaps (their query slices in the same arena), cdna_direction as
    there.  Returns a gmapdp_microexon_problem array."""
    import gmapdp
    k = np.arange(n) % len(gp)
    g = gp[k]
    mp = np.zeros(n, dtype=gmapdp.MICROEXON_PROBLEM_DTYPE)
    for f in ("qoff", "rlength", "roffset", "goffsetL", "rev_goffsetR", "cdna_direction", "chroffset", "chrhigh",
              "genestrand", "dynprogindex"):
        mp[f] = g[f]
    mp["watsonp"] = (g["flags"] & gmapdp.WATSON) != 0
    return mp


def block_seeds(b):
    """(read seed, intron-site seed) of block b of the read stream"""
    return 1000 + 7919 * b, 23 + b


def make_reads(genome, layout, reads, seed, site_seed=23, shape=CDNA2K, plant=True, sprob=True):
    """The per-read call stream of `reads` reads of `shape`: dict of descriptor arrays and arenas.
    With `plant`, genome gaps plant their intron motifs first (in place), then every other sub-problem
    is cut."""
    rng = np.random.default_rng(seed)
    ng = int(round(reads * shape.genome))
    # intron sites are rank-independent (site_seed), so every rank plants the same genome
    gp, gq, sp = make_genome_gaps(genome, layout, ng, np.random.default_rng(seed + 1), site_seed=site_seed,
                                  plant=plant, sprob=sprob)
    ns = int(round(reads * shape.single))
    n5 = int(round(reads * shape.end5))
    n3 = int(round(reads * shape.end3))
    sp_, sq = make_single(genome, layout, ns, rng, shape)
    ep, eq = make_end(genome, layout, n5, n3, rng)
    ep["qoff"] += len(sq)
    gp["qoff"] += len(sq) + len(eq)
    q = np.concatenate([sq, eq, gq])
    op, oq = make_stage2(genome, layout, reads, np.random.default_rng(seed + 3), exons=shape.exons,
                         exlen=shape.exlen, pad=shape.pad, subs=shape.subs, indel=shape.indel,
                         extra=shape.stage2 - 1.0)
    mp = make_microexon(gp, int(round(reads * shape.microexon)), np.random.default_rng(seed + 4))
    out = {"single": sp_, "end": ep, "genome": gp, "q": q, "oligo": op, "oq": oq, "microexon": mp,
           "reads": reads}
    if sprob:
        out["sprob"] = sp
    else:
        out["sprob_len"], out["sprob_hi"] = sp
    return out


def plant_stream(genome, layout, reads, blocks, shape=CDNA2K):
    """Plant the intron sites of every block of the stream, in block order (every rank does the same,
    so every rank holds the same genome)."""
    for b in blocks:
        plant_sites(genome, genome_gap_sites(layout, int(round(reads * shape.genome)), block_seeds(b)[1]))


def _block_worker(args):
    genome, layout, reads, b, shape, sprob = _POOL_STATE[0], _POOL_STATE[1], args[0], args[1], args[2], args[3]
    seed, site_seed = block_seeds(b)
    return make_reads(genome, layout, reads, seed, site_seed=site_seed, shape=shape, plant=False, sprob=sprob)


_POOL_STATE = [None, None]


def make_blocks(genome, layout, reads, blocks, shape=CDNA2K, sprob=True, workers=1):
    """The call streams of `blocks` (the genome already planted by plant_stream), generated in
    `workers` forked processes (the genome is shared copy-on-write; call before any GPU work)."""
    _POOL_STATE[0], _POOL_STATE[1] = genome, layout
    jobs = [(reads, b, shape, sprob) for b in blocks]
    try:
        if workers <= 1 or len(blocks) <= 1:
            return [_block_worker(j) for j in jobs]
        import multiprocessing as mp
        with mp.get_context("fork").Pool(min(workers, len(blocks))) as pool:
            return pool.map(_block_worker, jobs)
    finally:
        _POOL_STATE[0] = _POOL_STATE[1] = None
