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
"""
import numpy as np

# GRCh38 primary assembly chromosome lengths (chr1..chr22, chrX, chrY)
GRCH38 = [("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555),
          ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636),
          ("chr9", 138394717), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
          ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
          ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
          ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415)]
CHR22 = [("chr22", 50818468)]

SINGLE_PER_READ = 43.7         # Dynprog_single_gap calls per 2-kb read (nosimd)
END5_PER_READ = 7.1            # Dynprog_end5_gap
END3_PER_READ = 6.5            # Dynprog_end3_gap
GENOME_PER_READ = 49.4         # Dynprog_genome_gap
STAGE2_PER_READ = 1            # Stage2_compute seeding calls
MICROEXON_PER_READ = 25.6      # Dynprog_microexon_int

COMPL = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTN", b"TGCAN"):
    COMPL[_a] = _b
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


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


def make_single(genome, layout, n, rng):
    """Dynprog_single_gap sub-problems (stage3.c:9081): query slices with 2 % substitutions and
    occasional 1-3 nt indels, extraband 6, wide band."""
    import gmapdp
    g = np.clip(rng.gamma(3.0, 40.0, size=n).astype(np.int64), 1, 640)
    d = np.where(rng.random(n) < 0.15, rng.integers(-3, 4, size=n), 0)
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


def make_genome_gaps(genome, layout, n, rng, site_seed=23):
    """Dynprog_genome_gap sub-problems (stage3.c:9504-9539): a query gap of rlength nt = a exonic nt
    before a planted GT..AG intron + b after it; goffsetL = first genomic position after the left
    anchor, rev_goffsetR = last one before the right anchor, glengthL = glengthR = rlength + 8
    (extramaterial_paired), extraband_paired 14.  Plants the dinucleotides into `genome` (in place)
    at sites drawn from `site_seed`, so every rank builds the same genome; call it before the other
    sub-problems are cut from the genome.  Splice probabilities are synthetic host inputs (0.95 at
    the planted sites, U[0, 0.3) elsewhere)."""
    import gmapdp
    srng = np.random.default_rng(site_seed)
    r = np.clip(srng.gamma(2.2, 50.0, size=n).astype(np.int64), 2, 600)
    a = (srng.random(n) * (r + 1)).astype(np.int64)
    b = r - a
    intron = srng.integers(60, 5000, size=n)
    watson = srng.random(n) < 0.5
    choff, chrhigh, clen = layout.sample(srng, n, 8000)
    goffL = (srng.random(n) * (clen - 7200)).astype(np.int64) + 100
    revR = goffL + a + intron + b - 1
    x, y = goffL + a, revR - b            # first / last intron base, strand coordinates

    def plant(pos, ch):
        idx = np.where(watson, choff + pos, chrhigh - pos)
        genome[idx] = np.where(watson, ord(ch), COMPL[ord(ch)])
    plant(x, "G"); plant(x + 1, "T"); plant(y - 1, "A"); plant(y, "G")
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
    sprob = rng.random(int(p_off[-1])) * 0.3
    sprob[p_off[:-1] + a] = 0.95                 # left site (cL = a)
    sprob[p_off[:-1] + (r + 8) + b] = 0.95       # right site (cR = b)
    return gp, q.astype(np.uint8), sprob


def make_stage2(genome, layout, n, rng, exons=5, exlen=400, pad=1000):
    """Stage-2 seeding calls, one per 2-kb read: 5 exons x 400 nt cut from the genome with
    log-uniform [80, 20000] introns, 2 % substitutions, half reverse-complemented (seeded on the
    minus strand), against the window spanning the locus plus 1 kb each side (the gregion).
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
    q = genome[src]                                                   # (n, 2000)
    m = rng.random(q.shape) < 0.02
    q = np.where(m, ACGT[rng.integers(0, 4, size=q.shape, dtype=np.uint8)], q)
    plus = rng.random(n) < 0.5
    q = np.where(plus[:, None], q, COMPL[q[:, ::-1]]).astype(np.uint8)
    probs = np.zeros(n, dtype=gmapdp.OLIGO_PROBLEM_DTYPE)
    probs["qoff"] = np.arange(n) * q.shape[1]
    probs["querylength"] = q.shape[1]
    probs["chrstart"] = start - pad
    probs["chrend"] = start + span + pad
    probs["chroffset"] = choff
    probs["chrhigh"] = chrhigh
    probs["plusp"] = plus
    probs["minor"] = 0
    return probs, q.reshape(-1)


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


def make_reads(genome, layout, reads, seed, site_seed=23):
    """The per-read call stream of `reads` reads: dict of descriptor arrays and arenas.  Genome gaps
    plant their intron motifs first (in place), then every other sub-problem is cut."""
    rng = np.random.default_rng(seed)
    ng = int(round(reads * GENOME_PER_READ))
    # intron sites are rank-independent (site_seed), so every rank plants the same genome
    gp, gq, sprob = make_genome_gaps(genome, layout, ng, np.random.default_rng(seed + 1), site_seed=site_seed)
    ns = int(round(reads * SINGLE_PER_READ))
    n5 = int(round(reads * END5_PER_READ))
    n3 = int(round(reads * END3_PER_READ))
    sp, sq = make_single(genome, layout, ns, rng)
    ep, eq = make_end(genome, layout, n5, n3, rng)
    ep["qoff"] += len(sq)
    gp["qoff"] += len(sq) + len(eq)
    q = np.concatenate([sq, eq, gq])
    op, oq = make_stage2(genome, layout, reads, np.random.default_rng(seed + 3))
    mp = make_microexon(gp, int(round(reads * MICROEXON_PER_READ)), np.random.default_rng(seed + 4))
    return {"single": sp, "end": ep, "genome": gp, "q": q, "sprob": sprob, "oligo": op, "oq": oq,
            "microexon": mp, "reads": reads}
