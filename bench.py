"""bench.py -- MI355X Dynprog engine throughput (BASELINE.json metric, configs[1]).

Workload (configs[1]: "100k synthetic 2-kb cDNA vs human chr22, 1xMI355X,
Dynprog_single + Dynprog_end only"): a chr22-length (50,818,468 nt) i.i.d.
genome (seed 22) packed in the reference's .genomecomp format and resident
in HBM, and the stream of sub-problems GMAP issues per 2-kb read (nosimd
instrumented counts): 43.7 Dynprog_single_gap calls (query
slices with 2 % substitutions and occasional 1-3 nt indels, extraband 6,
wide band) plus 7.1 Dynprog_end5_gap + 6.5 Dynprog_end3_gap calls (read ends
beyond the last anchor, glength = rlength + extramaterial_end 10, mixed
endalign).  One "step" = one pass of the engine over the sub-problems of
--reads reads; all inputs are in HBM before the timed region.

value = reads whose DP sub-problems were processed per second, whole job
(all ranks).  This is the DP-engine throughput of the path, not end-to-end
GMAP (stage 1/2/3 orchestration stays on the host; DESIGN.md "Measurement").

The same JSON line carries "all_dynprog": the same measurement with the
Dynprog_genome_gap calls added (49.4 per read; the configs[2]
DP mix without stage 2): query gaps spanning a planted GT-AG intron,
glength = rlength + extramaterial_paired (8), extraband_paired 14.  Their
MaxEnt splice probabilities are a host input to the engine (the caller's
Maxent_hr_*_prob values); the bench supplies synthetic ones (0.95 at the
planted sites, U[0, 0.3) elsewhere).
"""
import argparse
import ctypes as C
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))

CHR22_LEN = 50_818_468
SINGLE_PER_READ = 43.7         # Dynprog_single_gap calls per 2-kb read (nosimd)
END5_PER_READ = 7.1            # Dynprog_end5_gap
END3_PER_READ = 6.5            # Dynprog_end3_gap
GENOME_PER_READ = 49.4         # Dynprog_genome_gap
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
COMPL = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTN", b"TGCAN"):
    COMPL[_a] = _b
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def make_genome(seed=22, length=CHR22_LEN):
    rng = np.random.default_rng(seed)
    return ACGT[rng.integers(0, 4, size=length, dtype=np.uint8)]


def genomic_chars(genome, pos, watson):
    """get_genomic_nt with chroffset 0, chrhigh = len(genome), positions in range."""
    glen = len(genome)
    fwd = genome[np.where(watson, pos, 0)]
    rev = COMPL[genome[np.where(watson, 0, glen - pos)]]
    return np.where(watson, fwd, rev)


def make_single(genome, n, rng):
    """Vectorised GMAP-shaped Dynprog_single_gap sub-problems."""
    import gmapdp
    glen = len(genome)
    g = np.clip(rng.gamma(3.0, 40.0, size=n).astype(np.int64), 1, 640)
    d = np.where(rng.random(n) < 0.15, rng.integers(-3, 4, size=n), 0)
    d = np.where(g + d < 1, 0, d)
    r = np.clip(g + d, 1, 660)
    d = r - g
    watson = rng.random(n) < 0.5
    goff = rng.integers(1, glen - 700, size=n)
    seg_off = np.concatenate([[0], np.cumsum(g)])
    pid = np.repeat(np.arange(n), g)
    i = np.arange(seg_off[-1]) - seg_off[pid]
    seg = genomic_chars(genome, goff[pid] + i, watson[pid])
    # query = segment with one indel of |d| at position a, then 2 % substitutions
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
    probs["chroffset"] = 0
    probs["chrhigh"] = glen
    probs["flags"] = (watson.astype(np.int32) * gmapdp.WATSON | (rng.random(n) < 0.5) * gmapdp.JUMP_LATE |
                      gmapdp.WIDEBAND)
    probs["genestrand"] = 0
    probs["extraband"] = 6
    probs["defect_rate"] = np.where(rng.random(n) < 0.7, 0.02, 0.01)
    probs["dynprogindex"] = rng.integers(1, 50, size=n) * np.where(rng.random(n) < 0.5, 1, -1)
    return probs, q


def make_end(genome, n5, n3, rng):
    """Vectorised Dynprog_end5_gap / Dynprog_end3_gap sub-problems: the read end beyond the last
    anchor (lognormal length, median 60 nt), genome = rlength + extramaterial_end (10)."""
    import gmapdp
    glen = len(genome)
    n = n5 + n3
    end3 = np.zeros(n, dtype=bool)
    end3[n5:] = True
    L = np.clip(rng.lognormal(np.log(60.0), 1.2, size=n).astype(np.int64), 1, 800)
    g = L + 10
    watson = rng.random(n) < 0.5
    # end3: genomic positions goffset .. goffset+L-1; end5: rev_goffset-L+1 .. rev_goffset
    goff = np.where(end3, rng.integers(1, glen - 900, size=n), rng.integers(900, glen - 2, size=n))
    first = np.where(end3, goff, goff - L + 1)
    q_off = np.concatenate([[0], np.cumsum(L)])
    qpid = np.repeat(np.arange(n), L)
    j = np.arange(q_off[-1]) - q_off[qpid]
    q = genomic_chars(genome, first[qpid] + j, watson[qpid])
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
    probs["chroffset"] = 0
    probs["chrhigh"] = glen
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


def make_genome_gaps(genome, n, rng, site_seed=23):
    """Vectorised Dynprog_genome_gap sub-problems (stage3.c:9504-9539): a query gap of rlength
    nt = a exonic nt before a planted GT..AG intron + b after it; goffsetL = first genomic
    position after the left anchor, rev_goffsetR = last one before the right anchor,
    glengthL = glengthR = rlength + 8.  Plants the dinucleotides into `genome` (in place) at
    sites drawn from `site_seed`, so every rank builds the same genome; call it before the
    other sub-problems are cut from the genome."""
    import gmapdp
    glen = len(genome)
    srng = np.random.default_rng(site_seed)
    r = np.clip(srng.gamma(2.2, 50.0, size=n).astype(np.int64), 2, 600)
    a = (srng.random(n) * (r + 1)).astype(np.int64)
    b = r - a
    intron = srng.integers(60, 5000, size=n)
    watson = srng.random(n) < 0.5
    goffL = srng.integers(100, glen - 7000, size=n)
    revR = goffL + a + intron + b - 1
    x, y = goffL + a, revR - b            # first / last intron base, strand coordinates
    # strand coordinate p -> genome index: watson p, minus glen - p (complemented)
    def plant(pos, ch):
        idx = np.where(watson, pos, glen - pos)
        genome[idx] = np.where(watson, ord(ch), COMPL[ord(ch)])
    plant(x, "G"); plant(x + 1, "T"); plant(y - 1, "A"); plant(y, "G")
    q_off = np.concatenate([[0], np.cumsum(r)])
    qpid = np.repeat(np.arange(n), r)
    j = np.arange(q_off[-1]) - q_off[qpid]
    src = np.where(j < a[qpid], goffL[qpid] + j, revR[qpid] - b[qpid] + 1 + (j - a[qpid]))
    q = genomic_chars(genome, src, watson[qpid])
    q = np.where(rng.random(q.size) < 0.02, ACGT[rng.integers(0, 4, size=q.size, dtype=np.uint8)], q)
    gp = np.zeros(n, dtype=gmapdp.GENOME_PROBLEM_DTYPE)
    gp["qoff"] = q_off[:-1]
    gp["rlength"] = r
    gp["glengthL"] = r + 8
    gp["glengthR"] = r + 8
    gp["roffset"] = rng.integers(0, 1500, size=n)
    gp["goffsetL"] = goffL
    gp["rev_goffsetR"] = revR
    gp["chroffset"] = 0
    gp["chrhigh"] = glen
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


def make_workload(genome, reads, seed):
    rng = np.random.default_rng(seed)
    ns = int(round(reads * SINGLE_PER_READ))
    n5 = int(round(reads * END5_PER_READ))
    n3 = int(round(reads * END3_PER_READ))
    sp, sq = make_single(genome, ns, rng)
    ep, eq = make_end(genome, n5, n3, rng)
    ep["qoff"] += len(sq)  # one query arena: singles then ends
    return sp, ep, np.concatenate([sq, eq])


def algorithmic_bytes(rlength, glength, npairs, desc_bytes):
    """HBM bytes the path must move (DESIGN.md "Roofline"): problem descriptor + query and
    upper-cased query (2 x rlength) + packed genome blocks covering the segment (12 B per
    32 nt) + result (32 B) + one 16-B Pair record per emitted pair."""
    r = np.asarray(rlength, dtype=np.int64)
    g = np.asarray(glength, dtype=np.int64)
    return int((desc_bytes + 2 * r + 12 * ((g + 62) // 32) + 32).sum() + 16 * int(np.asarray(npairs).sum()))


def pmc_traffic(name):
    """HBM bytes per dispatch of kernel template `name` from the newest committed rocprofv3 PMC
    summary (profiles/*/pmc_summary.json: 2 x FETCH_SIZE + WRITE_SIZE of the same bench command,
    per MI355X_MICROARCH.md's gfx950 correction), or (None, None)."""
    import glob
    if name == "oi_kernel+oi_map_kernel":  # stage-2 seeding: the two kernels of one launch, summed
        # oi_kernel<unsigned short>: the 16-bit-counter build every bench window (< 65536 starts) takes
        for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary.json")), reverse=True):
            try:
                ks = json.load(open(path))["kernels"]
            except (OSError, ValueError, KeyError):
                continue
            a = ks.get("gmapdp::oi_kernel<unsigned short>") or ks.get("gmapdp::oi_kernel")
            b = ks.get("gmapdp::oi_map_kernel")
            if a and b:
                return a["hbm_bytes_per_dispatch"] + b["hbm_bytes_per_dispatch"], os.path.relpath(path, ROOT)
        return None, None
    m = re.match(r"(\w+)<R=(\d+),dirs_lds=(\d)>", name)
    if not m:
        return None, None
    if m.group(1) == "dpx_kernel":  # dpx_kernel<S, GD>: GD = direction words in global scratch
        key = "gmapdp::dpx_kernel<%s, %s>" % (m.group(2), "false" if m.group(3) == "1" else "true")
    else:
        key = "gmapdp::%s<%s, %s>" % (m.group(1), m.group(2), "true" if m.group(3) == "1" else "false")
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary.json")), reverse=True):
        try:
            k = json.load(open(path))["kernels"].get(key)
        except (OSError, ValueError, KeyError):
            continue
        if k:
            return k["hbm_bytes_per_dispatch"], os.path.relpath(path, ROOT)
    return None, None


def genome_algorithmic_bytes(gp, npairs):
    """Dynprog_genome_gap: descriptor (80 B) + query and upper-cased query (2 x rlength) + the
    packed genome blocks of both segments + 8-B splice probability per column of both
    segments + result (72 B) + one 16-B record per emitted pair."""
    r = gp["rlength"].astype(np.int64)
    gL = gp["glengthL"].astype(np.int64)
    gR = gp["glengthR"].astype(np.int64)
    return int((80 + 2 * r + 12 * ((gL + 62) // 32) + 12 * ((gR + 62) // 32) + 8 * (gL + gR) + 72).sum()
               + 16 * int(np.asarray(npairs).sum()))


def banded_cells(sp, ep):
    """Banded DP cells of the fills (wide band for single/GAP/BEST_LOCAL, narrow for INDELS)."""
    r = sp["rlength"].astype(np.int64)
    g = sp["glength"].astype(np.int64)
    cells = int(np.minimum(np.abs(g - r) + 2 * sp["extraband"].astype(np.int64) + 1, r + 1).dot(g))
    r = np.minimum(ep["rlength"].astype(np.int64), 660)
    g = np.minimum(ep["glength"].astype(np.int64), 2000)
    eb = ep["extraband"].astype(np.int64)
    W = np.where(ep["endalign"] == 1, 2 * eb + 1, np.abs(g - r) + 2 * eb + 1)
    W = np.where(ep["endalign"] == 2, 0, W)
    return cells + int(np.minimum(W, r + 1).dot(g))


def make_stage2(genome, n, rng, exons=5, exlen=400, pad=1000):
    """Stage-2 seeding calls, one per 2-kb read (SURVEY §8d read model): 5 exons x 400 nt cut from
    the genome with log-uniform [80, 20000] introns, 2 % substitutions, half reverse-complemented
    (seeded on the minus strand), against the window spanning the locus plus 1 kb each side (the
    gregion).  Returns (gmapdp_oligo_problem array, upper-case query arena)."""
    import gmapdp
    glen = len(genome)
    probs = np.zeros(n, dtype=gmapdp.OLIGO_PROBLEM_DTYPE)
    parts, off = [], 0
    for i in range(n):
        introns = np.exp(rng.uniform(np.log(80), np.log(20000), size=exons - 1)).astype(np.int64)
        span = exons * exlen + int(introns.sum())
        start = int(rng.integers(pad, glen - span - pad))
        segs, p = [], start
        for e in range(exons):
            segs.append(genome[p:p + exlen])
            p += exlen + (int(introns[e]) if e < exons - 1 else 0)
        q = np.concatenate(segs)
        m = rng.random(q.size) < 0.02
        q[m] = ACGT[rng.integers(0, 4, size=int(m.sum()))]
        plus = rng.random() < 0.5
        if not plus:
            q = COMPL[q[::-1]]
        probs[i] = (off, q.size, start - pad, start + span + pad, 0, glen, int(plus), 0)
        parts.append(q)
        off += q.size
    return probs, np.concatenate(parts)


def stage2_algorithmic_bytes(op, res):
    """Stage-2 seeding per call: descriptor (32 B) + the query (1 B/nt) + the window's packed genome
    (12 B per 32 nt) + npositions and mappings (8 B per query position) + the table (4 B per stored
    position) + the result (32 B) + the diagonal records (16 B each)."""
    w = (op["chrend"].astype(np.int64) - op["chrstart"].astype(np.int64))
    ql = op["querylength"].astype(np.int64)
    return int((32 + ql + 12 * ((w + 31) // 32) + 8 * ql + 32).sum()
               + 4 * int(res["totalpositions"].astype(np.int64).sum())
               + 16 * int(res["ndiagonals"].astype(np.int64).sum()))


def cpu_baseline_stage2(op, oq, genome, budget_s=8.0):
    """The reference's Oligoindex_hr_tally + Oligoindex_get_mappings (1 core, nosimd objects) on a
    bounded prefix of the same seeding calls."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "librefdp_nosimd.so")
    if not os.path.exists(ref_so):
        return None
    lib = C.CDLL(ref_so)
    lib.refh_init(0, 0, 0)
    gb = genome.tobytes()
    lib.refh_set_genome(gb, len(gb))
    f = lib.refh_oligo_mappings
    f.restype = C.c_int
    f.argtypes = [C.c_char_p, C.c_int, C.c_uint, C.c_uint, C.c_uint, C.c_uint, C.c_int, C.c_int, C.c_void_p,
                  C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
    cap = 1 << 21
    pos = np.zeros(cap, dtype=np.uint32)
    npos = np.zeros(int(op["querylength"].max()) + 1, dtype=np.int32)
    sc = np.zeros(4, dtype=np.int32)
    dg = np.zeros(4 * 65536, dtype=np.int32)
    qb = oq.tobytes()
    t, n = 0.0, 0
    while t < budget_s and n < len(op):
        p = op[n]
        o, ql = int(p["qoff"]), int(p["querylength"])
        t0 = time.perf_counter()
        f(qb[o:o + ql], ql, int(p["chrstart"]), int(p["chrend"]), int(p["chroffset"]), int(p["chrhigh"]),
          int(p["plusp"]), 0, npos.ctypes.data, pos.ctypes.data, cap, sc.ctypes.data, dg.ctypes.data, 65536)
        t += time.perf_counter() - t0
        n += 1
    return {"value": n / t, "unit": "reads/s", "cores": 1, "kind": "reference",
            "sample": "%d seeding calls of the same stream (%.1f s, 1 thread, gmap nosimd oligoindex_hr.o via "
                      "oracle/_ref refh_oligo_mappings)" % (n, t)}


def cpu_baseline(sp, ep, q, genome, budget_s=12.0):
    """Time the reference itself (oracle/_ref/librefdp_nosimd.so, 1 core) on a bounded prefix of
    the same per-read problem mix; None if the reference objects are absent."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "librefdp_nosimd.so")
    if not os.path.exists(ref_so):
        return None
    lib = C.CDLL(ref_so)
    lib.refh_init(0, 0, 0)
    gb = genome.tobytes()
    lib.refh_set_genome(gb, len(gb))
    for name in ("refh_single_gap_batch", "refh_end_gap_batch"):
        f = getattr(lib, name)
        f.restype = C.c_long
        f.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_char_p]
    qb = q.tobytes()
    per_read_s = SINGLE_PER_READ / (SINGLE_PER_READ + END5_PER_READ + END3_PER_READ)
    t_single = t_end = 0.0
    ns = ne = 0
    chunk = 256
    while t_single + t_end < budget_s and ns + chunk <= len(sp) and ne + chunk <= len(ep):
        a = np.ascontiguousarray(sp[ns:ns + chunk])
        t0 = time.perf_counter()
        lib.refh_single_gap_batch(a.ctypes.data, chunk, qb, qb)
        t_single += time.perf_counter() - t0
        ns += chunk
        m = max(1, int(round(chunk * (1 - per_read_s) / per_read_s)))
        m = min(m, len(ep) - ne)
        b = np.ascontiguousarray(ep[ne:ne + m])
        t0 = time.perf_counter()
        lib.refh_end_gap_batch(b.ctypes.data, m, qb, qb)
        t_end += time.perf_counter() - t0
        ne += m
        chunk = min(chunk * 2, 8192)
    sec_per_read = SINGLE_PER_READ * t_single / ns + (END5_PER_READ + END3_PER_READ) * t_end / ne
    return {"value": 1.0 / sec_per_read, "unit": "reads/s", "cores": 1, "kind": "reference",
            "sample": "%d Dynprog_single_gap + %d Dynprog_end{5,3}_gap problems of the same stream "
                      "(%.1f s, 1 thread, gmap nosimd objects via oracle/_ref), weighted %.1f + %.1f calls/read"
                      % (ns, ne, t_single + t_end, SINGLE_PER_READ, END5_PER_READ + END3_PER_READ)}


def cpu_baseline_genome(gp, q, genome, budget_s=8.0):
    """The reference's Dynprog_genome_gap (1 core) on a bounded prefix of the genome-gap stream;
    it computes its own MaxEnt probabilities (maxent_hr.c) inside the timed calls."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "librefdp_nosimd.so")
    if not os.path.exists(ref_so):
        return None
    lib = C.CDLL(ref_so)
    lib.refh_init(0, 0, 0)
    gb = genome.tobytes()
    lib.refh_set_genome(gb, len(gb))
    f = lib.refh_genome_gap_batch
    f.restype = C.c_long
    f.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_char_p]
    qb = q.tobytes()
    t, n, chunk = 0.0, 0, 256
    while t < budget_s and n + chunk <= len(gp):
        a = np.ascontiguousarray(gp[n:n + chunk])
        t0 = time.perf_counter()
        f(a.ctypes.data, chunk, qb, qb)
        t += time.perf_counter() - t0
        n += chunk
        chunk = min(chunk * 2, 8192)
    return t / max(n, 1), n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=10000, help="reads per step per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import gmapdp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    genome = make_genome()
    rng_g = np.random.default_rng(2000 + rank)
    ng = int(round(args.reads * GENOME_PER_READ))
    gp, gq, sprob = make_genome_gaps(genome, ng, rng_g)   # plants intron motifs into the genome first
    sp, ep, q = make_workload(genome, args.reads, seed=1000 + rank)
    ns, ne = len(sp), len(ep)
    nprob = ns + ne
    gp["qoff"] += len(q)
    q_all = np.concatenate([q, gq])
    if world > 1:
        # the genome is replicated per GPU (read-only); the reads are this rank's --part=rank/world
        # share (gmapdp.shard): weak scaling, no collective on the data path
        from gmapdp import shard
        shard.check_replicated(shard.genome_digest(genome), dist)

    eng = gmapdp.Engine(local)
    eng.set_genome(genome.tobytes())
    lib = eng.lib
    d_q = torch.from_numpy(q_all).to(dev)
    d_sprob = torch.from_numpy(sprob).to(dev)

    def build(with_genome):
        host_res = np.zeros(nprob, dtype=gmapdp.RESULT_DTYPE)
        host_gres = np.zeros(max(ng, 1), dtype=gmapdp.GENOME_RESULT_DTYPE)
        plan = C.c_void_p()
        eng._check(lib.gmapdp_plan_create_all(eng.h, sp.ctypes.data, ns, ep.ctypes.data, ne,
                                              gp.ctypes.data if with_genome else None, ng if with_genome else 0,
                                              host_res.ctypes.data, host_gres.ctypes.data, C.byref(plan)),
                   "gmapdp_plan_create_all")
        P = {"plan": plan, "ngpu": lib.gmapdp_plan_gpu_problems(plan),
             "nggpu": lib.gmapdp_plan_genome_gpu_problems(plan), "cap": lib.gmapdp_plan_pair_capacity(plan)}
        P["d_res"] = torch.zeros(max(P["ngpu"], 1) * 32, dtype=torch.uint8, device=dev)
        P["d_gres"] = torch.zeros(max(P["nggpu"], 1) * 72, dtype=torch.uint8, device=dev)
        P["d_pairs"] = torch.empty(max(P["cap"], 1) * 16, dtype=torch.uint8, device=dev)
        eng._check(lib.gmapdp_plan_bind_genome(plan, C.c_void_p(d_sprob.data_ptr()),
                                               C.c_void_p(P["d_gres"].data_ptr())), "gmapdp_plan_bind_genome")
        nl = lib.gmapdp_plan_nlaunches(plan)
        info = []
        for li in range(nl):
            R, dl, cnt, lds = C.c_int(), C.c_int(), C.c_int(), C.c_size_t()
            lib.gmapdp_plan_launch_info(plan, li, C.byref(R), C.byref(dl), C.byref(cnt), C.byref(lds))
            info.append((R.value, dl.value, cnt.value, lds.value))
        P["nl"], P["info"] = nl, info
        P["kind"] = [lib.gmapdp_plan_launch_kind(plan, li) for li in range(nl)]
        P["tail"] = [lib.gmapdp_plan_launch_is_tail(plan, li) == 1 for li in range(nl)]
        P["stream"] = [lib.gmapdp_plan_launch_stream(plan, li) for li in range(nl)]
        return P

    # Same issue order as gmapdp_plan_run: tail classes (long problems, latency-bound) on side
    # streams, the bulk on the main stream, joined at the end of the step.  Real (non-null)
    # streams, so the per-launch events on the main stream see exactly the bulk launches.
    stream = torch.cuda.Stream(dev)
    sides = [torch.cuda.Stream(dev) for _ in range(3)]

    def timed(P, steps, warmup):
        plan, nl, tail = P["plan"], P["nl"], P["tail"]

        def launch(li, s):
            eng._check(lib.gmapdp_plan_run_launch(eng.h, plan, li, C.c_void_p(d_q.data_ptr()),
                                                  C.c_void_p(d_q.data_ptr()), C.c_void_p(P["d_res"].data_ptr()),
                                                  C.c_void_p(P["d_pairs"].data_ptr()), C.c_void_p(s.cuda_stream)),
                       "gmapdp_plan_run_launch")

        def step(ev=None):
            # the engine's schedule (gmapdp_plan_run): launches in issue order, each on its assigned
            # stream (0 = main, 1..3 = sides) after a fork from the main stream, joined at the end;
            # per-dispatch events on the stream each launch runs on (what rocprofv3's kernel trace times)
            fork = torch.cuda.Event()
            fork.record(stream)
            used = set()
            for li in range(nl):
                k = P["stream"][li]
                s = stream if k == 0 else sides[k - 1]
                if k and k not in used:
                    s.wait_event(fork)
                    used.add(k)
                if ev is not None:
                    ev[li][0].record(s)
                launch(li, s)
                if ev is not None:
                    ev[li][1].record(s)
            for k in used:
                stream.wait_stream(sides[k - 1])

        with torch.cuda.stream(stream):
            for _ in range(warmup):
                step()
            torch.cuda.synchronize()
            evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nl)]
                   for _ in range(steps)]
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(steps):
                step(evs[k])
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            elapsed = time.perf_counter() - t0
        if world > 1:
            from gmapdp import shard
            elapsed = shard.max_over_ranks(elapsed, dist, device=dev)
        launch_ms = [sum(evs[k][li][0].elapsed_time(evs[k][li][1]) for k in range(steps)) / steps
                     for li in range(nl)]
        return elapsed, launch_ms

    # ---- headline: configs[1] (Dynprog_single_gap + Dynprog_end{5,3}_gap) ----
    P = build(False)
    plan, nl, info, tail, ngpu = P["plan"], P["nl"], P["info"], P["tail"], P["ngpu"]
    elapsed, launch_ms = timed(P, args.steps, args.warmup)
    rl = np.concatenate([sp["rlength"], np.minimum(ep["rlength"], 660)]).astype(np.int64)
    gl = np.concatenate([sp["glength"], np.minimum(ep["glength"], 2000)]).astype(np.int64)
    desc = np.concatenate([np.full(ns, 56), np.full(ne, 64)])

    def dispatches(PP, lms, steps):
        """(kernel template, algorithmic bytes, ms, count) of every timed dispatch of a plan."""
        plan_, info_ = PP["plan"], PP["info"]
        res_ = np.frombuffer(PP["d_res"].cpu().numpy().tobytes(), dtype=gmapdp.RESULT_DTYPE)[:PP["ngpu"]]
        gres_ = np.frombuffer(PP["d_gres"].cpu().numpy().tobytes(), dtype=gmapdp.GENOME_RESULT_DTYPE)[:PP["nggpu"]]
        dev_index = np.array([lib.gmapdp_plan_dev_index(plan_, i) for i in range(nprob)])
        npairs = np.zeros(nprob, dtype=np.int64)
        npairs[dev_index >= 0] = res_["npairs"][dev_index[dev_index >= 0]]
        out_ = []
        for li in range(PP["nl"]):
            m = np.zeros(info_[li][2], dtype=np.int32)
            lib.gmapdp_plan_launch_members(plan_, li, m.ctypes.data)
            if PP["kind"][li] in (0, 2):
                name = ("dp_kernel<R=%d,dirs_lds=%d>" if PP["kind"][li] == 0 else "dpx_kernel<R=%d,dirs_lds=%d>") \
                    % (info_[li][0], info_[li][1])
                nbytes = algorithmic_bytes(rl[m], gl[m], npairs[m], desc[m])
            else:
                name = "gg_kernel<R=%d,dirs_lds=%d>" % (info_[li][0], info_[li][1])
                j = m - nprob
                gi = np.array([lib.gmapdp_plan_genome_dev_index(plan_, int(x)) for x in j])
                nbytes = genome_algorithmic_bytes(gp[j], gres_["npairs"][gi])
            out_.append((name, nbytes, lms[li], steps, info_[li][2]))
        return out_

    disp = dispatches(P, launch_ms, args.steps)
    cells = banded_cells(sp, ep)
    step_bytes = sum(d[1] for d in disp)
    counts = {}
    for name, _, _, _, cnt in disp:
        counts[name] = counts.get(name, 0) + cnt
    dominant = max(counts, key=counts.get)   # the kernel template that processes the most problems
    lib.gmapdp_plan_destroy(plan)
    del P
    reads_total = args.reads * world * args.steps
    value = reads_total / elapsed
    out = {
        "metric": "aligned cDNA reads/sec (2 kb, GRCh38) at 1/2/4/8 MI355X; DP HBM GB/s vs peak",
        "value": value,
        "unit": "reads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": "configs[1]: synthetic 2-kb cDNA DP sub-problem stream vs a chr22-length i.i.d. "
                               "genome (seed 22): %.1f Dynprog_single_gap + %.1f Dynprog_end5_gap + %.1f "
                               "Dynprog_end3_gap calls per read; DP engine only (host stages 1-3 excluded)"
                               % (SINGLE_PER_READ, END5_PER_READ, END3_PER_READ),
                   "reads_per_step_per_gpu": args.reads, "subproblems_per_step_per_gpu": nprob,
                   "banded_cells_per_step_per_gpu": cells,
                   "parallelism": "dp%d (reads sharded by rank, genome replicated)" % world,
                   "launch_classes": info, "launch_ms": launch_ms},
        "gcups": cells * world * args.steps / elapsed / 1e9,
        "step_algorithmic_bytes": step_bytes,
    }

    # ---- all Dynprog_* paths: + Dynprog_genome_gap ----
    PA = build(True)
    gsteps = max(1, args.steps // 2)
    elapsed_all, launch_ms_all = timed(PA, gsteps, max(1, args.warmup // 2))
    disp_all = dispatches(PA, launch_ms_all, gsteps)
    gk = [li for li in range(PA["nl"]) if PA["kind"][li] == 1]

    def roofline(name, dl):
        """Average algorithmic bytes / average duration over every timed dispatch of one kernel
        template (both phases) -- the quantity rocprofv3 --stats averages per kernel name."""
        sel = [d for d in dl if d[0] == name]
        n = sum(d[3] for d in sel)
        ms = sum(d[2] * d[3] for d in sel) / n
        nbytes = sum(d[1] * d[3] for d in sel) / n
        ach = nbytes / (ms * 1e-3) / 1e9
        traffic, src = pmc_traffic(name)
        return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                "traffic": traffic, "traffic_source": src, "kernel": name, "dispatches": n,
                "kernel_ms_per_launch": ms,
                "algorithmic_bytes_per_launch": nbytes,
                "note": "integer VALU/LDS-bound DP; HBM roofline reported as required (DESIGN.md)"}

    out["roofline"] = roofline(dominant, disp + disp_all)
    gcount = {}
    for d in disp_all:
        if d[0].startswith("gg_"):
            gcount[d[0]] = gcount.get(d[0], 0) + d[4]
    gr = gp["rlength"].astype(np.int64)
    gcells = int((2 * np.minimum(8 + 2 * 14 + 1, gr + 1) * (gr + 8)).sum())  # two fills, band W = 37
    out["all_dynprog"] = {
        "value": args.reads * world * gsteps / elapsed_all, "unit": "reads/s",
        "ms_per_step": elapsed_all / gsteps * 1e3, "steps": gsteps,
        "genome_gap_calls_per_read": GENOME_PER_READ, "genome_gap_subproblems_per_step_per_gpu": ng,
        "gcups": (cells + gcells) * world * gsteps / elapsed_all / 1e9,
        "genome_gap_launch_classes": [PA["info"][li] for li in gk],
        "genome_gap_launch_ms": [launch_ms_all[li] for li in gk],
        "roofline_genome_gap": roofline(max(gcount, key=gcount.get), disp_all),
        "splice_probabilities": "synthetic host input (0.95 at planted GT-AG sites, U[0,0.3) elsewhere)"}
    lib.gmapdp_plan_destroy(PA["plan"])

    # ---- stage-2 seeding: Oligoindex_hr_tally + Oligoindex_get_mappings ----
    op, oq = make_stage2(genome, args.reads, np.random.default_rng(3000 + rank))
    oplan = C.c_void_p()
    eng._check(lib.gmapdp_oligo_plan_create(eng.h, op.ctypes.data, len(op), oq.ctypes.data, len(oq), C.byref(oplan)),
               "gmapdp_oligo_plan_create")
    pcap = lib.gmapdp_oligo_plan_positions_capacity(oplan)
    dcap = lib.gmapdp_oligo_plan_diagonal_capacity(oplan)
    d_oq = torch.from_numpy(oq).to(dev)
    d_ores = torch.zeros(len(op) * 32, dtype=torch.uint8, device=dev)
    d_onpos = torch.empty(len(oq) * 4, dtype=torch.uint8, device=dev)
    d_omap = torch.empty(len(oq) * 4, dtype=torch.uint8, device=dev)
    d_opos = torch.empty(max(pcap, 1) * 4, dtype=torch.uint8, device=dev)
    d_odiag = torch.empty(max(dcap, 1) * 16, dtype=torch.uint8, device=dev)

    def orun():
        eng._check(lib.gmapdp_oligo_plan_run(eng.h, oplan, C.c_void_p(d_oq.data_ptr()), C.c_void_p(d_ores.data_ptr()),
                                             C.c_void_p(d_onpos.data_ptr()), C.c_void_p(d_omap.data_ptr()),
                                             C.c_void_p(d_opos.data_ptr()), C.c_void_p(d_odiag.data_ptr()),
                                             C.c_void_p(stream.cuda_stream)), "gmapdp_oligo_plan_run")

    osteps = max(1, args.steps // 2)
    with torch.cuda.stream(stream):
        orun()
        torch.cuda.synchronize()
        oev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(osteps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(osteps):
            oev[k][0].record(stream)
            orun()
            oev[k][1].record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        oelapsed = time.perf_counter() - t0
    if world > 1:
        from gmapdp import shard
        oelapsed = shard.max_over_ranks(oelapsed, dist, device=dev)
    oms = sum(a.elapsed_time(b) for a, b in oev) / osteps
    ores = np.frombuffer(d_ores.cpu().numpy().tobytes(), dtype=gmapdp.OLIGO_RESULT_DTYPE)
    obytes = stage2_algorithmic_bytes(op, ores)
    otraffic, osrc = pmc_traffic("oi_kernel+oi_map_kernel")
    nol = lib.gmapdp_oligo_plan_nlaunches(oplan)
    out["stage2_seeding"] = {
        "value": args.reads * world * osteps / oelapsed, "unit": "reads/s", "ms_per_step": oelapsed / osteps * 1e3,
        "steps": osteps, "calls_per_read": 1, "window_nt_per_step_per_gpu": int((op["chrend"] - op["chrstart"]).sum()),
        "totalpositions_per_step_per_gpu": int(ores["totalpositions"].astype(np.int64).sum()),
        "diagonals_per_step_per_gpu": int(ores["ndiagonals"].astype(np.int64).sum()),
        "roofline": {"bound": "hbm", "achieved": obytes / (oms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": obytes / (oms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": otraffic, "traffic_source": osrc,
                     "kernel": "oi_kernel+oi_map_kernel", "dispatches": nol * osteps, "kernel_ms_per_launch": oms / max(nol, 1),
                     "algorithmic_bytes_per_launch": obytes / max(nol, 1),
                     "note": "per launch oi_kernel (LDS counting sort of the window's 8-mers, one wave per read) "
                             "+ oi_map_kernel (get_mappings as a diagonal radix sort and segmented scans); "
                             "latency-bound (DESIGN.md)"}}
    lib.gmapdp_oligo_plan_destroy(oplan)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["stage2_seeding"]["cpu_baseline"] = cpu_baseline_stage2(op, oq, genome)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sp, ep, q_all, genome)
        cg = cpu_baseline_genome(gp, q_all, genome)
        if out["cpu_baseline"] is not None and cg is not None:
            spr = 1.0 / out["cpu_baseline"]["value"] + GENOME_PER_READ * cg[0]
            out["all_dynprog"]["cpu_baseline"] = {
                "value": 1.0 / spr, "unit": "reads/s", "cores": 1, "kind": "reference",
                "sample": "headline sample + %d Dynprog_genome_gap problems of the same stream (reference "
                          "computes its own MaxEnt probabilities), weighted %.1f calls/read" % (cg[1], GENOME_PER_READ)}
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
