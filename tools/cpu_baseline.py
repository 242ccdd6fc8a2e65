"""CPU baseline leg of bench.py (TEST/MEASUREMENT INFRASTRUCTURE: it loads the reference's own objects
from oracle/_ref, never the product library).

Times the reference GMAP 2024-02-22 path -- Stage2_compute (stage2.c:6325: seeding and chaining, as
gmap.c:1208 calls it) and Dynprog_single_gap / _end5_gap / _end3_gap / _genome_gap /
_microexon_int (with the reference's own MaxEnt) -- on the
host cores, one process per core, each on a bounded sample of the configs[2] per-read call stream
(gmapdp.workload, same generators and per-read mix as the GPU bench).  The reference's harness takes
an int genome length, so the CPU sample is cut from a chr22-length (50.8 Mnt) i.i.d. genome; the DP and
seeding costs depend on the sub-problem shapes, not on the genome size.  The reference computes its own
MaxEnt splice probabilities inside Dynprog_genome_gap (the GPU bench takes them as an input).

Run as a child process of bench.py (never forked from a process that has touched the GPU):
  python tools/cpu_baseline.py --build avx2 --cores 16 --budget 10
prints one JSON object.
"""
import argparse
import ctypes as C
import json
import multiprocessing as mp
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def ref_layout(arr):
    """a gmapdp problem array in the reference harness's struct layout (oracle/refharness.c: the same
    fields in the same order, 32-bit chroffset/chrhigh, C alignment)"""
    dt = np.dtype([(n, "<u4" if n in ("chroffset", "chrhigh") else arr.dtype.fields[n][0].str) for n in arr.dtype.names],
                  align=True)
    out = np.zeros(len(arr), dtype=dt)
    for n in arr.dtype.names:
        out[n] = arr[n]
    return out


def worker(args):
    wid, build, budget, reads, mix, config = args
    from gmapdp import workload as W
    shape = W.SHAPES[mix]
    layout = W.Layout(W.CHR22)
    genome = W.make_genome(layout, seed=22)
    d = W.make_reads(genome, layout, reads, seed=7000 + 17 * wid, shape=shape)
    lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "librefdp_%s.so" % build))
    lib.refh_init(0, 0, 0)
    lib.refh_set_genome(genome.tobytes(), len(genome))
    for name in ("refh_single_gap_batch", "refh_end_gap_batch", "refh_genome_gap_batch"):
        f = getattr(lib, name)
        f.restype = C.c_long
        f.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_char_p]
    fm = lib.refh_microexon_int
    fm.restype = C.c_int
    fm.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint, C.c_uint, C.c_int,
                   C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    msc = np.zeros(2, dtype=np.int32)
    mds = np.zeros(2, dtype=np.float64)
    fo = lib.refh_stage2_compute
    fo.restype = C.c_int
    fo.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_uint, C.c_uint, C.c_uint, C.c_uint, C.c_int, C.c_int, C.c_int,
                   C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int]
    qb = d["q"].tobytes()
    oq = d["oq"].tobytes()
    cap = 1 << 18
    pairs = np.zeros(cap * 32, dtype=np.uint8)  # RefPair records (oracle/refharness.c)
    paths = np.zeros(2 * 1024, dtype=np.int32)
    sc = np.zeros(8, dtype=np.int32)
    fams = [("single", lib.refh_single_gap_batch, ref_layout(d["single"]), shape.single),
            ("end", lib.refh_end_gap_batch, ref_layout(d["end"]), shape.end5 + shape.end3),
            ("genome", lib.refh_genome_gap_batch, ref_layout(d["genome"]), shape.genome)]
    if config == 1:  # configs[1]: Dynprog_single + Dynprog_end only
        fams = fams[:2]
    # The host MaxEnt work the GMAP drop-in does for a genome gap (gmapdp_genome_splice_sites: every
    # position of both sides but each side's last, the reference's own Maxent_hr_*_prob; none for the
    # calls the engine answers before reading them) -- the GPU bench takes these as device inputs.
    g = d["genome"]
    fm_b = lib.refh_maxent_batch
    fm_b.restype = None
    fm_b.argtypes = [C.c_void_p, C.c_void_p, C.c_uint, C.c_int, C.c_void_p]
    mx_models, mx_pos, mx_off = [], [], [0]
    for p in g:
        gl, gr, r = int(p["glengthL"]), int(p["glengthR"]), int(p["rlength"])
        if r > 1 and r <= 660 and 0 < gl <= 2000 and 0 < gr <= 2000:
            watson, sense = bool(int(p["flags"]) & 1), int(p["cdna_direction"]) > 0
            lo, ro, co, ch = int(p["goffsetL"]), int(p["rev_goffsetR"]), int(p["chroffset"]), int(p["chrhigh"])
            cl, cr = np.arange(gl - 1), np.arange(gr - 1)
            if watson:
                mx_pos += [co + lo + cl, co + ro - cr + 1]
                mx_models += [np.full(gl - 1, 0 if sense else 3), np.full(gr - 1, 1 if sense else 2)]
            else:
                mx_pos += [ch - lo - cl + 1, ch - ro + cr]
                mx_models += [np.full(gl - 1, 2 if sense else 1), np.full(gr - 1, 3 if sense else 0)]
            mx_off.append(mx_off[-1] + gl + gr - 2)
        else:
            mx_off.append(mx_off[-1])
    mx_models = np.ascontiguousarray(np.concatenate(mx_models).astype(np.int32)) if mx_models else np.zeros(1, np.int32)
    mx_pos = np.ascontiguousarray(np.concatenate(mx_pos).astype(np.uint32)) if mx_pos else np.zeros(1, np.uint32)
    mx_out = np.zeros(max(len(mx_pos), 1), dtype=np.float64)
    # every call's arguments sliced before its timed region (no Python slicing inside t0..t1)
    oligo_args = []
    for p in d["oligo"]:
        o, ql = int(p["qoff"]), int(p["querylength"])
        oligo_args.append((oq[o:o + ql], ql, int(p["chrstart"]), int(p["chrend"]), int(p["chroffset"]),
                           int(p["chrhigh"]), int(p["plusp"])))
    micro_args = []
    for m in d["microexon"]:
        mo, ml = int(m["qoff"]), int(m["rlength"])
        micro_args.append((qb[mo:mo + ml], ml, int(m["roffset"]), int(m["goffsetL"]), int(m["rev_goffsetR"]),
                           int(m["cdna_direction"]), int(m["chroffset"]), int(m["chrhigh"]), int(m["watsonp"]),
                           int(m["genestrand"]), int(m["dynprogindex"])))
    t = {k: 0.0 for k in ("single", "end", "genome", "oligo", "microexon", "host_maxent")}
    n = {k: 0 for k in t}
    t_start = time.perf_counter()
    # one read's worth of calls per round, so every family is sampled in proportion
    while time.perf_counter() - t_start < budget:
        for name, f, arr, per in fams:
            k = max(1, int(round(per)))
            i = n[name] % max(1, len(arr) - k)
            a = np.ascontiguousarray(arr[i:i + k])
            t0 = time.perf_counter()
            f(a.ctypes.data, k, qb, qb)
            t[name] += time.perf_counter() - t0
            if name == "genome":  # the same k calls' host MaxEnt, as the drop-in evaluates it
                a0, a1 = mx_off[i], mx_off[i + k]
                pm, pp, po = mx_models[a0:].ctypes.data, mx_pos[a0:].ctypes.data, mx_out.ctypes.data
                t0 = time.perf_counter()
                fm_b(pm, pp, 0, a1 - a0, po)
                t["host_maxent"] += time.perf_counter() - t0
                n["host_maxent"] += k
            n[name] += k
        if config == 1:
            continue
        qs, ql, c0, c1, co, ch, pl = oligo_args[n["oligo"] % len(oligo_args)]
        t0 = time.perf_counter()
        fo(qs, qs, ql, c0, c1, co, ch, pl, 1, 500000, sc.ctypes.data, paths.ctypes.data, 1024, pairs.ctypes.data, cap)
        t["oligo"] += time.perf_counter() - t0
        n["oligo"] += 1
        for _ in range(int(round(shape.microexon))):
            ma = micro_args[n["microexon"] % len(micro_args)]
            t0 = time.perf_counter()
            fm(ma[0], ma[0], *ma[1:], msc.ctypes.data, mds.ctypes.data, pairs.ctypes.data, cap)
            t["microexon"] += time.perf_counter() - t0
            n["microexon"] += 1
    per_call = {k: t[k] / max(n[k], 1) for k in t}
    sec_per_read = shape.single * per_call["single"] + (shape.end5 + shape.end3) * per_call["end"]
    if config != 1:
        sec_per_read += (shape.genome * per_call["genome"] + shape.stage2 * per_call["oligo"]
                         + shape.microexon * per_call["microexon"])
    return {"reads_per_s": 1.0 / sec_per_read, "calls": n, "seconds": t, "per_call_us":
            {k: v * 1e6 for k, v in per_call.items()},
            "host_maxent_reads_per_s": 1.0 / max(shape.genome * per_call["host_maxent"], 1e-12)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", default="avx2", choices=["avx2", "nosimd"])
    ap.add_argument("--cores", type=int, default=0, help="worker processes (0: the CPUs this process may use, <= 16)")
    ap.add_argument("--budget", type=float, default=10.0, help="seconds of timed calls per worker")
    ap.add_argument("--reads", type=int, default=200, help="reads generated per worker (the sample is cycled)")
    ap.add_argument("--mix", default="d", choices=["d", "appb"], help="per-read call mix (workload.SHAPES)")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2],
                    help="BASELINE configs index: 1 = Dynprog_single + Dynprog_end only; 2 = every family + stage 2")
    a = ap.parse_args()
    from gmapdp import workload as W
    shape = W.SHAPES[a.mix]
    so = os.path.join(ROOT, "oracle", "_ref", "librefdp_%s.so" % a.build)
    if not os.path.exists(so):
        print(json.dumps(None))
        return
    # at most 16 workers: the GPU box allots one MI355X job 16 host cores (os.cpu_count() there shows
    # the whole machine), and the GPU drop-in is measured on the same 16
    host_cpus = len(os.sched_getaffinity(0))
    cores = a.cores or min(16, host_cpus)
    with mp.get_context("fork").Pool(cores) as pool:
        res = pool.map(worker, [(w, a.build, a.budget, a.reads, a.mix, a.config) for w in range(cores)])
    genome_per_read = shape.genome
    total = sum(r["reads_per_s"] for r in res)
    maxent_total = sum(r["host_maxent_reads_per_s"] for r in res)
    calls = {k: sum(r["calls"][k] for r in res) for k in res[0]["calls"]}
    per_call = {k: float(np.mean([r["per_call_us"][k] for r in res])) for k in res[0]["per_call_us"]}
    print(json.dumps({
        "value": total, "unit": "reads/s", "cores": cores, "kind": "reference",
        "build": "gmap.%s objects (oracle/_ref/librefdp_%s.so)" % (a.build, a.build),
        "cpu_model": cpu_model(), "host_cpus_visible": host_cpus, "os_cpu_count": os.cpu_count(),
        "per_core_reads_per_s": total / cores, "per_call_us": per_call,
        "host_maxent": None if a.config == 1 else {"reads_per_s": maxent_total, "per_read_us": per_call["host_maxent"] * genome_per_read,
                        "note": "the drop-in's host MaxEnt (every splice-site position of every genome gap the engine "
                                "fills, reference Maxent_hr_*_prob) on the same cores: the ceiling it puts on a "
                                "pipeline that feeds the GPU bench's calls from host probabilities"},
        "sample": ("%d worker processes x %.0f s of timed reference calls (%s) on the configs[1] per-read mix "
                   "(%s: %.1f single + %.1f end calls per read, Dynprog_single + Dynprog_end only) cut from a chr22 "
                   "i.i.d. genome; per-read time composed from per-call averages"
                   % (cores, a.budget, ", ".join("%d %s" % (v, k) for k, v in calls.items() if v), shape.source,
                      shape.single, shape.end5 + shape.end3)) if a.config == 1 else
                  ("%d worker processes x %.0f s of timed reference calls (%s) on the configs[2] per-read mix "
                   "(%s: %.3g Stage2_compute calls over locus +- %d-nt windows + %.1f single + %.1f end + %.1f "
                   "genome-gap + %.1f microexon calls per read) cut from a chr22-length i.i.d. genome; per-read time "
                   "composed from per-call averages"
                   % (cores, a.budget, ", ".join("%d %s" % (v, k) for k, v in calls.items()), shape.source,
                      shape.stage2, shape.pad, shape.single, shape.end5 + shape.end3, shape.genome,
                      shape.microexon))}))


if __name__ == "__main__":
    main()
