"""Phase breakdown of oi_kernel (stage-2 seeding) / gg_kernel (`gg`) on the bench workload (chr22 layout).

Loads the GMAPDP_OI_TIMING variant of the library (make -C gmap-2024_amd timing), runs one plan and
prints, per phase, the wave-summed wall-clock time as a share of the total.  Diagnostic only."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
sys.path.insert(0, ROOT)
import gmapdp  # noqa: E402
from gmapdp import workload as W  # noqa: E402

PHASES = ["set_inquery (bitmap, ids)", "pass 1 (counts) + layout", "pass 2 (store)", "npositions/mappings/cum",
          "event pool allocation", "events", "radix sort", "sweep + records"]


GG_PHASES = ["stage", "genome_gap_simple", "fills (L and R waves)", "bridge", "traceback R + reverse",
             "traceback L", "maxnegscore + result"]


def main_gg(reads=10000):
    """gg_kernel phases on bench.py's genome-gap stream (GENOME_PER_READ calls per read)."""
    import torch
    lib = gmapdp.load_library(os.path.join(ROOT, "gmap-2024_amd", "lib", "libgmapdp_oitiming.so"))
    lib.gmapdp_debug_gg_marks.argtypes = [C.c_void_p]
    layout = W.Layout(W.CHR22)
    genome = W.make_genome(layout, seed=22)
    ng = int(round(reads * W.GENOME_PER_READ))
    gp, gq, sprob = W.make_genome_gaps(genome, layout, ng, np.random.default_rng(2000))
    eng = gmapdp.Engine(0)
    eng.set_genome(genome.tobytes())
    qb = gq.tobytes()
    # (the device MaxEnt, as bench.py's step runs it: the staging evaluates the splice sites' models)
    sp = gmapdp.DEVICE if os.environ.get("GG_HOST_PROBS") is None else sprob
    eng.genome_gap_batch_raw(gp, qb, qb, sp)
    marks = np.zeros(32, dtype=np.uint64)
    lib.gmapdp_debug_gg_marks(marks.ctypes.data)
    eng.genome_gap_batch_raw(gp, qb, qb, sp)
    torch.cuda.synchronize()
    lib.gmapdp_debug_gg_marks(marks.ctypes.data)
    t, c = marks[:16].astype(np.float64), marks[16:]
    dur = [float(t[k + 1] - t[k]) for k in range(7)]
    tot = sum(dur)
    print(json.dumps({"blocks": [int(x) for x in c[:8]], "phases": {n: round(d / tot, 4) for n, d in zip(GG_PHASES, dur)},
                      "mean_block_us": tot / 1e2 / max(int(c[0]), 1)}))
    eng.close()


S2_PHASES = ["coverage", "Diag_compute_bounds", "hit arrays", "lookback sweep", "cells", "traceback + filter",
             "convert_to_nucleotides"]


def main_s2(reads=10000):
    """s2c_kernel (Stage2_compute chaining) phases on bench.py's stage-2 stream."""
    import torch
    lib = gmapdp.load_library(os.path.join(ROOT, "gmap-2024_amd", "lib", "libgmapdp_oitiming.so"))
    lib.gmapdp_debug_s2_marks.argtypes = [C.c_void_p]
    lib.gmapdp_debug_s2_waves.argtypes = [C.c_void_p]
    lib.gmapdp_debug_s2_sub.argtypes = [C.c_void_p]
    layout = W.Layout(W.CHR22)
    genome = W.make_genome(layout, seed=22)
    eng = gmapdp.Engine(0)
    eng.set_genome(genome.tobytes())
    sh = W.CDNA2K  # the bench's configs[2] read shape and stage-2 windows (gmap -d: locus +- ~100 kb)
    op, oq = W.make_stage2(genome, layout, reads, np.random.default_rng(3000), pad=sh.pad, extra=sh.stage2 - 1.0)
    calls = [dict(quc=oq[int(p["qoff"]):int(p["qoff"]) + int(p["querylength"])].tobytes(),
                  **{k: int(p[k]) for k in ("chrstart", "chrend", "chroffset", "chrhigh", "plusp")}) for p in op]
    probs, qb, qub = eng.build_stage2_batch(calls)
    eng.stage2_batch_raw(probs, qb, qub)
    marks = np.zeros(32, dtype=np.uint64)
    sub = np.zeros(16, dtype=np.uint64)
    lib.gmapdp_debug_s2_marks(marks.ctypes.data)
    lib.gmapdp_debug_s2_sub(sub.ctypes.data)
    res, _, _ = eng.stage2_batch_raw(probs, qb, qub)
    torch.cuda.synchronize()
    lib.gmapdp_debug_s2_marks(marks.ctypes.data)
    lib.gmapdp_debug_s2_sub(sub.ctypes.data)
    t, c = marks[:16].astype(np.float64), marks[16:]
    dur = [float(t[k + 1] - t[k]) for k in range(7)]
    tot = sum(dur)
    s2c = {n: round(float(t[b] - t[a]) / 1e2 / max(int(c[0]), 1), 1)
           for n, a, b in (("cells_us", 12, 5), ("traceback_filter_us", 5, 6), ("convert_us", 6, 7))}
    nw = max(int(c[5]), 1)  # s2c waves that reached the traceback (mark 5)
    s2c["npaths_per_wave"] = round(float(marks[29]) / nw, 2)
    s2c["link_table_us"] = round(float(marks[30] - t[5]) / 1e2 / nw, 1)
    cnt = {k: round(float(marks[i]) / 1e2 / max(int(c[0]), 1), 1)
           for k, i in (("sweep_meta_us", 8), ("sweep_one_us", 9), ("sweep_mult_us", 10), ("sweep_tail_us", 11))}
    wv = np.zeros((3, 16384), dtype=np.uint32)
    lib.gmapdp_debug_s2_waves(wv.ctypes.data)
    k = min(len(probs), 16384)
    us, npq, nh = wv[0, :k] / 1e2, wv[1, :k].astype(np.float64), wv[2, :k].astype(np.float64)
    sweep = {"p50_us": float(np.percentile(us, 50)), "p90_us": float(np.percentile(us, 90)),
             "p99_us": float(np.percentile(us, 99)), "max_us": float(us.max()), "mean_us": float(us.mean()),
             "mean_positions": float(npq.mean()), "mean_hits": float(nh.mean()), "max_hits": float(nh.max()),
             "corr_us_hits": float(np.corrcoef(us, nh)[0, 1]), "corr_us_positions": float(np.corrcoef(us, npq)[0, 1]),
             "per_wave_candidate_visits": float(marks[13]) / max(int(c[0]), 1),
             "per_wave_fast_windows": float(marks[14]) / max(int(c[0]), 1),
             "per_wave_slow_entry_evals": float(marks[15]) / max(int(c[0]), 1),
             "per_wave_multi_windows": float(marks[31]) / max(int(c[0]), 1),
             "per_wave_runs": float(marks[24]) / max(int(c[0]), 1),
             "per_wave_run_positions": float(marks[25]) / max(int(c[0]), 1),
             "per_wave_one_hit_positions": float(marks[26]) / max(int(c[0]), 1),
             "per_wave_multi_hit_positions": float(marks[27]) / max(int(c[0]), 1),
             "slowest": [[float(us[i]), int(npq[i]), int(nh[i])] for i in np.argsort(-us)[:8]]}
    print(json.dumps({"waves": [int(x) for x in c[:8]], "phases": {n: round(d / tot, 4) for n, d in zip(S2_PHASES, dur)},
                      "mean_wave_us": tot / 1e2 / max(int(c[0]), 1), "status": np.bincount(res["status"] + 3).tolist(),
                      "counts": cnt, "s2c_per_wave": s2c, "s2b_sweep_per_wave": sweep,
                      "s2_one_parts_us_per_wave": {n: round(float(sub[i]) / 1e2 / max(int(c[0]), 1), 1)
                                                   for i, n in enumerate(("adjacent", "prefetch", "fast_window",
                                                                          "multi_windows", "entry_tail"))},
                      "s2_one_parts_calls_per_wave": {n: round(float(sub[8 + i]) / max(int(c[0]), 1), 1)
                                                      for i, n in enumerate(("adjacent", "prefetch", "fast_window",
                                                                             "multi_windows", "entry_tail"))}}))
    eng.close()


def main():
    import torch
    if len(sys.argv) > 1 and sys.argv[1] == "gg":
        return main_gg()
    if len(sys.argv) > 1 and sys.argv[1] == "s2":
        return main_s2(int(sys.argv[2]) if len(sys.argv) > 2 else 10000)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    lib = gmapdp.load_library(os.path.join(ROOT, "gmap-2024_amd", "lib", "libgmapdp_oitiming.so"))
    lib.gmapdp_debug_oi_marks.argtypes = [C.c_void_p]
    layout = W.Layout(W.CHR22)
    genome = W.make_genome(layout, seed=22)
    eng = gmapdp.Engine(0)
    eng.set_genome(genome.tobytes())
    sh = W.CDNA2K
    op, oq = W.make_stage2(genome, layout, n, np.random.default_rng(3000), pad=sh.pad, extra=sh.stage2 - 1.0)
    # the seeding as Stage2_compute runs it (the host-array seeding API keeps its table below 2^31 entries)
    calls = [dict(quc=oq[int(p["qoff"]):int(p["qoff"]) + int(p["querylength"])].tobytes(),
                  **{k: int(p[k]) for k in ("chrstart", "chrend", "chroffset", "chrhigh", "plusp")}) for p in op]
    probs, qb, qub = eng.build_stage2_batch(calls)
    res = eng.stage2_batch_raw(probs, qb, qub)
    marks = np.zeros(32, dtype=np.uint64)
    lib.gmapdp_debug_oi_marks(marks.ctypes.data)  # clear (includes the first run's warm-up)
    res = eng.stage2_batch_raw(probs, qb, qub)
    torch.cuda.synchronize()
    lib.gmapdp_debug_oi_marks(marks.ctypes.data)
    t, c = marks[:16].astype(np.float64), marks[16:]
    if int(c[10]):  # the split kernels (oi_scan_kernel 10 -> 11; oi_build_kernel 12, 2, 3, 4, 5, 13, 14, 15)
        per = lambda a, b, w: round(float(t[b] - t[a]) / 1e2 / max(int(c[w]), 1), 1)  # noqa: E731
        print(json.dumps({"waves": {k: int(c[k]) for k in (10, 11, 12, 2, 3, 4, 5, 13, 14, 15)},
                          "us_per_wave": {"scan (set_inquery + pass 1)": per(10, 11, 10), "counts": per(12, 2, 12),
                                          "layout": per(2, 3, 2), "placement + write-out": per(3, 4, 3),
                                          "prelude": per(4, 5, 4), "slot counts": per(5, 13, 13),
                                          "emit candidates": per(13, 14, 14), "sort + sweep": per(14, 15, 15)}}))
        eng.close()
        return
    # oi_kernel: marks 0..4; oi_map_kernel: 8 (start), 9 (pool allocated), 5, 6, 7
    spans = [(0, 1), (1, 2), (2, 3), (3, 4), (8, 9), (9, 5), (5, 6), (6, 7)]
    out = {"waves": [int(c[k]) for k in (0, 1, 2, 3, 4, 8, 9, 5, 6, 7)]}
    dur = [float(t[b] - t[a]) for a, b in spans]
    tot = sum(dur)
    out["wave_ms_total"] = tot / 1e5
    out["phases"] = {name: round(d / tot, 4) for name, d in zip(PHASES, dur)}
    out["mean_wave_us"] = {"oi_kernel": sum(dur[:4]) / 1e2 / max(int(c[0]), 1),
                           "oi_map_kernel": sum(dur[4:]) / 1e2 / max(int(c[8]), 1)}
    if hasattr(lib, "gmapdp_debug_oi_waves"):  # per-call wave durations: the kernels' tails
        lib.gmapdp_debug_oi_waves.argtypes = [C.c_void_p]
        wv = np.zeros((3, 16384), dtype=np.uint32)
        lib.gmapdp_debug_oi_waves(wv.ctypes.data)
        m = min(len(probs), 16384)
        for name, row in (("oi_kernel", 0), ("oi_map_kernel", 1)):
            us = wv[row, :m] / 1e2
            top = np.argsort(-us)[:8]
            out["waves_" + name] = {"p50_us": float(np.percentile(us, 50)), "p99_us": float(np.percentile(us, 99)),
                                    "max_us": float(us.max()),
                                    "slowest": [[int(i), float(us[i]), int(wv[2, i])] for i in top]}
        E = wv[2, :m].astype(np.float64)
        out["events"] = {"p50": float(np.percentile(E, 50)), "p99": float(np.percentile(E, 99)), "max": float(E.max())}
    print(json.dumps(out))
    eng.close()
    del res


if __name__ == "__main__":
    main()
