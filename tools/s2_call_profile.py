"""Diagnostic (GPU box): where one Stage2_compute sweep spends its time.  Loads the GMAPDP_OI_TIMING
build (make -C gmap-2024_amd timing), rebuilds bench.py's configs[2] block `b` and runs the listed calls
one at a time (each a one-call batch), printing per call the sweep's wall-clock split (metadata, one-hit
positions, several-hit positions, tail), s2_one's parts, the s2_mult time with the hits it handled, and
the s2_eval chunk counts (all / outside the LDS ring).

    python tools/s2_call_profile.py block call [call ...]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
import gmapdp  # noqa: E402
from gmapdp import workload as W  # noqa: E402


def main():
    b = int(sys.argv[1])
    calls = [int(x) for x in sys.argv[2:]]
    lib = gmapdp.load_library(os.path.join(ROOT, "gmap-2024_amd", "lib", "libgmapdp_oitiming.so"))
    for f in ("gmapdp_debug_s2_waves", "gmapdp_debug_s2_marks", "gmapdp_debug_s2_sub"):
        getattr(lib, f).argtypes = [C.c_void_p]
    lay = W.Layout(W.GRCH38)
    genome = W.PackedGenome(lay.total, seed=38)
    W.plant_stream(genome, lay, 10000, range(8), W.CDNA2K)
    d = W.make_blocks(genome, lay, 10000, [b], shape=W.CDNA2K, sprob=False)[0]
    op = d["oligo"]
    s2p = np.zeros(len(op), dtype=gmapdp.STAGE2_PROBLEM_DTYPE)
    for k in ("qoff", "querylength", "chrstart", "chrend", "chroffset", "chrhigh", "plusp"):
        s2p[k] = op[k]
    s2p["splicingp"] = 1
    s2p["maxintronlen"] = 500000
    q = d["oq"].tobytes()
    eng = gmapdp.Engine(0)
    eng.set_genome(blocks=genome.blocks, length=genome.length)
    marks = np.zeros(32, dtype=np.uint64)
    sub = np.zeros(16, dtype=np.uint64)
    wv = np.zeros((3, 16384), dtype=np.uint32)
    for c in calls:
        one = s2p[c:c + 1].copy()
        for rep in range(2):  # the first run warms the code and the tables
            lib.gmapdp_debug_s2_marks(marks.ctypes.data)
            lib.gmapdp_debug_s2_sub(sub.ctypes.data)
            res, _, _ = eng.stage2_batch_raw(one, q, q)
            lib.gmapdp_debug_s2_marks(marks.ctypes.data)
            lib.gmapdp_debug_s2_sub(sub.ctypes.data)
            lib.gmapdp_debug_s2_waves(wv.ctypes.data)
        m0 = marks[:16] / 100.0  # wall-clock ticks (100 MHz) -> us
        s0 = sub[:8].astype(np.float64)
        s1 = sub[8:].astype(np.int64)
        print(json.dumps({
            "call": c, "sweep_us": float(wv[0, 0] / 1e2), "positions": int(wv[1, 0]), "hits": int(wv[2, 0]),
            "us": {"meta": m0[8], "one": m0[9], "mult": m0[10], "tail": m0[11]},
            "counts": {"cand": int(marks[13]), "fast": int(marks[14]), "slow": int(marks[15]),
                       "multi": int(marks[16 + 15]), "runs": int(marks[16 + 8]), "runpos": int(marks[16 + 9]),
                       "onepos": int(marks[16 + 10]), "multpos": int(marks[16 + 11])},
            "s2_one_us": [float(x / 100.0) for x in s0[:5]], "s2_one_n": [int(x) for x in s1[:5]],
            "tail_or_s2_mult_us": float(s0[5] / 100.0), "tail_or_s2_mult_n": int(s1[5]),
            "multi_pos_pre_us": float(s0[6] / 100.0), "multi_pos_n": int(s1[6]),
            "multi_hit_dloop_us": float(s0[7] / 100.0), "multi_hit_n": int(s1[7]),
            "status": int(res["status"][0]) if "status" in res.dtype.names else None}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
