"""Diagnostic (GPU box): the slowest Stage2_compute sweeps (s2b waves) of one bench block.  Loads the
GMAPDP_OI_TIMING build (make -C gmap-2024_amd timing), generates bench.py's configs[2] block `b` (GRCh38
layout), runs gmapdp_stage2_batch over it and prints, for the slowest waves, the call's sweep time,
query positions, seeding hits and window, plus the block's time distribution.  Writes the slow calls'
problems (npz) so they can be studied on the CPU with the oracle.

    python tools/s2_slow.py [block] [out.npz]"""
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
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    out = sys.argv[2] if len(sys.argv) > 2 else None
    lib = gmapdp.load_library(os.path.join(ROOT, "gmap-2024_amd", "lib", "libgmapdp_oitiming.so"))
    lib.gmapdp_debug_s2_waves.argtypes = [C.c_void_p]
    lib.gmapdp_debug_s2_marks.argtypes = [C.c_void_p]
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
    eng.stage2_batch_raw(s2p, q, q)
    marks = np.zeros(32, dtype=np.uint64)
    lib.gmapdp_debug_s2_marks(marks.ctypes.data)
    wv0 = np.zeros((3, 16384), dtype=np.uint32)
    lib.gmapdp_debug_s2_waves(wv0.ctypes.data)
    res, _, _ = eng.stage2_batch_raw(s2p, q, q)
    wv = np.zeros((3, 16384), dtype=np.uint32)
    lib.gmapdp_debug_s2_waves(wv.ctypes.data)
    n = len(s2p)  # (g_s2_wave is indexed by call)
    us = wv[0, :n] / 1e2
    order_t = wv[2, :n]
    slow = np.argsort(-us)[:24]
    print(json.dumps({"block": b, "calls": n, "sweep_us": {"mean": float(us.mean()), "p50": float(np.percentile(us, 50)),
                                                            "p99": float(np.percentile(us, 99)), "max": float(us.max()),
                                                            "sum_ms": float(us.sum() / 1e3)},
                      "slowest_waves": [[int(i), float(us[i]), int(wv[1, i]), int(order_t[i])] for i in slow]}))
    if out:
        np.savez(out, probs=s2p, q=d["oq"], us=us, positions=wv[1, :n], hits=order_t)
    eng.close()


if __name__ == "__main__":
    main()
