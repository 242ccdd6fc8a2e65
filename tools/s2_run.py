"""Runs gmapdp_stage2_batch twice on bench.py's Stage2_compute calls (chr22 layout, the configs[2] read
shape and `gmap -d` windows, locus +- ~100 kb: workload.CDNA2K; `appb` as a second argument: App. B's
locus +- 1 kb); the driver for rocprofv3 passes over the stage-2 kernels alone (tools/profile_s2.sh).
Prints the second run's wall time."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
import gmapdp  # noqa: E402
from gmapdp import workload as W  # noqa: E402


def main(reads=10000, mix="d"):
    layout = W.Layout(W.CHR22)
    genome = W.make_genome(layout, seed=22)
    eng = gmapdp.Engine(0)
    eng.set_genome(genome.tobytes())
    if mix == "appb":
        op, oq = W.make_stage2(genome, layout, reads, np.random.default_rng(3000))
    else:
        sh = W.CDNA2K
        op, oq = W.make_stage2(genome, layout, reads, np.random.default_rng(3000), pad=sh.pad, extra=sh.stage2 - 1.0)
    calls = [dict(quc=oq[int(p["qoff"]):int(p["qoff"]) + int(p["querylength"])].tobytes(),
                  **{k: int(p[k]) for k in ("chrstart", "chrend", "chroffset", "chrhigh", "plusp")}) for p in op]
    probs, qb, qub = eng.build_stage2_batch(calls)
    eng.stage2_batch_raw(probs, qb, qub)
    t0 = time.perf_counter()
    res, paths, pairs = eng.stage2_batch_raw(probs, qb, qub)
    print("stage2 batch of %d: %.1f ms, %d results, %d pairs" % (reads, (time.perf_counter() - t0) * 1e3,
                                                                 int(res["nresults"].sum()), len(pairs)))
    eng.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10000, sys.argv[2] if len(sys.argv) > 2 else "d")
