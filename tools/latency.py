"""Round-trip latency of the synchronous batch entry points (what the drop-in shim pays per batch):
host arrays in, host arrays out, for batches of k calls drawn from bench.py's streams.  Measurement
tool, run on the GPU box:

    python tools/latency.py [reps]

Prints one JSON line: microseconds per batch for each entry point and batch size.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
import gmapdp  # noqa: E402
from gmapdp import workload as W  # noqa: E402


def _time(fn, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    layout = W.Layout(W.CHR22)
    genome = W.make_genome(layout, seed=22)
    eng = gmapdp.Engine(0)
    eng.set_genome(genome.tobytes())
    rng = np.random.default_rng(5)
    sp, sq = W.make_single(genome, layout, 256, rng)
    gp, gq, gprob = W.make_genome_gaps(genome, layout, 256, rng)
    # Stage2_compute over the windows `gmap -d` gives it (the read's locus +- ~100 kb, workload.CDNA2K)
    op, oq = W.make_stage2(genome, layout, 64, rng, pad=W.CDNA2K.pad)
    s2calls = [dict(quc=oq[int(p["qoff"]):int(p["qoff"]) + int(p["querylength"])].tobytes(),
                    **{k: int(p[k]) for k in ("chrstart", "chrend", "chroffset", "chrhigh", "plusp")}) for p in op]
    out = {"reps": reps, "us_per_batch": {}}
    sqb, gqb = sq.tobytes(), gq.tobytes()
    for k in (1, 8, 16, 64):
        out["us_per_batch"]["single_gap_%d" % k] = _time(lambda: eng.single_gap_batch_raw(sp[:k], sqb, sqb), reps)
        out["us_per_batch"]["genome_gap_%d" % k] = _time(lambda: eng.genome_gap_batch_raw(gp[:k], gqb, gqb, gprob),
                                                         reps)
        probs, qb, qub = eng.build_stage2_batch(s2calls[:k])
        out["us_per_batch"]["stage2_compute_%d" % k] = _time(lambda: eng.stage2_batch_raw(probs, qb, qub),
                                                             max(reps // 10, 5))
        print(json.dumps(out), file=sys.stderr, flush=True)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
