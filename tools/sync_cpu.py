"""Host CPU time per synchronous batch call, by context flags (diagnostic: does the waiting thread spin?).
    python tools/sync_cpu.py"""
import json
import os
import resource
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
import gmapdp  # noqa: E402
from gmapdp import workload as W  # noqa: E402


def cpu():
    r = resource.getrusage(resource.RUSAGE_THREAD)
    return r.ru_utime + r.ru_stime


def main():
    layout = W.Layout(W.CHR22)
    g = W.PackedGenome(layout.total, seed=22)
    rng = np.random.default_rng(5)
    sp, sq = W.make_single(g, layout, 64, rng)
    gp, gq, gprob = W.make_genome_gaps(g, layout, 64, rng)
    out = {}
    for name, flags in (("default", 0), ("one_stream", gmapdp.CTX_ONE_STREAM),
                        ("blocking", gmapdp.CTX_ONE_STREAM | gmapdp.CTX_BLOCKING_SYNC)):
        eng = gmapdp.Engine(0, flags=flags)
        eng.set_genome(blocks=g.blocks, length=g.length)
        sqb, gqb = sq.tobytes(), gq.tobytes()
        for what, fn in (("single64", lambda: eng.single_gap_batch_raw(sp, sqb, sqb)),
                         ("genome64", lambda: eng.genome_gap_batch_raw(gp, gqb, gqb, gprob))):
            fn()
            n = 200
            c0, t0 = cpu(), time.perf_counter()
            for _ in range(n):
                fn()
            c1, t1 = cpu(), time.perf_counter()
            out["%s_%s" % (name, what)] = {"wall_us": (t1 - t0) / n * 1e6, "cpu_us": (c1 - c0) / n * 1e6}
            print(json.dumps(out), file=sys.stderr, flush=True)
        eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
