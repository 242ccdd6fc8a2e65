#!/usr/bin/env python3
"""How much do the SIMD builds' Dynprog fills depend on what their arenas held before the call?

The reference's Dynprog_T arenas (dynprog.c:686-731) are posix_memalign'd once per worker and never cleared,
and the SIMD fills read cells outside the block they compute (e.g. dynprog_simd.c:3290, matrix[c-1][rlo-1]).
The engine, the oracle and the goldens define those cells as zero (tests/dpbind.py Ref._before_call zeroes the
reference arenas before every call).  This tool runs the S goldens' problems through the reference's own AVX2
objects the way gmap.avx2 runs them and counts the outputs that differ from the goldens:

  stale       one process, golden order, arenas never cleared (what a gmap.avx2 worker does);
  poison:B    every call on arenas filled with byte B (scores and directions);
  random      every call on arenas filled with a fresh random byte (seeded).

Each (golden, mode) runs in a child process: a fill that walks a poisoned direction can abort ("Bad dir",
dynprog_simd.c:9278), which is recorded as such.  Test infrastructure: loads only oracle/_ref (the reference
compiled here) and the committed goldens.

  python3 tools/stale_arena.py [--modes stale,poison:127,...] [--json out.json]
"""
import argparse
import json
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDENS = ("simd_single_gap_golden.npz", "simd_end_gap_golden.npz", "simd_genome_gap_golden.npz",
           "simd_cdna_gap_golden.npz")
MODES = ("stale", "poison:0", "poison:127", "poison:128", "poison:255", "poison:85", "random")


def load_golden(name):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load(os.path.join(ROOT, "tests", "golden", name))


def child(name, mode):
    from dpbind import Ref, call_end, call_single
    g, probs, outs = load_golden(name)
    exp = outs["ref_avx2"]
    rng = random.Random(4242)

    def before(self):
        if mode == "stale":
            return
        b = rng.randrange(256) if mode == "random" else int(mode.split(":")[1])
        self.lib.refh_poison_arenas(b, 3)

    Ref._before_call = before
    refs = {}

    def ref_for(p):
        # the genome-gap golden's halfp problems come from the --enable-alloca AVX2 build (make_golden.py)
        v = "avx2a" if name.startswith("simd_genome") and p["flags"] & 8 else "avx2"
        if v not in refs:
            refs[v] = Ref(v)
            refs[v].set_genome(g)
        return refs[v]

    if "single" in name:
        call = lambda p: call_single(ref_for(p), p)  # noqa: E731
    elif "end" in name:
        call = lambda p: call_end(ref_for(p), p)  # noqa: E731
    elif "genome" in name:
        call = lambda p: ref_for(p).genome_gap(p)  # noqa: E731
    else:
        call = lambda p: ref_for(p).cdna_gap(p)  # noqa: E731
    diff = []
    for i, p in enumerate(probs):
        if call(p) != exp[i]:
            diff.append(i)
    print(json.dumps({"golden": name, "mode": mode, "problems": len(probs), "differ": len(diff),
                      "first": diff[:20]}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default=",".join(MODES))
    ap.add_argument("--goldens", default=",".join(GOLDENS))
    ap.add_argument("--json", default=None)
    ap.add_argument("--child", nargs=2, default=None)
    a = ap.parse_args()
    if a.child:
        return child(*a.child)
    rows = []
    for name in a.goldens.split(","):
        for mode in a.modes.split(","):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", name, mode],
                               capture_output=True, text=True, timeout=1800)
            if r.returncode == 0:
                rows.append(json.loads(r.stdout.strip().splitlines()[-1]))
            else:
                rows.append({"golden": name, "mode": mode, "aborted": r.returncode,
                             "stderr": r.stderr.strip().splitlines()[-3:]})
            print(json.dumps(rows[-1]), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": rows, "note": __doc__.split("\n\n")[1]}, f, indent=1)


if __name__ == "__main__":
    main()
