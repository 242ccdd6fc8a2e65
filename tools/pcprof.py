"""Resolve tools/pcprof.c's samples to functions (measurement tool, run where the programs were built or
on the GPU box beside them):

    python tools/pcprof.py pcprof_gmap_gpu_prof_nosimd.txt [--top 40] [--json out.json]

Each sample is a program counter and a thread role; the owning mapping in the dumped /proc/self/maps gives
the file and its offset, `nm` (the symbol table, or the dynamic one for stripped libraries) the function.
The table lists samples per function and role, as a share of all samples (CPU time).
"""
import argparse
import bisect
import collections
import json
import os
import subprocess

ROLES = ("gmap", "fibers", "dispatch", "other")


def load(path):
    maps, pcs = [], []
    for line in open(path):
        if line.startswith("M "):
            f = line[2:].split()
            lo, hi = (int(x, 16) for x in f[0].split("-"))
            if "x" in f[1] and len(f) >= 6:
                maps.append((lo, hi, int(f[2], 16), f[5]))
        elif line.startswith("S "):
            v = int(line[2:], 16)
            pcs.append((v & ((1 << 56) - 1), v >> 56))
    return sorted(maps), pcs


_syms = {}


def symbols(path):
    if path in _syms:
        return _syms[path]
    out = []
    for args in (["nm", "-n", "--defined-only", path], ["nm", "-n", "-D", "--defined-only", path]):
        try:
            r = subprocess.run(args, capture_output=True, text=True, timeout=120)
        except (OSError, subprocess.TimeoutExpired):
            continue
        for l in r.stdout.splitlines():
            f = l.split()
            if len(f) >= 3 and f[1] in "tTwWiI":
                out.append((int(f[0], 16), f[2]))
        if out:
            break
    out.sort()
    _syms[path] = ([a for a, _ in out], [n for _, n in out])
    return _syms[path]


def elf_is_exec(path):
    try:
        with open(path, "rb") as fh:
            h = fh.read(18)
        return h[16] == 2  # ET_EXEC: symbols at absolute addresses
    except OSError:
        return False


def resolve(maps, pcs):
    starts = [m[0] for m in maps]
    agg = collections.Counter()
    for pc, role in pcs:
        i = bisect.bisect_right(starts, pc) - 1
        if i < 0 or pc >= maps[i][1]:
            agg[("?", "?", role)] += 1
            continue
        lo, _, off, path = maps[i]
        addr = pc if elf_is_exec(path) else pc - lo + off
        addrs, names = symbols(path)
        j = bisect.bisect_right(addrs, addr) - 1
        name = names[j] if j >= 0 else "?"
        agg[(os.path.basename(path), name, role)] += 1
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = {}
    for f in a.files:
        maps, pcs = load(f)
        agg = resolve(maps, pcs)
        n = max(1, len(pcs))
        by_role = collections.Counter()
        by_lib = collections.Counter()
        for (lib, _, role), c in agg.items():
            by_role[ROLES[role]] += c
            by_lib[lib] += c
        top = sorted(agg.items(), key=lambda kv: -kv[1])[:a.top]
        print("== %s: %d samples" % (f, len(pcs)))
        print("roles: " + ", ".join("%s %.1f%%" % (k, 100.0 * v / n) for k, v in by_role.most_common()))
        print("objects: " + ", ".join("%s %.1f%%" % (k, 100.0 * v / n) for k, v in by_lib.most_common(8)))
        for (lib, name, role), c in top:
            print("%6.2f%%  %-8s %-28s %s" % (100.0 * c / n, ROLES[role], lib[:28], name))
        res[os.path.basename(f)] = {
            "samples": len(pcs),
            "roles": {k: round(v / n, 4) for k, v in by_role.items()},
            "objects": {k: round(v / n, 4) for k, v in by_lib.most_common(12)},
            "top": [{"share": round(c / n, 4), "role": ROLES[role], "object": lib, "function": name}
                    for (lib, name, role), c in top],
        }
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
