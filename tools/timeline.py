"""The bench step's kernel timeline from a rocprofv3 --kernel-trace CSV (diagnostic).

Steps are separated where a dispatch starts after every earlier one has ended (bench.py's steps fork
from and join into one stream).  Prints, for the chosen steps, each kernel name's first start / last end
relative to the step start, its dispatch count and summed duration.

    python tools/timeline.py <kernel_trace.csv> [first_step] [nsteps]
    python tools/timeline.py <kernel_trace.csv> around <name> <k> <window_ms>
        (the window from the k-th dispatch of a kernel whose name contains <name>)"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    if len(sys.argv) > 2 and sys.argv[2] == "around":
        return around(path, sys.argv[3], int(sys.argv[4]), float(sys.argv[5]))
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    nst = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    steps, cur, hi = [], [], 0
    for s, e, n in rows:
        if cur and s > hi:
            steps.append(cur)
            cur = []
        cur.append((s, e, n))
        hi = max(hi, e) if len(cur) > 1 else e
    if cur:
        steps.append(cur)
    out = []
    for k in range(first, min(first + nst, len(steps))):
        st = steps[k]
        t0 = st[0][0]
        t1 = max(e for _, e, _ in st)
        per = defaultdict(lambda: [1e30, 0, 0, 0.0])
        for s, e, n in st:
            n = n.split("(")[0].replace("void ", "")
            p = per[n]
            p[0] = min(p[0], s - t0)
            p[1] = max(p[1], e - t0)
            p[2] += 1
            p[3] += (e - s) / 1e6
        out.append({"step": k, "ms": (t1 - t0) / 1e6,
                    "kernels": {n: {"first_ms": round(p[0] / 1e6, 3), "last_ms": round(p[1] / 1e6, 3), "n": p[2],
                                    "sum_ms": round(p[3], 3)} for n, p in sorted(per.items(), key=lambda x: x[1][0])}})
    print(json.dumps({"nsteps_found": len(steps), "step_ms": [round((max(e for _, e, _ in st) - st[0][0]) / 1e6, 2)
                                                            for st in steps[:40]], "steps": out}, indent=1))


def around(path, name, k, win):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    hits = [s for s, _, n in rows if name in n]
    t0 = hits[k] - 200000
    t1 = t0 + int(win * 1e6)
    per = defaultdict(lambda: [1e30, 0, 0, 0.0])
    busy = []
    for s, e, n in rows:
        if s < t0 or s > t1:
            continue
        n = n.split("(")[0].replace("void ", "")
        p = per[n]
        p[0] = min(p[0], s - t0)
        p[1] = max(p[1], e - t0)
        p[2] += 1
        p[3] += (e - s) / 1e6
        busy.append((s - t0, e - t0, n))
    # how many kernels run at once, per 0.5 ms bin
    nb = int(win / 0.5) + 1
    conc = [0.0] * nb
    for s, e, _ in busy:
        for b in range(max(0, int(s / 5e5)), min(nb, int(e / 5e5) + 1)):
            lo, hi = max(s, b * 5e5), min(e, (b + 1) * 5e5)
            if hi > lo:
                conc[b] += (hi - lo) / 5e5
    print(json.dumps({"t0_ns": t0, "kernels": {n: {"first_ms": round(p[0] / 1e6, 3), "last_ms": round(p[1] / 1e6, 3),
                                                    "n": p[2], "sum_ms": round(p[3], 3)}
                                                for n, p in sorted(per.items(), key=lambda x: x[1][0])},
                      "concurrency_per_0.5ms": [round(c, 2) for c in conc]}, indent=1))


if __name__ == "__main__":
    main()
