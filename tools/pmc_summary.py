#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>/ (kernel stats + PMC summary).

Usage: python3 tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>

Writes kernel_stats.csv (rocprofv3 --kernel-trace --stats), the counter CSVs trimmed to
the gmapdp kernels, and pmc_summary.json: per kernel template the dispatch count, average
duration, FETCH_SIZE / WRITE_SIZE averages and HBM bytes per dispatch
= (2 * FETCH_SIZE + WRITE_SIZE) KB * 1024 (MI355X_MICROARCH.md, HBM section: on gfx950
FETCH_SIZE counts wide reads at half their size), plus the SQ counter averages.
bench.py's pmc_traffic() reads hbm_bytes_per_dispatch from the newest such summary.
"""
import csv
import json
import os
import re
import shutil
import sys
import time
from collections import defaultdict


def short(name):
    """'void gmapdp::dpx_kernel<16, true>(...)' -> 'gmapdp::dpx_kernel<16, true>'."""
    m = re.match(r"(?:void )?(gmapdp::\w+(?:<[^>]*>)?)", name)
    return m.group(1) if m else None


def counters(path):
    """{kernel: {counter: [value per dispatch]}} from a run_counter_collection.csv."""
    out = defaultdict(lambda: defaultdict(dict))
    rows = []
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if not k:
                continue
            rows.append(row)
            d = out[k][row["Counter_Name"]]
            d[row["Dispatch_Id"]] = d.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in out.items()}, rows


def find(root, sub, name):
    for dp, _, files in os.walk(os.path.join(root, sub)):
        if name in files:
            return os.path.join(dp, name)
    return None


def workload_of(src):
    """the bench workload id tools/profile.sh recorded (bench.py workload_id: c<config>[-appb][-simd])"""
    try:
        return open(os.path.join(src, "workload.txt")).read().strip() or None
    except OSError:
        return None


def bench_block_runs(src):
    """block_runs of the bench line the kernel-trace pass printed (stats.log), or None"""
    try:
        lines = open(os.path.join(src, "stats.log")).read().splitlines()
    except OSError:
        return None
    for ln in reversed(lines):
        if ln.startswith("{") and '"block_runs"' in ln:
            try:
                return json.loads(ln).get("block_runs")
            except ValueError:
                return None
    return None


def main(src, dst, iso=False):
    os.makedirs(dst, exist_ok=True)
    stats = find(src, "stats", "run_kernel_stats.csv")
    kern = {}
    if stats:
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
        with open(stats) as f:
            for row in csv.DictReader(f):
                k = short(row["Name"])
                if k:
                    kern[k] = {"dispatches": int(row["Calls"]), "avg_duration_ns": float(row["AverageNs"]),
                               "total_ms": float(row["TotalDurationNs"]) / 1e6}
    for sub in ("fetch", "write", "sq", "sq2"):
        path = find(src, sub, "run_counter_collection.csv")
        if not path:
            continue
        per, rows = counters(path)
        with open(os.path.join(dst, "pmc_%s.csv" % sub), "w", newline="") as f:
            if rows:
                w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
        for k, cs in per.items():
            e = kern.setdefault(k, {})
            for c, vals in cs.items():
                avg = sum(vals) / len(vals)
                if c == "FETCH_SIZE":
                    e["fetch_size_kb_avg"] = avg
                elif c == "WRITE_SIZE":
                    e["write_size_kb_avg"] = avg
                else:
                    e["sq_%s_sum_avg" % c] = avg
    for e in kern.values():
        if "fetch_size_kb_avg" in e and "write_size_kb_avg" in e:
            e["hbm_bytes_per_dispatch"] = (2 * e["fetch_size_kb_avg"] + e["write_size_kb_avg"]) * 1024
    if iso:
        return write_iso(src, dst, kern)
    summary = {
        "recorded": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),  # bench.py selects summaries by this
        "workload": workload_of(src),  # ... and only those of its own workload
        "command": "python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline %s(under rocprofv3, tools/profile.sh)"
                   % (open(os.path.join(src, "bench_args.txt")).read().strip() + " "
                      if os.path.exists(os.path.join(src, "bench_args.txt")) else ""),
        "hbm_bytes_rule": "2*FETCH_SIZE + WRITE_SIZE, KB -> bytes x1024 (MI355X_MICROARCH.md HBM: gfx950 "
                          "FETCH_SIZE counts half of wide reads)",
        "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1].get("total_ms", 0.0))),
    }
    # the bench line's count of stage-2 kernel runs over a block in the profiled process (bench.py
    # pmc_entry: dispatch totals / runs = bytes per block, whatever the seeding's launch chunks per block)
    runs = bench_block_runs(src)
    if runs:
        summary["block_runs"] = runs
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    shutil.copy(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profile.sh"),
                os.path.join(dst, "recipe.sh"))
    print("wrote", dst, "kernels:", ", ".join(kern))


def write_iso(src, dst, kern):
    """iso_summary.json: the rocprofv3 record of `bench.py --iso-kernel K` (K's launch classes run alone, one
    launch at a time) -- the average duration the bench line's roofline cites, the bench's own HIP-event
    timing and algorithmic bytes of the same launches, and that kernel's counters (per dispatch)."""
    bench = {}
    try:
        bench = json.loads(open(os.path.join(src, "iso_bench.json")).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        pass
    k = bench.get("iso_kernel")
    e = kern.get(k, {}) if k else {}
    out = {"recorded": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "workload": workload_of(src),
           "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --iso-kernel '%s' --iso-reps 3 "
                      "(tools/profile.sh <tag> iso)" % k,
           "kernel": k, "dispatches": e.get("dispatches"), "avg_duration_ns": e.get("avg_duration_ns"),
           "algorithmic_bytes_per_launch": bench.get("algorithmic_bytes_per_launch"),
           "bench_hip_event_ms_per_launch": bench.get("ms_per_launch"),
           "hbm_rule": "2*FETCH_SIZE + WRITE_SIZE, KB -> bytes x1024 (MI355X_MICROARCH.md)",
           "counters": e, "other_kernels": {n: v for n, v in kern.items() if n != k}}
    if out["avg_duration_ns"] and out["algorithmic_bytes_per_launch"]:
        out["achieved_gbs"] = out["algorithmic_bytes_per_launch"] / out["avg_duration_ns"]
        out["frac_of_8tbs"] = out["achieved_gbs"] / 8000.0
    with open(os.path.join(dst, "iso_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(dst, "iso_summary.json"), "kernel:", k)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--iso"]
    main(args[0], args[1], iso="--iso" in sys.argv[1:])
