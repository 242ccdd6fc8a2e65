"""bench.py -- MI355X GMAP hot path throughput (BASELINE.json metric on configs[2]; configs[4] with --config 4).

Workload (gmap-2024_amd/gmapdp/workload.py):
  * configs[2] (default; "1M synthetic 2-kb cDNA (5 exons, 2 % mismatch) vs GRCh38, 1xMI355X, full stage2 +
    all Dynprog_* paths"): an i.i.d. ACGT genome laid out as GRCh38's 24 primary chromosomes (3.09 Gnt,
    universal coordinates past 2^31), generated directly as the reference's .genomecomp blocks and resident
    in HBM (1.16 GB); per 2-kb read the calls GMAP's own program makes into the path, measured with the
    reference `gmap -d` over a gmap_build index (tools/callmix.py --index, profiles/r04_callmix/callmix_d.json;
    workload.CDNA2K): 1.585 Stage2_compute calls (gmap.c:1208: Oligoindex_hr_tally + Oligoindex_get_mappings
    over the read's locus +- 100 kb, gregion.c:899, then the chaining -- Diag_compute_bounds,
    align_compute_lookback, convert_to_nucleotides, Stage2_filter_unique) and 21.1 Dynprog_single_gap +
    6.78 Dynprog_end5_gap + 6.38 Dynprog_end3_gap + 49.7 Dynprog_genome_gap + 7.53 Dynprog_microexon_int
    (`--mix appb`: SURVEY App. B's mix of rounds 1-3);
  * configs[4] (--config 4; gmapl, "500k 5-kb Iso-Seq-style reads vs 17-Gb wheat genome"): 5-kb reads of
    10 exons with 1 % substitutions + 1 % indels against a 17-Gnt wheat-layout genome (6.4 GB packed,
    universal coordinates past 2^32), the per-read call mix of that read shape (workload.ISOSEQ5K).
The splice probabilities of the genome gaps and the microexon candidates' sites are GMAP's MaxEnt models
evaluated by the engine on the device inside the step (gmapdp_plan_bind_genome_maxent, the microexon plan
with device probabilities); the genome-gap introns carry strong planted splice sites.

Read stream: blocks of --reads reads, each generated from its own seeds; rank r of N takes the blocks
b % N == r (GMAP's --part=r/N rule, inbuffer.c:283, per block) and cycles through --batches of them, so
consecutive steps process different reads and genomic windows (a stream, not one warm replay).  One step
= one pass of the engine over every call of one block (Stage2_compute on its own stream, the DP launch
classes on three more).  The timed steps stream the blocks as two pipelines, the stage-2 chains and the DP
classes, each block's work complete inside the timed region (GMAPDP_BENCH_PIPE=0: each step joined at its
end; its time is reported beside the headline as step_split_ms.together_serial).  Inputs (descriptors, query arenas, splice
probabilities) are resident in HBM before the timed region (the contract's `value`); the host plans
(bands, launch classes) are made once per block and their cost is reported as plan_ms.

value = reads whose Stage2_compute and DP calls were processed per second, whole job (all ranks).  Stage
1/3 orchestration stays on the host and is not in the step.

Multi-GPU: `--gpus N` without a WORLD_SIZE in the environment starts N rank processes (this file, with
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set) before anything touches the GPU and exits with their
status; under torch.distributed.run the ranks come from the environment.  One process per GPU, RCCL
(backend nccl) for the barrier and the max-over-ranks step time only: the path has no exchange step.
`--dry-run` runs the launcher, the process group (gloo), the block sharding and the workload generation on
the CPU without a GPU (tests/test_bench_launcher.py).
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
# VALU issue: a wave64 instruction issues over 2 cycles on a SIMD-32 (MI355X_MICROARCH.md), 4 SIMDs x 256 CUs
# at 2.4 GHz: 1.2288 T wave-instructions/s; lane-ops: 256 x 4 x 32 x 2.4 GHz = 78.6 T int32 ops/s
VALU_WAVE_INSTR_PEAK = 256 * 4 * 2.4e9 / 2
INT_OPS_PEAK = 256 * 4 * 32 * 2.4e9
OPS_PER_CELL = 11                # E 3 + F 3 + H 4 + clamp 1 integer ops per banded cell
METRIC = "aligned cDNA reads/sec (2 kb, GRCh38) at 1/2/4/8 MI355X; DP HBM GB/s vs peak"
T_START = time.perf_counter()


def progress(msg):
    """a progress line on stderr (stdout carries only the result line)"""
    r = os.environ.get("RANK")
    err_line("[bench%s %.0fs] %s" % ("" if r is None else " r" + r, time.perf_counter() - T_START, msg))


def err_line(text):
    """One stderr line in ONE write: the ranks share the pipe, and print's separate newline write could let
    another rank's line land in the middle of this one."""
    sys.stderr.write(text + "\n")
    sys.stderr.flush()


# ---------------------------------------------------------------------------------------------------
# algorithmic bytes and cells
# ---------------------------------------------------------------------------------------------------
def algorithmic_bytes(rlength, glength, npairs, desc_bytes):
    """Dynprog_single_gap / _end{5,3}_gap: descriptor + query and upper-cased query (2 x rlength) +
    packed genome blocks covering the segment (12 B per 32 nt) + result (32 B) + one 16-B Pair
    record per emitted pair."""
    r = np.asarray(rlength, dtype=np.int64)
    g = np.asarray(glength, dtype=np.int64)
    return int((desc_bytes + 2 * r + 12 * ((g + 62) // 32) + 32).sum() + 16 * int(np.asarray(npairs).sum()))


def genome_algorithmic_bytes(gp, npairs, sprob_arena=False):
    """Dynprog_genome_gap with its splice-site MaxEnt (the fused operation gg_kernel runs): descriptor (96 B)
    + query and upper-cased query (2 x rlength) + the packed genome blocks of both segments + result (72 B)
    + one 16-B record per emitted pair.  The splice probabilities are computed in the kernel from the same
    segments and the L2-resident model tables, so they are not counted (no probability arena exists).
    `sprob_arena`: the SIMD builds' uxg_kernel still reads the 8-B-per-column probability arena that its
    me_gap_kernel prologue writes, so its classes count 8 x (glengthL + glengthR) more."""
    r = gp["rlength"].astype(np.int64)
    gL = gp["glengthL"].astype(np.int64)
    gR = gp["glengthR"].astype(np.int64)
    arena = 8 * (gL + gR) if sprob_arena else 0
    return int((96 + 2 * r + 12 * ((gL + 62) // 32) + 12 * ((gR + 62) // 32) + 72 + arena).sum()
               + 16 * int(np.asarray(npairs).sum()))


S2_SEED = "gmapdp::oi_kernel+gmapdp::oi_map_kernel"  # the seeding (Oligoindex_hr_tally + get_mappings)
# stage-2 kernels timed alone: gmapdp_stage2_plan_run's `what` (1 seeding, 4 s2a, 8 s2b, 16 s2c)
CHAIN_FUSED = "chaining_fused"  # s2a + s2b + s2c against the fused operation's bytes
S2_WHAT = {S2_SEED: 1, "gmapdp::s2a_kernel": 4, "gmapdp::s2b_kernel": 8, "gmapdp::s2c_kernel": 16}


def stage2_algorithmic_bytes(op, ores, s2res):
    """Per stage-2 kernel, the algorithmic bytes of one block's calls: ql = querylength,
    T = totalpositions (seeding hits kept), nd = ndiagonals, W = window length.
      seeding: descriptor 48 + query ql + genome blocks 12 x ceil((W + 16) / 32) + npositions and mappings 8 ql
               + table 4 T + result 32 + diagonals 16 nd
      s2a:     descriptors 48 + 32 + npositions / mappings 8 ql + diagonals 16 nd + table 4 T + chrpos and
               score arrays out 8 T + per-position offsets, active bounds and ranges 24 ql + result 32
      s2b:     per-position metadata 20 ql + the chrpos of every hit 4 T + one 36-B link per query position (the
               chain; a lower bound: the sweep scores every hit in the active ranges)
      s2c:     the score array 4 T + the kept paths' walk (32 B per pair) + 20-B pair records + 16-B path records
               + the query twice 2 ql + result 32
      chaining (the three as one fused operation, no intermediates): what the seeding hands over (descriptor
               48 + 32, npositions / mappings 8 ql, table 4 T, diagonals 16 nd) + the query twice 2 ql, and the
               outputs (20-B pair records, 16-B path records, result 32)"""
    ql = op["querylength"].astype(np.int64)
    T = np.maximum(ores["totalpositions"].astype(np.int64), 0)
    nd = np.maximum(ores["ndiagonals"].astype(np.int64), 0)
    W = (op["chrend"].astype(np.int64) - op["chrstart"].astype(np.int64)).clip(min=0)
    npairs = int(s2res["npairs"].sum())
    return {S2_SEED: int((48 + ql + 12 * ((W + 16 + 31) // 32) + 8 * ql + 4 * T + 32 + 16 * nd).sum()),
            "gmapdp::s2a_kernel": int((80 + 8 * ql + 16 * nd + 4 * T + 8 * T + 24 * ql + 32).sum()),
            "gmapdp::s2b_kernel": int((20 * ql + 4 * T + 36 * ql).sum()),
            "gmapdp::s2c_kernel": int((4 * T + 2 * ql + 32).sum()) + 52 * npairs + 16 * int(s2res["nresults"].sum()),
            CHAIN_FUSED: int((80 + 8 * ql + 4 * T + 16 * nd + 2 * ql + 32).sum()) + 20 * npairs
            + 16 * int(s2res["nresults"].sum())}


def workload_id(args):
    """The committed PMC / iso summaries a bench line may cite are the ones of its own workload:
    c<config>[-appb][-simd] (tools/profile.sh records it)."""
    return "c%d%s%s" % (args.config, "-appb" if args.mix == "appb" else "", "-simd" if args.simd else "")


def band_cells(rlength, glength, lband, uband):
    """Cells of a banded fill: sum over columns c = 1..glength of |[max(1, c - uband), min(rlength,
    c + lband)]| (dynprog.c:1411-1449 row range), per problem."""
    R = np.asarray(rlength, dtype=np.int64)
    G = np.asarray(glength, dtype=np.int64)
    lo, up = np.asarray(lband, dtype=np.int64), np.asarray(uband, dtype=np.int64)
    tot = np.zeros(len(R), dtype=np.int64)
    for c in range(1, int(G.max(initial=0)) + 1):
        live = G >= c
        tot += np.where(live, np.maximum(0, np.minimum(R, c + lo) - np.maximum(1, c - up) + 1), 0)
    return tot


def dp_cells(sp, ep, gp, g_fills):
    """Banded DP cells of the step: single gaps (wide band), end gaps (wide band, INDELS narrow, NOGAPS
    none), two fills per genome gap where `g_fills` (False where genome_gap_simple answered)."""
    r, g = sp["rlength"].astype(np.int64), sp["glength"].astype(np.int64)
    eb = sp["extraband"].astype(np.int64)
    cells = int(np.minimum(np.abs(g - r) + 2 * eb + 1, r + 1).dot(g))
    r = np.minimum(ep["rlength"].astype(np.int64), 660)
    g = np.minimum(ep["glength"].astype(np.int64), 2000)
    eb = ep["extraband"].astype(np.int64)
    W = np.where(ep["endalign"] == 1, 2 * eb + 1, np.abs(g - r) + 2 * eb + 1)
    W = np.where(ep["endalign"] == 2, 0, W)
    cells += int(np.minimum(W, r + 1).dot(g))
    return cells + int(genome_cells(gp, g_fills).sum())


def genome_cells(gp, g_fills):
    """Cells of the two fills of each genome gap (L: lbandL, ubandL; R: lbandL, ubandR, as
    dynprog_genome.c:3801-3813 calls them), zero where genome_gap_simple answered."""
    r = gp["rlength"].astype(np.int64)
    eb = gp["extraband"].astype(np.int64)
    gL, gR = gp["glengthL"].astype(np.int64), gp["glengthR"].astype(np.int64)
    c = band_cells(r, gL, eb, gL - r + eb) + band_cells(r, gR, eb, gR - r + eb)
    return np.where(g_fills, c, 0)


# ---------------------------------------------------------------------------------------------------
# committed profiles (profiles/*): PMC traffic, VALU instructions, rocprof average duration
# ---------------------------------------------------------------------------------------------------
def profile_record(kind, name, workload):
    """The committed record of `kind` for `workload` (workload_id) the bench line cites: the one
    profiles/current.json names for it ({kind: {workload: path}}), else the newest of that workload by the
    "recorded" time the writing tool stored in it (tools/pmc_summary.py); records without one rank oldest.
    Never by path name or file mtime (a checkout sets mtimes in checkout order), and never a record of
    another workload (a summary whose "workload" differs is skipped).  Returns (parsed json, path relative
    to ROOT) or (None, None)."""
    import glob
    try:
        cur = json.load(open(os.path.join(ROOT, "profiles", "current.json"))).get(kind)
    except (OSError, ValueError):
        cur = None
    if isinstance(cur, dict):
        cur = cur.get(workload)
    paths = [os.path.join(ROOT, cur)] if cur else glob.glob(os.path.join(ROOT, "profiles", "*", name))
    best = None
    for path in paths:
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if workload is not None and d.get("workload") != workload:
            continue
        key = d.get("recorded") or ""
        if best is None or key > best[0]:
            best = (key, d, os.path.relpath(path, ROOT))
    return (best[1], best[2]) if best else (None, None)


def pmc_entry(key, workload):
    """The PMC summary of this workload's step (tools/profile.sh + tools/pmc_summary.py): the record of kernel
    `key` ('+'-joined names and template instances of one kernel are summed per step), or (None, source)."""
    d, src = profile_record("pmc_summary", "pmc_summary.json", workload)
    if not d:
        return None, None
    ks = d.get("kernels", {})
    rec = {}
    # a stage-2 kernel: the profiled process's dispatch totals over its block runs (bench block_runs)
    runs = (d.get("block_runs") or {}).get(key)
    parts = key.split("+")
    # a plain name (gmapdp::s2c_kernel) covers its template instances (s2c_kernel<false>, <true>)
    members = [[k for k in ks if k == p or (("<" not in p) and k.startswith(p + "<"))] for p in parts]
    if not all(members):
        return None, src
    for f in ("hbm_bytes_per_dispatch", "sq_SQ_INSTS_VALU_sum_avg", "avg_duration_ns"):
        tot = 0.0
        for m in members:
            for k in m:
                v = ks[k].get(f)
                if v is None:
                    tot = None
                    break
                # per bench launch: a template instance dispatched on fewer blocks counts in proportion
                disp = ks[k].get("dispatches") or 1
                ref = runs or max(ks[x].get("dispatches") or 1 for x in m)
                tot += v * disp / ref
            if tot is None:
                break
        rec[f] = tot
    return rec, src


def iso_entry(key, workload):
    """The committed rocprofv3 --kernel-trace --stats record of `bench.py --iso-kernel <key>` on this
    workload (tools/pmc_summary.py --iso): {avg_duration_ns, dispatches, ...}."""
    d, src = profile_record("iso_summary", "iso_summary.json", workload)
    if not d or d.get("kernel") != key:
        return None, src
    return d, src


def rocprof_name(kind, R, dl, lds=0):
    """The rocprofv3 kernel name(s) of a DP launch class ('+'-joined when a class is several kernels)."""
    if kind == 0:
        return "gmapdp::dp_kernel<%d, %s>" % (R, "true" if dl else "false")
    if kind == 7:  # lanes over query rows (bands wider than the query)
        return "gmapdp::dpr_kernel<%d, %s>" % (R, "true" if dl else "false")
    if kind == 2:  # dpx_kernel<S, GD>: GD = direction words in global scratch
        return "gmapdp::dpx_kernel<%d, %s>" % (R, "false" if dl else "true")
    if kind == 3:
        return "gmapdp::sx_kernel<%d>" % R
    if kind == 4:
        return "gmapdp::uxe_kernel<%d>" % R
    if kind == 5:
        return "gmapdp::uxg_kernel<%d>" % R
    return "gmapdp::gg_kernel<%d, %s>" % (R, "true" if dl else "false")


def latest_e2e(kind="e2e"):
    """The cited GMAP end-to-end record (tools/e2e_timing.py, profiles/*/e2e.json, or e2e_avx2.json for the
    AVX2 builds; profile_record's rule): the unmodified gmap and the drop-in on the same reads and host cores."""
    d, src = profile_record(kind, kind + ".json", None)
    try:
        runs = d["runs"]
    except (TypeError, KeyError):
        return None
    cpu = [r for r in runs if "gpu" not in r["program"]]
    gpu = [r for r in runs if "gpu" in r["program"]]
    if not cpu or not gpu:
        return None
    # repeated drop-in runs at one thread count (the record's configurations): their median, and the spread
    by_t = {}
    for r in gpu:
        by_t.setdefault(r["threads"], []).append(r["reads_per_s"])
    t_best = max(by_t, key=lambda t: float(np.median(by_t[t])))
    cpu_v = max(r["reads_per_s"] for r in cpu)
    med = float(np.median(by_t[t_best]))
    return {"source": src, "recorded": d.get("recorded"), "reads": d.get("reads"), "mode": d.get("mode", "-g"),
            "cpu_gmap_reads_per_s": cpu_v,
            "cpu_gmap_threads": max(cpu, key=lambda r: r["reads_per_s"])["threads"],
            "drop_in_reads_per_s": med, "drop_in_runs": sorted(by_t[t_best]), "drop_in_threads": t_best,
            "ratio": med / cpu_v, "outputs_identical": d.get("outputs_identical")}


def like_for_like(out, pcie_ms, up, down, compact=None, pipelined=None):
    """The headline next to what it leaves out: the step's own host-to-device and device-to-host copies and
    GMAP end to end through the drop-in.  MaxEnt is in the step (device), as it is in the CPU baseline's
    reference objects.  With the compact pair stream (`compact`), the down copy is the run-length stream
    plus the results, and the compaction kernels are added; reads_per_s_incl_pcie takes the cheaper of the
    two transports (the host's expansion back to records replaces reading the records, and is reported
    beside it, not added: neither transport counts the consumer's own pass over the pairs)."""
    v = out["value"]
    ms = out["ms_per_step"]
    reads = out["config"]["reads_per_step_per_gpu"]
    raw = reads / ((ms + pcie_ms) * 1e-3) * out["n_gpus"]
    with_pcie = raw
    if compact and compact.get("expanded_equals_records"):
        compact["reads_per_s_incl_pcie"] = reads / ((ms + compact["pcie_ms_per_step"]) * 1e-3) * out["n_gpus"]
        with_pcie = max(raw, compact["reads_per_s_incl_pcie"])
    serial = with_pcie
    if pipelined:
        with_pcie = max(with_pcie, pipelined["reads_per_s"] * out["n_gpus"])
    cb = out.get("cpu_baseline") or {}
    cpu = cb.get("value")
    return {"pcie_ms_per_step": pcie_ms, "pcie_bytes_up": up, "pcie_bytes_down": down,
            "reads_per_s_incl_pcie_records": raw, "compact_pair_stream": compact,
            "reads_per_s_incl_pcie": with_pcie, "reads_per_s_incl_pcie_serial": serial,
            "pipelined_compact_with_pcie": pipelined,
            "ratio_vs_cpu": v / cpu if cpu else None,
            "ratio_vs_cpu_incl_pcie": with_pcie / cpu if cpu else None,
            "drop_in_end_to_end": latest_e2e(),
            "drop_in_end_to_end_avx2": latest_e2e("e2e_avx2"),
            "note": "reads_per_s_incl_pcie_serial: the copies measured after the step and added to it; "
                    "pipelined_compact_with_pcie: the same bytes copied on a copy stream overlapped with the next "
                    "step (reads_per_s_incl_pcie: the better of the two); the end-to-end record is GMAP's own "
                    "program on the same reads and cores (tools/e2e_timing.py)"}


def cpu_baselines(mix, config=2):
    """tools/cpu_baseline.py as a child process (the reference's own objects, all usable host cores,
    AVX2 and nosimd builds, the bench's call mix: configs[1] times the single and end gaps alone);
    {build: result or None}."""
    out = {}
    for build in ("avx2", "nosimd"):
        progress("CPU baseline (%s build)" % build)
        try:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "cpu_baseline.py"), "--build", build,
                                "--budget", "10", "--mix", mix, "--config", str(config)],
                               capture_output=True, timeout=240, text=True)
            out[build] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else None
        except (subprocess.TimeoutExpired, ValueError, IndexError):
            out[build] = None
    return out


# ---------------------------------------------------------------------------------------------------
# launcher: N rank processes, started before anything touches the GPU
# ---------------------------------------------------------------------------------------------------
def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """Start n copies of this script as ranks 0..n-1 (torchrun's environment contract, rendezvous on
    127.0.0.1), wait for them, and return the first nonzero exit status (0 when all succeed).  A rank
    that fails ends the others (their exact PIDs)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


# ---------------------------------------------------------------------------------------------------
# one rank
# ---------------------------------------------------------------------------------------------------
def config_of(args):
    from gmapdp import workload as W
    if args.config == 1:  # "100k synthetic 2-kb cDNA vs human chr22, Dynprog_single + Dynprog_end only"
        return W.Layout(W.CHR22), W.SHAPES[args.mix], "chr22"
    if args.config == 4:
        return W.Layout(W.WHEAT17), (W.ISOSEQ5K if args.mix == "d" else W.ISOSEQ5K_G), "wheat17"
    shape = W.SHAPES[args.mix]
    if args.genome == "chr22":
        return W.Layout(W.CHR22), shape, "chr22"
    return W.Layout(W.GRCH38), shape, "grch38"


def make_stream(args, rank, world):
    """genome (planted for the whole stream) + this rank's blocks; no GPU work"""
    from gmapdp import workload as W
    from gmapdp import shard
    layout, shape, gname = config_of(args)
    mine = shard.blocks_of_rank(rank, world, args.batches)
    t0 = time.perf_counter()
    genome = W.PackedGenome(layout.total, seed=38)
    W.plant_stream(genome, layout, args.reads, range(world * args.batches), shape)
    workers = int(os.environ.get("GMAPDP_BENCH_WORKERS", "0")) or max(1, min(args.batches, 16 // world))
    data = W.make_blocks(genome, layout, args.reads, mine, shape=shape, sprob=False, workers=workers)
    if args.config == 1:  # configs[1] times the single and end gaps alone
        for d in data:
            for k in ("genome", "microexon", "oligo"):
                d[k] = d[k][:0]
    progress("genome (%s, %d nt) and %d blocks of %d reads ready (%.0f s, %d workers)"
             % (gname, layout.total, len(mine), args.reads, time.perf_counter() - t0, workers))
    return layout, shape, gname, genome, mine, data, time.perf_counter() - t0


def dry_run(args, rank, world):
    """The launcher / process group / sharding / generation path without a GPU (gloo)."""
    import torch
    import torch.distributed as dist
    from gmapdp import shard
    layout, shape, gname, genome, mine, data, t_gen = make_stream(args, rank, world)
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    digest = shard.genome_digest(genome.blocks[::4097])
    rec = shard.gather_blocks(mine, [int(d["reads"]) for d in data], dist if world > 1 else None)
    if world > 1:
        shard.check_replicated(digest, dist)
    rank_line = {"rank": rank, "world_size": dist.get_world_size() if world > 1 else 1,
                 "backend": dist.get_backend() if world > 1 else None, "blocks": mine,
                 "stage2_calls": [int(len(d["oligo"])) for d in data]}
    err_line(json.dumps({"rank_line": rank_line}))
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "config": gname, "shard": rec,
                          "genome_digest": digest.hex(), "setup_s": t_gen}))
    if world > 1:
        dist.destroy_process_group()
    _ = torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=None,
                    help="reads per step per GPU (one block; default 10000, 2000 for --config 4's 5-kb reads)")
    ap.add_argument("--batches", type=int, default=None,
                    help="distinct read blocks per rank, cycled over the steps (default 8; 10 for --config 1)")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 4],
                    help="BASELINE.json configs index: 1 = chr22, Dynprog_single + Dynprog_end only (10 blocks of "
                         "10 000 reads: 100 k distinct reads per cycle); 2 = GRCh38, full stage 2 + every Dynprog_* "
                         "family (default); 4 = gmapl, 5-kb Iso-Seq reads vs a 17-Gnt wheat layout")
    ap.add_argument("--genome", default="grch38", choices=["grch38", "chr22"], help="configs[2] genome layout")
    ap.add_argument("--simd", action="store_true", help="the SIMD builds' semantics (gmap.avx2: sx/uxe/uxg kernels)")
    ap.add_argument("--mix", default="d", choices=["d", "appb"],
                    help="per-read call mix: d = measured with the reference's gmap -d (stage 1 included; 1.585 "
                         "Stage2_compute calls per read over ~214-kb windows), appb = SURVEY App. B (rounds 1-3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true", help="CPU only: launcher, gloo process group, sharding")
    ap.add_argument("--iso-kernel", default=None,
                    help="profiling mode: run only this kernel template's launch classes, one launch at a time on one "
                         "stream (what the line's roofline times), print their timing and exit; run under rocprofv3 "
                         "--kernel-trace --stats for the committed isolated average (tools/profile.sh iso)")
    ap.add_argument("--iso-reps", type=int, default=3)
    args = ap.parse_args()

    if args.reads is None:
        args.reads = 2000 if args.config == 4 else 10000
    if args.batches is None:
        args.batches = 10 if args.config == 1 else 8
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "WORLD_SIZE" in os.environ and args.gpus != 1:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.dry_run:
        return dry_run(args, rank, world)

    # ---- workload first (forked generator workers must not inherit a GPU context) ----
    layout, shape, gname, genome, mine, data, t_gen = make_stream(args, rank, world)

    import torch
    import torch.distributed as dist
    import gmapdp
    from gmapdp import shard

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://", device_id=dev)
    # the plans' launch classes over three streams (the caller's and two sides): stage 2 takes the fourth
    eng = gmapdp.Engine(local, flags=gmapdp.CTX_TWO_SIDES if int(os.environ.get("GMAPDP_BENCH_SIDES", "2")) < 3 else 0)
    if world > 1:
        shard.check_replicated(shard.genome_digest(genome.blocks[::4097]), dist)
    eng.set_genome(blocks=genome.blocks, length=genome.length)
    del genome
    lib = eng.lib
    gen = torch.Generator(device=dev)

    # ---- per block: device arenas and plans (host: bands, launch classes, offsets) ----
    B = []
    t_plan = t_oplan = 0.0
    plan_ms, oplan_ms = [], []  # per block
    for bi, d in zip(mine, data):
        sp, ep, gp, op, mp = d["single"], d["end"], d["genome"], d["oligo"], d["microexon"]
        if args.simd:
            sp["flags"] |= gmapdp.SIMD
            ep["flags"] |= gmapdp.SIMD
            gp["flags"] |= gmapdp.SIMD
        blk = {"id": bi, "d": d, "ns": len(sp), "ne": len(ep), "ng": len(gp)}
        blk["d_q"] = torch.from_numpy(d["q"]).to(dev)
        blk["d_oq"] = torch.from_numpy(d["oq"]).to(dev)
        # the genome gaps' splice-probability arena: scratch the device MaxEnt fills in the step
        blk["d_sprob"] = torch.zeros(max(d["sprob_len"], 1), dtype=torch.float64, device=dev)
        nprob = len(sp) + len(ep)
        blk["host_res"] = np.zeros(nprob, dtype=gmapdp.RESULT_DTYPE)
        blk["host_gres"] = np.zeros(max(len(gp), 1), dtype=gmapdp.GENOME_RESULT_DTYPE)
        t0 = time.perf_counter()
        plan = C.c_void_p()
        eng._check(lib.gmapdp_plan_create_all(eng.h, sp.ctypes.data, len(sp), ep.ctypes.data, len(ep),
                                              gp.ctypes.data, len(gp), blk["host_res"].ctypes.data,
                                              blk["host_gres"].ctypes.data, C.byref(plan)), "gmapdp_plan_create_all")
        t_plan += time.perf_counter() - t0
        plan_ms.append((time.perf_counter() - t0) * 1e3)
        blk["plan"] = plan
        # Stage2_compute per read (gmap.c:1208): seeding + chaining, GMAP's defaults (splicing on,
        # maxintronlen 500000)
        s2p = np.zeros(len(op), dtype=gmapdp.STAGE2_PROBLEM_DTYPE)
        for k in ("qoff", "querylength", "chrstart", "chrend", "chroffset", "chrhigh", "plusp"):
            s2p[k] = op[k]
        s2p["splicingp"] = 1
        s2p["maxintronlen"] = 500000
        t0 = time.perf_counter()
        oplan = None
        if len(s2p):
            oplan = C.c_void_p()
            eng._check(lib.gmapdp_stage2_plan_create(eng.h, s2p.ctypes.data, len(s2p), d["oq"].ctypes.data,
                                                     d["oq"].ctypes.data, len(d["oq"]), C.byref(oplan)),
                       "gmapdp_stage2_plan_create")
        t_oplan += time.perf_counter() - t0
        oplan_ms.append((time.perf_counter() - t0) * 1e3)
        blk["oplan"] = oplan
        # Dynprog_microexon_int per read (stage3.c:9664) over genome-gap gaps: search + choice
        mplan = None
        if len(mp):
            mplan = C.c_void_p()
            eng._check(lib.gmapdp_microexon_plan_create(eng.h, mp.ctypes.data, len(mp), d["q"].ctypes.data,
                                                        d["q"].ctypes.data, len(d["q"]), C.byref(mplan)),
                       "gmapdp_microexon_plan_create")
        blk["mplan"] = mplan
        blk["ncands"] = lib.gmapdp_microexon_plan_candidates(mplan) if mplan else 0
        blk["ngpu"], blk["nggpu"] = lib.gmapdp_plan_gpu_problems(plan), lib.gmapdp_plan_genome_gpu_problems(plan)
        blk["cap"] = lib.gmapdp_plan_pair_capacity(plan)
        blk["mcap"] = lib.gmapdp_microexon_plan_pair_capacity(mplan) if mplan else 0
        nl = lib.gmapdp_plan_nlaunches(plan)
        blk["info"], blk["kinds"], blk["lstream"] = [], [], []
        for li in range(nl):
            R, dl, cnt, lds = C.c_int(), C.c_int(), C.c_int(), C.c_size_t()
            lib.gmapdp_plan_launch_info(plan, li, C.byref(R), C.byref(dl), C.byref(cnt), C.byref(lds))
            blk["info"].append((R.value, dl.value, cnt.value, lds.value))
            blk["kinds"].append(lib.gmapdp_plan_launch_kind(plan, li))
            blk["lstream"].append(lib.gmapdp_plan_launch_stream(plan, li))
        blk["names"] = [rocprof_name(blk["kinds"][li], *blk["info"][li][:2], blk["info"][li][3]) for li in range(nl)]
        B.append(blk)
    # outputs shared by the blocks (the steps are serialised: each forks from and joins into `stream`)
    mx = lambda k: max(b[k] for b in B)  # noqa: E731
    d_res = torch.zeros(max(mx("ngpu"), 1) * 32, dtype=torch.uint8, device=dev)
    d_gres = torch.zeros(max(mx("nggpu"), 1) * 72, dtype=torch.uint8, device=dev)
    d_pairs = torch.empty(max(mx("cap"), 1) * 16, dtype=torch.uint8, device=dev)
    d_s2res = torch.zeros(args.reads * 32, dtype=torch.uint8, device=dev)
    d_mres = torch.zeros(max(max(len(b["d"]["microexon"]) for b in B), 1) * gmapdp.MICROEXON_RESULT_DTYPE.itemsize,
                         dtype=torch.uint8, device=dev)
    d_mpairs = torch.empty(max(mx("mcap"), 1) * 16, dtype=torch.uint8, device=dev)
    for b in B:
        eng._check(lib.gmapdp_plan_bind_genome_maxent(eng.h, b["plan"], C.c_void_p(b["d_sprob"].data_ptr()),
                                                      C.c_void_p(d_gres.data_ptr())), "gmapdp_plan_bind_genome_maxent")
    progress("plans ready (%d blocks, %.2f s DP plans, %.2f s stage-2 plans)" % (len(B), t_plan, t_oplan))

    # Streams: stage 2 on its own stream, the DP launch classes on the engine's schedule (0 = main,
    # 1..2 = sides, longest-processing-time first over these three: the context is created with
    # GMAPDP_CTX_TWO_SIDES), forked from and joined into main; the microexon plan runs on the last side.
    # The process has four hardware queues (GPU_MAX_HW_QUEUES, HIP's default), so four streams.  Real
    # (non-null) streams, so per-launch events time exactly the launches on their stream.
    stream = torch.cuda.Stream(dev)
    # GMAPDP_BENCH_SIDES=3 (with GPU_MAX_HW_QUEUES >= 5): each of the plan's side lists on its own stream
    sides = [torch.cuda.Stream(dev) for _ in range(int(os.environ.get("GMAPDP_BENCH_SIDES", "2")))]
    # stage 2 (the step's longest chain) may take the high-priority queue: GMAPDP_BENCH_S2_PRIORITY=1
    s2prio = int(os.environ.get("GMAPDP_BENCH_S2_PRIORITY", "0"))
    # (=2: only the seeding launch on a high-priority stream, the chaining back on a normal one)
    # (=3: the chaining kernels there, the seeding on a normal-priority stream of its own)
    ostream = torch.cuda.Stream(dev, priority=-1) if s2prio in (1, 3) else torch.cuda.Stream(dev)
    sstream = torch.cuda.Stream(dev, priority=-1) if s2prio == 2 else (torch.cuda.Stream(dev) if s2prio == 3
                                                                       else ostream)
    # The timed steps as a deployment streams blocks (GMAPDP_BENCH_PIPE, default 3): the stage-2 chains (on
    # their stream) and the DP classes (forked from and joined into `stream`) run as two pipelines over the
    # blocks -- a block's chain starts when the previous block's chain ends, not when its DP classes end, and
    # the next block's DP classes do not wait for this block's sweep tail.  The two share no buffer (plans,
    # result and pair arenas are per pipeline), every block's work completes inside the timed region, and the
    # line reports the serialised step beside it (step_split_ms.together_serial).  0 = serialised steps (each
    # joins its chain); 1 = chains not joined but still forked from `stream`; 2 = 1 with consecutive chains on
    # two streams (measured slower: DESIGN.md §7).
    pipe = int(os.environ.get("GMAPDP_BENCH_PIPE", "3"))
    ostream2 = torch.cuda.Stream(dev) if pipe == 2 else None
    d_s2res2 = torch.zeros(args.reads * 32, dtype=torch.uint8, device=dev) if pipe == 2 else None
    nstep = [0]
    side_of = lambda k: min(k, len(sides))  # noqa: E731  plan stream k >= 1 -> side index + 1

    def launch(b, li, s, kernel_only=False):
        f = lib.gmapdp_plan_run_launch_kernel if kernel_only else lib.gmapdp_plan_run_launch
        eng._check(f(eng.h, b["plan"], li, C.c_void_p(b["d_q"].data_ptr()),
                     C.c_void_p(b["d_q"].data_ptr()), C.c_void_p(d_res.data_ptr()),
                     C.c_void_p(d_pairs.data_ptr()), C.c_void_p(s.cuda_stream)),
                   "gmapdp_plan_run_launch")

    # how many times this process ran each stage-2 kernel over a block (every leg: warmup, timed steps, the
    # outputs pass, the kernels alone, the PCIe legs), printed with the line so that tools/pmc_summary.py can
    # turn a profile's dispatch totals into bytes per block (the seeding's launch chunks vary per block; the
    # plans' sizing runs launch under other names and count nowhere)
    block_runs = {k: 0 for k in S2_WHAT}

    def orun(b, s, what, res=None):
        for k, w in S2_WHAT.items():
            if what & w or (what & 2 and w > 1):
                block_runs[k] += 1
        res = d_s2res if res is None else res
        eng._check(lib.gmapdp_stage2_plan_run(eng.h, b["oplan"], C.c_void_p(b["d_oq"].data_ptr()),
                                              C.c_void_p(b["d_oq"].data_ptr()), C.c_void_p(res.data_ptr()),
                                              what, C.c_void_p(s.cuda_stream)), "gmapdp_stage2_plan_run")

    def mrun(b, s, what):
        eng._check(lib.gmapdp_microexon_plan_run(eng.h, b["mplan"], C.c_void_p(b["d_q"].data_ptr()),
                                                 C.c_void_p(b["d_q"].data_ptr()), None,
                                                 C.c_void_p(d_mres.data_ptr()), C.c_void_p(d_mpairs.data_ptr()),
                                                 what, C.c_void_p(s.cuda_stream)), "gmapdp_microexon_plan_run")

    def step(b, do_oligo=True, do_dp=True, ev=None, piped=False):
        do_oligo = do_oligo and b["oplan"] is not None
        fork = torch.cuda.Event()
        fork.record(stream)
        used = set()
        alt = piped and pipe == 2 and nstep[0] % 2 == 1
        nstep[0] += 1
        os_, ss_, res = (ostream2, ostream2, d_s2res2) if alt else (ostream, sstream, None)
        if do_oligo:
            if not (piped and pipe == 3):
                ss_.wait_event(fork)
            if ev is not None:
                ev["oligo"][0].record(ss_)
            orun(b, ss_, 1, res)
            if ev is not None:
                ev["oligo"][1].record(ss_)
            if ss_ is not os_:
                os_.wait_stream(ss_)
            # the chaining as its three kernels (what 4 / 8 / 16: s2a, the s2b sweep, s2c), events between
            orun(b, os_, 4, res)
            if ev is not None:
                ev["s2a"].record(os_)
            orun(b, os_, 8, res)
            if ev is not None:
                ev["s2b"].record(os_)
            orun(b, os_, 16, res)
            if ev is not None:
                ev["chain"][1].record(os_)
        if do_dp:
            for li in range(len(b["names"])):
                k = side_of(b["lstream"][li])
                s = stream if k == 0 else sides[k - 1]
                if k and k not in used:
                    s.wait_event(fork)
                    used.add(k)
                if ev is not None:
                    ev["dp"][li][0].record(s)
                launch(b, li, s)
                if ev is not None:
                    ev["dp"][li][1].record(s)
            ms = sides[-1]
            if len(sides) not in used:
                ms.wait_event(fork)
                used.add(len(sides))
            if ev is not None:
                ev["mx"][0].record(ms)
            if b["mplan"] is not None:
                mrun(b, ms, 3)
            if ev is not None:
                ev["mx"][1].record(ms)
        for k in used:
            stream.wait_stream(sides[k - 1])
        if do_oligo and not (piped and pipe):
            stream.wait_stream(ostream)

    mk = lambda: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))  # noqa: E731

    def class_outputs(b, res, gres):
        """Per problem of block b: pairs emitted (single/end, genome), genome_gap_simple answered, and the
        genome gaps that ran both fills, from the results the launches left in res / gres."""
        d = b["d"]
        ns, ne, ng = b["ns"], b["ne"], b["ng"]
        nprob = ns + ne
        dev_index = np.array([lib.gmapdp_plan_dev_index(b["plan"], i) for i in range(nprob)], dtype=np.int64)
        gdev_index = np.array([lib.gmapdp_plan_genome_dev_index(b["plan"], j) for j in range(ng)], dtype=np.int64)
        npairs = np.zeros(nprob, dtype=np.int64)
        npairs[dev_index >= 0] = res["npairs"][dev_index[dev_index >= 0]]
        gnp = np.zeros(ng, dtype=np.int64)
        gsel = gdev_index >= 0
        gnp[gsel] = gres["npairs"][gdev_index[gsel]]
        # genome_gap_simple answered (dynprog_genome.c:3479): its result sets exonhead = new_rightgenomepos
        gsimple = np.zeros(ng, dtype=bool)
        gr = gres[gdev_index[gsel]]
        gsimple[gsel] = (gr["npairs"] > 0) & (gr["exonhead"] == gr["new_rightgenomepos"])
        _ = d
        return npairs, gnp, gsimple, gsel & ~gsimple

    def class_bytes(b, li, npairs, gnp, g_fills):
        """Algorithmic bytes and banded cells (genome-gap classes) of launch class li."""
        d = b["d"]
        sp, ep, gp = d["single"], d["end"], d["genome"]
        ns, ne = b["ns"], b["ne"]
        nprob = ns + ne
        m = np.zeros(b["info"][li][2], dtype=np.int32)
        lib.gmapdp_plan_launch_members(b["plan"], li, m.ctypes.data)
        if b["kinds"][li] not in (1, 5):  # every class but the genome-gap kernels (gg, uxg)
            rl = np.concatenate([sp["rlength"], np.minimum(ep["rlength"], 660)]).astype(np.int64)
            gl = np.concatenate([sp["glength"], np.minimum(ep["glength"], 2000)]).astype(np.int64)
            desc = np.concatenate([np.full(ns, gmapdp.PROBLEM_DTYPE.itemsize),
                                   np.full(ne, gmapdp.END_PROBLEM_DTYPE.itemsize)])
            return algorithmic_bytes(rl[m], gl[m], npairs[m], desc[m]), None
        j = m - nprob
        return (genome_algorithmic_bytes(gp[j], gnp[j], sprob_arena=b["kinds"][li] == 5),
                int(genome_cells(gp[j], g_fills[j]).sum()))

    def fetch_results(b):
        res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=gmapdp.RESULT_DTYPE)[:b["ngpu"]]
        gres = np.frombuffer(d_gres.cpu().numpy().tobytes(), dtype=gmapdp.GENOME_RESULT_DTYPE)[:b["nggpu"]]
        return res, gres

    def iso_launches(name, reps, with_bytes):
        """Every launch class of kernel `name`, one launch at a time on one stream, HIP events around each
        (on the stream it runs on); per dispatch: (ms, algorithmic bytes, cells).  A stage-2 kernel (S2_WHAT)
        runs alone over the scratch of a full untimed stage-2 run of the same block."""
        out = []
        if name in S2_WHAT:
            with torch.cuda.stream(stream):
                for rep in range(reps):
                    for b in B:
                        if b["oplan"] is None:
                            continue
                        orun(b, stream, 3)
                        e0, e1 = mk()
                        e0.record(stream)
                        orun(b, stream, S2_WHAT[name])
                        e1.record(stream)
                        torch.cuda.synchronize()
                        if "s2bytes" not in b:
                            b["s2bytes"] = stage2_bytes(b)
                        out.append((e0.elapsed_time(e1), b["s2bytes"][name], 0))
            return out
        with torch.cuda.stream(stream):
            for rep in range(reps):
                for b in B:
                    for li, nm in enumerate(b["names"]):
                        if nm != name:
                            continue
                        launch(b, li, stream)  # (the class's MaxEnt prologue, untimed)
                        e0, e1 = mk()
                        e0.record(stream)
                        launch(b, li, stream, kernel_only=True)  # the kernel alone, as rocprof times it
                        e1.record(stream)
                        torch.cuda.synchronize()
                        if with_bytes and rep == 0:
                            npairs, gnp, _, g_fills = class_outputs(b, *fetch_results(b))
                            b.setdefault("iso_bytes", {})[li] = class_bytes(b, li, npairs, gnp, g_fills)
                        nbytes, cells = b["iso_bytes"][li] if with_bytes else (b["bytes"][li], b["cells"][li])
                        out.append((e0.elapsed_time(e1), nbytes, cells or 0))
        return out


    def timed(steps, warmup, **kw):
        if not kw:  # the whole step (not a leg alone): GMAPDP_BENCH_PIPE applies
            kw = {"piped": True}
        with torch.cuda.stream(stream):
            for k in range(warmup):
                step(B[k % len(B)], **kw)
            torch.cuda.synchronize()
            evs = [{"oligo": mk(), "chain": mk(), "mx": mk(), "s2a": mk()[0], "s2b": mk()[0],
                    "dp": [mk() for _ in B[k % len(B)]["names"]]} for k in range(steps)]
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(steps):
                step(B[k % len(B)], ev=evs[k], **kw)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            elapsed = time.perf_counter() - t0
        if world > 1:
            elapsed = shard.max_over_ranks(elapsed, dist, device=dev)
        return elapsed, evs

    def stage2_bytes(b):
        """Algorithmic bytes of block b's stage-2 kernels, from its last run's seeding and
        chaining results."""
        op = b["d"]["oligo"]
        ores = np.zeros(len(op), dtype=gmapdp.OLIGO_RESULT_DTYPE)
        eng._check(lib.gmapdp_stage2_plan_seeding_results(eng.h, b["oplan"], C.c_void_p(stream.cuda_stream),
                                                          ores.ctypes.data), "gmapdp_stage2_plan_seeding_results")
        torch.cuda.synchronize()
        s2res = np.frombuffer(d_s2res.cpu().numpy().tobytes(), dtype=gmapdp.STAGE2_RESULT_DTYPE)[:len(op)]
        return stage2_algorithmic_bytes(op, ores, s2res)

    if args.iso_kernel:
        if args.iso_kernel in S2_WHAT:
            if not all(b["oplan"] is not None for b in B):
                raise SystemExit("bench: no Stage2_compute calls in this workload")
        elif not any(args.iso_kernel in b["names"] for b in B):
            raise SystemExit("bench: no launch class of %s in this workload" % args.iso_kernel)
        rows = iso_launches(args.iso_kernel, args.iso_reps, True)
        ms = [r[0] for r in rows]
        nbytes = float(np.mean([r[1] for r in rows]))
        if rank == 0:
            print(json.dumps({"iso_kernel": args.iso_kernel, "dispatches": len(rows), "ms_per_launch": float(np.mean(ms)),
                              "ms_each": [round(x, 3) for x in ms],
                              "ms_min": min(ms), "ms_max": max(ms), "algorithmic_bytes_per_launch": nbytes,
                              "achieved_gbs": nbytes / (np.mean(ms) * 1e-3) / 1e9,
                              "cells_per_launch": float(np.mean([r[2] for r in rows]))}), flush=True)
        for b in B:
            lib.gmapdp_plan_destroy(b["plan"])
            if b["oplan"] is not None:
                lib.gmapdp_stage2_plan_destroy(b["oplan"])
            if b["mplan"] is not None:
                lib.gmapdp_microexon_plan_destroy(b["mplan"])
        return

    # every block once before anything is timed: the context's grow-only scratch reaches its size
    with torch.cuda.stream(stream):
        for b in B:
            step(b)
    torch.cuda.synchronize()

    # ---- headline: Stage2_compute + every Dynprog_* call of a block per step ----
    progress("timing %d steps over %d blocks" % (args.steps, len(B)))
    elapsed, evs = timed(args.steps, args.warmup)
    progress("headline %.2f ms per step" % (elapsed / args.steps * 1e3))
    el_serial, _ = timed(args.steps, 1, piped=False)
    half = max(2, args.steps // 4)
    el_dp, _ = timed(half, 1, do_oligo=False)
    has_s2 = all(b["oplan"] is not None for b in B)
    el_o = s2_seed_ms = s2_chain_ms = None
    if has_s2:
        el_o, evs_o = timed(half, 1, do_dp=False)
        # stage 2 alone, split at the seeding / chaining boundary (HIP events on its stream)
        s2_seed_ms = float(np.mean([e["oligo"][0].elapsed_time(e["oligo"][1]) for e in evs_o]))
        s2_chain_ms = float(np.mean([e["oligo"][1].elapsed_time(e["chain"][1]) for e in evs_o]))

    # ---- per-launch times of the timed steps, by kernel template ----
    per_kernel = {}   # name -> [ms total, dispatches, algorithmic bytes total]

    def add(name, ms, nbytes, n=1):
        e = per_kernel.setdefault(name, [0.0, 0, 0])
        e[0] += ms
        e[1] += n
        e[2] += nbytes if nbytes is not None else 0

    # outputs and algorithmic bytes per launch class, per block (each block's outputs: re-run it once)
    checks = {"pairs": 0, "genome_gaps_bridged": 0, "genome_gap_simple": 0, "stage2_chained": 0, "stage2_results": 0,
              "stage2_path_pairs": 0, "microexon_candidates": 0, "microexons_found": 0, "reads": 0}
    cells_total = 0
    for b in B:
        with torch.cuda.stream(stream):
            step(b)
        torch.cuda.synchronize()
        d = b["d"]
        sp, ep, gp, op, mp = d["single"], d["end"], d["genome"], d["oligo"], d["microexon"]
        res, gres = fetch_results(b)
        s2res = np.frombuffer(d_s2res.cpu().numpy().tobytes(), dtype=gmapdp.STAGE2_RESULT_DTYPE)[:len(op)]
        mres = np.frombuffer(d_mres.cpu().numpy().tobytes(), dtype=gmapdp.MICROEXON_RESULT_DTYPE)[:len(mp)]
        # size-independent invariants of the step's outputs (the oracle parity of this same workload is
        # tests/test_gpu_bench_workload.py)
        assert np.all(res["npairs"] >= 0) and np.all(gres["npairs"] >= 0) and np.all(s2res["status"] >= 0)
        assert np.all(mres["ncandidates"] >= 0) and np.all(mres["cand_offset"] >= 0)
        npairs, gnp, gsimple, g_fills = class_outputs(b, res, gres)
        cells_total += dp_cells(sp, ep, gp, g_fills)
        b["bytes"], b["cells"] = zip(*[class_bytes(b, li, npairs, gnp, g_fills) for li in range(len(b["names"]))])
        if b["oplan"] is not None:
            b["s2bytes"] = stage2_bytes(b)
        checks["pairs"] += int(npairs.sum() + gnp.sum())
        checks["genome_gaps_bridged"] += int((gnp > 0).sum())
        checks["genome_gap_simple"] += int(gsimple.sum())
        checks["stage2_chained"] += int((s2res["status"] == 2).sum())
        checks["stage2_results"] += int(s2res["nresults"].sum())
        checks["stage2_path_pairs"] += int(s2res["npairs"].sum())
        checks["microexon_candidates"] += int(b["ncands"])
        checks["microexons_found"] += int((mres["npairs"] > 0).sum())
        checks["reads"] += args.reads
    for k, e in enumerate(evs):
        b = B[k % len(B)]
        for li, name in enumerate(b["names"]):
            add(name, e["dp"][li][0].elapsed_time(e["dp"][li][1]), b["bytes"][li])
        if b["oplan"] is not None:
            sb = b["s2bytes"]
            add(S2_SEED, e["oligo"][0].elapsed_time(e["oligo"][1]), sb[S2_SEED])
            add("gmapdp::s2a_kernel", e["oligo"][1].elapsed_time(e["s2a"]), sb["gmapdp::s2a_kernel"])
            add("gmapdp::s2b_kernel", e["s2a"].elapsed_time(e["s2b"]), sb["gmapdp::s2b_kernel"])
            add("gmapdp::s2c_kernel", e["s2b"].elapsed_time(e["chain"][1]), sb["gmapdp::s2c_kernel"])
        if b["mplan"] is not None:
            add("gmapdp::mx_search_kernel+gmapdp::mx_finish_kernel", e["mx"][0].elapsed_time(e["mx"][1]), None)
    # the dominant kernel: the largest in-step time among the single kernels (and the seeding pair)
    dominant = max((n for n in per_kernel if per_kernel[n][2] > 0), key=lambda n: per_kernel[n][0])
    dms, dn, dbytes = per_kernel[dominant]
    wl = workload_id(args)

    def kernel_roofline(name, reps):
        """`name`'s launches alone (every block, one at a time on one stream, HIP events) against its
        algorithmic bytes, with the committed PMC summary of this workload's step (traffic, VALU)."""
        rows = iso_launches(name, reps, False)
        n = len(rows)
        ms = sum(r[0] for r in rows) / n
        nbytes = sum(r[1] for r in rows) / n
        cells = sum(r[2] for r in rows) / n
        ach = nbytes / (ms * 1e-3) / 1e9
        pmc, psrc = pmc_entry(name, wl)
        traffic = pmc["hbm_bytes_per_dispatch"] if pmc else None
        valu = pmc["sq_SQ_INSTS_VALU_sum_avg"] if pmc else None
        return {"kernel": name, "dispatches_timed": n, "ms_per_launch": ms, "algorithmic_bytes_per_launch": nbytes,
                "achieved": ach, "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_over_algorithmic": traffic / nbytes if traffic and nbytes else None, "traffic_source": psrc,
                "valu_insts_per_launch": valu,
                "valu_issue_frac": valu / (VALU_WAVE_INSTR_PEAK * ms * 1e-3) if valu else None,
                "rocprof_avg_ms_in_step_committed": pmc["avg_duration_ns"] / 1e6 if pmc and pmc.get("avg_duration_ns")
                else None,
                "ms_per_launch_in_step": per_kernel[name][0] / per_kernel[name][1] if name in per_kernel else None,
                "cells_per_launch": cells}

    # ---- the dominant kernel alone (its launches of every block, one at a time on one stream) ----
    dom = kernel_roofline(dominant, 3)
    kms, kbytes, kcells, ach = dom["ms_per_launch"], dom["algorithmic_bytes_per_launch"], dom["cells_per_launch"], \
        dom["achieved"]
    traffic, psrc, valu = dom["traffic"], dom["traffic_source"], dom["valu_insts_per_launch"]
    prof_ms = dom["rocprof_avg_ms_in_step_committed"]
    iso, isrc = iso_entry(dominant, wl)
    iso_prof_ms = iso["avg_duration_ns"] / 1e6 if iso else None
    # beside it: the stage-2 kernels (the step's long pole) and the largest DP class
    others = [n for n in list(S2_WHAT) + [max((n for n in per_kernel if n not in S2_WHAT),
                                              key=lambda n: per_kernel[n][0], default=None)]
              if n and n != dominant and n in per_kernel]
    roofline_others = [kernel_roofline(n, 1) for n in others]
    # the chaining as one operation: its three kernels' traffic and time against the bytes
    # a fused chaining would move (no s2a -> s2b -> s2c intermediates)
    chain = {r["kernel"]: r for r in roofline_others if r["kernel"] in ("gmapdp::s2a_kernel", "gmapdp::s2b_kernel",
                                                                      "gmapdp::s2c_kernel")}
    chaining_fused = None
    if len(chain) == 3 and all("s2bytes" in bb for bb in B):
        fb = float(np.mean([bb["s2bytes"][CHAIN_FUSED] for bb in B]))
        tr = [r["traffic"] for r in chain.values()]
        ms3 = sum(r["ms_per_launch"] for r in chain.values())
        chaining_fused = {"kernels": sorted(chain), "ms_alone_per_block": ms3, "fused_algorithmic_bytes_per_block": fb,
                          "traffic_per_block": sum(tr) if all(t is not None for t in tr) else None,
                          "traffic_over_fused": sum(tr) / fb if all(t is not None for t in tr) and fb else None,
                          "achieved_fused": fb / (ms3 * 1e-3) / 1e9, "frac_fused": fb / (ms3 * 1e-3) / 1e9 / HBM_PEAK_GBS}

    # ---- PCIe: one block's inputs up and outputs down through pinned host memory (outside the step) ----
    b = B[0]
    d = b["d"]
    # (the splice and microexon probabilities are computed on the device: no probability crosses PCIe)
    up = d["q"].nbytes + d["oq"].nbytes + sum(d[k].nbytes for k in ("single", "end", "genome", "oligo", "microexon"))
    # the outputs as produced: results, the DP and microexon pairs, the stage-2 results and path pairs
    down = int(32 * b["ngpu"] + 72 * b["nggpu"] + 16 * checks["pairs"] / len(B) + 32 * len(d["oligo"])
               + 20 * checks["stage2_path_pairs"] / len(B))
    h_up = torch.empty(up, dtype=torch.uint8, pin_memory=True)
    h_down = torch.empty(down, dtype=torch.uint8, pin_memory=True)
    g_up = torch.empty(up, dtype=torch.uint8, device=dev)
    g_down = torch.empty(down, dtype=torch.uint8, device=dev)
    pcie_ms = []
    with torch.cuda.stream(stream):
        for _ in range(4):
            e0, e1 = mk()
            e0.record(stream)
            g_up.copy_(h_up, non_blocking=True)
            h_down.copy_(g_down, non_blocking=True)
            e1.record(stream)
            torch.cuda.synchronize()
            pcie_ms.append(e0.elapsed_time(e1))
    pcie_ms = float(np.median(pcie_ms[1:]))
    up_ms = []
    with torch.cuda.stream(stream):
        for _ in range(4):
            e0, e1 = mk()
            e0.record(stream)
            g_up.copy_(h_up, non_blocking=True)
            e1.record(stream)
            torch.cuda.synchronize()
            up_ms.append(e0.elapsed_time(e1))
    up_ms = float(np.median(up_ms[1:]))
    del h_up, h_down, g_up, g_down

    # ---- the compact pair stream: block b's DP pairs as run-length ops
    # (gmapdp_plan_compact_pairs), copied down with the results and the stage-2 outputs, then expanded on the
    # host (gmapdp_expand_pairs, 16 threads) and checked against the records themselves ----
    compact = None
    with torch.cuda.stream(stream):
        step(b)
        torch.cuda.synchronize()
        nprob = b["ngpu"] + b["nggpu"]
        d_off = torch.empty(nprob + 1, dtype=torch.int64, device=dev)
        d_cmp = torch.empty(max(int(lib.gmapdp_plan_compact_bound(b["plan"])), 16), dtype=torch.uint8, device=dev)
        # stage 2's path pairs too (gmapdp_stage2_plan_compact_pairs: one list per path record)
        has_s2 = b["oplan"] is not None
        if has_s2:
            pcap = C.c_size_t()
            s2bound = int(lib.gmapdp_stage2_plan_compact_bound(b["oplan"], C.byref(pcap)))
            d_s2off = torch.empty(pcap.value + 1, dtype=torch.int64, device=dev)
            d_s2cmp = torch.empty(max(s2bound, 16), dtype=torch.uint8, device=dev)
        cms = []
        for _ in range(3):
            e0, e1 = mk()
            e0.record(stream)
            eng._check(lib.gmapdp_plan_compact_pairs(eng.h, b["plan"], C.c_void_p(d_res.data_ptr()),
                                                     C.c_void_p(d_pairs.data_ptr()), C.c_void_p(d_cmp.data_ptr()),
                                                     C.c_void_p(d_off.data_ptr()), C.c_void_p(stream.cuda_stream)),
                       "gmapdp_plan_compact_pairs")
            if has_s2:
                eng._check(lib.gmapdp_stage2_plan_compact_pairs(eng.h, b["oplan"], C.c_void_p(d_s2cmp.data_ptr()),
                                                                C.c_void_p(d_s2off.data_ptr()),
                                                                C.c_void_p(stream.cuda_stream)),
                           "gmapdp_stage2_plan_compact_pairs")
            e1.record(stream)
            torch.cuda.synchronize()
            cms.append(e0.elapsed_time(e1))
        offs = d_off.cpu().numpy().view(np.uint64)
        nbytes = int(offs[-1])
        s2same, s2bytes, s2expand_ms, s2records, npaths = True, 0, 0.0, 0, 0
        if has_s2:
            s2r = np.zeros(len(b["d"]["oligo"]), dtype=gmapdp.STAGE2_RESULT_DTYPE)
            pn, qn = C.c_size_t(), C.c_size_t()
            rc = lib.gmapdp_stage2_plan_fetch(eng.h, b["oplan"], C.c_void_p(d_s2res.data_ptr()),
                                              C.c_void_p(stream.cuda_stream), s2r.ctypes.data, None, 0, None, 0,
                                              C.byref(pn), C.byref(qn))
            if rc not in (0, -6):
                eng._check(rc, "gmapdp_stage2_plan_fetch")
            s2paths = np.zeros(max(pn.value, 1), dtype=gmapdp.PATH_DTYPE)
            s2pairs = np.zeros(max(qn.value, 1), dtype=gmapdp.PATH_PAIR_DTYPE)
            eng._check(lib.gmapdp_stage2_plan_fetch(eng.h, b["oplan"], C.c_void_p(d_s2res.data_ptr()),
                                                    C.c_void_p(stream.cuda_stream), s2r.ctypes.data,
                                                    s2paths.ctypes.data, len(s2paths), s2pairs.ctypes.data,
                                                    len(s2pairs), C.byref(pn), C.byref(qn)), "gmapdp_stage2_plan_fetch")
            npaths = int(pn.value)
            s2offs = d_s2off[:npaths + 1].cpu().numpy().view(np.uint64)
            s2bytes = int(s2offs[-1])
            s2stream = d_s2cmp[:max(s2bytes, 1)].cpu().numpy()
            t0 = time.perf_counter()
            s2exp = gmapdp.expand_path_pairs(s2stream, s2offs, s2paths[:npaths], len(s2pairs), nthreads=16)
            s2expand_ms = (time.perf_counter() - t0) * 1e3
            pc = np.maximum(s2paths[:npaths]["npairs"].astype(np.int64), 0)
            pidx = np.repeat(s2paths[:npaths]["pair_offset"], pc) + (np.arange(int(pc.sum()))
                                                                      - np.repeat(np.cumsum(pc) - pc, pc))
            s2same = bool(np.array_equal(s2exp[pidx], s2pairs[pidx]))
            s2records = int(pc.sum())
            del d_s2cmp, s2exp, s2pairs, s2stream
        # the rest of the outputs as records: the DP results and stream offsets, the stage-2 results, path
        # records and stream offsets
        other = int(32 * b["ngpu"] + 72 * b["nggpu"] + 8 * (nprob + 1) + 32 * len(b["d"]["oligo"])
                    + (16 * npaths + 8 * (npaths + 1) if has_s2 else 0))
        cdown = nbytes + s2bytes + other
        h_c = torch.empty(cdown, dtype=torch.uint8, pin_memory=True)
        g_c = torch.empty(cdown, dtype=torch.uint8, device=dev)
        down_ms = []
        for _ in range(4):
            e0, e1 = mk()
            e0.record(stream)
            h_c.copy_(g_c, non_blocking=True)
            e1.record(stream)
            torch.cuda.synchronize()
            down_ms.append(e0.elapsed_time(e1))
        stream_host = d_cmp[:max(nbytes, 1)].cpu().numpy()
        res_h, gres_h = fetch_results(b)
        npc = np.concatenate([res_h["npairs"], gres_h["npairs"]]).astype(np.int32)
        poff = np.concatenate([res_h["pair_offset"], gres_h["pair_offset"]]).astype(np.int64)
        t0 = time.perf_counter()
        exp = gmapdp.expand_pairs(stream_host, offs, npc, poff, b["cap"], nthreads=16)
        expand_ms = (time.perf_counter() - t0) * 1e3
        allp = np.frombuffer(d_pairs[:16 * b["cap"]].cpu().numpy().tobytes(), dtype=gmapdp.PAIR_DTYPE)
        cnt = np.maximum(npc.astype(np.int64), 0)
        idx = np.repeat(poff, cnt) + (np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt))
        same = bool(np.array_equal(exp[idx], allp[idx])) and s2same
        del h_c, g_c, d_cmp, allp, exp
        compact = {"records": int(cnt.sum()), "stream_bytes": nbytes, "bytes_per_record": nbytes / max(int(cnt.sum()), 1),
                   "stage2_path_pair_records": s2records, "stage2_stream_bytes": s2bytes,
                   "stage2_bytes_per_record": s2bytes / max(s2records, 1),
                   "compact_kernels_ms": float(np.median(cms[1:])), "pcie_bytes_down": cdown,
                   "pcie_down_ms": float(np.median(down_ms[1:])), "pcie_up_ms": up_ms,
                   "host_expand_ms_16_threads": expand_ms, "stage2_host_expand_ms_16_threads": s2expand_ms,
                   "expanded_equals_records": same}
        compact["pcie_ms_per_step"] = compact["pcie_up_ms"] + compact["compact_kernels_ms"] + compact["pcie_down_ms"]
        progress("compact pair stream: %d DP records in %d bytes, %d stage-2 path pairs in %d bytes, expanded %s"
                 % (compact["records"], nbytes, s2records, s2bytes, "identically" if same else "DIFFERENTLY"))

    # ---- pipelined: the loop a deployment runs -- each step followed by its compaction on the compute
    # stream, and on a copy stream (the DMA engines) the next block's inputs up and the finished step's
    # compact outputs down, double-buffered so the copies overlap the next step.  Byte counts per step are
    # the ones measured above (block b's inputs, its compact stream plus results); the host's expansion
    # (the consumer's pass over the pairs) is not counted, as in the serial figure ----
    pipelined = None
    if compact is not None and same and world == 1 and has_s2:
        # (the copies go on the microexon side stream: a fifth stream would share a hardware queue with one of
        # the step's four and wait behind its kernels -- GPU_MAX_HW_QUEUES is 4 -- serialising the copies)
        cstream = sides[-1]
        dbound = max(int(lib.gmapdp_plan_compact_bound(x["plan"])) for x in B)
        pc_, s2max, pmax = C.c_size_t(), 16, 0
        for x in B:
            s2max = max(s2max, int(lib.gmapdp_stage2_plan_compact_bound(x["oplan"], C.byref(pc_))))
            pmax = max(pmax, int(pc_.value))
        nmax = max(x["ngpu"] + x["nggpu"] for x in B)
        slots = [{"cmp": torch.empty(max(dbound, cdown, 16), dtype=torch.uint8, device=dev),
                  "off": torch.empty(nmax + 1, dtype=torch.int64, device=dev),
                  "s2cmp": torch.empty(s2max, dtype=torch.uint8, device=dev),
                  "s2off": torch.empty(pmax + 1, dtype=torch.int64, device=dev),
                  "h_down": torch.empty(cdown, dtype=torch.uint8, pin_memory=True),
                  "h_up": torch.empty(up, dtype=torch.uint8, pin_memory=True),
                  "g_up": torch.empty(up, dtype=torch.uint8, device=dev),
                  "arrived": torch.cuda.Event(), "done": torch.cuda.Event()} for _ in range(2)]

        def pstep(k):
            bb, sl, nx = B[k % len(B)], slots[k % 2], slots[(k + 1) % 2]
            with torch.cuda.stream(cstream):  # the next block's inputs, once step k - 1 released its slot
                if k > 0:
                    cstream.wait_event(nx["done"])
                nx["g_up"].copy_(nx["h_up"], non_blocking=True)
                nx["arrived"].record(cstream)
            with torch.cuda.stream(stream):
                stream.wait_event(sl["arrived"])
                step(bb)
                eng._check(lib.gmapdp_plan_compact_pairs(eng.h, bb["plan"], C.c_void_p(d_res.data_ptr()),
                                                         C.c_void_p(d_pairs.data_ptr()), C.c_void_p(sl["cmp"].data_ptr()),
                                                         C.c_void_p(sl["off"].data_ptr()), C.c_void_p(stream.cuda_stream)),
                           "gmapdp_plan_compact_pairs")
                eng._check(lib.gmapdp_stage2_plan_compact_pairs(eng.h, bb["oplan"], C.c_void_p(sl["s2cmp"].data_ptr()),
                                                                C.c_void_p(sl["s2off"].data_ptr()),
                                                                C.c_void_p(stream.cuda_stream)),
                           "gmapdp_stage2_plan_compact_pairs")
                sl["done"].record(stream)
            with torch.cuda.stream(cstream):  # this step's outputs down
                cstream.wait_event(sl["done"])
                sl["h_down"].copy_(sl["cmp"][:cdown], non_blocking=True)

        with torch.cuda.stream(cstream):
            slots[0]["g_up"].copy_(slots[0]["h_up"], non_blocking=True)
            slots[0]["arrived"].record(cstream)
        for k in range(args.warmup):
            pstep(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.warmup, args.warmup + args.steps):
            pstep(k)
        torch.cuda.synchronize()
        pel = time.perf_counter() - t0
        pipelined = {"reads_per_s": args.reads * args.steps / pel, "ms_per_step": pel / args.steps * 1e3,
                     "steps": args.steps, "bytes_up_per_step": up, "bytes_down_per_step": cdown,
                     "note": "compute stream: step + both compactions; copy stream: inputs up one step ahead, "
                             "compact outputs down one step behind, double-buffered"}
        del slots
        progress("pipelined with PCIe: %.2f ms per step" % pipelined["ms_per_step"])

    ms_step = elapsed / args.steps * 1e3
    reads_total = args.reads * world * args.steps
    nsub = {k: int(np.mean([len(b["d"][k]) for b in B])) for k in ("oligo", "single", "end", "genome", "microexon")}
    nsub_end3 = float(np.mean([int((b["d"]["end"]["end3p"] != 0).sum()) for b in B]))
    nsub_end5 = nsub["end"] - nsub_end3
    out = {
        "metric": METRIC,
        "value": reads_total / elapsed,
        "unit": "reads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16/int8 saturating (SIMD-build semantics)" if args.simd else "int32",
        "data": "synthetic",
        "config": {"workload": "configs[%d]: synthetic %d-nt %s reads (%d exons x %d nt, %g %% subs, %g %% indels) vs a "
                               "%s-layout i.i.d. genome (%d chromosomes, %d nt, universal coordinates to %d): per read "
                               "%.3g Stage2_compute calls (seeding + chaining, locus +- %d-nt windows) + %.1f "
                               "Dynprog_single_gap + %.1f "
                               "Dynprog_end5_gap + %.1f Dynprog_end3_gap + %.1f Dynprog_genome_gap + %.1f "
                               "Dynprog_microexon_int (%s semantics)%s; %d distinct blocks of %d reads cycled per rank; "
                               "inputs HBM-resident; host stages 1/3 not in the step"
                               % (args.config, shape.readlength, "Iso-Seq-style" if args.config == 4 else "cDNA",
                                  shape.exons, shape.exlen, 100 * shape.subs, 100 * shape.indel, gname,
                                  len(layout.lens), layout.total, layout.total - 1, nsub["oligo"] / args.reads,
                                  shape.pad, nsub["single"] / args.reads,
                                  nsub_end5 / args.reads, nsub_end3 / args.reads, nsub["genome"] / args.reads,
                                  nsub["microexon"] / args.reads, "gmap.avx2" if args.simd else "nosimd",
                                  " -- Dynprog_single + Dynprog_end only, as configs[1] names it" if args.config == 1
                                  else "", len(B), args.reads),
                   "genome": gname, "reads_per_step_per_gpu": args.reads, "blocks_per_rank": len(B),
                   "call_mix_source": shape.source,
                   "subproblems_per_step_per_gpu": {"stage2_compute": nsub["oligo"], "single": nsub["single"],
                                                    "end": nsub["end"], "genome": nsub["genome"],
                                                    "microexon": nsub["microexon"]},
                   "banded_cells_per_step_per_gpu": cells_total // len(B),
                   "parallelism": "dp%d (reads sharded by rank, --part=r/%d over read blocks; genome replicated)"
                                  % (world, world)},
        "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": psrc, "kernel": dominant,
                     "kernel_ms_per_launch": kms, "algorithmic_bytes_per_launch": kbytes,
                     "timing": "HIP events around each of the kernel's launches run alone on one stream (%d "
                               "dispatches, after the timed region); in the timed steps, which share the CUs "
                               "four streams wide, its launches average %.3f ms" % (dom["dispatches_timed"], dms / dn),
                     "traffic_over_algorithmic": dom["traffic_over_algorithmic"], "workload_id": wl,
                     "kernel_ms_per_launch_in_step": dms / dn, "rocprof_avg_ms_committed": prof_ms,
                     "rocprof_isolated": {"source": isrc, "avg_ms": iso_prof_ms,
                                          "dispatches": iso["dispatches"] if iso else None,
                                          "algorithmic_bytes_per_launch": iso.get("algorithmic_bytes_per_launch")
                                          if iso else None,
                                          "frac": (iso["algorithmic_bytes_per_launch"] / (iso_prof_ms * 1e-3) / 1e9
                                                   / HBM_PEAK_GBS) if iso and iso.get("algorithmic_bytes_per_launch")
                                          else None,
                                          "live_over_rocprof": kms / iso_prof_ms if iso_prof_ms else None,
                                          "note": "rocprofv3 --kernel-trace --stats of `bench.py --iso-kernel <kernel>` "
                                                  "(the same isolated launches this line times with HIP events)"},
                     "step_algorithmic_gbs": sum(e[2] for e in per_kernel.values()) / args.steps
                                             / (ms_step * 1e-3) / 1e9,
                     "valu": {"insts_per_launch": valu,
                              "issue_frac": valu / (VALU_WAVE_INSTR_PEAK * kms * 1e-3) if valu else None,
                              "peak_wave_insts_per_s": VALU_WAVE_INSTR_PEAK,
                              "source": psrc},
                     "int_ops": {"cells_per_launch": kcells, "ops_per_cell": OPS_PER_CELL,
                                 "frac": OPS_PER_CELL * kcells / (INT_OPS_PEAK * kms * 1e-3) if kcells else None,
                                 "peak_ops_per_s": INT_OPS_PEAK,
                                 # issued lanes (VALU wave-instructions x 64) per algorithmic
                                 # int op of the launch -- the instruction overhead the issue fraction hides
                                 "lane_slots_per_op": 64.0 * valu / (OPS_PER_CELL * kcells) if valu and kcells
                                 else None,
                                 "note": "genome-gap fills counted only where genome_gap_simple did not answer"},
                     "note": "integer VALU/LDS/latency-bound DP and a serial stage-2 sweep (SURVEY §8d); the HBM "
                             "roofline is reported as required, the VALU issue fraction (and for DP fills the "
                             "algorithmic int-op fraction) are the binding bounds (BASELINE.md §3(i))"},
        "roofline_other_kernels": roofline_others,
        "chaining_fused": chaining_fused,
        "gcups": cells_total / len(B) * world * args.steps / elapsed / 1e9,
        "step_split_ms": {"stage2_alone": el_o / half * 1e3 if el_o is not None else None,
                          "stage2_alone_seeding": s2_seed_ms,
                          "stage2_alone_chaining": s2_chain_ms, "dynprog_alone": el_dp / half * 1e3,
                          "together": ms_step, "together_serial": el_serial / args.steps * 1e3,
                          "pipelined_blocks": pipe},
        "block_runs": dict(block_runs),
        "launch_classes": sorted(({"kernel": n, "dispatches": e[1], "ms_per_step": round(e[0] / args.steps, 4)}
                                  for n, e in per_kernel.items()), key=lambda x: -x["ms_per_step"]),
        # the host's per-block planning (gmapdp_plan_create_all, gmapdp_stage2_plan_create: 16 host threads),
        # the median block's (the first block also pays the process's first device allocations: listed apart)
        "host": {"plan_ms_per_block": float(np.median(plan_ms)), "stage2_plan_ms_per_block": float(np.median(oplan_ms)),
                 "plan_ms_first_block": plan_ms[0], "stage2_plan_ms_first_block": oplan_ms[0],
                 "plan_threads": int(os.environ.get("GMAPDP_PLAN_THREADS", "16")),
                 "setup_s": t_gen},
        "checks": {"pairs_per_read": checks["pairs"] / checks["reads"],
                   "genome_gaps_bridged": checks["genome_gaps_bridged"],
                   "genome_gap_simple": checks["genome_gap_simple"],
                   "stage2_chained": checks["stage2_chained"], "stage2_results": checks["stage2_results"],
                   "stage2_path_pairs_per_read": checks["stage2_path_pairs"] / checks["reads"],
                   "microexon_candidates": checks["microexon_candidates"],
                   "microexons_found": checks["microexons_found"], "reads_checked": checks["reads"]},
    }
    # shard record: every rank's blocks, checked disjoint and complete
    out["shard"] = shard.gather_blocks(mine, [b["d"]["reads"] for b in B], dist if world > 1 else None)
    rank_line = {"rank": rank, "world_size": dist.get_world_size() if world > 1 else 1,
                 "backend": dist.get_backend() if world > 1 else None, "device": local,
                 "blocks": mine, "ms_per_step_local": ms_step}
    err_line(json.dumps({"rank_line": rank_line}))
    for b in B:
        lib.gmapdp_plan_destroy(b["plan"])
        if b["oplan"] is not None:
            lib.gmapdp_stage2_plan_destroy(b["oplan"])
        if b["mplan"] is not None:
            lib.gmapdp_microexon_plan_destroy(b["mplan"])
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config in (1, 2) and not args.simd:
        progress("CPU baselines")
        cb = cpu_baselines(args.mix, args.config)
        # the faster of the reference's two builds is the baseline; the other is kept beside it
        done = sorted((c for c in cb.values() if c), key=lambda c: -c["value"])
        out["cpu_baseline"] = done[0] if done else None
        out["cpu_baseline_other_build"] = done[1] if len(done) > 1 else None
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        out["like_for_like"] = like_for_like(out, pcie_ms, up, down, compact, pipelined)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
