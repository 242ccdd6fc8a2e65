"""bench.py -- MI355X Dynprog engine throughput (BASELINE.json metric, configs[1]).

Workload (configs[1]: "100k synthetic 2-kb cDNA vs human chr22, 1xMI355X,
Dynprog_single + Dynprog_end only"): a chr22-length (50,818,468 nt) i.i.d.
genome (seed 22) packed in the reference's .genomecomp format and resident
in HBM, and the stream of Dynprog_single_gap sub-problems that GMAP issues
for 2-kb reads (43.7 calls per read): query slices of the
genome with 2 % substitutions and occasional 1-3 nt indels, GMAP's default
extraband 6 / wide band, MEDQ/LOWQ defect rates.  One "step" = one pass of
the engine over the sub-problems of --reads reads (all inputs already in
HBM; host->device copies are outside the timed region).

value = reads whose sub-problems were processed per second, whole job (all
ranks).  This is the DP-engine throughput of the path, not end-to-end GMAP
(stage 1/2/3 orchestration stays on the host; DESIGN.md "Measurement").
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

CHR22_LEN = 50_818_468
CALLS_PER_READ = 43.7          # Dynprog_single_gap calls per 2-kb read
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
COMPL = np.zeros(256, dtype=np.uint8)
for a, b in zip(b"ACGTN", b"TGCAN"):
    COMPL[a] = b


def make_genome(seed=22, length=CHR22_LEN):
    rng = np.random.default_rng(seed)
    return np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=length, dtype=np.uint8)]


def make_problems(genome, nprob, seed):
    """Vectorised GMAP-shaped single-gap sub-problems (see module docstring)."""
    import gmapdp
    rng = np.random.default_rng(seed)
    glen = len(genome)
    g = np.clip(rng.gamma(3.0, 40.0, size=nprob).astype(np.int64), 1, 640)
    d = np.where(rng.random(nprob) < 0.15, rng.integers(-3, 4, size=nprob), 0)
    d = np.where(g + d < 1, 0, d)
    r = np.clip(g + d, 1, 660)
    d = r - g
    watson = rng.random(nprob) < 0.5
    goff = rng.integers(1, glen - 700, size=nprob)
    # segment characters as the engine sees them
    seg_off = np.concatenate([[0], np.cumsum(g)])
    pid = np.repeat(np.arange(nprob), g)
    i = np.arange(seg_off[-1]) - seg_off[pid]
    gpos = np.where(watson[pid], goff[pid] + i, glen - goff[pid] - i)
    seg = genome[gpos]
    seg = np.where(watson[pid], seg, COMPL[seg])
    # query = segment with one indel of |d| at position a, then 2 % substitutions
    q_off = np.concatenate([[0], np.cumsum(r)])
    qpid = np.repeat(np.arange(nprob), r)
    j = np.arange(q_off[-1]) - q_off[qpid]
    a = (rng.random(nprob) * np.maximum(r - np.maximum(d, 0), 1)).astype(np.int64)
    dd, aa = d[qpid], a[qpid]
    src = np.where((dd < 0) & (j >= aa), j - dd, j)                      # deletion: skip -d bases
    ins = (dd > 0) & (j >= aa) & (j < aa + dd)
    src = np.where((dd > 0) & (j >= aa + dd), j - dd, src)               # insertion: shift back
    src = np.clip(src, 0, g[qpid] - 1)
    q = seg[seg_off[qpid] + src]
    rnd = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=q.size, dtype=np.uint8)]
    q = np.where(ins | (rng.random(q.size) < 0.02), rnd, q).astype(np.uint8)
    probs = np.zeros(nprob, dtype=gmapdp.PROBLEM_DTYPE)
    probs["qoff"] = q_off[:-1]
    probs["rlength"] = r
    probs["glength"] = g
    probs["roffset"] = rng.integers(0, 1800, size=nprob)
    probs["goffset"] = goff
    probs["chroffset"] = 0
    probs["chrhigh"] = glen
    probs["flags"] = (watson.astype(np.int32) * gmapdp.WATSON | (rng.random(nprob) < 0.5) * gmapdp.JUMP_LATE |
                      gmapdp.WIDEBAND)
    probs["genestrand"] = 0
    probs["extraband"] = 6
    probs["defect_rate"] = np.where(rng.random(nprob) < 0.7, 0.02, 0.01)
    probs["dynprogindex"] = rng.integers(1, 50, size=nprob) * np.where(rng.random(nprob) < 0.5, 1, -1)
    return probs, q


def algorithmic_bytes(probs, npairs):
    """HBM bytes the path must move per launch (DESIGN.md "Roofline"): problem
    descriptor (56 B) + query and upper-cased query (2 x rlength) + the packed
    genome blocks covering the segment (12 B per 32 nt) + result (32 B) + one
    16-B Pair record per emitted pair."""
    g = probs["glength"].astype(np.int64)
    return int((56 + 2 * probs["rlength"].astype(np.int64) + 12 * ((g + 62) // 32) + 32).sum()
               + 16 * int(npairs.sum()))


def banded_cells(probs):
    import gmapdp
    lib = gmapdp.load_library()
    lb, ub = C.c_int(), C.c_int()
    r = probs["rlength"].astype(np.int64)
    g = probs["glength"].astype(np.int64)
    # widebandp, extraband 6: W = |g - r| + 13; cells ~ g * W clipped by r (exact count not needed)
    W = np.abs(g - r) + 2 * probs["extraband"].astype(np.int64) + 1
    return int(np.minimum(W, r + 1).dot(g))


def cpu_baseline(probs, q, genome, budget_s=12.0):
    """Time the reference itself (oracle/_ref/librefdp_nosimd.so, 1 core) on a
    bounded prefix of the same problem stream; fall back to the repo's oracle
    port if the reference objects are absent."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "librefdp_nosimd.so")
    qb = q.tobytes()
    if os.path.exists(ref_so):
        lib = C.CDLL(ref_so)
        lib.refh_init(0, 0, 0)
        gb = genome.tobytes()
        lib.refh_set_genome(gb, len(gb))
        fn = lib.refh_single_gap_batch
        fn.restype = C.c_long
        fn.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_char_p]
        kind = "reference"
    else:
        return None
    n, done, t_total = 256, 0, 0.0
    while t_total < budget_s and done + n <= len(probs):
        sub = np.ascontiguousarray(probs[done:done + n])
        t0 = time.perf_counter()
        fn(sub.ctypes.data, n, qb, qb)
        t_total += time.perf_counter() - t0
        done += n
        n = min(n * 2, 8192)
    per_s = done / t_total
    return {"value": per_s / CALLS_PER_READ, "unit": "reads/s", "cores": 1, "kind": kind,
            "sample": "%d Dynprog_single_gap problems of the same stream (%.1f s, 1 thread, gmap nosimd "
                      "objects via oracle/_ref); %.0f problems/s / %.1f calls per read" %
                      (done, t_total, per_s, CALLS_PER_READ)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=10000, help="reads per step per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import gmapdp

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    genome = make_genome()
    nprob = int(round(args.reads * CALLS_PER_READ))
    probs, q = make_problems(genome, nprob, seed=1000 + rank)

    eng = gmapdp.Engine(local)
    eng.set_genome(genome.tobytes())
    lib = eng.lib
    host_res = np.zeros(nprob, dtype=gmapdp.RESULT_DTYPE)
    plan = C.c_void_p()
    eng._check(lib.gmapdp_plan_single(eng.h, probs.ctypes.data, nprob, host_res.ctypes.data, C.byref(plan)),
               "gmapdp_plan_single")
    ngpu = lib.gmapdp_plan_gpu_problems(plan)
    cap = lib.gmapdp_plan_pair_capacity(plan)
    d_q = torch.from_numpy(q).to(dev)
    d_res = torch.zeros(max(ngpu, 1) * 32, dtype=torch.uint8, device=dev)
    d_pairs = torch.empty(max(cap, 1) * 16, dtype=torch.uint8, device=dev)
    nl = lib.gmapdp_plan_nlaunches(plan)
    info = []
    for li in range(nl):
        R, dl, cnt, lds = C.c_int(), C.c_int(), C.c_int(), C.c_size_t()
        lib.gmapdp_plan_launch_info(plan, li, C.byref(R), C.byref(dl), C.byref(cnt), C.byref(lds))
        info.append((R.value, dl.value, cnt.value, lds.value))
    # the kernel template each launch runs; the dominant kernel is the template with most problems
    kname = ["single_gap_kernel<R=%d,dirs_lds=%d>" % (i[0], i[1]) for i in info]
    per_kernel = {}
    for li in range(nl):
        per_kernel.setdefault(kname[li], []).append(li)
    dominant = max(per_kernel, key=lambda k: sum(info[li][2] for li in per_kernel[k]))
    stream = torch.cuda.Stream(dev)  # a real (non-null) stream: the events below see exactly these launches

    def step(ev=None):
        for li in range(nl):
            if ev is not None:
                ev[li][0].record(stream)
            eng._check(lib.gmapdp_plan_run_launch(eng.h, plan, li, C.c_void_p(d_q.data_ptr()),
                                                  C.c_void_p(d_q.data_ptr()), C.c_void_p(d_res.data_ptr()),
                                                  C.c_void_p(d_pairs.data_ptr()), C.c_void_p(stream.cuda_stream)),
                       "gmapdp_plan_run_launch")
            if ev is not None:
                ev[li][1].record(stream)

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nl)]
               for _ in range(args.steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(evs[k])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    launch_ms = [sum(evs[k][li][0].elapsed_time(evs[k][li][1]) for k in range(args.steps)) / args.steps
                 for li in range(nl)]

    # results of the last pass (for algorithmic byte accounting)
    res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=gmapdp.RESULT_DTYPE)[:ngpu]
    dev_index = np.array([lib.gmapdp_plan_dev_index(plan, i) for i in range(nprob)])
    gpu_mask = dev_index >= 0
    npairs = np.zeros(nprob, dtype=np.int64)
    npairs[gpu_mask] = res["npairs"][dev_index[gpu_mask]]
    dom_launches = per_kernel[dominant]
    dom_bytes_total = 0
    for li in dom_launches:
        members = np.zeros(info[li][2], dtype=np.int32)
        lib.gmapdp_plan_launch_members(plan, li, members.ctypes.data)
        dom_bytes_total += algorithmic_bytes(probs[members], npairs[members])
    dom_ms = sum(launch_ms[li] for li in dom_launches) / len(dom_launches)   # average dispatch duration
    dom_bytes = dom_bytes_total / len(dom_launches)                          # average bytes per dispatch
    step_bytes = algorithmic_bytes(probs[gpu_mask], npairs[gpu_mask])
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9

    reads_total = args.reads * world * args.steps
    value = reads_total / elapsed
    out = {
        "metric": "aligned cDNA reads/sec (2 kb, GRCh38) at 1/2/4/8 MI355X; DP HBM GB/s vs peak",
        "value": value,
        "unit": "reads/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {"workload": "configs[1]: synthetic 2-kb cDNA Dynprog_single_gap sub-problem stream vs a "
                               "chr22-length i.i.d. genome (seed 22), %.1f calls/read; DP engine only "
                               "(Dynprog_end on GPU not yet in this round)" % CALLS_PER_READ,
                   "reads_per_step_per_gpu": args.reads, "subproblems_per_step_per_gpu": nprob,
                   "banded_cells_per_step_per_gpu": banded_cells(probs),
                   "parallelism": "dp%d (reads sharded by rank, genome replicated)" % world,
                   "launch_classes": info},
        "gcups": banded_cells(probs) * world * args.steps / elapsed / 1e9,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": dominant, "dispatches_per_step": len(dom_launches),
                     "kernel_ms_per_launch": dom_ms, "algorithmic_bytes_per_launch": dom_bytes,
                     "launch_ms": launch_ms,
                     "note": "integer VALU/LDS-bound DP; HBM roofline reported as required (DESIGN.md)"},
        "step_algorithmic_bytes": step_bytes,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(probs, q, genome)
    elif rank == 0:
        out["cpu_baseline"] = None
    lib.gmapdp_plan_destroy(plan)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
