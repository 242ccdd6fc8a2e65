"""Genome-gap kernel timing on one bench block (diagnostic): the block's Dynprog_genome_gap calls planned
once and their launch classes run alone on one stream, timed with HIP events; variants are selected
through the engine's environment switches, one child process each (they are read once per process).

  python tools/gg_bench.py [--reads 10000] [--reps 5] [--simd]

--simd times the SIMD builds' genome gaps (uxg_kernel) on the same block.
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
VARIANTS = {"gg_kernel": {}, "gg_kernel_lds_dirs": {"GMAPDP_GG_LDS_DIRS_MAX": str(48 * 1024)},
            # an earlier build of the library kept under gmap-2024_amd/lib_base (A/B of a kernel change)
            "lib_base": {"GMAPDP_LIB": os.path.join(ROOT, "gmap-2024_amd", "lib_base", "libgmapdp.so")}}


def variant_env(v):
    """A named variant, or lib_<x>: a build kept under gmap-2024_amd/lib_<x> (A/B of a kernel change)."""
    if v in VARIANTS:
        return VARIANTS[v]
    if v.startswith("lib_"):
        return {"GMAPDP_LIB": os.path.join(ROOT, "gmap-2024_amd", v, "libgmapdp.so")}
    raise SystemExit("unknown variant " + v)


def child(reads, reps, simd):
    import numpy as np
    import torch
    import gmapdp
    from gmapdp import workload as W
    lay = W.Layout(W.GRCH38)
    g = W.PackedGenome(lay.total, seed=38)
    W.plant_stream(g, lay, reads, range(1))
    d = W.make_blocks(g, lay, reads, [0], sprob=True)[0]
    eng = gmapdp.Engine(0)
    eng.set_genome(blocks=g.blocks, length=g.length)
    lib = eng.lib
    gp = d["genome"]
    if simd:
        gp["flags"] |= gmapdp.SIMD
    dev = torch.device("cuda", 0)
    d_q = torch.from_numpy(d["q"]).to(dev)
    d_sp = torch.from_numpy(d["sprob"]).to(dev)
    hres = np.zeros(1, dtype=gmapdp.RESULT_DTYPE)
    hg = np.zeros(len(gp), dtype=gmapdp.GENOME_RESULT_DTYPE)
    plan = C.c_void_p()
    eng._check(lib.gmapdp_plan_create_all(eng.h, None, 0, None, 0, gp.ctypes.data, len(gp), hres.ctypes.data,
                                          hg.ctypes.data, C.byref(plan)), "plan")
    d_gres = torch.zeros(len(gp) * 72, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(64, dtype=torch.uint8, device=dev)
    d_pairs = torch.empty(lib.gmapdp_plan_pair_capacity(plan) * 16, dtype=torch.uint8, device=dev)
    eng._check(lib.gmapdp_plan_bind_genome(plan, C.c_void_p(d_sp.data_ptr()), C.c_void_p(d_gres.data_ptr())), "bind")
    s = torch.cuda.Stream(dev)
    nl = lib.gmapdp_plan_nlaunches(plan)

    def run():
        for li in range(nl):
            eng._check(lib.gmapdp_plan_run_launch(eng.h, plan, li, C.c_void_p(d_q.data_ptr()),
                                                  C.c_void_p(d_q.data_ptr()), C.c_void_p(d_res.data_ptr()),
                                                  C.c_void_p(d_pairs.data_ptr()), C.c_void_p(s.cuda_stream)), "run")
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    out = np.frombuffer(d_gres.cpu().numpy().tobytes(), dtype=gmapdp.GENOME_RESULT_DTYPE)
    digest = int(np.frombuffer(out.tobytes(), dtype=np.uint64).sum() % (1 << 61))
    info = []
    for li in range(nl):
        R, dl, cnt, lds = C.c_int(), C.c_int(), C.c_int(), C.c_size_t()
        lib.gmapdp_plan_launch_info(plan, li, C.byref(R), C.byref(dl), C.byref(cnt), C.byref(lds))
        info.append((R.value, dl.value, cnt.value, lds.value))
    print(json.dumps({"ms_per_block": e0.elapsed_time(e1) / reps, "launches": info, "results_digest": digest}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--simd", action="store_true")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    a = ap.parse_args()
    if a.child:
        return child(a.reads, a.reps, a.simd)
    res = {}
    for v in a.variants.split(","):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--reads", str(a.reads), "--reps",
                            str(a.reps)] + (["--simd"] if a.simd else []), capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, **variant_env(v)))
        if r.returncode != 0:
            res[v] = {"error": r.stderr[-1500:]}
            break
        res[v] = json.loads(r.stdout.strip().splitlines()[-1])
        print(v, json.dumps(res[v]), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
