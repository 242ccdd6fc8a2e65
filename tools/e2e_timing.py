"""End-to-end timing of GMAP's own per-read pipeline: the unmodified reference `gmap` (CPU) against the
same program linked with the drop-in shim (every Dynprog_* call and stage-2 seeding on the MI355X
engine), on the same host cores.  Measurement tool, run on the GPU box:

    python tools/e2e_timing.py --reads 2000 --threads 1,16

Reads are tests/golden/make_e2e.py's synthetic 2-kb spliced reads (5 exons x 400 nt, 2 % subs) against
its 300-kb segment, in user-segment mode (-g: stage 2 over the whole segment, then stage 3).  With
--index DIR (made by tools/e2e_index.py) the reads are DIR/r.fa and both programs run on DIR's genome
index (`-D DIR/db -d NAME`: stage 1, then stage 2 over each locus +- 100 kb, then stage 3 -- the mix the
headline bench restates).  Both programs' SAM outputs are compared; the JSON line gives reads/s per
program and thread count and the shim's call counts.
"""
import argparse
import json
import os
import resource
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2000)
    ap.add_argument("--index", default=None, help="tools/e2e_index.py's directory: gmap -d over its index")
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--build", default="nosimd", choices=["nosimd", "avx2"])
    ap.add_argument("--gpu-threads", default=None, help="thread counts for the GPU program (default: --threads)")
    ap.add_argument("--dispatchers", type=int, default=3, help="GMAPDP_SHIM_DISPATCHERS")
    ap.add_argument("--trace", default=None, help="directory for the shim's per-batch traces (GMAPDP_SHIM_TRACE)")
    ap.add_argument("--configs", default="default:",
                    help="shim configurations for the GPU runs, 'name:VAR=V,VAR=V;name2:...' (environment overrides)")
    ap.add_argument("--cpu-configs", default="cpu:",
                    help="environment configurations for the unmodified program's runs, same syntax (e.g. the same "
                         "malloc tunables as a GPU configuration, for a like-for-like comparison)")
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--thread-cpu", action="store_true", help="per-thread-name CPU seconds of each run")
    ap.add_argument("--prof", default=None,
                    help="directory for sampled CPU profiles: runs the unstripped gmap_prof_V / gmap_gpu_prof_V "
                         "programs with tools/pcprof.c's sampler on and resolves them (tools/pcprof.py)")
    a = ap.parse_args()
    import make_e2e as M
    tmp = tempfile.mkdtemp(prefix="e2e_")
    if a.index:
        idx = os.path.abspath(a.index)
        meta = json.load(open(os.path.join(idx, "meta.json")))
        # the first --reads reads of the index's read set
        with open(os.path.join(idx, "r.fa")) as f, open(os.path.join(tmp, "r.fa"), "w") as g:
            n = 0
            for line in f:
                if line.startswith(">"):
                    n += 1
                    if n > a.reads:
                        break
                g.write(line)
        a.reads = min(a.reads, n)
        gargs = ["-D", os.path.join(idx, "db"), "-d", meta["name"]]
    else:
        genome = list(M.synth_genome())
        reads = [M.synth_read(genome, i) for i in range(a.reads)]
        M.write_fasta(os.path.join(tmp, "g.fa"), [("synseg", "".join(genome))])
        M.write_fasta(os.path.join(tmp, "r.fa"), reads)
        gargs = ["-g", "g.fa"]
    ref = os.path.join(ROOT, "oracle", "_ref")
    out = {"reads": a.reads, "build": a.build, "mode": "-d %s" % meta["name"] if a.index else "-g", "cpu_model": None,
           "runs": []}
    try:
        out["cpu_model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    sams = {}
    cpu_t = [int(x) for x in a.threads.split(",")]
    gpu_t = [int(x) for x in (a.gpu_threads or a.threads).split(",")]
    def parse_configs(spec):
        out = []
        for c in spec.split(";"):
            name, _, kv = c.partition(":")
            out.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
        return out
    configs = parse_configs(a.configs)
    pv = "prof_" if a.prof else ""
    runs = [] if a.skip_cpu else [("gmap_%s%s" % (pv, a.build), t, name, cenv)
                                  for name, cenv in parse_configs(a.cpu_configs) for t in cpu_t]
    runs += [("gmap_gpu_%s%s" % (pv, a.build), t, name, cenv) for name, cenv in configs for t in gpu_t]
    profs = []
    out["dispatchers"] = a.dispatchers
    for prog, t, cname, cenv in runs:
        if True:
            env = dict(os.environ, GMAPDP_SHIM_STATS="1", GMAPDP_SHIM_DISPATCHERS=str(a.dispatchers))
            env.update(cenv)
            if a.trace and "gpu" in prog:
                os.makedirs(a.trace, exist_ok=True)
                env["GMAPDP_SHIM_TRACE"] = os.path.abspath(os.path.join(a.trace, "trace_%s_t%d.txt" % (cname, t)))
            if a.prof:
                os.makedirs(a.prof, exist_ok=True)
                env["PCPROF_OUT"] = os.path.abspath(os.path.join(a.prof, "pcprof_%s_%s_t%d.txt" % (prog, cname, t)))
                profs.append(env["PCPROF_OUT"])
            args = [os.path.join(ref, prog), "-t", str(t), "-O"] + gargs + ["-f", "samse", "--no-sam-headers", "r.fa"]
            t0 = time.perf_counter()
            ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
            threads = None
            if a.thread_cpu:  # per-thread-name CPU seconds (fiber hosts, dispatchers, GMAP's own threads)
                import collections
                from thread_cpu import sample
                seen = {}
                p = subprocess.Popen(args, cwd=tmp, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                import threading
                res = {}
                th = threading.Thread(target=lambda: res.update(zip(("out", "err"), p.communicate())))
                th.start()
                while th.is_alive():
                    sample(p.pid, seen)
                    time.sleep(0.2)
                th.join()
                agg = collections.defaultdict(float)
                for name, secs in seen.values():
                    agg[name] += secs
                threads = {k: round(v, 2) for k, v in sorted(agg.items(), key=lambda kv: -kv[1])}
                r = subprocess.CompletedProcess(args, p.returncode, res.get("out", ""), res.get("err", ""))
            else:
                r = subprocess.run(args, cwd=tmp, env=env, capture_output=True, text=True, timeout=1500)
            dt = time.perf_counter() - t0
            ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
            cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
            if r.returncode != 0:
                raise SystemExit("%s failed: %s" % (prog, r.stderr[-2000:]))
            sams[(prog, t, cname)] = r.stdout
            stats = [l for l in r.stderr.splitlines() if l.startswith("gmapdp shim calls")]
            # GMAPDP_BATCH_TIMING=1 in a configuration: the engine's per-phase means of the mixed batches
            bt = [l for l in r.stderr.splitlines() if l.startswith("[gmapdp batch timing]")]
            out["runs"].append({"program": prog, "threads": t, "config": cname, "env": cenv, "seconds": dt, "reads_per_s": a.reads / dt,
                                "cpu_seconds": cpu, "cpu_cores_busy": cpu / dt,
                                "shim_calls": stats[0] if stats else None, "thread_cpu_s": threads,
                                "batch_timing": bt[0] if bt else None})
            print(json.dumps(out["runs"][-1]), file=sys.stderr, flush=True)
    base = next(iter(sams.values())) if a.skip_cpu else next(v for k, v in sams.items() if k[0] == "gmap_%s%s" % (pv, a.build))
    out["outputs_identical"] = all(v == base for v in sams.values())
    out["recorded"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())  # bench.py selects records by this
    print(json.dumps(out))
    if profs:
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pcprof.py"), "--json",
                        os.path.join(a.prof, "pcprof_summary.json")] + profs, check=False, stdout=sys.stderr)


if __name__ == "__main__":
    main()
