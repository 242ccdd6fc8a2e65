"""Per-thread CPU time of a program, grouped by thread name (diagnostic): runs the command, samples
/proc/<pid>/task/*/stat every 0.2 s, and prints the last user+system seconds seen per thread name.

    python tools/thread_cpu.py -- oracle/_ref/gmap_gpu_nosimd -t 512 ...
"""
import collections
import json
import os
import subprocess
import sys
import time

TICK = os.sysconf("SC_CLK_TCK")


def sample(pid, seen):
    base = "/proc/%d/task" % pid
    try:
        tids = os.listdir(base)
    except OSError:
        return
    for t in tids:
        try:
            txt = open("%s/%s/stat" % (base, t)).read()
        except OSError:
            continue
        name = txt[txt.index("(") + 1:txt.rindex(")")]
        f = txt[txt.rindex(")") + 2:].split()
        seen[int(t)] = (name, (int(f[11]) + int(f[12])) / TICK)


def main():
    cmd = sys.argv[1:]
    if cmd and cmd[0] == "--":
        cmd = cmd[1:]
    seen = {}
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    while p.poll() is None:
        sample(p.pid, seen)
        time.sleep(0.2)
    err = p.stderr.read().decode(errors="replace")
    by = collections.defaultdict(lambda: [0, 0.0])
    for name, cpu in seen.values():
        by[name][0] += 1
        by[name][1] += cpu
    print(json.dumps({"seconds": time.perf_counter() - t0, "rc": p.returncode,
                      "threads": {k: {"n": v[0], "cpu_s": round(v[1], 2)} for k, v in
                                  sorted(by.items(), key=lambda kv: -kv[1][1])},
                      "stderr_tail": err[-400:]}))


if __name__ == "__main__":
    main()
