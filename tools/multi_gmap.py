"""Run GMAP over N GPUs of one node the way the reference splits a read stream over processes
(configs[3]: reads sharded, genome replicated per GPU): read `inputid` goes to copy inputid % N -- the
rule of GMAP's own --part=i/N (gmap.c:5077 parse_part, inbuffer.c:392) -- each copy runs on
GMAPDP_DEVICE = i % devices (the drop-in's device, gmapdp_gmap_shim.c), and the N outputs are merged back
into input order.

The split is done here, on the FASTA input, rather than with the program's --part option: in this
reference snapshot --part crashes whenever the input is not a pairalign stream (inbuffer.c:392-394 calls
Sequence_free(&genomeseq) on an uninitialised `genomeseq`; the unmodified gmap_nosimd segfaults on
`--part=0/2 -g ...`), so the copies read pre-split files holding exactly the reads --part would give them.

Each copy aligns its reads in input order (add -O with -t > 1), so the merge takes one read's records
from copy 0, the next read's from copy 1, and so on; a read's records are its consecutive lines with the
same name (SAM QNAME, the first field).

    python tools/multi_gmap.py --parts 8 --reads reads.fa -- oracle/_ref/gmap_gpu_nosimd -t 64 -O \
        -g g.fa -f samse --no-sam-headers > out.sam

The copies are separate processes, each with its own device, and share nothing (no collective): weak
scaling by reads.
"""
import argparse
import os
import subprocess
import sys
import tempfile
import time


def groups(lines):
    """consecutive lines with the same first field -> list of groups"""
    out, cur, name = [], [], None
    for ln in lines:
        q = ln.split("\t", 1)[0]
        if cur and q != name:
            out.append(cur)
            cur = []
        cur.append(ln)
        name = q
    if cur:
        out.append(cur)
    return out


def merge(parts):
    """round-robin over the copies' read groups (read i came from copy i % N)"""
    gs = [groups(p.splitlines(keepends=True)) for p in parts]
    out, k = [], 0
    while any(k < len(g) for g in gs):
        for g in gs:
            if k < len(g):
                out.extend(g[k])
        k += 1
    return "".join(out)


def split_fasta(path, parts, tmp):
    """read i of the FASTA file -> part i % parts (the --part=i/N rule); returns the part files"""
    outs = [open(os.path.join(tmp, "reads%d.fa" % i), "w") for i in range(parts)]
    k = -1
    with open(path) as f:
        for ln in f:
            if ln.startswith(">"):
                k += 1
            if k >= 0:
                outs[k % parts].write(ln)
    for o in outs:
        o.close()
    return [o.name for o in outs]


def run(parts, devices, cmd, reads, cwd=None):
    procs, files = [], []
    tmp = tempfile.mkdtemp(prefix="multi_gmap_")
    inputs = split_fasta(os.path.join(cwd or ".", reads), parts, tmp)
    t0 = time.perf_counter()
    for i in range(parts):
        f = open(os.path.join(tmp, "part%d" % i), "w+")
        env = dict(os.environ, GMAPDP_DEVICE=str(i % max(devices, 1)))
        procs.append(subprocess.Popen(cmd + [inputs[i]], stdout=f, stderr=subprocess.PIPE, env=env, cwd=cwd))
        files.append(f)
    errs, rc = [], 0
    for p in procs:
        _, err = p.communicate()
        errs.append(err.decode(errors="replace"))
        rc = rc or p.returncode
    dt = time.perf_counter() - t0
    outs = []
    for f in files:
        f.seek(0)
        outs.append(f.read())
        f.close()
    return rc, merge(outs), errs, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, required=True)
    ap.add_argument("--devices", type=int, default=0, help="GPUs to spread the copies over (default: --parts)")
    ap.add_argument("--reads", required=True, help="the query FASTA (split here by the --part rule)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    rc, out, errs, dt = run(a.parts, a.devices or a.parts, cmd, os.path.abspath(a.reads))
    sys.stdout.write(out)
    for i, e in enumerate(errs):
        if e.strip():
            sys.stderr.write("[part %d] %s" % (i, e))
    sys.stderr.write("multi_gmap: %d parts in %.3f s\n" % (a.parts, dt))
    return rc


if __name__ == "__main__":
    sys.exit(main())
