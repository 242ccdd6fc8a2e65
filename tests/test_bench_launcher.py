"""CPU tests of bench.py's multi-GPU path (no GPU): `--gpus N` starts N rank processes itself, and the
driver's torch.distributed.run launch reaches the same code; both run the gloo process group, the
--part=r/N block sharding (inbuffer.c:283 applied to blocks of reads), the replicated-genome check and
the workload generation (--dry-run)."""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))


def _run(cmd, timeout=300):
    env = dict(os.environ, GMAPDP_BENCH_WORKERS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 alone prints the result line
    ranks = [json.loads(ln)["rank_line"] for ln in r.stderr.splitlines() if ln.startswith('{"rank_line"')]
    return json.loads(lines[0]), ranks


def _check(out, ranks, world, batches, reads):
    assert out["dry_run"] and out["n_gpus"] == world
    sh = out["shard"]
    assert sh["disjoint"]
    flat = sorted(b for ids in sh["blocks_per_rank"] for b in ids)
    assert flat == list(range(world * batches))
    for r, ids in enumerate(sh["blocks_per_rank"]):
        assert all(b % world == r for b in ids)
    assert sh["reads_total"] == world * batches * reads
    assert sorted(x["rank"] for x in ranks) == list(range(world))
    assert all(x["world_size"] == world and x["backend"] == "gloo" for x in ranks)


def test_bench_launcher_spawns_ranks():
    out, ranks = _run([sys.executable, "bench.py", "--gpus", "2", "--dry-run", "--reads", "200", "--batches", "2",
                       "--genome", "chr22"])
    _check(out, ranks, 2, 2, 200)


def test_bench_under_torchrun():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:  # a free port (a fixed one can be taken)
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    out, ranks = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                       "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--dry-run",
                       "--reads", "200", "--batches", "2", "--genome", "chr22"])
    _check(out, ranks, 2, 2, 200)


def test_stream_blocks_independent_of_world_size():
    """Block b's calls are the same whichever rank generates it (the stream does not depend on N), and
    every rank's planted genome is the same."""
    from gmapdp import workload as W
    layout = W.Layout(W.CHR22)
    outs = []
    for world in (1, 2):
        g = W.PackedGenome(layout.total, seed=38)
        W.plant_stream(g, layout, 100, range(2 * 2), W.CDNA2K)   # same stream length in both runs
        outs.append((g.blocks[::997].copy(), W.make_blocks(g, layout, 100, [1], sprob=False)[0]))
    assert np.array_equal(outs[0][0], outs[1][0])
    for k in ("single", "end", "genome", "oligo", "microexon", "q", "oq"):
        assert np.array_equal(outs[0][1][k], outs[1][1][k]), k


def test_isoseq_reads_shape():
    """configs[4] read shape: 10 exons x 500 nt with 1 % indels gives ragged queries near 5 kb."""
    from gmapdp import workload as W
    layout = W.Layout(W.CHR22)
    g = W.PackedGenome(layout.total, seed=5)
    op, oq = W.make_stage2(g, layout, 50, np.random.default_rng(3), exons=10, exlen=500, subs=0.01, indel=0.01)
    L = op["querylength"].astype(np.int64)
    assert len(oq) == L.sum() and L.min() > 4800 and L.max() < 5200 and len(set(L.tolist())) > 5
    assert np.array_equal(op["qoff"][1:], np.cumsum(L)[:-1])


def test_wheat_layout_past_2_32():
    from gmapdp import workload as W
    lay = W.Layout(W.WHEAT17)
    assert abs(lay.total - 17e9) < 1e6
    assert lay.total > 2 ** 32 and lay.lens.max() < 2 ** 31
