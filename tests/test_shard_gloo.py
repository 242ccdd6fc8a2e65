"""World-size-2 CPU test (gloo) of the multi-GPU path: --part sharding covers every
read exactly once, each rank's DP results for its shard equal the single-process
results, the replicated-genome check and the max-over-ranks timing reduction."""
import os
import random
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from gmapdp import shard
    from dpbind import Oracle, call_single, random_genome, single_gap_problem
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = random.Random(11)                      # same stream on every rank
        g = random_genome(rng, 20000)
        probs = [single_gap_problem(rng, g) for _ in range(120)]
        shard.check_replicated(shard.genome_digest(np.frombuffer(g, dtype=np.uint8)), dist)
        mine = np.nonzero(shard.part_mask(np.arange(len(probs)), rank, world))[0]
        orc = Oracle()
        orc.set_genome(g)
        out = {int(i): call_single(orc, probs[i]) for i in mine}
        t = shard.max_over_ranks(0.25 * (rank + 1), dist)
        q.put((rank, out, t))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_gloo():
    sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
    from dpbind import Oracle, call_single, random_genome, single_gap_problem
    if not os.path.exists(os.path.join(ROOT, "oracle", "libgmapdp_oracle.so")):
        pytest.fail("oracle not built")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = {}
    for rank, out, t in got:
        assert t == 0.5                              # max over ranks
        assert not set(out) & set(merged)            # disjoint shards
        merged.update(out)
    rng = random.Random(11)
    g = random_genome(rng, 20000)
    probs = [single_gap_problem(rng, g) for _ in range(120)]
    assert sorted(merged) == list(range(len(probs)))  # every read exactly once
    orc = Oracle()
    orc.set_genome(g)
    assert all(merged[i] == call_single(orc, probs[i]) for i in range(len(probs)))


def test_part_rule_matches_gmap():
    sys.path.insert(0, os.path.join(ROOT, "gmap-2024_amd"))
    from gmapdp import shard
    ids = np.arange(1000)
    masks = [shard.part_mask(ids, r, 8) for r in range(8)]
    assert (np.sum(masks, axis=0) == 1).all()
    assert list(np.nonzero(masks[3])[0][:3]) == [3, 11, 19]    # inputid % 8 == 3 (inbuffer.c:283)
    with pytest.raises(ValueError):
        shard.part_mask(ids, 8, 8)
