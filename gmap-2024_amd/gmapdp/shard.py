"""Read sharding across GPUs (one process per GPU, no data-path collective).

GMAP's own rule for splitting a read stream over processes is --part=i/n:
input read `inputid` is aligned by the process whose part_modulus equals
inputid % part_interval (inbuffer.c:270-283, gmap.c:5077-5100).  Rank r of a
world of n plays --part=r/n.  Every rank holds the whole packed genome (it is
read-only); the only cross-rank traffic is for reporting (the max step time)
and a one-time check that the replicated genomes are identical.
"""
import hashlib

import numpy as np


def part_mask(inputids, rank, world):
    """Boolean mask of the reads rank `rank` aligns (--part=rank/world)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad part %d/%d" % (rank, world))
    return (np.asarray(inputids, dtype=np.int64) % world) == rank


def genome_digest(genome):
    """32-byte digest of a genome array (checked equal across ranks)."""
    return hashlib.blake2b(np.ascontiguousarray(genome).tobytes(), digest_size=32).digest()


def check_replicated(digest, dist):
    """all_gather the ranks' genome digests; raise if any rank holds a different genome."""
    import torch
    world = dist.get_world_size()
    mine = torch.tensor(list(digest), dtype=torch.uint8)
    backend = dist.get_backend()
    if backend == "nccl":
        mine = mine.cuda()
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    if any(not torch.equal(g.cpu(), mine.cpu()) for g in gathered):
        raise RuntimeError("ranks hold different genomes")


def max_over_ranks(value, dist, device=None):
    """The step time the job is judged by: the slowest rank's."""
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def blocks_of_rank(rank, world, nbatches):
    """The read blocks rank `rank` of `world` processes: block b of the stream's first world x nbatches
    blocks goes to the rank with b % world == rank (--part=rank/world applied to blocks of reads)."""
    ids = np.arange(world * nbatches)
    return [int(b) for b in ids[part_mask(ids, rank, world)]]


def gather_blocks(mine, reads, dist=None):
    """all_gather every rank's (block ids, reads per block); check that the blocks are disjoint and
    together cover 0 .. nblocks-1, and return the shard record bench.py reports."""
    world = dist.get_world_size() if dist is not None else 1
    if dist is None:
        every = [list(mine)]
        every_reads = [list(reads)]
    else:
        every = [None] * world
        every_reads = [None] * world
        dist.all_gather_object(every, list(mine))
        dist.all_gather_object(every_reads, [int(r) for r in reads])
    flat = [b for ids in every for b in ids]
    if len(set(flat)) != len(flat):
        raise RuntimeError("read blocks assigned to more than one rank: %s" % every)
    if sorted(flat) != list(range(len(flat))):
        raise RuntimeError("read blocks missing from the shard: %s" % every)
    return {"rule": "--part=r/N over blocks of reads (inbuffer.c:283)", "blocks_per_rank": every,
            "reads_per_rank": [int(sum(r)) for r in every_reads], "reads_total": int(sum(sum(r) for r in every_reads)),
            "disjoint": True}
