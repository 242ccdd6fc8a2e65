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
