"""The engine plans a batch in one of two ways (gmapdp_engine.cpp classify): throughput mode (launch
classes by band width and LDS bucket, packed narrow-band kernels; large batches such as bench.py's) and
latency mode (batches of at most GMAPDP_LATENCY_BATCH problems, 1024 by default: one class per kernel
and band width sized for its largest member, no packed kernels; the GMAP drop-in's dispatcher batches).
The same problems run both ways must give the same results, and those equal the oracle's."""
import random

import pytest

import gmapdp
from dpbind import (Oracle, call_end, call_single, edge_single_gap_problem, end_gap_problem, genome_gap_problem,
                    random_genome, single_gap_problem)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0, flags=gmapdp.CTX_ONE_STREAM | gmapdp.CTX_PRIO_HIGH)
    yield e
    e.close()


def _chunks(xs, n):
    return [xs[i:i + n] for i in range(0, len(xs), n)]


def test_single_and_end_gaps_both_modes(engine):
    rng = random.Random(606)
    g = random_genome(rng, 60000)
    singles = [single_gap_problem(rng, g) for _ in range(1700)] + [edge_single_gap_problem(rng, g) for _ in range(300)]
    ends = [end_gap_problem(rng, g, edge=(i % 4 == 0)) for i in range(1500)]
    engine.set_genome(g)
    big_s = engine.single_gap_batch(singles)             # 2000 problems: throughput mode
    big_e = engine.end_gap_batch(ends)                   # 1500 problems: throughput mode
    small_s = [x for c in _chunks(singles, 150) for x in engine.single_gap_batch(c)]
    small_e = [x for c in _chunks(ends, 150) for x in engine.end_gap_batch(c)]
    assert small_s == big_s
    assert small_e == big_e
    orc = Oracle()
    orc.set_genome(g)
    for i in range(0, len(singles), 7):
        assert small_s[i] == call_single(orc, singles[i]), i
    for i in range(0, len(ends), 7):
        assert small_e[i] == call_end(orc, ends[i]), i


def test_genome_gaps_both_modes(engine):
    rng = random.Random(707)
    g = bytearray(random_genome(rng, 120000))
    probs = [genome_gap_problem(rng, g, edge=(i % 5 == 0)) for i in range(2100)]
    g = bytes(g)
    vals = [0.0, 0.3, 0.5, 0.9, 0.95, 1.0]
    sp = [([rng.choice(vals) for _ in range(max(0, p["glengthL"]))],
           [rng.choice(vals) for _ in range(max(0, p["glengthR"]))]) for p in probs]
    engine.set_genome(g)
    big = engine.genome_gap_batch(probs, sp)
    small = [x for c, s in zip(_chunks(probs, 200), _chunks(sp, 200)) for x in engine.genome_gap_batch(c, s)]
    assert small == big
    orc = Oracle()
    orc.set_genome(g)
    for i in range(0, len(probs), 5):
        assert small[i] == orc.genome_gap(probs[i], *sp[i]), i


def test_shared_genome_context(engine):
    """gmapdp_share_genome: a second context answers from the first one's HBM genome."""
    rng = random.Random(808)
    g = random_genome(rng, 40000)
    engine.set_genome(g)
    other = gmapdp.Engine(0, flags=gmapdp.CTX_ONE_STREAM | gmapdp.CTX_PRIO_LOW | gmapdp.CTX_BLOCKING_SYNC)
    try:
        other.share_genome(engine)
        probs = [single_gap_problem(rng, g) for _ in range(300)]
        assert other.single_gap_batch(probs) == engine.single_gap_batch(probs)
    finally:
        other.close()
