"""GPU parity tests for Stage2_compute: oi_kernel / oi_map_kernel seeding, then
s2c_kernel's Diag_update_coverage, Diag_compute_bounds, align_compute_lookback, traceback_one,
convert_to_nucleotides and Stage2_filter_unique (stage2.c:6325, diag.c:597), against the golden from
the reference's own Stage2_compute, the oracle restatement (oracle/stage2_chain_oracle.c) and the
reference objects directly.  Bar: bit-exact result lists (number, order) and every pair record of
every kept path (querypos, genomepos, gap holders' queryjump / genomejump, cdna, comp, genome,
genomealt)."""
import os
import random

import pytest

import gmapdp
from dpbind import Oracle, Ref, random_genome, ref_available, repeat_genome, stage2_problem

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.load_stage2(os.path.join(HERE, "golden", "stage2_golden.npz"))


@pytest.fixture(scope="module")
def engine():
    e = gmapdp.Engine(0)
    yield e
    e.close()


def _check(got, exp, probs, what):
    for i, (a, b) in enumerate(zip(got, exp)):
        if a != b:
            p = {k: v for k, v in probs[i].items() if k not in ("q", "quc")}
            detail = ""
            if a[0] == b[0]:
                for k, (x, y) in enumerate(zip(a[1], b[1])):
                    if x != y:
                        j = next((j for j, (u, v) in enumerate(zip(x, y)) if u != v), min(len(x), len(y)))
                        detail = "result %d (len %d vs %d) first difference at record %d: %s vs %s" % (
                            k, len(x), len(y), j, x[j] if j < len(x) else None, y[j] if j < len(y) else None)
                        break
            raise AssertionError("problem %d (%s, qlen %d): gpu %d results vs %s %d; %s"
                                 % (i, p, len(probs[i]["quc"]), a[0], what, b[0], detail))


def test_gpu_stage2_matches_reference_golden(engine):
    g, probs, exp = _golden()
    engine.set_genome(g)
    _check(engine.stage2_batch(probs), exp, probs, "ref")


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_stage2_matches_oracle_random(engine, seed):
    rng = random.Random(9100 + seed)
    g = repeat_genome(rng, 400000) if seed % 2 else random_genome(rng, 400000)
    engine.set_genome(g)
    orc = Oracle()
    orc.set_genome(g)
    probs = [stage2_problem(rng, g, edge=(i % 5 == 0)) for i in range(500)]
    got = engine.stage2_batch(probs)
    _check(got, [orc.stage2_compute(p) for p in probs], probs, "oracle")
    assert sum(1 for r in got if r[0] > 1) > 0  # several kept results occur


@pytest.mark.skipif(not ref_available("nosimd"), reason="reference objects did not travel")
def test_gpu_stage2_matches_reference_objects(engine):
    rng = random.Random(9200)
    g = repeat_genome(rng, 300000)
    engine.set_genome(g)
    ref = Ref("nosimd")
    ref.set_genome(g)
    probs = [stage2_problem(rng, g, edge=(i % 4 == 0)) for i in range(300)]
    _check(engine.stage2_batch(probs), [ref.stage2_compute(p) for p in probs], probs, "ref")


def test_gpu_stage2_empty_and_single(engine):
    rng = random.Random(9300)
    g = random_genome(rng, 100000)
    engine.set_genome(g)
    assert engine.stage2_batch([]) == []
    orc = Oracle()
    orc.set_genome(g)
    p = stage2_problem(rng, g)
    assert engine.stage2_batch([p]) == [orc.stage2_compute(p)]
