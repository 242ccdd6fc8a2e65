"""CPU checks of the arithmetic oi_map_kernel's event keys rest on (oi_kernel.hip, OiKeyT32 / OiKeyQT):

- get_mappings' run test, q - q_prev >= diag_lookback + cum[q] - cum[q_prev] (oligoindex_hr.c:34127's
  Genomicdiag_T walk, with cum_nohits as oi_kernel computes it: an inclusive prefix count of the query
  positions whose 8-mer has no hit, a position without a full 8-mer carrying it forward), equals
  t(q) - t(q_prev) >= diag_lookback with t = q - cum[q];
- t is strictly increasing over the positions that have hits (the only positions events come from), so
  (t, diagi) orders events as (q, diagi) does and q is recovered as the first position with
  q - cum[q] >= t (the kernel's binary search, oi_q_of_t)."""
import random

import numpy as np


def cum_nohits(npos):
    """oi_kernel's cum_nohits: npos[q] = -1 (no full 8-mer), 0 (no hit) or > 0 (hits)."""
    return np.cumsum(np.asarray(npos) == 0)


def q_of_t(t, cum):
    lo, hi = 0, len(cum) - 1
    while lo < hi:
        mid = (lo + hi) // 2
        if mid - cum[mid] >= t:
            hi = mid
        else:
            lo = mid + 1
    return lo


def test_t_recovers_q_and_orders_events():
    rng = random.Random(5)
    for _ in range(300):
        n = rng.randint(1, 3000)
        pz, pn = rng.random(), rng.random() * 0.1
        npos = [-1 if rng.random() < pn else (0 if rng.random() < pz else rng.randint(1, 9)) for _ in range(n)]
        cum = cum_nohits(npos)
        t = np.arange(n) - cum
        hits = [q for q in range(n) if npos[q] > 0]
        assert np.all(np.diff(t) >= 0) and np.all(np.diff(t) <= 1)  # non-decreasing by steps of 0 or 1
        th = t[hits]
        assert np.all(np.diff(th) > 0)  # strictly increasing over the positions with hits
        for q in hits:
            assert q_of_t(int(t[q]), cum) == q


def test_run_test_on_t_equals_reference_form():
    rng = random.Random(6)
    for _ in range(200):
        n = rng.randint(2, 2500)
        npos = [rng.choice([-1, 0, 0, 1, 2, 3]) for _ in range(n)]
        cum = cum_nohits(npos)
        hits = [q for q in range(n) if npos[q] > 0]
        for lookback in (60, 120):
            for a, b in zip(hits, hits[1:]):
                ref = b - a >= lookback + int(cum[b]) - int(cum[a])
                assert ref == ((b - int(cum[b])) - (a - int(cum[a])) >= lookback)
