"""classic_stats (metacov_amd/engine.py, the host half of the reference's
pileup.classic, metacov/pileup.py:18-26) against numpy's own float64
computation on the full column vector (oracle/classic_np.py), which is what
the reference runs.

classic_stats sees only the exact integer row the GPU returns (n, sum, sum of
squares, min, max, the two median ranks, the trimmed q23 sum).  The claims
this file checks:
  * avg and q23: float64(sum) / n is exactly np.mean's value for integer data
    (its pairwise sum of integers below 2**53 is exact, then one division);
  * std: sqrt(float(exact variance)).  When the mean is an integer, numpy's
    deviations, squares and their sum are exact too, so np.std is
    sqrt(fl(sum / n)) and the two agree to the bit — including the
    constructed cases whose std is exactly k + 0.005 (a round(x, 2) tie);
  * med: (med_lo + med_hi) // 2 is int(np.median) for non-negative data.
With a non-integer mean np.std's value depends on its summation order (its
rounding errors are position-dependent), so a vector whose exact std lies
within ~1e-13 of a .xx5 boundary can round the other way in numpy.  Those
rows are flagged (engine.std_near_tie) and given numpy's own value,
computed on the device in numpy's order: tests/test_npstd.py pins them
against the real classic() on constructed ties (tests/golden/std_ties.json).
"""
import numpy as np
import pytest

from metacov_amd.engine import classic_stats
from oracle.classic_np import classic_from_vector


def exact_row(vec):
    """The mc_region_stat row of a depth vector (exact integers)."""
    v = np.asarray(vec, np.int64)
    n = len(v)
    s = np.sort(v)
    sq = v * v
    assert float(sq.sum(dtype=np.float64)) < 9.0e18      # int64 sum of squares exact
    return {"n": n, "sum": int(v.sum()), "sumsq": int(sq.sum(dtype=np.int64)),
            "min": int(s[0]), "max": int(s[-1]), "med_lo": int(s[(n - 1) // 2]), "med_hi": int(s[n // 2]),
            "q23_sum": int(s[n // 4:n - n // 4].sum()), "q23_cnt": n - 2 * (n // 4)}


def check(vec):
    got = classic_stats(exact_row(vec))
    want = classic_from_vector(np.asarray(vec, np.float64))
    assert got == want, (len(vec), got, want)


def test_random_vectors():
    """10^4 random depth vectors: Poisson bodies over 5 orders of magnitude of
    depth, zero runs (positions past the contig end), ramps, constant runs."""
    rng = np.random.default_rng(2024)
    for _ in range(10_000):
        n = int(np.exp(rng.uniform(0, np.log(6000))))
        lam = float(np.exp(rng.uniform(np.log(0.05), np.log(2.5e4))))
        v = rng.poisson(lam, size=n)
        r = rng.random()
        if r < 0.15:                                  # zeros past the data
            v[rng.integers(0, n + 1):] = 0
        elif r < 0.25:                                # ramp at one end
            k = min(n, int(rng.integers(1, 300)))
            v[:k] = np.minimum(v[:k], np.arange(k))
        elif r < 0.30:
            v[:] = v[0]
        check(v)


@pytest.mark.parametrize("lam", [30.0, 1.5e4])
def test_large_vectors(lam):
    """n > 10^7 positions (a whole C3 / C5 contig is 0.05-1.8 M; a 12 M
    region covers the ceiling of what one pileup.classic call allocates),
    depth above 10^4."""
    rng = np.random.default_rng(int(lam))
    v = rng.poisson(lam, size=12_000_000)
    v[:1000] = 0
    check(v)


@pytest.mark.parametrize("q", [1, 3, 5, 7, 49, 201, 4001])
@pytest.mark.parametrize("pairs", [1, 150])
def test_std_exact_ties(q, pairs):
    """Integer mean m, deviations +q / -q on `pairs` pairs among n = 80000 *
    pairs positions: var = q^2 / 40000 exactly, std = q / 200 = x.xx5 — a tie
    for round(std, 2).  pairs = 150: n = 1.2 x 10^7."""
    n = 80_000 * pairs
    m = 1000
    v = np.full(n, m, np.int64)
    v[:pairs] += q
    v[pairs:2 * pairs] -= q
    np.random.default_rng(q).shuffle(v)
    row = exact_row(v)
    assert row["sum"] == m * n
    assert classic_stats(row)["std"] == classic_from_vector(v.astype(np.float64))["std"]
    check(v)


@pytest.mark.parametrize("k", [0, 1, 7, 123, 20000])
def test_avg_and_q23_exact_ties(k):
    """avg = k + 0.005 and q23 = k + 0.005 exactly (sum = 200 k + 1 over 200
    values; the trimmed middle of 400 values holds 200)."""
    v = np.full(200, k, np.int64)
    v[0] += 1
    check(v)
    w = np.concatenate([np.zeros(100, np.int64), v, np.full(100, k + 10 ** 6, np.int64)])
    row = exact_row(w)
    assert row["q23_cnt"] == 200 and row["q23_sum"] == 200 * k + 1
    check(w)


def test_median_truncation():
    for v in ([1, 2], [0, 3], [5, 8, 9, 10], [2, 2, 3, 3], [0]):
        check(np.array(v))
