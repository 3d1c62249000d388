"""Depth vectors whose np.std lies on a round(x, 2) tie (tests/golden/std_ties.json).

A vector of n = 200 t positions at depth y, with a positions at y + d1 and b
at y + d2, has n^2 var = D = a b (d1 - d2)^2 + c (a d1^2 + b d2^2) (c = n - a
- b; Lagrange's identity).  When D = (t (2k + 1))^2 the exact std is (2k +
1) / 200 = x.xx5, a tie for round(std, 2), and the mean is not an integer
unless n divides a d1 + b d2.  numpy's float64 value then lies a rounding
error above or below the tie, and its position order (the vector is
shuffled) decides which: exactly the cases where round(sqrt(exact var), 2)
and the reference's round(np.std(columns), 2) can differ.
"""
import math

import numpy as np


def tie_params(t, amax=40, dmax=12):
    """(n, a, b, d1, d2) with an exact x.xx5 std and a non-integer mean."""
    n = 200 * t
    out = []
    for a in range(1, amax):
        for b in range(1, amax):
            c = n - a - b
            for d1 in range(1, dmax):
                for d2 in range(-dmax + 1, dmax):
                    if d2 == 0 or d2 == d1:
                        continue
                    D = a * b * (d1 - d2) ** 2 + c * (a * d1 * d1 + b * d2 * d2)
                    e = math.isqrt(D)
                    if e * e != D or e % t or (e // t) % 2 == 0 or (a * d1 + b * d2) % n == 0:
                        continue
                    out.append((n, a, b, d1, d2))
    return out


def tie_vector(n, a, b, d1, d2, y, seed):
    v = np.full(n, y, np.int64)
    v[:a] += d1
    v[a:a + b] += d2
    np.random.default_rng(seed).shuffle(v)
    return v


def skyline_reads(v, start=0):
    """(pos, span) of reads whose per-position count is exactly v on
    [start, start + len(v)): a stack of open reads, one pushed per unit
    step up, the latest popped per unit step down; sorted by position."""
    v = np.asarray(v, np.int64)
    pos, span = [], []
    stack = []
    prev = 0
    for i, x in enumerate(list(v) + [0]):
        x = int(x)
        for _ in range(x - prev):
            stack.append(i)
        for _ in range(prev - x):
            s = stack.pop()
            pos.append(start + s)
            span.append(i - s)
        prev = x
    order = np.argsort(np.asarray(pos, np.int64), kind="stable")
    return np.asarray(pos, np.int32)[order], np.asarray(span, np.int32)[order]
