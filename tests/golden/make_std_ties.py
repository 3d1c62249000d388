"""Generates tests/golden/std_ties.json: depth vectors on an exact round(x, 2)
tie of their standard deviation, with the reference's own classic() result.

Run ONLY in the build container: it imports the reference's real
`metacov.pileup.classic` (/root/reference/metacov/pileup.py:9-26, whose std
is round(np.std(columns), 2) at :22) and feeds it each vector's columns
through make_golden.DuckBam.  Each case keeps the vector's parameters
(tests/std_ties.py rebuilds it), numpy's std as a float64 hex string, the
reference's dict, and whether the exact variance's rounding differs.
"""
import json
import math
import os
import sys
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from std_ties import tie_params, tie_vector  # noqa: E402
from make_golden import DuckBam, run_classic  # noqa: E402  (imports the real reference)


def exact_round(v):
    n, s, q = len(v), int(v.sum()), int((v.astype(object) ** 2).sum())
    return float(np.round(np.float64(math.sqrt(Fraction(n * q - s * s, n * n))), 2))


def main():
    cases = []
    for t, want in ((8, 24), (128, 16)):
        got = 0
        for (n, a, b, d1, d2) in tie_params(t):
            for y, seed in ((20, 1), (20, 2), (31, 3)):
                if got >= want:
                    break
                if y + min(d1, d2) < 0:
                    continue
                v = tie_vector(n, a, b, d1, d2, y, seed)
                cols = v.astype(np.float64)
                npstd = float(np.std(cols))
                differs = float(np.round(np.float64(npstd), 2)) != exact_round(v)
                if not differs and got % 4:
                    continue              # mostly cases where the two roundings differ
                stats = run_classic(DuckBam(["c"], [v]), "c", 0, n)
                cases.append({"n": n, "a": a, "b": b, "d1": d1, "d2": d2, "y": y, "seed": seed,
                              "np_std_hex": npstd.hex(), "exact_rounding_differs": differs,
                              "stats": stats})
                got += 1
    with open(os.path.join(HERE, "std_ties.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_std_ties.py", "cases": cases}, fh, indent=1)
    print(len(cases), sum(c["exact_rounding_differs"] for c in cases))


if __name__ == "__main__":
    main()
