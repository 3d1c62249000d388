"""ORACLE / TEST INFRASTRUCTURE ONLY.

numpy restatement of the reference's region statistics, metacov/pileup.py:
  :10-16  float64 column vector of the region, positions past the data 0
  :18-26  min/max int(np.amin/np.amax), med int(np.median), std/avg
          round(np.std / np.mean, 2), q23 round(mean of the middle half of
          the sorted vector, 2), sum int(np.sum)
numpy (2.2 here) is the library the reference itself computes these with.
"""
import numpy as np


def region_vector(depth_1d, start, end):
    """classic's `columns` for [start, end) of one contig's depth vector."""
    out = np.zeros(end - start)
    a, b = min(start, len(depth_1d)), min(end, len(depth_1d))
    if b > a:
        out[a - start:b - start] = depth_1d[a:b]
    return out


def classic_from_vector(columns):
    n = len(columns)
    srt = np.sort(columns)
    return {
        "min": int(np.amin(columns)),
        "max": int(np.amax(columns)),
        "med": int(np.median(columns)),
        "std": round(np.std(columns), 2),
        "avg": round(np.mean(columns), 2),
        "q23": round(np.mean(srt[n // 4:n - n // 4]), 2),
        "sum": int(np.sum(columns)),
    }


# ---- np.std's float64 order (pileup.py:22), restated -----------------------
# numpy 2.2's _var: arrmean = umr_sum(arr) / n; x = arr - arrmean; x = x * x;
# ret = umr_sum(x) / n; sqrt.  umr_sum of a float64 vector walks it in
# reduction buffers of NPY_BUFSIZE = 8192 elements, adding each buffer's
# pairwise_sum (numpy/_core/src/umath/loops_utils.h.src: PW_BLOCKSIZE 128,
# eight accumulators, split at n/2 rounded down to a multiple of 8) to the
# running total in turn.  tests/test_npstd.py checks this against np.std bit
# for bit; metacov_amd/csrc/npstd.h is the device version.
NPY_BUFSIZE = 8192


def np_pairwise_sum(a):
    """numpy's pairwise_sum over a float64 sequence (Python floats)."""
    n = len(a)
    if n < 8:
        res = 0.0
        for x in a:
            res += float(x)
        return res
    if n <= 128:
        r = [float(a[j]) for j in range(8)]
        i = 8
        while i < n - n % 8:
            for j in range(8):
                r[j] += float(a[i + j])
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += float(a[i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return np_pairwise_sum(a[:n2]) + np_pairwise_sum(a[n2:])


def np_buffered_sum(a):
    """umr_sum of a float64 vector: buffer sums added in turn from 0."""
    t = 0.0
    for i in range(0, len(a), NPY_BUFSIZE):
        t += np_pairwise_sum(a[i:i + NPY_BUFSIZE])
    return t


def np_std_restated(columns):
    """np.std(columns) (ddof 0) in numpy's own operation order."""
    a = np.asarray(columns, np.float64)
    n = len(a)
    m = np.float64(np_buffered_sum(a)) / np.float64(n)
    x = a - m
    x = x * x
    return float(np.sqrt(np.float64(np_buffered_sum(x)) / np.float64(n)))
