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
