"""htslib's pileup read cap, opt-in (`max_depth`).

The reference's depth is pysam's `AlignmentFile.pileup(ref, start, end)`
(metacov/pileup.py:13), i.e. htslib's pileup with pysam's default
max_depth=8000: `bam_plp_push` drops a read that starts where its
predecessor started once the pileup's read pool holds more than max_depth
nodes (include/metacov_amd.h, mc_depth_cap_mask).  The engine never caps by
default (exact depth); `classic(..., max_depth=8000)` / `metacov pileup
--max-depth 8000` reproduce the cap, per region query as pysam sees it: the
records overlapping [start, end) of the region's contig.  Parity unpinned
(version-dependent htslib behaviour, htslib absent here).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check

HTSLIB_MAX_DEPTH = 8000   # pysam pileup's default max_depth


def cap_mask(tid, pos, span, max_depth=HTSLIB_MAX_DEPTH, n_threads=0):
    """bool keep mask of coordinate-sorted reads under the cap, and the number
    of reads dropped."""
    tid = np.ascontiguousarray(tid, np.int32)
    pos = np.ascontiguousarray(pos, np.int32)
    span = np.ascontiguousarray(span, np.int32)
    keep = np.zeros(len(tid), np.uint8)
    dropped = ctypes.c_int64()
    check(_lib.load().mc_depth_cap_mask(len(tid), _lib.ptr(tid), _lib.ptr(pos), _lib.ptr(span),
                                        int(max_depth), int(n_threads), _lib.ptr(keep),
                                        ctypes.byref(dropped)))
    return keep.view(bool), dropped.value


def region_reads(tid, pos, span, t, start, end):
    """Indices of the records of contig t overlapping [start, end) — what
    htslib's region iterator hands the pileup (bam_endpos: at least pos + 1)."""
    lo, hi = np.searchsorted(tid, t, "left"), np.searchsorted(tid, t, "right")
    p = pos[lo:hi].astype(np.int64)
    e = p + np.maximum(span[lo:hi], 1)
    return lo + np.nonzero((p < end) & (e > start))[0]


def capped_rows(bf, tids, starts, ends, max_depth=HTSLIB_MAX_DEPTH, device=0):
    """Exact stat rows of regions (header contig ids) as pysam's capped
    pileup would fill classic()'s column vector: per region, the overlapping
    records, the cap, then the depth and statistics of the kept reads on the
    GPU (one small engine call per region)."""
    from .engine import CoverageEngine, REGION_STAT_DTYPE
    rows = np.zeros(len(tids), dtype=REGION_STAT_DTYPE)
    dropped = 0
    eng = CoverageEngine(device)
    try:
        for i, (t, s, e) in enumerate(zip(tids, starts, ends)):
            t, s, e = int(t), int(s), int(e)
            idx = region_reads(bf.tid, bf.pos, bf.span, t, s, e)
            keep, d = cap_mask(np.zeros(len(idx), np.int32), bf.pos[idx], bf.span[idx], max_depth)
            dropped += d
            idx = idx[keep]
            eng.set_contigs(np.array([bf.lengths[t]], np.int64))
            eng.add_reads(np.zeros(len(idx), np.int32), bf.pos[idx], bf.span[idx])
            rows[i] = eng.compute_depth_stats(np.zeros(1, np.int32), np.array([s], np.int64),
                                              np.array([e], np.int64))[0]
    finally:
        eng.close()
    return rows, dropped
