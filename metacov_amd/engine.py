"""Python handle of one GPU coverage context (mc_ctx).

    eng = CoverageEngine(device=0)
    eng.set_contigs(lengths)
    eng.add_reads(tid, pos, span)          # numpy (host) or torch (device)
    eng.compute_depth()                    # K2 on the GPU
    eng.depth(tid, start, end)             # int32 numpy
    eng.region_stats(tids, starts, ends)   # structured numpy, exact integers
    classic_stats(row)                     # -> the dict pileup.classic returns

The statistics formatting here is the host half of the reference's
`pileup.classic` (metacov/pileup.py:18-26): every value classic reports is a
closed form of the exact integer row the GPU returns (see
include/metacov_amd.h, mc_region_stat).
"""
import ctypes
import math
from fractions import Fraction

import numpy as np

from . import _lib
from ._lib import check, ptr

REGION_STAT_DTYPE = np.dtype([("n", "<i8"), ("sum", "<i8"), ("sumsq", "<u8"), ("min", "<i8"),
                              ("max", "<i8"), ("med_lo", "<i8"), ("med_hi", "<i8"),
                              ("q23_sum", "<i8"), ("q23_cnt", "<i8")])
assert REGION_STAT_DTYPE.itemsize == ctypes.sizeof(_lib.RegionStat) == 72


def _np_round2(x):
    """round(np.float64, 2) as numpy implements it (np.round: rint(x*100)/100)."""
    return float(np.round(np.float64(x), 2))


STD_TIE_REL = 1e-9   # |100 std - (k + 1/2)| below this (relative): numpy's own value decides


def std_near_tie(rows, rel=None):
    """bool mask of the rows whose round(np.std, 2) could differ from the
    rounding of the exact standard deviation: 100 * std within `rel`
    (relative) of a k + 1/2 boundary.  numpy's float64 std is within a few
    ulps times log2(n) of the exact value (~1e-14 relative), so outside this
    window both round alike; inside it, numpy_std() computes numpy's value.
    rel None: STD_TIE_REL (read at call time)."""
    rel = STD_TIE_REL if rel is None else rel
    out = np.zeros(len(rows), bool)
    for i, r in enumerate(rows):
        n = int(r["n"])
        if n <= 0:
            continue
        s = int(r["sum"])
        num = n * int(r["sumsq"]) - s * s
        if num <= 0:
            continue
        x = 100.0 * math.sqrt(num / (n * n))
        out[i] = abs(x - math.floor(x) - 0.5) <= rel * max(x, 1.0)
    return out


def numpy_std(eng, rows, tids, starts, ends, rel=None):
    """float64 per row: np.std(columns) bit for bit (pileup.py:22) for the
    rows near a rounding tie (std_near_tie), NaN elsewhere.  `eng` holds the
    depth vector the rows came from; tids are its contig ids.  numpy's
    summation order runs on the device (mc_region_np_sqdev)."""
    out = np.full(len(rows), np.nan)
    need = np.nonzero(std_near_tie(rows, rel))[0]
    if len(need) == 0:
        return out
    n = rows["n"][need].astype(np.float64)
    means = rows["sum"][need].astype(np.float64) / n          # np.mean (exact sum, one division)
    t = eng.np_sqdev(np.asarray(tids)[need], np.asarray(starts)[need], np.asarray(ends)[need], means)
    out[need] = np.sqrt(t / n)                                # ret / rcount, then sqrt
    return out


def classic_stats(row, np_std=None):
    """dict(min, max, med, std, avg, q23, sum) from one exact stat row.

    Mirrors metacov/pileup.py:18-26 on the float64 column vector:
      min/max/sum  int(np.amin/np.amax/np.sum)          -> exact integers
      med          int(np.median): mean of ranks (n-1)//2 and n//2, truncated
      avg          round(np.mean, 2): float64(sum)/n is what np.mean returns
                   for integer-valued float64 data (its pairwise sum is exact)
      q23          round(np.mean(sorted(c)[n//4 : n-n//4]), 2), likewise exact
      std          round(np.std, 2) (ddof=0): numpy's own float64 value when
                   given (`np_std`, from numpy_std() for rows near a rounding
                   tie), else from the exact variance
    Raises ValueError for an empty region as classic does (zero-size
    reduction in np.amin).
    """
    n = int(row["n"])
    if n <= 0:
        raise ValueError("zero-size array to reduction operation minimum which has no identity")
    s = int(row["sum"])
    sq = int(row["sumsq"])
    if np_std is not None and not math.isnan(np_std):
        std = float(np_std)
    else:
        var = Fraction(n * sq - s * s, n * n)
        std = math.sqrt(float(var)) if var > 0 else 0.0
    avg = float(np.float64(s) / np.float64(n))
    q23 = float(np.float64(int(row["q23_sum"])) / np.float64(int(row["q23_cnt"])))
    med = (int(row["med_lo"]) + int(row["med_hi"])) // 2
    return {
        "min": int(row["min"]),
        "max": int(row["max"]),
        "med": med,
        "std": _np_round2(std),
        "avg": _np_round2(avg),
        "q23": _np_round2(q23),
        "sum": s,
    }


def _is_torch(x):
    return type(x).__module__.startswith("torch")


class CoverageEngine:
    """One mc_ctx on one GPU.  Not thread-safe (one engine per thread/GPU)."""

    def __init__(self, device=0, lib_path=None):
        self._lib = _lib.load(lib_path)
        h = ctypes.c_void_p()
        check(self._lib.mc_ctx_create(int(device), ctypes.byref(h)), self._lib)
        self._check = lambda rc: check(rc, self._lib)
        self._h = h
        self.device = int(device)
        self.lengths = np.zeros(0, dtype=np.int64)
        self._rcache = None   # the last region arrays passed as-is and their C arguments

    # -- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            self._lib.mc_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_stream(self, hip_stream_ptr):
        self._check(self._lib.mc_ctx_set_stream(self._h, ctypes.c_void_p(hip_stream_ptr or None)))

    # -- inputs
    def set_contigs(self, lengths):
        lengths = np.ascontiguousarray(lengths, dtype=np.int64)
        self._check(self._lib.mc_set_contigs(self._h, len(lengths), ptr(lengths)))
        self.lengths = lengths

    def add_reads(self, tid, pos, span):
        """Coordinate-sorted pileup intervals.  numpy arrays are copied from
        host memory; torch tensors on this ctx's GPU are copied device-side."""
        if _is_torch(tid):
            import torch
            ts = [t.contiguous().to(torch.int32) for t in (tid, pos, span)]
            torch.cuda.current_stream(ts[0].device).synchronize()   # producer stream -> ctx stream
            n = ts[0].numel()
            if not all(t.is_cuda and t.numel() == n for t in ts):
                raise ValueError("tid/pos/span must be equally sized device tensors")
            self._check(self._lib.mc_add_reads_device(self._h, n, *[ctypes.c_void_p(t.data_ptr()) for t in ts]))
            return
        arrs = [np.ascontiguousarray(a, dtype=np.int32) for a in (tid, pos, span)]
        n = len(arrs[0])
        if not all(len(a) == n for a in arrs):
            raise ValueError("tid/pos/span lengths differ")
        self._check(self._lib.mc_add_reads(self._h, n, *[ptr(a) for a in arrs]))

    def add_reads_async(self, tid, pos, span):
        """Host int32 arrays (pinned for a real overlap) copied asynchronously
        on the ctx stream; keep them unchanged until synchronize()."""
        arrs = [np.ascontiguousarray(a, dtype=np.int32) for a in (tid, pos, span)]
        if any(a.ctypes.data != np.asarray(b).ctypes.data for a, b in zip(arrs, (tid, pos, span))):
            raise ValueError("add_reads_async needs contiguous int32 arrays (no copies)")
        n = len(arrs[0])
        self._check(self._lib.mc_add_reads_async(self._h, n, *[ptr(a) for a in arrs]))

    def add_reads_cigar(self, tid, pos, cig_off, cigar):
        tid = np.ascontiguousarray(tid, dtype=np.int32)
        pos = np.ascontiguousarray(pos, dtype=np.int32)
        cig_off = np.ascontiguousarray(cig_off, dtype=np.int64)
        cigar = np.ascontiguousarray(cigar, dtype=np.uint32)
        if len(cig_off) != len(tid) + 1:
            raise ValueError("cig_off must have n + 1 entries")
        self._check(self._lib.mc_add_reads_cigar(self._h, len(tid), ptr(tid), ptr(pos), ptr(cig_off),
                                           ptr(cigar)))

    def add_reads_cigar_device(self, tid, pos, cig_off, cigar):
        """Raw-CIGAR batch already in this GPU's memory (torch tensors: int32
        tid/pos, int64 cig_off with n + 1 entries starting at 0, int32/uint32
        cigar words).  tid/pos (any integer dtype) are copied before this
        returns; cig_off/cigar are borrowed until the next prepare() (K1 reads
        them there) — this engine keeps references to them until then."""
        import torch
        tid = tid.contiguous().to(torch.int32)
        pos = pos.contiguous().to(torch.int32)
        if not (cig_off.is_contiguous() and cig_off.dtype == torch.int64 and cigar.is_contiguous()
                and cigar.dtype in (torch.int32, torch.uint32)):
            raise ValueError("cig_off must be contiguous int64 and cigar contiguous 32-bit")
        n = tid.numel()
        if pos.numel() != n or cig_off.numel() != n + 1:
            raise ValueError("need n tid/pos and n + 1 cig_off entries")
        torch.cuda.current_stream(tid.device).synchronize()
        self._borrowed = (cig_off, cigar)
        self._check(self._lib.mc_add_reads_cigar_device(
            self._h, n, ctypes.c_void_p(tid.data_ptr()), ctypes.c_void_p(pos.data_ptr()),
            ctypes.c_void_p(cig_off.data_ptr()), ctypes.c_void_p(cigar.data_ptr())))

    def add_reads_capped(self, n, d_tid, d_pos, d_span, qtid, qstart, qend, max_depth):
        """The capped recompute's batch from device intervals (addresses of
        n coordinate-sorted int32 tid / pos / span): region r's pileup query,
        capped, as contig r (mc_add_reads_capped).  Returns the reads
        dropped."""
        qtid = np.ascontiguousarray(qtid, dtype=np.int32)
        qstart = np.ascontiguousarray(qstart, dtype=np.int64)
        qend = np.ascontiguousarray(qend, dtype=np.int64)
        dropped = ctypes.c_int64()
        self._check(self._lib.mc_add_reads_capped(
            self._h, int(n), ctypes.c_void_p(d_tid), ctypes.c_void_p(d_pos), ctypes.c_void_p(d_span), len(qtid),
            ptr(qtid), ptr(qstart), ptr(qend), int(max_depth), ctypes.byref(dropped)))
        return dropped.value

    def clear_reads(self):
        """Drop the reads (contigs stay): the next batch starts empty."""
        self._check(self._lib.mc_clear_reads(self._h))
        self._borrowed = None

    def prepare(self):
        self._check(self._lib.mc_prepare(self._h))

    def set_direct_prepare(self, enable=True):
        """Direct per-batch prepare on (default) or off (always mc_prepare):
        see include/metacov_amd.h."""
        self._check(self._lib.mc_set_direct_prepare(self._h, 1 if enable else 0))

    def set_legacy_endpos(self, legacy=True):
        """K1's span for a CIGAR without reference-consuming ops: 1 (htslib
        <= 1.9 bam_endpos) instead of 0 (current bam_plp_push)."""
        self._check(self._lib.mc_set_legacy_endpos(self._h, 1 if legacy else 0))

    def invalidate(self):
        """Drop the prepared index: the next compute call re-prepares the
        same device reads, as for a fresh batch."""
        self._check(self._lib.mc_invalidate(self._h))

    # -- compute
    def compute_depth(self):
        self._check(self._lib.mc_compute_depth(self._h))

    def depth(self, tid, start=0, end=None):
        if end is None:
            end = int(self.lengths[tid])
        out = np.empty(max(0, end - start), dtype=np.int32)
        self._check(self._lib.mc_get_depth(self._h, int(tid), int(start), int(end), ptr(out)))
        return out

    def depth_device(self):
        p = ctypes.c_void_p()
        n = ctypes.c_int64()
        self._check(self._lib.mc_depth_device(self._h, ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def contig_offset(self, tid):
        o, e = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._lib.mc_contig_offset(self._h, int(tid), ctypes.byref(o), ctypes.byref(e)))
        return o.value, e.value

    def region_stats(self, tids, starts, ends):
        tids = np.ascontiguousarray(tids, dtype=np.int32)
        starts = np.ascontiguousarray(starts, dtype=np.int64)
        ends = np.ascontiguousarray(ends, dtype=np.int64)
        out = np.zeros(len(tids), dtype=REGION_STAT_DTYPE)
        self._check(self._lib.mc_region_stats(self._h, len(tids), ptr(tids), ptr(starts), ptr(ends),
                                        ptr(out)))
        return out

    def region_stats_device(self, tids, starts, ends, d_out_ptr):
        tids = np.ascontiguousarray(tids, dtype=np.int32)
        starts = np.ascontiguousarray(starts, dtype=np.int64)
        ends = np.ascontiguousarray(ends, dtype=np.int64)
        self._check(self._lib.mc_region_stats_device(self._h, len(tids), ptr(tids), ptr(starts), ptr(ends),
                                               ctypes.c_void_p(d_out_ptr)))

    def np_sqdev(self, tids, starts, ends, means):
        """numpy's float64 sum of squared deviations from `means` of each
        region's column vector, in numpy's summation order (float64 array)."""
        tids = np.ascontiguousarray(tids, dtype=np.int32)
        starts = np.ascontiguousarray(starts, dtype=np.int64)
        ends = np.ascontiguousarray(ends, dtype=np.int64)
        means = np.ascontiguousarray(means, dtype=np.float64)
        out = np.zeros(len(tids), dtype=np.float64)
        self._check(self._lib.mc_region_np_sqdev(self._h, len(tids), ptr(tids), ptr(starts), ptr(ends),
                                                 ptr(means), ptr(out)))
        return out

    def compute_depth_stats(self, tids, starts, ends):
        """K2 with the region statistics fused in (non-overlapping regions),
        else K2 + K3.  Returns the exact rows like region_stats()."""
        tids = np.ascontiguousarray(tids, dtype=np.int32)
        starts = np.ascontiguousarray(starts, dtype=np.int64)
        ends = np.ascontiguousarray(ends, dtype=np.int64)
        out = np.zeros(len(tids), dtype=REGION_STAT_DTYPE)
        self._check(self._lib.mc_compute_depth_stats(self._h, len(tids), ptr(tids), ptr(starts), ptr(ends),
                                               ptr(out)))
        return out

    def _region_args(self, tids, starts, ends):
        """(R, tid, start, end) C arguments.  When the caller passes the same
        int32 / int64 contiguous arrays as last time, their pointers are
        reused (taking three ctypes pointers was ~6 us of a call; the cache
        holds the arrays, so numpy cannot move their data).  The library
        compares the region contents itself."""
        c = self._rcache
        if c is not None and c[0] is tids and c[1] is starts and c[2] is ends:
            return c[3], None
        t = np.ascontiguousarray(tids, dtype=np.int32)
        s = np.ascontiguousarray(starts, dtype=np.int64)
        e = np.ascontiguousarray(ends, dtype=np.int64)
        args = (len(t), ptr(t), ptr(s), ptr(e))
        if t is tids and s is starts and e is ends:
            self._rcache = (tids, starts, ends, args)
        return args, (t, s, e)   # (the converted arrays live through the call)

    def compute_depth_stats_device(self, tids, starts, ends, d_out_ptr):
        args, keep = self._region_args(tids, starts, ends)
        self._check(self._lib.mc_compute_depth_stats_device(self._h, *args, ctypes.c_void_p(d_out_ptr)))
        del keep

    def fused_fallbacks(self):
        """Regions of the last fused call the host's K3 recomputed."""
        v = ctypes.c_int64()
        self._check(self._lib.mc_fused_fallbacks(self._h, ctypes.byref(v)))
        return v.value

    def fused_recomputes(self):
        """Regions of the last fused call recomputed on the device in the call."""
        v = ctypes.c_int64()
        self._check(self._lib.mc_fused_recomputes(self._h, ctypes.byref(v)))
        return v.value

    def aligned_bases(self):
        v = ctypes.c_int64()
        self._check(self._lib.mc_aligned_bases(self._h, ctypes.byref(v)))
        return v.value

    def max_depth(self):
        v = ctypes.c_int32()
        self._check(self._lib.mc_max_depth(self._h, ctypes.byref(v)))
        return v.value

    def timings(self):
        t = _lib.Timings()
        self._check(self._lib.mc_get_timings(self._h, ctypes.byref(t)))
        return {k: getattr(t, k) for k, _ in t._fields_}

    def synchronize(self):
        self._check(self._lib.mc_synchronize(self._h))
