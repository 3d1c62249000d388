"""htslib's pileup read cap (pysam's `max_depth`, 8000 by default) — on by
default, as in the reference.

The reference's depth is pysam's `AlignmentFile.pileup(ref, start, end)`
(metacov/pileup.py:13), i.e. htslib's pileup with pysam's default
max_depth=8000: `bam_plp_push` drops a read that starts where its
predecessor started once the pileup's read pool holds more than max_depth
nodes (include/metacov_amd.h, mc_depth_cap_mask).  Each region is its own
query: the records overlapping [start, end) of the region's contig.

The cap can only change a region whose exact maximum depth M is large: at a
push the pool holds the tail node, the kept reads still covering the
previous column (<= M) and the reads of the current start group buffered so
far (<= M + 1, the group's first read may be a span-0 one), so no read is
dropped while 2 + 2M <= max_depth (M <= 3999 for 8000).  `apply_cap` checks
that on the exact rows and recomputes only the regions that fail it, all in
one engine call (`capped_rows`).  Parity with htslib itself is unpinned
(version-dependent, htslib absent here).
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check

HTSLIB_MAX_DEPTH = 8000   # pysam pileup's default max_depth


def cap_mask(tid, pos, span, max_depth=HTSLIB_MAX_DEPTH, n_threads=0):
    """bool keep mask of coordinate-sorted reads under the cap, and the number
    of reads dropped.  Each distinct tid is one pileup query."""
    tid = np.ascontiguousarray(tid, np.int32)
    pos = np.ascontiguousarray(pos, np.int32)
    span = np.ascontiguousarray(span, np.int32)
    keep = np.zeros(len(tid), np.uint8)
    dropped = ctypes.c_int64()
    check(_lib.load().mc_depth_cap_mask(len(tid), _lib.ptr(tid), _lib.ptr(pos), _lib.ptr(span),
                                        int(max_depth), int(n_threads), _lib.ptr(keep),
                                        ctypes.byref(dropped)))
    return keep.view(bool), dropped.value


def cap_mask_device(tid, pos, span, max_depth=HTSLIB_MAX_DEPTH):
    """cap_mask on the device (mc_depth_cap_mask_device) for int32 torch
    tensors on one GPU: (uint8 keep tensor, reads dropped)."""
    import torch
    ts = [t.contiguous().to(torch.int32) for t in (tid, pos, span)]
    n = ts[0].numel()
    keep = torch.empty(n, dtype=torch.uint8, device=ts[0].device)
    torch.cuda.current_stream(ts[0].device).synchronize()
    dropped = ctypes.c_int64()
    check(_lib.load().mc_depth_cap_mask_device(ts[0].device.index or 0, n, *[ctypes.c_void_p(t.data_ptr())
                                                                           for t in ts],
                                               int(max_depth), ctypes.c_void_p(keep.data_ptr()),
                                               ctypes.byref(dropped)))
    return keep, dropped.value


def region_reads(tid, pos, span, t, start, end, max_span=None):
    """Indices of the records of contig t overlapping [start, end) — what
    htslib's region iterator hands the pileup (hts_itr_next tests overlap
    with bam_endpos, at least pos + 1, in every htslib version).  The
    records are coordinate-sorted, so only those starting in
    [start - max_span, end) are examined (max_span: the longest span, at
    least 1; None: computed here)."""
    lo, hi = np.searchsorted(tid, t, "left"), np.searchsorted(tid, t, "right")
    if max_span is None:
        max_span = int(span[lo:hi].max()) if hi > lo else 1
    p = pos[lo:hi]
    a = lo + int(np.searchsorted(p, start - max(int(max_span), 1), "left"))
    b = lo + int(np.searchsorted(p, end, "left"))
    pp = pos[a:b].astype(np.int64)
    e = pp + np.maximum(span[a:b], 1)
    return a + np.nonzero(e > start)[0]


def may_cap(rows, max_depth):
    """Regions whose exact rows the cap could change (2 + 2 * max > cap)."""
    return 2 + 2 * rows["max"].astype(np.int64) > int(max_depth)


def host_intervals(src, contigs):
    """(tid, pos, span) host arrays (header contig ids) holding at least the
    records of `contigs`, from any of the library's BAM sources: a decoded
    BamFile keeps them; a GpuBamFile copies just those contigs' records back
    from HBM; a StreamedBam (intervals never kept on the host) decodes those
    contigs again, through the BAI when there is one, else in bounded
    windows keeping only their records."""
    if hasattr(src, "tid") and getattr(src, "tid", None) is not None:
        return src.tid, src.pos, src.span
    if hasattr(src, "intervals"):
        return src.intervals(contigs)
    from .bam import BamFile, BamStream
    path = src.filename
    legacy = getattr(src, "legacy_endpos", False)
    want = np.unique(np.asarray(contigs, np.int64))
    if os.path.exists(path + ".bai"):
        bf = BamFile(path, contigs=want, legacy_endpos=legacy)
        return bf.tid, bf.pos, bf.span
    parts = []
    with BamStream(path, legacy_endpos=legacy) as st:
        while True:
            k, (t, p, sp) = st.read(1 << 22)
            if k == 0:
                break
            keep = np.isin(t[:k], want)
            parts.append((t[:k][keep], p[:k][keep], sp[:k][keep]))
    if not parts:
        return tuple(np.zeros(0, np.int32) for _ in range(3))
    return tuple(np.concatenate([q[i] for q in parts]) for i in range(3))


def device_intervals(src):
    """(n, (tid, pos, span) device addresses) of a GPU-decoded source's kept
    intervals (GpuBamFile), else None."""
    dptr = getattr(src, "_dptr", None)
    if dptr is None or getattr(src, "_h", None) is None:
        return None
    return int(src.n_kept), tuple(int(p.value or 0) for p in dptr)


def capped_rows(src, tids, starts, ends, lengths, max_depth=HTSLIB_MAX_DEPTH, device=0, with_std=False):
    """Exact stat rows of regions (header contig ids) as pysam's capped
    pileup would fill classic()'s column vector: per region the overlapping
    records and the cap; then ONE engine call over all of them, each region
    its own contig of the batch (the same contig's reads repeated when
    regions share it).  Returns (rows, reads dropped), and with_std:
    engine.numpy_std of the rows on that batch's depth as a third value."""
    from .engine import CoverageEngine, REGION_STAT_DTYPE, numpy_std
    tids = np.asarray(tids, np.int64)
    starts = np.asarray(starts, np.int64)
    ends = np.asarray(ends, np.int64)
    if len(tids) == 0:
        empty = np.zeros(0, dtype=REGION_STAT_DTYPE)
        return (empty, 0, np.zeros(0)) if with_std else (empty, 0)
    local = np.arange(len(tids), dtype=np.int32)
    dev = device_intervals(src)
    if dev is not None:
        # the GPU decode's intervals stay in HBM: query gather, cap and the
        # batch on the device (mc_add_reads_capped)
        eng = CoverageEngine(device)
        try:
            eng.set_contigs(np.asarray(lengths, np.int64)[tids])
            try:
                dropped = eng.add_reads_capped(dev[0], *dev[1], src.local_tid(tids), starts, ends, max_depth)
            except _lib.MetacovError as e:
                if e.code != _lib.MC_E_RANGE:
                    raise
                dev = None   # a span beyond the device walk's ring: the host sweep below
            if dev is not None:
                rows = eng.compute_depth_stats(local, starts, ends)
                std = numpy_std(eng, rows, local, starts, ends) if with_std else None
                return (rows, dropped, std) if with_std else (rows, dropped)
        finally:
            eng.close()
    tid, pos, span = host_intervals(src, tids)
    max_span = int(span.max()) if len(span) else 1
    idx = [region_reads(tid, pos, span, int(t), int(s), int(e), max_span)
           for t, s, e in zip(tids, starts, ends)]
    counts = np.array([len(i) for i in idx], np.int64)
    sel = np.concatenate(idx) if len(idx) else np.zeros(0, np.int64)
    vt = np.repeat(np.arange(len(tids), dtype=np.int32), counts)
    vpos, vspan = pos[sel], span[sel]
    keep, dropped = cap_mask(vt, vpos, vspan, max_depth)
    eng = CoverageEngine(device)
    try:
        eng.set_contigs(np.asarray(lengths, np.int64)[tids])
        eng.add_reads(vt[keep], vpos[keep], vspan[keep])
        rows = eng.compute_depth_stats(local, starts, ends)
        std = numpy_std(eng, rows, local, starts, ends) if with_std else None
    finally:
        eng.close()
    return (rows, dropped, std) if with_std else (rows, dropped)


def apply_cap(src, rows, tids, starts, ends, lengths, max_depth=HTSLIB_MAX_DEPTH, device=0, std=None):
    """Rows of the same regions under the cap: the exact `rows` where the cap
    cannot act (may_cap), the capped recompute elsewhere.  Returns (rows,
    regions recomputed, reads dropped).  std (optional, engine.numpy_std of
    `rows`): its recomputed regions' entries are replaced in place by those
    of the capped rows."""
    if not max_depth or len(rows) == 0:
        return rows, 0, 0
    need = np.nonzero(may_cap(rows, max_depth))[0]
    if len(need) == 0:
        return rows, 0, 0
    sub, dropped, sub_std = capped_rows(src, np.asarray(tids)[need], np.asarray(starts)[need],
                                        np.asarray(ends)[need], lengths, max_depth, device, with_std=True)
    out = rows.copy()
    out[need] = sub
    if std is not None:
        std[need] = sub_std
    return out, len(need), dropped
