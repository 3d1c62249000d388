"""ORACLE / TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/liboracle.so
(the C restatement in oracle/oracle.c).  Imported by tests/ and by bench.py's
cpu_baseline leg only."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

STAT_DTYPE = np.dtype([("n", "<i8"), ("sum", "<i8"), ("sumsq", "<u8"), ("min", "<i8"),
                       ("max", "<i8"), ("med_lo", "<i8"), ("med_hi", "<i8"),
                       ("q23_sum", "<i8"), ("q23_cnt", "<i8")])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
                os.path.getmtime(os.path.join(HERE, f)) for f in ("oracle.c", "scan_oracle.c")):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.orc_pileup_classic.restype = ctypes.c_int64
        _lib.orc_scan.restype = ctypes.c_int64
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else None


def layout(lengths, tid, pos, span):
    """extents (max of length and furthest read end) and offsets."""
    lengths = np.asarray(lengths, dtype=np.int64)
    ext = lengths.copy()
    if len(tid):
        ends = pos.astype(np.int64) + span
        np.maximum.at(ext, tid, ends)
    coff = np.zeros(len(ext) + 1, dtype=np.int64)
    coff[1:] = np.cumsum(ext)
    return ext, coff


def depth(lengths, tid, pos, span, method="interval"):
    """Concatenated depth vector and (extent, offset) per contig."""
    tid = np.ascontiguousarray(tid, np.int32)
    pos = np.ascontiguousarray(pos, np.int32)
    span = np.ascontiguousarray(span, np.int32)
    ext, coff = layout(lengths, tid, pos, span)
    out = np.zeros(int(coff[-1]), dtype=np.int32)
    fn = load().orc_depth_interval if method == "interval" else load().orc_depth_columnwalk
    fn(ctypes.c_int32(len(ext)), _p(ext), _p(coff), ctypes.c_int64(len(tid)), _p(tid), _p(pos),
       _p(span), _p(out))
    return out, ext, coff


def region_stats(depth_vec, ext, coff, rtid, rstart, rend):
    rtid = np.ascontiguousarray(rtid, np.int32)
    rstart = np.ascontiguousarray(rstart, np.int64)
    rend = np.ascontiguousarray(rend, np.int64)
    out = np.zeros(len(rtid), dtype=STAT_DTYPE)
    load().orc_region_stats(_p(depth_vec), _p(coff), _p(ext), ctypes.c_int64(len(rtid)), _p(rtid),
                            _p(rstart), _p(rend), _p(out))
    return out


def pileup_classic(tid, pos, span, rtid, rstart, rend):
    """classic() per region, end to end on one core; returns (out7, columns)."""
    tid = np.ascontiguousarray(tid, np.int32)
    pos = np.ascontiguousarray(pos, np.int32)
    span = np.ascontiguousarray(span, np.int32)
    rtid = np.ascontiguousarray(rtid, np.int32)
    rstart = np.ascontiguousarray(rstart, np.int64)
    rend = np.ascontiguousarray(rend, np.int64)
    out = np.zeros((len(rtid), 7), dtype=np.float64)
    ms = int(span.max()) if len(span) else 0
    cols = load().orc_pileup_classic(ctypes.c_int64(len(tid)), _p(tid), _p(pos), _p(span),
                                     ctypes.c_int32(ms), ctypes.c_int64(len(rtid)), _p(rtid),
                                     _p(rstart), _p(rend), _p(out))
    return out, cols


def pileup_classic_parallel(tid, pos, span, rtid, rstart, rend, threads):
    """pileup_classic with the regions spread over `threads` host threads
    (contig-parallel: the C call releases the GIL; one task per region, the
    costliest first — positions plus aligned bases — from a shared queue, so
    deep contigs do not pile onto one thread).  Same rows as the one-core
    call."""
    from concurrent.futures import ThreadPoolExecutor
    tid = np.ascontiguousarray(tid, np.int32)
    pos = np.ascontiguousarray(pos, np.int32)
    span = np.ascontiguousarray(span, np.int32)
    rtid = np.ascontiguousarray(rtid, np.int32)
    rstart = np.ascontiguousarray(rstart, np.int64)
    rend = np.ascontiguousarray(rend, np.int64)
    out = np.zeros((len(rtid), 7), dtype=np.float64)
    ms = int(span.max()) if len(span) else 0
    per_tid = np.bincount(tid, weights=span.astype(np.float64),
                          minlength=int(max(rtid.max(initial=-1), tid.max(initial=-1))) + 1)
    cost = (rend - rstart).astype(np.float64) + per_tid[rtid]
    order = np.argsort(-cost, kind="stable")
    groups = [order[k:k + 1] for k in range(len(order))]
    lib = load()

    def run(g):
        g = np.sort(g)
        o = np.zeros((len(g), 7), dtype=np.float64)
        gt, gs, ge = (np.ascontiguousarray(x[g]) for x in (rtid, rstart, rend))
        c = lib.orc_pileup_classic(ctypes.c_int64(len(tid)), _p(tid), _p(pos), _p(span),
                                   ctypes.c_int32(ms), ctypes.c_int64(len(g)), _p(gt), _p(gs),
                                   _p(ge), _p(o))
        out[g] = o
        return c

    with ThreadPoolExecutor(threads) as ex:
        cols = sum(ex.map(run, [g for g in groups if len(g)]))
    return out, cols


def scan(cfg, batch, ref=None, ref_off=None, ref_len=None, base_rows=0, isize_cap=128):
    """orc_scan over one SoA batch (rlen, flag, gpos, gisize, ref_id, seq_off,
    seq); cfg is a metacov_amd._lib.ScanConfig (same layout).  Returns the
    group-major tables (base, kmer, mirror, isize, isize_max) and the read
    count."""
    lib = load()
    G = 1 << cfg.n_flags
    rlen, flag, gpos, gisize, ref_id, seq_off, seq = batch
    base = np.zeros((G, base_rows, 5), np.uint32)
    kmer = np.zeros((G, (4 ** cfg.kmer_k + 1) if cfg.kmer_on else 0, cfg.kmer_nk), np.uint32)
    mirror = np.zeros((G, cfg.mirror_n + 1, 2), np.uint32)
    isize = np.zeros((G, isize_cap), np.uint32)
    isize_max = np.zeros(G, np.int32)
    ref = np.zeros(1, np.uint8) if ref is None else ref
    ref_off = np.zeros(1, np.int64) if ref_off is None else ref_off
    n_ref = 0 if ref_len is None else len(ref_len)
    ref_len = np.zeros(1, np.int64) if ref_len is None else ref_len
    done = lib.orc_scan(ctypes.byref(cfg), ctypes.c_int64(len(rlen)), *[_p(a) for a in (
        rlen, flag, gpos, gisize, ref_id, seq_off, seq, ref, ref_off, ref_len)],
        ctypes.c_int32(n_ref), ctypes.c_int64(base_rows), _p(base), _p(kmer), _p(mirror),
        ctypes.c_int64(isize_cap), _p(isize), _p(isize_max))
    return (base, kmer, mirror, isize, isize_max), done
