"""BAM input through the library's C++ decoder (mc_bam_*).

`BamFile(path)` decodes the whole file once (multi-threaded BGZF inflate)
into coordinate-sorted pileup intervals and keeps the header.  It offers the
parts of `pysam.AlignmentFile` the reference's pileup path touches:
`references` / `lengths` (metacov/cli.py:80, metacov/util.py:64-69),
`mapped` / `unmapped` (cli.py:67-76) and `filename`.

`BamFile(path, contigs=[...])` decodes only those contigs' records through
the BAI index (`<path>.bai`, or `index=`), the way one rank of a multi-GPU
run reads its shard; `contigs=[]` reads the header and the index counts only.
Its engine holds just those contigs (`local_tid` maps header ids to them).
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check

FLAG_FILTER = 0x704   # pysam pileup stepper "all": UNMAP|SECONDARY|QCFAIL|DUP
# include/metacov_amd.h MC_LEGACY_ENDPOS: a mapped read without a
# reference-consuming CIGAR op spans [pos, pos + 1) (htslib <= 1.9
# bam_endpos) instead of current htslib's raw rlen 0 (bam_plp_push)
LEGACY_ENDPOS = 0x10000


def _filter(flag_filter, legacy_endpos):
    return int(flag_filter) | (LEGACY_ENDPOS if legacy_endpos else 0)


def build_index(path, index=None, n_threads=0):
    """Writes the BAI of a coordinate-sorted BAM (`samtools index`), by
    default next to it as <path>.bai."""
    lib = _lib.load()
    check(lib.mc_bam_index_build(os.fspath(path).encode(),
                                 os.fspath(index).encode() if index else None, int(n_threads)))
    return os.fspath(index) if index else os.fspath(path) + ".bai"


def index_stats(index, n_ref):
    """Per-reference (mapped, unmapped) record counts and the records without
    coordinates, from a BAI's pseudo-bins."""
    lib = _lib.load()
    m = np.zeros(n_ref, np.int64)
    u = np.zeros(n_ref, np.int64)
    nc = ctypes.c_int64()
    check(lib.mc_bam_index_stats(os.fspath(index).encode(), int(n_ref), _lib.ptr(m), _lib.ptr(u),
                                 ctypes.byref(nc)))
    return m, u, nc.value


class BamFile:
    def __init__(self, path, n_threads=0, flag_filter=FLAG_FILTER, keep_cigar=False,
                 contigs=None, index=None, legacy_endpos=False):
        if hasattr(path, "filename"):          # pysam.AlignmentFile
            path = path.filename
        if isinstance(path, bytes):
            path = path.decode()
        self.filename = os.fspath(path)
        self.index = os.fspath(index) if index else None
        self.legacy_endpos = bool(legacy_endpos)
        flag_filter = _filter(flag_filter, legacy_endpos)
        lib = _lib.load()
        h = ctypes.c_void_p()
        if contigs is None:
            self.contigs = None
            check(lib.mc_bam_open(self.filename.encode(), int(n_threads), int(flag_filter),
                                  1 if keep_cigar else 0, ctypes.byref(h)))
        else:
            self.contigs = np.unique(np.asarray(contigs, dtype=np.int32))
            check(lib.mc_bam_open_contigs(self.filename.encode(),
                                          self.index.encode() if self.index else None,
                                          int(n_threads), int(flag_filter), 1 if keep_cigar else 0,
                                          len(self.contigs), _lib.ptr(self.contigs),
                                          ctypes.byref(h)))
        try:
            n = ctypes.c_int32()
            check(lib.mc_bam_n_targets(h, ctypes.byref(n)))
            names, lengths = [], []
            for i in range(n.value):
                nm = ctypes.c_char_p()
                ln = ctypes.c_int64()
                check(lib.mc_bam_target(h, i, ctypes.byref(nm), ctypes.byref(ln)))
                names.append(nm.value.decode())
                lengths.append(ln.value)
            self.references = tuple(names)
            self.lengths = tuple(lengths)
            c = [ctypes.c_int64() for _ in range(4)]
            check(lib.mc_bam_counts(h, *[ctypes.byref(x) for x in c]))
            self.n_records, n_kept, self.mapped, self.unmapped = (x.value for x in c)
            self.tid = np.empty(n_kept, dtype=np.int32)
            self.pos = np.empty(n_kept, dtype=np.int32)
            self.span = np.empty(n_kept, dtype=np.int32)
            if n_kept:
                check(lib.mc_bam_intervals(h, _lib.ptr(self.tid), _lib.ptr(self.pos),
                                           _lib.ptr(self.span)))
            self.cig_off = self.cigar = None
            if keep_cigar:
                nw = ctypes.c_int64()
                check(lib.mc_bam_n_cigar_words(h, ctypes.byref(nw)))
                self.cig_off = np.empty(n_kept + 1, dtype=np.int64)
                self.cigar = np.empty(nw.value, dtype=np.uint32)
                check(lib.mc_bam_cigars(h, _lib.ptr(self.cig_off), _lib.ptr(self.cigar)))
        finally:
            lib.mc_bam_close(h)
        self._engines = {}

    @property
    def nreferences(self):
        return len(self.references)

    def get_tid(self, name):
        try:
            return self.references.index(name)
        except ValueError:
            raise KeyError(name)

    def aligned_bases(self):
        return int(self.span.astype(np.int64).sum())

    def restrict(self, contigs):
        """This file's records of `contigs` only, as a contig-shard BamFile
        (the no-index fallback of a multi-GPU run: decode all, keep a shard)."""
        out = object.__new__(BamFile)
        out.__dict__.update(self.__dict__)
        out.contigs = np.unique(np.asarray(contigs, dtype=np.int32))
        keep = np.isin(self.tid, out.contigs)
        out.tid, out.pos, out.span = self.tid[keep], self.pos[keep], self.span[keep]
        if self.cig_off is not None:
            idx = np.nonzero(keep)[0]
            lens = (self.cig_off[idx + 1] - self.cig_off[idx]).astype(np.int64)
            out.cig_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
            sel = np.concatenate([np.arange(self.cig_off[i], self.cig_off[i + 1]) for i in idx]) \
                if len(idx) else np.zeros(0, np.int64)
            out.cigar = self.cigar[sel]
        out._engines = {}
        return out

    def local_tid(self, tid):
        """Engine contig id of header contig id(s) `tid` (identity for a
        whole-file BamFile; KeyError for a contig outside the shard)."""
        if self.contigs is None:
            return tid
        t = np.asarray(tid, dtype=np.int64)
        k = np.searchsorted(self.contigs, t)
        if np.any(k >= len(self.contigs)) or np.any(self.contigs[np.minimum(k, len(self.contigs) - 1)] != t):
            raise KeyError("contig outside this shard: %r" % (tid,))
        return k.astype(np.int32) if t.ndim else int(k)

    def engine(self, device=0, compute=True):
        """A CoverageEngine holding this file's reads (cached per device);
        with compute=True its depth is computed (once).  A contig shard's
        engine holds only its contigs (ids from local_tid)."""
        eng = self._engines.get(device)
        if eng is None:
            from .engine import CoverageEngine
            eng = CoverageEngine(device)
            lengths = np.asarray(self.lengths, dtype=np.int64)
            tid = self.tid
            if self.contigs is not None:
                lengths = lengths[self.contigs]
                tid = np.searchsorted(self.contigs, self.tid).astype(np.int32)
            eng.set_contigs(lengths)
            eng.add_reads(tid, self.pos, self.span)
            # (no explicit prepare: the first compute call prepares the batch,
            # by the direct path when it can take it)
            eng._depth_ready = False
            self._engines[device] = eng
        if compute and not eng._depth_ready:
            eng.compute_depth()
            eng._depth_ready = True
        return eng

    def close(self):
        for e in self._engines.values():
            e.close()
        self._engines.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class BamStream:
    """Bounded-memory decode (mc_bam_stream_*): the BGZF blocks are inflated a
    window at a time and the kept records' intervals are read out in batches,
    in file order.  references / lengths come from the header; record counts
    grow as the file is consumed."""

    def __init__(self, path, n_threads=0, flag_filter=FLAG_FILTER, window_bytes=0,
                 legacy_endpos=False):
        self.filename = os.fspath(getattr(path, "filename", path))
        self._lib = _lib.load()
        self._h = ctypes.c_void_p()
        flag_filter = _filter(flag_filter, legacy_endpos)
        check(self._lib.mc_bam_stream_open(self.filename.encode(), int(n_threads), int(flag_filter),
                                           int(window_bytes), ctypes.byref(self._h)))
        hdr = ctypes.c_void_p()
        check(self._lib.mc_bam_stream_header(self._h, ctypes.byref(hdr)))
        self._hdr = hdr
        n = ctypes.c_int32()
        check(self._lib.mc_bam_n_targets(hdr, ctypes.byref(n)))
        names, lengths = [], []
        for i in range(n.value):
            nm = ctypes.c_char_p()
            ln = ctypes.c_int64()
            check(self._lib.mc_bam_target(hdr, i, ctypes.byref(nm), ctypes.byref(ln)))
            names.append(nm.value.decode())
            lengths.append(ln.value)
        self.references = tuple(names)
        self.lengths = tuple(lengths)

    def counts(self):
        """(records, mapped, unmapped) decoded so far."""
        c = [ctypes.c_int64() for _ in range(4)]
        check(self._lib.mc_bam_counts(self._hdr, *[ctypes.byref(x) for x in c]))
        return c[0].value, c[2].value, c[3].value

    def read(self, cap, out=None):
        """Up to `cap` intervals into `out` = (tid, pos, span) int32 arrays
        (allocated if None); returns (k, out); k = 0 at the end."""
        if out is None:
            out = tuple(np.empty(cap, np.int32) for _ in range(3))
        k = ctypes.c_int64()
        check(self._lib.mc_bam_stream_next(self._h, int(cap), *[_lib.ptr(a) for a in out],
                                           ctypes.byref(k)))
        return k.value, out

    def close(self):
        if self._h:
            self._lib.mc_bam_stream_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()


def _header_of(lib, hdr):
    n = ctypes.c_int32()
    check(lib.mc_bam_n_targets(hdr, ctypes.byref(n)))
    names, lengths = [], []
    for i in range(n.value):
        nm = ctypes.c_char_p()
        ln = ctypes.c_int64()
        check(lib.mc_bam_target(hdr, i, ctypes.byref(nm), ctypes.byref(ln)))
        names.append(nm.value.decode())
        lengths.append(ln.value)
    c = [ctypes.c_int64() for _ in range(4)]
    check(lib.mc_bam_counts(hdr, *[ctypes.byref(x) for x in c]))
    return tuple(names), tuple(lengths), (c[0].value, c[2].value, c[3].value)


# mc_contig_extent: where a contig's records lie (a BAI pseudo-bin)
EXTENT_DTYPE = np.dtype([("beg_voff", "<i8"), ("end_voff", "<i8"), ("n_mapped", "<i8"),
                         ("n_unmapped", "<i8"), ("n_kept", "<i8")])


def index_extents(index, n_ref):
    """The extents table of a BAI (per contig: virtual offsets of its first
    record and of the end of its last one, mapped / unmapped counts) and its
    count of records without coordinates."""
    ext = np.zeros(n_ref, EXTENT_DTYPE)
    nc = ctypes.c_int64()
    check(_lib.load().mc_bam_index_extents(os.fspath(index).encode(), int(n_ref), _lib.ptr(ext),
                                           ctypes.byref(nc)))
    return ext, nc.value


class GpuBamFile:
    """A BAM decoded on the GPU (mc_bam_gpu_*: BGZF inflate and record parse
    in HBM).  Same header, counts and kept intervals as BamFile(path); the
    intervals stay on `device` and go into the engine by a device copy
    (mc_add_reads_device).  Offers what the CLI uses of BamFile: references,
    lengths, mapped, unmapped, engine(), local_tid().

    contigs=[...]: one rank's shard: only the BGZF blocks of
    those contigs are read and inflated, located by the BAI (`index`, default
    <path>.bai) or by an `extents` table (ext, n_no_coor) of a whole-file
    decode (GpuBamFile.extents() on another rank, for a BAM without an
    index).  Its engine holds just those contigs (local_tid maps header ids
    to them); mapped / unmapped are the whole file's, as an index reports."""

    def __init__(self, path, device=0, n_threads=0, flag_filter=FLAG_FILTER, window_bytes=0,
                 legacy_endpos=False, contigs=None, index=None, extents=None):
        self.filename = os.fspath(getattr(path, "filename", path))
        self.device = device
        self.legacy_endpos = bool(legacy_endpos)
        flag_filter = _filter(flag_filter, legacy_endpos)
        self._lib = _lib.load()
        self._h = ctypes.c_void_p()
        self._eng = None
        self._ext = None
        if contigs is None:
            self.contigs = None
            check(self._lib.mc_bam_gpu_open(self.filename.encode(), int(device), int(n_threads),
                                            int(flag_filter), int(window_bytes), ctypes.byref(self._h)))
        else:
            self.contigs = np.unique(np.asarray(contigs, dtype=np.int32))
            if extents is None:
                check(self._lib.mc_bam_gpu_open_contigs(
                    self.filename.encode(), os.fspath(index).encode() if index else None, int(device),
                    int(n_threads), int(flag_filter), len(self.contigs), _lib.ptr(self.contigs),
                    ctypes.byref(self._h)))
            else:
                ext = np.ascontiguousarray(extents[0], EXTENT_DTYPE)
                check(self._lib.mc_bam_gpu_open_extents(
                    self.filename.encode(), int(device), int(n_threads), int(flag_filter), len(ext),
                    _lib.ptr(ext), int(extents[1]), len(self.contigs), _lib.ptr(self.contigs),
                    ctypes.byref(self._h)))
        hdr = ctypes.c_void_p()
        check(self._lib.mc_bam_gpu_header(self._h, ctypes.byref(hdr)))
        self.references, self.lengths, (self.n_records, self.mapped, self.unmapped) = \
            _header_of(self._lib, hdr)
        n = ctypes.c_int64()
        self._dptr = [ctypes.c_void_p() for _ in range(3)]
        check(self._lib.mc_bam_gpu_intervals_device(self._h, ctypes.byref(n),
                                                    *[ctypes.byref(p) for p in self._dptr]))
        self.n_kept = n.value

    @property
    def nreferences(self):
        return len(self.references)

    def get_tid(self, name):
        try:
            return self.references.index(name)
        except ValueError:
            raise KeyError(name)

    local_tid = BamFile.local_tid

    def extents(self):
        """(EXTENT_DTYPE table, records without coordinates): per contig the
        virtual offsets of its first record and of the end of its last one,
        mapped / unmapped / kept counts — computed on the device during the
        decode (a whole file), what its BAI would hold."""
        if self._ext is None:
            ext = np.zeros(len(self.references), EXTENT_DTYPE)
            nc = ctypes.c_int64()
            check(self._lib.mc_bam_gpu_extents(self._h, len(ext), _lib.ptr(ext), ctypes.byref(nc)))
            self._ext = (ext, nc.value)
        return self._ext

    def restrict(self, contigs):
        """Keeps only `contigs`' records (a rank's shard of this whole-file
        decode), in place on the device; returns self, now a contig-subset
        file (local_tid, engine over those contigs)."""
        if self.contigs is not None:
            raise ValueError("already a contig subset")
        sel = np.unique(np.asarray(contigs, dtype=np.int32))
        self.extents()                  # the whole file's table, before the subset
        if self._eng is not None:
            self._eng.close()
            self._eng = None
        check(self._lib.mc_bam_gpu_restrict(self._h, len(sel), _lib.ptr(sel)))
        self.contigs = sel
        self._ext = None
        n = ctypes.c_int64()
        check(self._lib.mc_bam_gpu_intervals_device(self._h, ctypes.byref(n),
                                                    *[ctypes.byref(p) for p in self._dptr]))
        self.n_kept = n.value
        return self

    def _range(self, first, count):
        out = tuple(np.empty(count, np.int32) for _ in range(3))
        if count:
            check(self._lib.mc_bam_gpu_intervals_range(self._h, int(first), int(count),
                                                       *[_lib.ptr(a) for a in out]))
        return out

    def intervals(self, contigs=None):
        """(tid, pos, span) host arrays with header contig ids, in file order:
        every kept record, or (contigs=[...]) only the records of those
        contigs, copied back from HBM slice by slice."""
        if contigs is None:
            tid, pos, span = self._range(0, self.n_kept)
        else:
            ext, _ = self.extents()
            kept = ext["n_kept"]
            order = np.argsort(ext["beg_voff"], kind="stable")
            first = np.zeros(len(kept), np.int64)
            first[order] = np.cumsum(kept[order]) - kept[order]
            want = np.unique(np.asarray(contigs, np.int64))
            want = want[kept[want] > 0]
            want = want[np.argsort(first[want], kind="stable")]
            parts = [self._range(first[t], kept[t]) for t in want]
            tid, pos, span = (np.concatenate([p[i] for p in parts]) if parts else np.zeros(0, np.int32)
                              for i in range(3))
        if self.contigs is not None and len(tid):
            tid = self.contigs[tid]
        return tid, pos, span

    def trim(self):
        """Releases the decode's staging buffers in HBM (compressed file,
        inflated stream, block and segment tables); the intervals, the
        extents table and the engine stay.  Returns the bytes released."""
        freed = ctypes.c_int64()
        check(self._lib.mc_bam_gpu_trim(self._h, ctypes.byref(freed)))
        return freed.value

    def timings(self):
        t = _lib.GpuDecodeTimings()
        check(self._lib.mc_bam_gpu_stats(self._h, ctypes.byref(t)))
        return {k: getattr(t, k) for k, _ in t._fields_}

    def engine(self, device=None, compute=True):
        if device is not None and device != self.device:
            raise ValueError("a GpuBamFile's reads live on device %d" % self.device)
        if self._eng is None:
            from .engine import CoverageEngine
            eng = CoverageEngine(self.device)
            lengths = np.asarray(self.lengths, dtype=np.int64)
            eng.set_contigs(lengths if self.contigs is None else lengths[self.contigs])
            if self.n_kept:
                eng._check(self._lib.mc_add_reads_device(eng._h, self.n_kept, *self._dptr))
            eng._depth_ready = False
            self._eng = eng
        if compute and not self._eng._depth_ready:
            self._eng.compute_depth()
            self._eng._depth_ready = True
        return self._eng

    def close(self):
        if self._eng is not None:
            self._eng.close()
            self._eng = None
        if self._h:
            self._lib.mc_bam_gpu_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedInt32:
    """int32 numpy array over page-locked host memory (mc_pinned_alloc), so
    mc_add_reads_async's DMA overlaps the host's next decode."""

    def __init__(self, n):
        self._lib = _lib.load()
        self._p = ctypes.c_void_p()
        check(self._lib.mc_pinned_alloc(int(n) * 4, ctypes.byref(self._p)))
        self.array = np.ctypeslib.as_array((ctypes.c_int32 * int(n)).from_address(self._p.value))

    def free(self):
        if self._p:
            self.array = None
            self._lib.mc_pinned_free(self._p)
            self._p = None

    def __del__(self):
        self.free()


def _host_batch(n, pinned):
    if pinned:
        bufs = [PinnedInt32(n) for _ in range(3)]
        return tuple(b.array for b in bufs), bufs
    return tuple(np.empty(n, np.int32) for _ in range(3)), None


class StreamedBam:
    """The pileup path over a BAM of any size: the file is decoded in windows
    and fed to the GPU through two pinned host batches (the H2D copy of one
    overlaps the decode of the next), so host memory stays bounded.  Offers
    what the CLI uses of BamFile: references, lengths, mapped, unmapped,
    engine(), local_tid()."""

    def __init__(self, path, device=0, n_threads=0, flag_filter=FLAG_FILTER,
                 batch_reads=1 << 22, window_bytes=0, pinned=True, legacy_endpos=False):
        from .engine import CoverageEngine
        self.filename = os.fspath(getattr(path, "filename", path))
        self.contigs = None
        self.legacy_endpos = bool(legacy_endpos)
        with BamStream(self.filename, n_threads, flag_filter, window_bytes, legacy_endpos) as st:
            self.references, self.lengths = st.references, st.lengths
            eng = CoverageEngine(device)
            eng.set_contigs(np.asarray(self.lengths, dtype=np.int64))
            bufs = [_host_batch(batch_reads, pinned) for _ in range(2)]
            k, _ = st.read(batch_reads, bufs[0][0])
            if k:
                eng.add_reads_async(*[a[:k] for a in bufs[0][0]])
            i = 1
            while True:
                k, _ = st.read(batch_reads, bufs[i][0])     # overlaps the other batch's copy
                eng.synchronize()
                if k == 0:
                    break
                eng.add_reads_async(*[a[:k] for a in bufs[i][0]])
                i ^= 1
            eng.synchronize()
            self.n_records, self.mapped, self.unmapped = st.counts()
        eng._depth_ready = False
        self._eng, self._device = eng, device

    def local_tid(self, tid):
        return tid

    def engine(self, device=0, compute=True):
        if device != self._device:
            raise ValueError("a StreamedBam's reads live on device %d" % self._device)
        if compute and not self._eng._depth_ready:
            self._eng.compute_depth()
            self._eng._depth_ready = True
        return self._eng

    def close(self):
        self._eng.close()
