"""`pileup.experimental` and `pileup.load_kmerhist` on the MI355X engine
(reference metacov/pileup.py:29-173; SURVEY.md §8 f).

    k_cor = load_kmerhist(open("khist.csv"))                 # pileup.py:29-35
    row = experimental(bam, k_cor, 7, fasta, ref, start, end)  # pileup.py:38-173

Same arguments, result keys, value types, rounding, printed "RCOR is ZERO"
lines and exceptions as the reference.  `bam` is a BAM path or a
`ReadTable`; `fasta` a FASTA path, a `FastaFile` or None.  The work splits
where the data does:

* reads (host C++, `mc_experimental_reads`): one pass over the records each
  region fetches -- mate pairing by name, the k-mer correction of each read,
  pair spans -- reduced to exact aggregates instead of the reference's
  per-position arrays, exact for every field (`covc` keeps its per-position
  float sums, in read order, once a read with 1/rcor != 1 covers the region);
* sequence (GPU, `mc_ecor_run`): the k-mer weights of every window and the
  900-tap normal-pdf correlation, O(length x 900) fp64 per region -- the
  part that dominates the reference's run time (a Python loop with one
  np.inner per position, pileup.py:80-83); `ecor` agrees with the reference
  to floating-point re-association (np.inner is a BLAS dot).

`experimental_batch` runs many regions in one pass each (the CLI's path).
K-mer keys must be K-long A/C/G/T strings (what `metacov scan` counts, and
the only keys a K-long window can match once it is cut at an N); any other
key is dropped with a warning.
"""
import gzip
import logging
import os
import time
import warnings

import numpy as np

from . import _lib

log = logging.getLogger(__name__)

INSERT, SD = 450, 150            # pileup.py:55-56
N_TAPS = 2 * INSERT              # l <= iend - istart (pileup.py:82)
STATUS_ERRORS = {
    1: "'NoneType' object is not subscriptable (read without SEQ: query_alignment_sequence "
       "is None)",
    2: "unsupported operand type(s) for -: 'int' and 'NoneType' (reference_length is None)",
    3: "'NoneType' object is not subscriptable (k_cor is None)",
}


def norm_taps():
    """N(450, 150).pdf(0..900) evaluated as scipy.stats.norm does
    (pileup.py:61): exp(-x^2/2) / sqrt(2 pi) / scale at x = (v - loc) / scale."""
    x = (np.arange(0, 2 * INSERT + 1, dtype=np.float64) - INSERT) / SD
    return np.exp(-x ** 2 / 2.0) / np.sqrt(2 * np.pi) / SD


def load_kmerhist(f, k_len=7):
    """pileup.py:29-35: per R1 / R2, the first count column over the row mean
    of the remaining numeric columns, keyed by k-mer, after dropping
    `Mapped == "Unmapped"` rows and the all-N k-mer.  Non-numeric columns
    (R, Mapped, other flag columns of `metacov scan`) are left out of the
    mean, as pandas < 2.0 did for the reference."""
    import pandas as pd
    table = pd.read_csv(f)
    # attribute access, as the reference's (AttributeError for a missing column)
    drop = (table.Mapped == "Unmapped") | (table.kmer == "N" * k_len)
    table = table.loc[~drop].set_index("kmer")
    numer = table[table.columns[0]]
    denom = table[list(table.columns[1:])].select_dtypes(include="number").mean(axis=1)
    ratio = numer / denom
    by_read = table.R.to_numpy()
    return [ratio[by_read == tag].to_dict() for tag in ("R1", "R2")]


# ------------------------------------------------------------------ inputs

def check_faidx(path):
    """Raises OSError where pysam.FastaFile(path) fails to open a reference
    (metacov/cli.py:59 opens one for every `pileup -f`).  With an existing
    `<path>.fai` (and `.gzi` for BGZF) htslib's fai_load takes the index as
    it is, so nothing is checked.  Otherwise it builds one, and faidx needs
    plain text or BGZF (not plain gzip: "Cannot index files compressed with
    gzip, please use bgzip"), '>' headers, and within a sequence every line
    but the last of one length ("Different line length in sequence").  The
    lines are checked as numpy arrays of their bounds, not one by one."""
    def fail(why):
        raise OSError("error when opening file `%s`: %s" % (path, why))
    with open(path, "rb") as fh:
        head = fh.read(18)
    gz = head[:2] == b"\x1f\x8b"
    if gz:
        bgzf = len(head) >= 16 and head[3] & 4 and head[12:14] == b"BC"
        if not bgzf:
            fail("Cannot index files compressed with gzip, please use bgzip")
    if os.path.exists(path + ".fai") and (not gz or os.path.exists(path + ".gzi")):
        return
    if gz:
        with gzip.open(path, "rb") as fh:
            data = fh.read()
    else:
        with open(path, "rb") as fh:
            data = fh.read()
    buf = np.frombuffer(data, np.uint8)
    nl = np.flatnonzero(buf == 10)
    starts = np.concatenate([[0], nl + 1])
    ends = np.concatenate([nl, [len(buf)]])
    lens = ends - starts
    cr = np.zeros(len(lens), bool)
    has = lens > 0
    cr[has] = buf[ends[has] - 1] == 13
    lens = lens - cr
    nonempty = lens > 0
    first = np.zeros(len(lens), np.uint8)
    first[nonempty] = buf[starts[nonempty]]
    is_head = nonempty & (first == ord(">"))
    grp = np.cumsum(is_head)
    seq = np.flatnonzero(nonempty & ~is_head)
    bad = []                                   # (line index, message)
    orphan = seq[grp[seq] == 0]
    if len(orphan):
        i = int(orphan[0])
        bad.append((i, "Format error, unexpected \"%s\" at line %d" % (chr(first[i]), i + 1)))
    seq = seq[grp[seq] > 0]
    if len(seq) > 1:
        g = grp[seq]
        new_grp = np.concatenate([[True], g[1:] != g[:-1]])
        w1 = lens[seq[new_grp]][np.cumsum(new_grp) - 1]      # each group's first line width
        cont = ~new_grp[1:]                                   # line k+1 continues line k's sequence
        prev, cur = seq[:-1], seq[1:]
        broken = cont & ((cur - prev > 1) | (lens[prev] < w1[1:]) | (lens[cur] > w1[1:]))
        if broken.any():
            i = int(cur[np.flatnonzero(broken)[0]])
            h = int(np.flatnonzero(is_head[:i])[-1])
            words = data[starts[h] + 1:ends[h] - cr[h]].split()
            bad.append((i, "Different line length in sequence '%s'" % (words[0].decode() if words else "")))
    if bad:
        fail(min(bad)[1])


class FastaFile:
    """pysam.FastaFile.fetch over a plain or gzip FASTA, held as one byte
    buffer (the sequence the GPU reads).  Names are the first word of each
    '>' line (faidx)."""

    def __init__(self, path):
        with open(path, "rb") as fh:
            gz = fh.read(2) == b"\x1f\x8b"
        with (gzip.open if gz else open)(path, "rb") as fh:
            data = fh.read()
        names, offsets, lengths, parts = [], [], [], []
        total = 0
        for block in data.split(b">")[1:]:
            head, _, body = block.partition(b"\n")
            seq = b"".join(body.split())
            names.append(head.split()[0].decode() if head.split() else "")
            offsets.append(total)
            lengths.append(len(seq))
            parts.append(seq)
            total += len(seq)
        self.filename = path
        self.references = tuple(names)
        self.lengths = tuple(lengths)
        self._index = {n: i for i, n in enumerate(names)}
        self._off = np.array(offsets, np.int64)
        self.buffer = np.frombuffer(b"".join(parts), dtype=np.uint8)

    def span(self, ref, start, end):
        """(offset into `buffer`, bases available) of fetch(ref, start, end);
        KeyError for an unknown sequence, as pysam."""
        i = self._index.get(ref)
        if i is None:
            raise KeyError("sequence '%s' not present" % ref)
        L = self.lengths[i]
        a = min(max(start, 0), L)
        return int(self._off[i]) + a, max(0, min(end, L) - a)

    def fetch(self, ref, start, end):
        off, n = self.span(ref, start, end)
        return self.buffer[off:off + n].tobytes().decode()


class ReadTable:
    """The placed records of a coordinate-sorted BAM as experimental() reads
    them; plays the role of the reference's indexed pysam.AlignmentFile for
    bam.fetch (pileup.py:101).  decode: "host" (mc_reads_open: BGZF inflate
    and record walk on n_threads host threads) or "gpu" (mc_reads_open_gpu:
    the file inflated and walked on GPU `device`, the table copied back);
    None: MC_READS_DECODE, else "host".

    contigs=[...] (GPU decode): one rank's shard -- only the
    placed records of those header contigs, decoded from their BGZF blocks
    alone, located by the BAI (`index`, default <path>.bai) or an `extents`
    table (ext, n_no_coor) as GpuBamFile takes it."""

    def __init__(self, path, k_len=7, n_threads=0, decode=None, device=0, contigs=None, index=None,
                 extents=None):
        self._lib = _lib.load()
        decode = decode or os.environ.get("MC_READS_DECODE", "host")
        if decode not in ("gpu", "host"):
            raise ValueError("decode must be 'gpu' or 'host'")
        if contigs is not None and decode != "gpu":
            raise ValueError("a contig subset is read with decode='gpu'")
        h = _lib.ctypes.c_void_p()
        if contigs is not None:
            from . import bam as _bam
            sel = np.unique(np.asarray(contigs, dtype=np.int32))
            if extents is None:
                n_ref = len(_bam.BamFile(path, contigs=[], index=index).lengths)
                extents = _bam.index_extents(index or str(path) + ".bai", n_ref)
            ext = np.ascontiguousarray(extents[0], _bam.EXTENT_DTYPE)
            rc = self._lib.mc_reads_open_gpu_extents(str(path).encode(), int(device), n_threads, k_len, len(ext),
                                                     _lib.ptr(ext), int(extents[1]), len(sel), _lib.ptr(sel),
                                                     _lib.ctypes.byref(h))
        elif decode == "gpu":
            rc = self._lib.mc_reads_open_gpu(str(path).encode(), int(device), n_threads, k_len,
                                             _lib.ctypes.byref(h))
        else:
            rc = self._lib.mc_reads_open(str(path).encode(), n_threads, k_len, _lib.ctypes.byref(h))
        _lib.check(rc, self._lib)
        self.decode = decode
        self._h = h
        self.k_len = k_len
        self.filename = str(path)
        n_ref = _lib.ctypes.c_int32()
        n_rec = _lib.ctypes.c_int64()
        n_placed = _lib.ctypes.c_int64()
        _lib.check(self._lib.mc_reads_header(h, _lib.ctypes.byref(n_ref), _lib.ctypes.byref(n_rec),
                                             _lib.ctypes.byref(n_placed)), self._lib)
        names, lengths = [], []
        for i in range(n_ref.value):
            nm = _lib.ctypes.c_char_p()
            ln = _lib.ctypes.c_int64()
            _lib.check(self._lib.mc_reads_target(h, i, _lib.ctypes.byref(nm),
                                                 _lib.ctypes.byref(ln)), self._lib)
            names.append(nm.value.decode())
            lengths.append(ln.value)
        self.references = tuple(names)
        self.lengths = tuple(lengths)
        self.n_records = n_rec.value
        self.n_placed = n_placed.value
        self._tid = {n: i for i, n in enumerate(names)}

    def fields(self):
        """The placed records as numpy copies: pos, end, flag, bits, kmer,
        name (bytes), plus per contig first (n_ref + 1) and max_span."""
        c = _lib.ctypes
        ptrs = [c.c_void_p() for _ in range(8)]
        nb = c.c_int64()
        first, span = c.c_void_p(), c.c_void_p()
        _lib.check(self._lib.mc_reads_fields(self._h, *[c.byref(p) for p in ptrs], c.byref(nb),
                                             c.byref(first), c.byref(span)), self._lib)
        n, n_ref = self.n_placed, len(self.references)

        def arr(p, dt, count):
            if count == 0 or not p.value:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(c.cast(p, c.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         (count,)).copy()
        out = {k: arr(p, dt, n) for k, p, dt in zip(
            ("pos", "end", "flag", "bits", "kmer", "name_off", "name_len"), ptrs[:7],
            (np.int32, np.int64, np.uint16, np.uint8, np.uint32, np.uint64, np.uint8))}
        arena = c.string_at(ptrs[7], nb.value) if nb.value else b""
        out["name"] = [arena[o:o + ln] for o, ln in zip(out.pop("name_off").tolist(),
                                                         out.pop("name_len").tolist())]
        out["first"] = arr(first, np.int64, n_ref + 1)
        out["max_span"] = arr(span, np.int64, n_ref)
        return out

    def get_tid(self, ref):
        if ref not in self._tid:
            raise ValueError("invalid contig `%s`" % ref)
        return self._tid[ref]

    def close(self):
        if getattr(self, "_h", None):
            self._lib.mc_reads_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class KmerTables:
    """k_cor (two dicts, R1 / R2: pileup.py:35) as dense tables over the 4^K
    A/C/G/T codes (first base most significant)."""

    def __init__(self, k_cor, k_len):
        if not 1 <= k_len <= 13:
            raise ValueError("k-mer length %d outside 1..13" % k_len)
        self.k_len = k_len
        n = 4 ** k_len
        self.val = np.zeros((2, n), np.float64)
        self.has = np.zeros((2, n), np.uint8)
        code = {b: i for i, b in enumerate("ACGT")}
        dropped = 0
        for which, table in enumerate(k_cor):
            for key, v in table.items():
                if not isinstance(key, str) or len(key) != k_len or any(c not in code for c in key):
                    dropped += 1
                    continue
                c = 0
                for ch in key:
                    c = (c << 2) | code[ch]
                self.val[which, c] = float(v)
                self.has[which, c] = 1
        if dropped:
            log.warning("%d k-mer keys are not %d-long A/C/G/T strings and can never match; "
                        "dropped", dropped, k_len)

    def decode(self, c):
        return "".join("ACGT"[(c >> (2 * (self.k_len - 1 - m))) & 3] for m in range(self.k_len))


class EcorEngine:
    """The GPU side (mc_ecor_*): one FASTA resident in HBM, one k_cor."""

    def __init__(self, device=0):
        self._lib = _lib.load()
        h = _lib.ctypes.c_void_p()
        _lib.check(self._lib.mc_ecor_create(device, _lib.ctypes.byref(h)), self._lib)
        self._h = h
        self._fasta = None
        self._tables = None
        self.kernel_ms = 0.0

    def set_sequence(self, fasta):
        if self._fasta is not fasta:
            buf = np.ascontiguousarray(fasta.buffer)
            _lib.check(self._lib.mc_ecor_set_sequence(self._h, buf.size, buf.ctypes.data),
                       self._lib)
            self._fasta = fasta

    def set_tables(self, tables):
        if self._tables is not tables:
            fwd = np.ascontiguousarray(tables.val[0] * tables.has[0])
            rev = np.ascontiguousarray(tables.val[1] * tables.has[1])
            taps = np.ascontiguousarray(norm_taps()[:N_TAPS])
            _lib.check(self._lib.mc_ecor_set_tables(self._h, tables.k_len, fwd.ctypes.data,
                                                    rev.ctypes.data, N_TAPS, taps.ctypes.data),
                       self._lib)
            self._tables = tables

    def run(self, base, n_avail, length):
        base = np.ascontiguousarray(base, np.int64)
        n_avail = np.ascontiguousarray(n_avail, np.int64)
        length = np.ascontiguousarray(length, np.int64)
        R = length.size
        inner = np.zeros(R, np.float64)
        gc = np.zeros(R, np.int64)
        at = np.zeros(R, np.int64)
        ms = _lib.ctypes.c_float()
        _lib.check(self._lib.mc_ecor_run(self._h, R, base.ctypes.data, n_avail.ctypes.data,
                                         length.ctypes.data, inner.ctypes.data, gc.ctypes.data,
                                         at.ctypes.data, _lib.ctypes.byref(ms)), self._lib)
        self.kernel_ms = ms.value
        return inner, gc, at

    def close(self):
        if getattr(self, "_h", None):
            self._lib.mc_ecor_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


# ------------------------------------------------------------------ estimator

def _as_reads(bam, k_len, n_threads, decode=None, device=0, contigs=None, extents=None):
    if isinstance(bam, ReadTable):
        if bam.k_len != k_len:
            raise ValueError("ReadTable was opened for k=%d, not %d" % (bam.k_len, k_len))
        return bam, False
    path = getattr(bam, "filename", bam)            # pysam.AlignmentFile, BamFile
    if isinstance(path, bytes):
        path = path.decode()
    if isinstance(path, (str, os.PathLike)):
        if contigs is not None and decode == "gpu":
            return ReadTable(path, k_len, n_threads, decode, device, contigs=contigs, extents=extents), True
        return ReadTable(path, k_len, n_threads, decode, device), True
    raise TypeError("bam must be a BAM path or a metacov_amd.experimental.ReadTable")


def _as_fasta(fasta):
    if fasta is None or isinstance(fasta, FastaFile):
        return fasta
    path = getattr(fasta, "filename", fasta)        # pysam.FastaFile
    if isinstance(path, bytes):
        path = path.decode()
    if isinstance(path, (str, os.PathLike)):
        return FastaFile(path)
    raise TypeError("fasta must be None, a FASTA path or a metacov_amd.experimental.FastaFile")


def _finish(L, counts, sums, seq):
    """The result dict of pileup.py:153-173 from the exact aggregates, with
    the reference's value types: numpy means are np.float64 (and so round()
    is numpy's), ratios of Python numbers are Python floats."""
    _status, secondary, improper, nreads, cov_sum, n_starts, cov2_sum, _nev = (int(x) for x in counts)
    covc_sum, cor_seq, cor_np, wnf = (float(x) for x in sums)
    gc, ecor = seq
    nz = L - n_starts
    nz_e = L * (1 - 1 / L) ** nreads
    nzef = nz / nz_e
    allreads = secondary + nreads + improper
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)   # numpy's 0/0, x/0 (the reference warns)
        return {
            'cov': np.float64(cov_sum) / L,
            'covc': np.float64(covc_sum) / L,
            'den': round(np.float64(n_starts) / L, 3),
            'denc': round(np.float64(cor_np) / L, 3),
            'cov2': round(np.float64(cov2_sum) / L),
            'cf': round(np.float64(cor_seq) / np.float64(n_starts), 3),
            'ambig': round(secondary / allreads, 3) if allreads > 0 else 0,
            'improper': round(improper / allreads, 3) if allreads > 0 else 0,
            'nzef': round(nzef, 3),
            'gc': round(gc, 3),
            'ecor': round(ecor(), 3),
            'wnf': round(wnf / L, 3),
            'cov3': round(200 * (wnf / ecor()) / nzef / L, 3),
        }


def _unbound_ecor():
    raise UnboundLocalError("cannot access local variable 'ecor' where it is not associated "
                            "with a value")


class RegionResult:
    """One region of experimental_batch: `row` (dict) or `error` (the
    exception the reference raises for it), and the "RCOR is ZERO" lines it
    prints first."""
    __slots__ = ("row", "error", "zero_lines")

    def __init__(self, row=None, error=None, zero_lines=()):
        self.row, self.error, self.zero_lines = row, error, list(zero_lines)

    def emit(self, out=None):
        """Print the zero-correction lines, then return the row or raise."""
        for line in self.zero_lines:
            print(line, file=out)
        if self.error is not None:
            raise self.error
        return self.row


def experimental_batch(bam, k_cor, k_len, fasta, regions, device=0, n_threads=0, timings=None, contigs=None,
                       extents=None):
    """pileup.experimental for every (ref, start, end) in `regions`; a list
    of RegionResult in input order.  Reads: one host pass per region on
    n_threads threads; sequence: one GPU launch for all regions.  A BAM
    path is decoded on the GPU when there is a FASTA (the run uses `device`
    anyway; MC_READS_DECODE overrides), else on the host.  contigs /
    extents (a GPU decode): only those header contigs' records are decoded
    (a distributed rank's shard; every region must lie on one of them)."""
    decode = os.environ.get("MC_READS_DECODE") or ("gpu" if fasta is not None else "host")
    reads, own_reads = _as_reads(bam, k_len, n_threads, decode, device, contigs, extents)
    fasta = _as_fasta(fasta)
    try:
        return _batch(reads, k_cor, k_len, fasta, list(regions), device, n_threads, timings)
    finally:
        if own_reads:
            reads.close()


def _batch(reads, k_cor, k_len, fasta, regions, device, n_threads, timings):
    R = len(regions)
    results = [None] * R
    tids = np.zeros(R, np.int32)
    starts = np.zeros(R, np.int64)
    ends = np.ones(R, np.int64)
    live = np.zeros(R, bool)
    seq_base, seq_n = np.zeros(R, np.int64), np.zeros(R, np.int64)
    for q, (ref, start, end) in enumerate(regions):
        start, end = int(start), int(end)
        if end - start == 0:
            results[q] = RegionResult(error=Exception("Length must be > 0"))
            continue
        try:
            if fasta is not None:
                seq_base[q], seq_n[q] = fasta.span(ref, start, end)
            tids[q] = reads.get_tid(ref)
        except (KeyError, ValueError) as e:
            results[q] = RegionResult(error=e)
            continue
        starts[q], ends[q] = start, end
        live[q] = True
    idx = np.nonzero(live)[0]
    tables = KmerTables(k_cor, k_len) if k_cor is not None else None
    # sequence side (GPU): k-mer correlation and G/C counts of every region
    inner = np.zeros(R)
    gcn = np.zeros(R, np.int64)
    atn = np.zeros(R, np.int64)
    if fasta is not None and idx.size:
        eng = EcorEngine(device)
        try:
            eng.set_sequence(fasta)
            eng.set_tables(tables if k_cor else KmerTables([{}, {}], k_len))
            i_, g_, a_ = eng.run(seq_base[idx], seq_n[idx], ends[idx] - starts[idx])
            if timings is not None:
                timings["ecor_kernel_ms"] = eng.kernel_ms
        finally:
            eng.close()
        inner[idx], gcn[idx], atn[idx] = i_, g_, a_
    # read side (host)
    counts = np.zeros((R, 8), np.int64)
    sums = np.zeros((R, 4), np.float64)
    if idx.size:
        c_ = np.zeros((idx.size, 8), np.int64)
        s_ = np.zeros((idx.size, 4), np.float64)
        lib = _lib.load()
        if tables is not None:
            ptrs = (tables.val[0].ctypes.data, tables.has[0].ctypes.data,
                    tables.val[1].ctypes.data, tables.has[1].ctypes.data)
        else:
            ptrs = (None, None, None, None)
        t_ = np.ascontiguousarray(tids[idx])
        a_ = np.ascontiguousarray(starts[idx])
        b_ = np.ascontiguousarray(ends[idx])
        t_pass = time.perf_counter()
        _lib.check(lib.mc_experimental_reads(reads._h, k_len, *ptrs, idx.size, t_.ctypes.data,
                                             a_.ctypes.data, b_.ctypes.data, n_threads,
                                             c_.ctypes.data, s_.ctypes.data), lib)
        if timings is not None:
            timings["reads_pass_ms"] = (time.perf_counter() - t_pass) * 1e3
        counts[idx], sums[idx] = c_, s_
        events = []
        for j in range(idx.size):
            n = _lib.ctypes.c_int64()
            _lib.check(lib.mc_experimental_events(reads._h, j, 0, None, _lib.ctypes.byref(n)), lib)
            ev = np.zeros(n.value, np.uint64)
            if n.value:
                _lib.check(lib.mc_experimental_events(reads._h, j, n.value, ev.ctypes.data,
                                                      _lib.ctypes.byref(n)), lib)
            events.append(ev)
    for j, q in enumerate(idx):
        L = int(ends[q] - starts[q])
        zero_lines = ["RCOR is ZERO: {} {}".format(("R1", "R2")[int(e >> 32)],
                                                   tables.decode(int(e & 0xFFFFFFFF)))
                      for e in events[j]]
        try:
            if fasta is not None:
                g, a = int(gcn[q]), int(atn[q])
                gc = g / (g + a)
                if k_cor:
                    ecor_v = np.float64(inner[q]) / L
                    ecor = (lambda v=ecor_v: v)
                else:
                    ecor = _unbound_ecor
            else:
                gc = -1
                ecor = (lambda: -1)
            status = int(counts[q, 0])
            if status:
                raise TypeError(STATUS_ERRORS[status])
            row = _finish(L, counts[q], sums[q], (gc, ecor))
            results[q] = RegionResult(row=row, zero_lines=zero_lines)
        except Exception as e:  # noqa: BLE001 - mirrored per region, raised by emit()
            results[q] = RegionResult(error=e, zero_lines=zero_lines)
    return results


def experimental(bam, k_cor, k_len, fasta, ref, start, end, device=0, n_threads=0):
    """pileup.experimental(bam, k_cor, k_len, fasta, ref, start, end)."""
    return experimental_batch(bam, k_cor, k_len, fasta, [(ref, start, end)], device,
                              n_threads)[0].emit()


__all__ = ["load_kmerhist", "experimental", "experimental_batch", "FastaFile", "ReadTable",
           "KmerTables", "EcorEngine", "RegionResult", "norm_taps"]
