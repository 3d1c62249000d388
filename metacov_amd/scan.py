"""`scan` read histograms on the MI355X (reference metacov/scan.pyx, SURVEY.md
§8 f rank 3), with the reference module's names:

    counters = ByFlag([BaseHist(0), KmerHist(7, 8, 7, 0), MirrorHist(4, 10), IsizeHist()],
                      [Flags["Mapped"]])
    nreads = scan_reads("reads.bam", "ref.fa", counters, maxreads=0)
    rows = counters.get_rows(1)       # the KmerHist table, as the CLI writes it

The processor objects are descriptions plus their counts; the reads never
pass through Python.  scan_reads hands the file to the library's C++ source
(all BAM records, or FASTQ lines, decoded into SoA batches; scan_src.cpp),
and one HIP kernel (scan.hip) runs every processor of every group over each
batch, one lane per read, with the hot bins privatised in LDS.  The results
are added into each processor's `counts` in the reference's layouts and
integer type (uint32, wrapping like the reference's arrays).

Semantics restated from scan.pyx (see scan.hip's header for the per-read
rules and oracle/scan.py for the line-by-line restatement); behaviour kept
on purpose:
* BaseHist's header names A,G,C,T,N over columns in A,C,G,T,N order
  (scan.pyx:472-476); its row count is max(50, longest read seen in this
  call) + start_pos, and each scan_reads call first cuts the table back to
  50 + start_pos rows (set_max_readlen(50) resizes, :636, :437-440);
* MirrorHist writes N of its N+1 rows (:549-552);
* IsizeHist writes rows 0..max |isize| of its own group (:583-588);
* ByFlag appends the group columns in reverse -g order (:395-405).
Where the reference reads memory it does not own (reference positions
outside the sequence, no FASTA, k-mer bases outside the read), this build
reads N -- DESIGN.md §4c.
"""
import ctypes
import logging
import os

import numpy as np

from . import _lib

log = logging.getLogger(__name__)


class Flag:
    """scan.pyx:78-83."""

    def __init__(self, flag, name_true, name_false, name_col):
        self.flag = flag
        self.name_true = name_true
        self.name_false = name_false
        self.name_col = name_col


FLAG_PAIRED = Flag(0x1, "Paired", "Unpaired", "Paired")
FLAG_PROPER_PAIR = Flag(0x2, "Paired", "Unpaired", "PairedProperly")
FLAG_MAPPED = Flag(0x4, "Unmapped", "Mapped", "Mapped")
FLAG_MMAPPED = Flag(0x8, "Unmapped", "Mapped", "MateMapped")
FLAG_REVERSE = Flag(0x10, "Reverse", "Forward", "Readdir")
FLAG_MREVERSE = Flag(0x20, "Reverse", "Forward", "MateReaddir")
FLAG_READ1 = Flag(0x40, "R1", "R2", "IsRead1")
FLAG_READ2 = Flag(0x80, "R2", "R1", "IsRead2")
FLAG_SECONDARY = Flag(0x100, "Secondary", "Primary", "Alignment")
FLAG_QCFAIL = Flag(0x200, "Fail", "Pass", "QC")
FLAG_DUP = Flag(0x400, "Duplicate", "Singleton", "Duplicate")

Flags = {flag.name_col: flag for flag in (
    FLAG_PAIRED, FLAG_PROPER_PAIR, FLAG_MAPPED, FLAG_MMAPPED, FLAG_REVERSE, FLAG_MREVERSE,
    FLAG_READ1, FLAG_READ2, FLAG_SECONDARY, FLAG_QCFAIL, FLAG_DUP)}


def kmer_base2_to_ascii(kmer, k):
    """scan.pyx:72-74: base j of the k-mer at bits 2j, 'ACGT'."""
    return "".join("ACGTN"[(kmer >> n) & 3] for n in range(0, 2 * k, 2))


def _add_u32(a, b):
    return (a.astype(np.uint64) + b.astype(np.uint64)).astype(np.uint32)


# ------------------------------------------------------------- processors

class ReadProcessor:
    """Base class for read stats accumulators (scan.pyx:345-352)."""
    kind = None

    def set_max_readlen(self, rlen):
        pass

    def __copy__(self):
        raise NotImplementedError


class BaseHist(ReadProcessor):
    """Base counts along the read, plus `start_pos` reference bases before it
    (scan.pyx:422-476)."""
    kind = "base"

    def __init__(self, start_pos):
        self.start_pos = int(start_pos)
        self._counts_data = np.zeros((10, 5), dtype=np.uint32)

    def __copy__(self):
        return BaseHist(self.start_pos)

    def set_max_readlen(self, rlen):
        rows = rlen + self.start_pos
        c = np.zeros((rows, 5), dtype=np.uint32)
        k = min(rows, self._counts_data.shape[0])
        c[:k] = self._counts_data[:k]
        self._counts_data = c

    def _add(self, counts):
        rows = max(counts.shape[0], self._counts_data.shape[0])
        self.set_max_readlen(rows - self.start_pos)
        self._counts_data[:counts.shape[0]] = _add_u32(self._counts_data[:counts.shape[0]], counts)

    @property
    def counts(self):
        return self._counts_data

    def get_rows(self):
        yield ["Pos", "A", "G", "C", "T", "N"]
        for i in range(self._counts_data.shape[0]):
            yield [i - self.start_pos] + list(self._counts_data[i])


class KmerHist(ReadProcessor):
    """NK k-mers of length K, STEP apart from OFFSET (scan.pyx:479-511)."""
    kind = "kmer"

    def __init__(self, K, NK, STEP, OFFSET):
        self.K, self.NK, self.STEP, self.OFFSET = int(K), int(NK), int(STEP), int(OFFSET)
        self._counts_data = np.zeros((4 ** self.K + 1, self.NK), dtype=np.uint32)

    def __copy__(self):
        return KmerHist(self.K, self.NK, self.STEP, self.OFFSET)

    def _add(self, counts):
        self._counts_data = _add_u32(self._counts_data, counts)

    @property
    def counts(self):
        return self._counts_data

    def get_rows(self):
        yield ["kmer"] + ["n{}".format(i) for i in range(self.NK)]
        yield ["N" * self.K] + list(self.counts[4 ** self.K])
        for i in range(4 ** self.K):
            yield [kmer_base2_to_ascii(i, self.K)] + list(self._counts_data[i])


class MirrorHist(ReadProcessor):
    """Mismatches against a palindrome around read start + OFFSET
    (scan.pyx:514-552)."""
    kind = "mirror"

    def __init__(self, OFFSET=4, N=10):
        self.OFFSET, self.N = int(OFFSET), int(N)
        self._counts_data = np.zeros((self.N + 1, 2), dtype=np.uint32)

    def __copy__(self):
        return MirrorHist(self.OFFSET, self.N)

    def _add(self, counts):
        self._counts_data = _add_u32(self._counts_data, counts)

    @property
    def counts(self):
        return self._counts_data

    def get_rows(self):
        yield ["n", "plain", "comp"]
        for i in range(self.N):
            yield [i, self._counts_data[i, 0], self._counts_data[i, 1]]


class IsizeHist(ReadProcessor):
    """Insert sizes of properly paired reads (scan.pyx:555-588)."""
    kind = "isize"

    def __init__(self):
        self._counts_data = np.zeros(128, dtype=np.uint32)
        self.max_isize = 0

    def __copy__(self):
        return IsizeHist()

    def _add(self, counts, max_isize):
        self.max_isize = max(self.max_isize, int(max_isize))
        size = self._counts_data.shape[0]
        while size <= self.max_isize:
            size *= 2
        c = np.zeros(size, dtype=np.uint32)
        c[:self._counts_data.shape[0]] = self._counts_data
        n = min(size, counts.shape[0])
        c[:n] = _add_u32(c[:n], counts[:n])
        self._counts_data = c

    @property
    def counts(self):
        return self._counts_data

    def get_rows(self):
        yield ["n", "count"]
        for i in range(self.max_isize + 1):
            yield [i, self._counts_data[i]]


class ReadProcessorList(ReadProcessor):
    """Several processors fed the same reads (scan.pyx:355-383)."""

    def __init__(self, processors):
        self.processors = processors
        for processor in processors:
            assert isinstance(processor, ReadProcessor)

    def __copy__(self):
        from copy import copy
        return ReadProcessorList([copy(p) for p in self.processors])

    def set_max_readlen(self, rlen):
        for p in self.processors:
            p.set_max_readlen(rlen)

    def get_rows(self, i):
        return self.processors[i].get_rows()


class ByFlag(ReadProcessorList):
    """One copy of `processor` per combination of the flags (scan.pyx:386-419):
    group n has bit (nflags-1-i) set when flags[i] is set on the read."""

    def __init__(self, processor, flags):
        from copy import copy
        if isinstance(processor, list):
            processor = ReadProcessorList(processor)
        assert isinstance(processor, ReadProcessor)
        self.nflags = len(flags)
        self.flags = flags
        self.processors = [copy(processor) for _ in range(2 ** self.nflags)]
        super().__init__(self.processors)

    def get_rows(self, i):
        tag_head = [flag.name_col for flag in reversed(self.flags)]
        yield next(self.processors[0].get_rows(i)) + tag_head
        for n, processor in enumerate(self.processors):
            tag = []
            for m, flag in enumerate(reversed(self.flags)):
                tag.append(flag.name_true if 1 << m & n else flag.name_false)
            rows = processor.get_rows(i)
            next(rows)
            for row in rows:
                yield row + tag


# ---------------------------------------------------------------- driver

def _groups(counters):
    """(flags, [per group: list of leaf processors])."""
    if isinstance(counters, list):
        counters = ReadProcessorList(counters)
    if not isinstance(counters, ReadProcessor):
        raise Exception("mah")                                       # scan.pyx:649
    if isinstance(counters, ByFlag):
        flags, groups = counters.flags, counters.processors
    else:
        flags, groups = [], [counters]
    out = []
    for g in groups:
        leaves = g.processors if isinstance(g, ReadProcessorList) else [g]
        for p in leaves:
            if p.kind is None:
                raise NotImplementedError("nested processor lists are not supported: %r" % (p,))
        out.append(leaves)
    return flags, out


def _source(lib, infile, n_threads, decode="host", device=0):
    """(handle, kind) for a path, a pyfq FastQFile / FastQFilePair or an
    object with .filename (pysam AlignmentFile): an mc_scan_src, or for a BAM
    with decode="gpu" an mc_bam_gpu decoded on `device` (kind "gbam")."""
    from . import pyfq
    h = ctypes.c_void_p()
    if isinstance(infile, pyfq.FastQFilePair):
        _lib.check(lib.mc_scan_src_open_fastq(infile.read1.filename.encode(),
                                              infile.read2.filename.encode(), ctypes.byref(h)), lib)
        return h, "fq"
    if isinstance(infile, pyfq.FastQFile):
        _lib.check(lib.mc_scan_src_open_fastq(infile.filename.encode(), None, ctypes.byref(h)), lib)
        return h, "fq"
    path = infile if isinstance(infile, (str, os.PathLike)) else getattr(infile, "filename", None)
    if isinstance(path, bytes):
        path = path.decode()
    if path is None:
        raise Exception("meh")                                       # scan.pyx:642
    path = os.fspath(path)
    if path.endswith((".fq", ".fq.gz", ".fastq", ".fastq.gz")):
        _lib.check(lib.mc_scan_src_open_fastq(path.encode(), None, ctypes.byref(h)), lib)
        return h, "fq"
    if is_sam(path):   # pysam tells SAM from BAM by content, whatever the name
        _lib.check(lib.mc_scan_src_open_sam(path.encode(), ctypes.byref(h)), lib)
        return h, "bam"
    if decode == "gpu":
        window = int(os.environ.get("MC_SCAN_GPU_WINDOW", "0"))   # (tests: force the windowed decode)
        _lib.check(lib.mc_bam_gpu_open_scan(path.encode(), int(device), int(n_threads), window, ctypes.byref(h)),
                   lib)
        return h, "gbam"
    _lib.check(lib.mc_scan_src_open_bam(path.encode(), n_threads, ctypes.byref(h)), lib)
    return h, "bam"


def is_sam(path):
    """True for SAM text (plain, gzip or BGZF), False for BAM: htslib's
    format detection looks at the (inflated) first bytes, "BAM\\1" or text."""
    import gzip
    with open(path, "rb") as fh:
        head = fh.read(2)
    if head == b"\x1f\x8b":
        try:
            with gzip.open(path, "rb") as fh:
                return fh.read(4) != b"BAM\x01"
        except (OSError, EOFError):
            return False
    return True


def _fasta(fasta):
    if fasta is None:
        return None
    from .experimental import FastaFile
    if isinstance(fasta, FastaFile):
        return fasta
    return FastaFile(os.fspath(getattr(fasta, "filename", fasta)))


def _config(flags, leaves):
    cfg = _lib.ScanConfig()
    cfg.n_flags = len(flags)
    for i, f in enumerate(flags):
        cfg.flags[i] = f.flag
    for p in leaves:
        if p.kind == "base":
            cfg.base_on, cfg.base_start = 1, p.start_pos
        elif p.kind == "kmer":
            cfg.kmer_on, cfg.kmer_k, cfg.kmer_nk = 1, p.K, p.NK
            cfg.kmer_step, cfg.kmer_offset = p.STEP, p.OFFSET
        elif p.kind == "mirror":
            cfg.mirror_on, cfg.mirror_offset, cfg.mirror_n = 1, p.OFFSET, p.N
        elif p.kind == "isize":
            cfg.isize_on = 1
    return cfg


def scan_reads(infile, fasta, counters, progress_interval=10000000, progress_cb=None,
               maxreads=0, device=0, n_threads=0, batch_reads=1 << 21, decode=None):
    """scan.pyx:623-672: runs `counters` over every read of `infile` (a BAM
    path / pysam-like object with .filename, a FASTQ path, or a pyfq
    FastQFile / FastQFilePair) and returns the number of reads processed.
    `fasta` (path or experimental.FastaFile) supplies the reference for
    BaseHist / MirrorHist.  progress_cb is called once per progress_interval
    reads, after the GPU pass.  decode: "gpu" (default; MC_SCAN_DECODE
    overrides) inflates and walks a BAM on the GPU, "host" with the C++
    source (SAM and FASTQ always take the host source).  With maxreads the
    host source streams and stops there; a GPU decode that does not fit in
    device memory falls back to it."""
    decode = decode or os.environ.get("MC_SCAN_DECODE", "gpu")
    if decode not in ("gpu", "host"):
        raise ValueError("decode must be 'gpu' or 'host'")
    lib = _lib.load()
    flags, groups = _groups(counters)
    if len(flags) > 11:
        raise ValueError("at most 11 group-by flags")
    # one GPU pass per layer of distinct processor kinds (the CLI has one)
    n_layers = max(max((sum(1 for p in g if p.kind == k) for k in ("base", "kmer", "mirror", "isize")),
                       default=0) for g in groups)
    fa = _fasta(fasta)
    for leaves in groups:
        for p in leaves:
            if p.kind == "base":
                p.set_max_readlen(50)                                # scan.pyx:636
    nreads = 0
    for layer in range(max(n_layers, 1)):
        per_group = []
        for leaves in groups:
            seen, sel = {}, []
            for p in leaves:
                seen[p.kind] = seen.get(p.kind, -1) + 1
                if seen[p.kind] == layer:
                    sel.append(p)
            per_group.append(sel)
        nreads = _run_layer(lib, infile, fa, flags, per_group, maxreads, device, n_threads,
                            batch_reads, decode)
    if progress_cb and progress_interval > 0:
        for _ in range(nreads // progress_interval):
            progress_cb()
    return nreads


def _target_names(lib, src, kind):
    if kind == "gbam":
        from .bam import _header_of
        hdr = ctypes.c_void_p()
        _lib.check(lib.mc_bam_gpu_header(src, ctypes.byref(hdr)), lib)
        return list(_header_of(lib, hdr)[0])
    n_t = ctypes.c_int32()
    _lib.check(lib.mc_scan_src_n_targets(src, ctypes.byref(n_t)), lib)
    name = ctypes.c_char_p()
    ln = ctypes.c_int64()
    names = []
    for t in range(n_t.value):
        _lib.check(lib.mc_scan_src_target(src, t, ctypes.byref(name), ctypes.byref(ln)), lib)
        names.append(name.value.decode())
    return names


def _run_layer(lib, infile, fa, flags, per_group, maxreads, device, n_threads, batch_reads, decode="host"):
    if maxreads:
        # the GPU decode inflates and walks the whole file into HBM before
        # the first batch; the host source streams and stops at maxreads
        decode = "host"
    try:
        return _run_layer_on(lib, infile, fa, flags, per_group, maxreads, device, n_threads, batch_reads,
                             decode)
    except _lib.MetacovError as e:
        # a BAM whose whole-file SoA batch does not fit in HBM (allocation
        # failure or a batch past the engine's range): the streaming host
        # source, in bounded windows, feeds the same GPU histograms
        if decode != "gpu" or e.code not in (_lib.MC_E_HIP, _lib.MC_E_RANGE):
            raise
        log.warning("GPU BAM decode for scan failed (%s); reading on the host instead", e)
        return _run_layer_on(lib, infile, fa, flags, per_group, maxreads, device, n_threads, batch_reads,
                             "host")


def _run_layer_on(lib, infile, fa, flags, per_group, maxreads, device, n_threads, batch_reads, decode):
    src, kind = _source(lib, infile, n_threads, decode, device)
    scan = ctypes.c_void_p()
    try:
        cfg = _config(flags, per_group[0])
        _lib.check(lib.mc_scan_create(device, ctypes.byref(cfg), ctypes.byref(scan)), lib)
        tid_map = np.zeros(0, np.int32)
        if fa is not None and kind in ("bam", "gbam"):
            names = _target_names(lib, src, kind)
            tid_map = np.full(len(names), -1, np.int32)
            for t, nm in enumerate(names):
                i = fa._index.get(nm)
                if i is not None and fa.lengths[i] > 0:
                    tid_map[t] = i
            off = np.ascontiguousarray(fa._off, np.int64)
            lens = np.ascontiguousarray(fa.lengths, np.int64)
            buf = np.ascontiguousarray(fa.buffer)
            _lib.check(lib.mc_scan_set_reference(scan, len(lens), _lib.ptr(off), _lib.ptr(lens),
                                                 buf.size, _lib.ptr(buf)), lib)
        done = ctypes.c_int64()
        if kind == "gbam":
            _lib.check(lib.mc_scan_run_gpu(scan, src, tid_map.size, _lib.ptr(tid_map), int(maxreads or 0),
                                           ctypes.byref(done)), lib)
        else:
            _lib.check(lib.mc_scan_run(scan, src, tid_map.size, _lib.ptr(tid_map), int(maxreads or 0),
                                       int(batch_reads), ctypes.byref(done)), lib)
        _collect(lib, scan, cfg, per_group)
        return done.value
    finally:
        if scan:
            lib.mc_scan_destroy(scan)
        if kind == "gbam":
            lib.mc_bam_gpu_close(src)
        else:
            lib.mc_scan_src_close(src)


def _collect(lib, scan, cfg, per_group):
    G = ctypes.c_int32()
    rows = ctypes.c_int64()
    cap = ctypes.c_int64()
    _lib.check(lib.mc_scan_dims(scan, ctypes.byref(G), ctypes.byref(rows), ctypes.byref(cap),
                                None, None), lib)
    G = G.value
    base = np.zeros((G, rows.value, 5), np.uint32) if cfg.base_on else None
    kmer = (np.zeros((G, 4 ** cfg.kmer_k + 1, cfg.kmer_nk), np.uint32) if cfg.kmer_on else None)
    mirror = np.zeros((G, cfg.mirror_n + 1, 2), np.uint32) if cfg.mirror_on else None
    isize = np.zeros((G, cap.value), np.uint32) if cfg.isize_on else None
    isize_max = np.zeros(G, np.int32) if cfg.isize_on else None
    _lib.check(lib.mc_scan_results(scan, _lib.ptr(base), _lib.ptr(kmer), _lib.ptr(mirror),
                                   _lib.ptr(isize), _lib.ptr(isize_max)), lib)
    for g, leaves in enumerate(per_group):
        for p in leaves:
            if p.kind == "base":
                p._add(base[g])
            elif p.kind == "kmer":
                p._add(kmer[g])
            elif p.kind == "mirror":
                p._add(mirror[g])
            elif p.kind == "isize":
                p._add(isize[g], isize_max[g])
