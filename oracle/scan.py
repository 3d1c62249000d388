"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Pure-Python restatement of `metacov scan` (reference metacov/cli.py:112-285)
and what it runs: the read iterators (scan.AlignmentFileIterator
metacov/scan.pyx:188-294, scan.FastQFileIterator :297-340 over
pyfq.FastQFile / FastQFilePair metacov/pyfq.pyx:60-270), the ReadProcessor
plugins (ReadProcessorList :355-383, ByFlag :386-419, BaseHist :422-476,
KmerHist :479-511, MirrorHist :514-552, IsizeHist :555-588) and the driver
scan_reads (:623-672).  One record at a time, exactly in the reference's
order; small inputs only.

Pinning: the reference's scan / pyfq are Cython over pysam's cdef API and
cannot be built here (SURVEY.md §8 c), and no reference test checks a
histogram value (tests/test_cli.py:22-29 checks exit codes).  The FASTQ
reader IS pinned: tests/golden/pyfq.json holds the known answers of the
reference's tests/test_pyfq.py:12-45 (sizes, read-length histograms, base
frequencies), which tests/test_scan.py checks this reader against.  The
histogram arithmetic is "parity unpinned" beyond this restatement.

Where the reference reads memory it does not own the result is undefined;
this restatement fixes it as the product does:
  * reference positions outside [0, L) after Cython's one negative wrap,
    and every position when the read has no reference sequence (no FASTA,
    FASTQ input, or no sequence loaded yet), read as N (4);
  * k-mer positions outside [0, rlen) read as N (stale buffer bytes in the
    reference).
"""
import gzip

from . import bamread

NT16_NT4 = [4, 0, 1, 4, 2, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4]     # scan.pyx:26-29


def iupac_nt4(c):
    """scan.pyx:37-60 / pyfq.pyx:26-49 (one byte)."""
    return {65: 0, 97: 0, 67: 1, 99: 1, 71: 2, 103: 2, 84: 3, 116: 3}.get(c, 4)


def nt4_comp(n):
    """scan.pyx:63-64: 3-n + ((3-n & 4) >> 2) * 5, in C ints, as uint8."""
    return (3 - n + (((3 - n) & 4) >> 2) * 5) & 0xFF


def kmer_base2_to_ascii(kmer, k):
    """scan.pyx:72-74."""
    return "".join("ACGTN"[(kmer >> n) & 3] for n in range(0, 2 * k, 2))


# ------------------------------------------------------------------ flags

class Flag:
    """scan.pyx:78-83."""

    def __init__(self, flag, name_true, name_false, name_col):
        self.flag, self.name_true, self.name_false, self.name_col = \
            flag, name_true, name_false, name_col


FLAGS = [Flag(0x1, "Paired", "Unpaired", "Paired"),             # scan.pyx:86-107
         Flag(0x2, "Paired", "Unpaired", "PairedProperly"),
         Flag(0x4, "Unmapped", "Mapped", "Mapped"),
         Flag(0x8, "Unmapped", "Mapped", "MateMapped"),
         Flag(0x10, "Reverse", "Forward", "Readdir"),
         Flag(0x20, "Reverse", "Forward", "MateReaddir"),
         Flag(0x40, "R1", "R2", "IsRead1"),
         Flag(0x80, "R2", "R1", "IsRead2"),
         Flag(0x100, "Secondary", "Primary", "Alignment"),
         Flag(0x200, "Fail", "Pass", "QC"),
         Flag(0x400, "Duplicate", "Singleton", "Duplicate")]
Flags = {f.name_col: f for f in FLAGS}                          # scan.pyx:123-135


# -------------------------------------------------------------- iterators

class Read:
    """What a ReadProcessor sees of one record."""
    __slots__ = ("rlen", "seq", "flags", "pos", "isize", "ref")

    def ref_at(self, i):
        """Cython memoryview index with wraparound, boundscheck off: one
        negative wrap; anything still outside [0, L) reads as N."""
        ref = self.ref
        if ref is None:
            return 4
        L = len(ref)
        if i < 0:
            i += L
        return ref[i] if 0 <= i < L else 4


def bam_reads(path, fasta=None):
    """AlignmentFileIterator over every record in file order (IteratorRowAll,
    scan.pyx:204).  fasta: {name: sequence str} or None."""
    names, _lengths, recs = bamread.read_bam(path)
    cur_tid, curseq = -1, None
    for rec in recs:
        if fasta is not None and cur_tid != rec.tid:                # scan.pyx:219-232
            cur_tid = rec.tid
            name = names[rec.tid] if rec.tid >= 0 else ""
            seq = fasta.get(name)
            if seq:                                                 # faidx length > 0
                curseq = [iupac_nt4(c) for c in seq.encode()]
        r = Read()
        r.rlen = rec.l_seq                                          # :261-262
        codes = [NT16_NT4[bamread.NT16.index(c)] for c in rec.seq]
        if rec.flag & 0x10:                                         # :247-253
            r.seq = [nt4_comp(c) for c in reversed(codes)]
        else:
            r.seq = codes
        r.flags = rec.flag
        r.pos = rec.pos + rec.l_seq if rec.flag & 0x10 else rec.pos  # :273-277
        r.isize = rec.tlen if rec.flag & 0x2 else 0                  # :267-271
        r.ref = curseq
        yield r


def _fastq_records(path):
    """FastQFile.cnext (pyfq.pyx:166-175): 4 getline calls per record; a
    file ending inside a record ends the stream.  Yields the sequence line
    with its newline."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as fh:
        while True:
            lines = [fh.readline() for _ in range(4)]
            if any(len(ln) == 0 for ln in lines):
                return
            yield lines[1]


def fastq_reads(path1, path2=None):
    """FastQFileIterator over a FastQFile, or a FastQFilePair alternating
    from the SECOND file (pyfq.pyx:264-269) with PAIRED|READ2 / PAIRED|READ1
    flags (:213-215, :278-282)."""
    def mk(line, flags):
        r = Read()
        r.rlen = len(line)
        r.seq = [iupac_nt4(c) for c in line]
        r.flags, r.pos, r.isize, r.ref = flags, -1, -1, None
        return r

    if path2 is None:
        for line in _fastq_records(path1):
            yield mk(line, 0)
        return
    it1, it2 = _fastq_records(path1), _fastq_records(path2)
    cur = 0
    while True:
        cur ^= 1
        line = next(it2 if cur else it1, None)
        if line is None:
            return
        yield mk(line, 0x81 if cur else 0x41)


class FastQFile:
    """pyfq.FastQFile as the reference's tests use it (pyfq.pyx:60-187)."""

    def __init__(self, filename):
        self.filename = filename

    @property
    def size(self):
        """kB, floor; gzip: the ISIZE trailer, wrapped up past 2x the
        compressed size (gzip_get_size, pyfq.pyx:52-62)."""
        import os
        size = os.path.getsize(self.filename)
        if self.filename.endswith(".gz"):
            with open(self.filename, "rb") as fh:
                fh.seek(size - 4)
                guess = int.from_bytes(fh.read(4), "little")
            while guess < size * 2:
                guess += 2 ** 32
            size = guess
        return int(size / 1024)

    def reads(self):
        return fastq_reads(self.filename)


class FastQFilePair(FastQFile):
    def __init__(self, read1, read2):
        self.read1, self.read2 = FastQFile(read1), FastQFile(read2)

    @property
    def size(self):
        return self.read1.size + self.read2.size

    def reads(self):
        return fastq_reads(self.read1.filename, self.read2.filename)


# ------------------------------------------------------------- processors

class BaseHist:
    """scan.pyx:422-476."""

    def __init__(self, start_pos):
        self.start_pos = start_pos
        self.counts = [[0] * 5 for _ in range(10)]

    def copy(self):
        return BaseHist(self.start_pos)

    def set_max_readlen(self, rlen):
        rows = rlen + self.start_pos
        # ndarray.resize of a C-contiguous (r, 5) array: rows kept, new rows 0
        self.counts = (self.counts + [[0] * 5 for _ in range(rows)])[:rows]

    def process_read(self, r):
        pos, sp = r.pos, self.start_pos
        if pos < sp:
            return
        mismatch = 0
        if r.flags & 0x10:
            for i in range(r.rlen):
                if r.seq[i] != nt4_comp(r.ref_at(pos - i - 1)):
                    mismatch += 1
            if mismatch * 32 > r.rlen:
                return
            for i in range(sp):
                self.counts[i][nt4_comp(r.ref_at(pos - i - 1 + sp))] += 1
        else:
            for i in range(r.rlen):
                if r.seq[i] != r.ref_at(pos + i):
                    mismatch += 1
            if mismatch * 32 > r.rlen:
                return
            for i in range(sp):
                self.counts[i][r.ref_at(pos + i - sp)] += 1
        for i in range(r.rlen):
            self.counts[i + sp][r.seq[i]] += 1

    def get_rows(self):
        yield ["Pos", "A", "G", "C", "T", "N"]
        for i, row in enumerate(self.counts):
            yield [i - self.start_pos] + [v & 0xFFFFFFFF for v in row]


class KmerHist:
    """scan.pyx:479-511."""

    def __init__(self, K, NK, STEP, OFFSET):
        self.K, self.NK, self.STEP, self.OFFSET = K, NK, STEP, OFFSET
        self.counts = [[0] * NK for _ in range(4 ** K + 1)]

    def copy(self):
        return KmerHist(self.K, self.NK, self.STEP, self.OFFSET)

    def set_max_readlen(self, rlen):
        pass

    def process_read(self, r):
        if r.rlen < self.OFFSET + self.STEP * self.NK:
            return
        for i in range(self.NK):
            k = 0
            for j in range(self.K):
                x = self.OFFSET + i * self.STEP + j
                c = r.seq[x] if 0 <= x < r.rlen else 4
                if c > 3:
                    k = 4 ** self.K
                    break
                k = k | c << (2 * j)
            self.counts[k][i] += 1

    def get_rows(self):
        yield ["kmer"] + ["n{}".format(i) for i in range(self.NK)]
        yield ["N" * self.K] + [v & 0xFFFFFFFF for v in self.counts[4 ** self.K]]
        for i in range(4 ** self.K):
            yield [kmer_base2_to_ascii(i, self.K)] + [v & 0xFFFFFFFF for v in self.counts[i]]


class MirrorHist:
    """scan.pyx:514-552."""

    def __init__(self, OFFSET=4, N=10):
        self.OFFSET, self.N = OFFSET, N
        self.counts = [[0, 0] for _ in range(N + 1)]

    def copy(self):
        return MirrorHist(self.OFFSET, self.N)

    def set_max_readlen(self, rlen):
        pass

    def process_read(self, r):
        pos = r.pos + self.OFFSET
        if pos < self.N - self.OFFSET:
            return
        plain = comp = 0
        for i in range(self.N):
            a, b = r.ref_at(pos + i + 1), r.ref_at(pos - i - 1)
            if a != b:
                plain += 1
            if a != nt4_comp(b):
                comp += 1
        self.counts[plain][0] += 1
        self.counts[comp][1] += 1

    def get_rows(self):
        yield ["n", "plain", "comp"]
        for i in range(self.N):                                     # N of the N+1 rows
            yield [i, self.counts[i][0] & 0xFFFFFFFF, self.counts[i][1] & 0xFFFFFFFF]


class IsizeHist:
    """scan.pyx:555-588."""

    def __init__(self):
        self.counts = {}
        self.max_isize = 0

    def copy(self):
        return IsizeHist()

    def set_max_readlen(self, rlen):
        pass

    def process_read(self, r):
        isize = -r.isize if r.isize < 0 else r.isize
        self.max_isize = max(self.max_isize, isize)
        self.counts[isize] = self.counts.get(isize, 0) + 1

    def get_rows(self):
        yield ["n", "count"]
        for i in range(self.max_isize + 1):
            yield [i, self.counts.get(i, 0) & 0xFFFFFFFF]


class ReadProcessorList:
    """scan.pyx:355-383."""

    def __init__(self, processors):
        self.processors = processors

    def copy(self):
        return ReadProcessorList([p.copy() for p in self.processors])

    def set_max_readlen(self, rlen):
        for p in self.processors:
            p.set_max_readlen(rlen)

    def process_read(self, r):
        for p in self.processors:
            p.process_read(r)

    def get_rows(self, i):
        return self.processors[i].get_rows()


class ByFlag(ReadProcessorList):
    """scan.pyx:386-419."""

    def __init__(self, processor, flags):
        if isinstance(processor, list):
            processor = ReadProcessorList(processor)
        self.flags = flags
        super().__init__([processor.copy() for _ in range(2 ** len(flags))])

    def get_rows(self, i):
        tag_head = [f.name_col for f in reversed(self.flags)]
        yield next(self.processors[0].get_rows(i)) + tag_head
        for n, p in enumerate(self.processors):
            tag = [f.name_true if (1 << m) & n else f.name_false
                   for m, f in enumerate(reversed(self.flags))]
            it = p.get_rows(i)
            next(it)
            for row in it:
                yield row + tag

    def process_read(self, r):
        n = 0
        for f in self.flags:
            n <<= 1
            if f.flag & r.flags:
                n += 1
        self.processors[n].process_read(r)


def scan_reads(reads, counters, maxreads=0):
    """scan.pyx:623-672 over an iterator of Read."""
    max_readlen = 50
    counters.set_max_readlen(max_readlen)
    readno = 0
    for r in reads:
        readno += 1
        if r.rlen > max_readlen:
            max_readlen = r.rlen
            counters.set_max_readlen(max_readlen)
        counters.process_read(r)
        if maxreads and readno >= maxreads:
            break
    return readno


def read_fasta(path):
    """{name: sequence} of a plain or gzip FASTA (first word of each '>')."""
    with open(path, "rb") as fh:
        gz = fh.read(2) == b"\x1f\x8b"
    with (gzip.open if gz else open)(path, "rt") as fh:
        text = fh.read()
    out = {}
    for block in text.split(">")[1:]:
        head, _, body = block.partition("\n")
        out[head.split()[0] if head.split() else ""] = "".join(body.split())
    return out


def scan_csv(readfile, out, fasta=None, group_by=(), boffset=0, k=7, number=8, step=7,
             offset=0, mirror_offset=4, mirror_length=10, max_reads=0):
    """The CSV files `metacov scan` writes (cli.py:247-285), as {name: text}.
    readfile: [bam] or [fq] or [fq1, fq2]; out: subset of base/kmer/mirror/
    isize.  Keeps the reference's output index sequence, including the
    missing `n += 1` after the k-mer table (cli.py:274-277)."""
    import csv
    import io
    counters = []
    if "base" in out:
        counters.append(BaseHist(boffset))
    if "kmer" in out:
        counters.append(KmerHist(k, number, step, offset))
    if "mirror" in out:
        counters.append(MirrorHist(mirror_offset, mirror_length))
    if "isize" in out:
        counters.append(IsizeHist())
    counters = ByFlag(counters, [Flags[f] for f in group_by])
    if readfile[0].endswith((".bam", ".sam")):
        reads = bam_reads(readfile[0], read_fasta(fasta) if fasta else None)
    else:
        reads = fastq_reads(*readfile)
    scan_reads(reads, counters, max_reads)
    texts = {}
    n = 0
    for name, bump in (("base", True), ("kmer", False), ("mirror", True), ("isize", True)):
        if name in out:
            buf = io.StringIO()
            csv.writer(buf).writerows(counters.get_rows(n))
            texts[name] = buf.getvalue()
            if bump:
                n += 1
    return texts
