"""FASTQ reader / writer with the reference's pyfq API (metacov/pyfq.pyx:60-352,
SURVEY.md §8 f rank 4).

    with FastQFile("r1.fq.gz") as fq:
        for read in fq:            # read.rlen, read.seq (ACGTN -> 01234), read.char_seq
            ...
    with FastQFilePair("r1.fq.gz", "r2.fq.gz") as fq: ...   # alternates, second file first
    with FastQWriter("out.fq.gz") as out: out.write(read)

Host I/O only.  Semantics kept from pyfq:
* a record is 4 `getline` lines; a file ending inside a record ends the
  iteration (FastQFile.cnext, pyfq.pyx:166-175);
* `rlen` is the length of the sequence line INCLUDING its newline, and
  `seq` converts all of it (the newline becomes 4 = N; pyfq.pyx:178-183);
* `pos` / `size` are kB (floor); a gzip file's size is its ISIZE trailer,
  wrapped up past twice the compressed size (gzip_get_size, :52-62);
* FastQFilePair reads the second file first (`cur` flips to 1 before the
  first read, :264-269) and stops when the file whose turn it is ends;
* FastQWriter writes the 4 raw lines of a FastQFile record, gzip when the
  name ends in .gz (:296-346).
The reference pipes .gz files through unpigz/gunzip; here Python's gzip
module does it in-process.

`metacov scan` does not iterate reads in Python: it hands the file names to
the library's C++ source (mc_scan_src_open_fastq, scan_src.cpp), which
implements the same record rules and feeds the GPU.
"""
import gzip
import os

_NT4 = bytes(0 if c in b"Aa" else 1 if c in b"Cc" else 2 if c in b"Gg" else 3 if c in b"Tt" else 4
             for c in range(256))


def gzip_get_size(filename):
    """pyfq.pyx:52-62."""
    size = os.path.getsize(filename)
    with open(filename, "rb") as f:
        f.seek(size - 4)
        guess = int.from_bytes(f.read(4), "little")
    while guess < size * 2:
        guess = guess + 2 ** 32
    return guess


class FastQFile:
    """pyfq.FastQFile (read only)."""

    def __init__(self, filename, max_linelen=1000):
        self.filename = filename
        self.max_linelen = max_linelen
        self._fh = None
        self._buf = [b"", b"", b"", b""]
        self._pos = 0
        self._file_size = 0

    def __enter__(self):
        if self.filename.endswith(".gz"):
            self._fh = gzip.open(self.filename, "rb")
        else:
            self._fh = open(self.filename, "rb")
        return self

    def __exit__(self, exception_type, exception_value, traceback):
        if self._fh:
            self._fh.close()
            self._fh = None

    def __iter__(self):
        return self

    def __next__(self):
        if self.cnext() <= 0:
            raise StopIteration()
        return self

    def cnext(self):
        """Parse the next read: 1, or -1 at the end, -2 when not open."""
        if self._fh is None:
            return -2
        for i in range(4):
            line = self._fh.readline()
            if not line:
                return -1
            self._pos += len(line)
            self._buf[i] = line
        return 1

    @property
    def rlen(self):
        """Length of the current read (with its newline)."""
        return len(self._buf[1])

    @property
    def seq(self):
        """List of bases of the current read (ACGTN -> 01234)."""
        return list(self._buf[1].translate(_NT4))

    @property
    def char_seq(self):
        return self._buf[1].decode("ascii")

    @property
    def pos(self):
        """Position in the file in kB."""
        return int(self._pos / 1024)

    @property
    def size(self):
        """Size of the file in kB."""
        if not self._file_size:
            if self.filename.endswith(".gz"):
                self._file_size = gzip_get_size(self.filename)
            else:
                self._file_size = os.path.getsize(self.filename)
        return int(self._file_size / 1024)

    def get_flags(self):
        return 0

    def raw_lines(self):
        return tuple(self._buf)


class FastQFilePair(FastQFile):
    """pyfq.FastQFilePair: zip(FastQFile, FastQFile), second file first."""

    def __init__(self, read1, read2, max_linelen=1000):
        self.read1 = FastQFile(read1, max_linelen)
        self.read2 = FastQFile(read2, max_linelen)
        self.flags1 = 0x1 | 0x40       # BAM_FPAIRED | BAM_FREAD1
        self.flags2 = 0x1 | 0x80       # BAM_FPAIRED | BAM_FREAD2
        self.cur = 0
        self.filename = read1

    def __enter__(self):
        self.read1.__enter__()
        self.read2.__enter__()
        self.cur = 0
        return self

    def __exit__(self, exception_type, exception_value, traceback):
        self.read1.__exit__(exception_type, exception_value, traceback)
        self.read2.__exit__(exception_type, exception_value, traceback)

    def _current(self):
        return self.read2 if self.cur > 0 else self.read1

    def cnext(self):
        self.cur = self.cur ^ 1
        return self._current().cnext()

    @property
    def rlen(self):
        return self._current().rlen

    @property
    def seq(self):
        return self._current().seq

    @property
    def char_seq(self):
        return self._current().char_seq

    @property
    def pos(self):
        return int(self.read1.pos + self.read2.pos)

    @property
    def size(self):
        return int(self.read1.size + self.read2.size)

    def get_flags(self):
        return self.flags2 if self.cur > 0 else self.flags1

    def raw_lines(self):
        return self._current().raw_lines()


class FastQWriter:
    """pyfq.FastQWriter: writes FastQFile records (the 4 raw lines)."""

    def __init__(self, fileobj):
        self.filename = None
        self.file = None
        if hasattr(fileobj, "fileno"):
            self.file = fileobj
        else:
            self.filename = fileobj
        self._out = None

    def __enter__(self):
        if self.filename is not None:
            self.file = open(self.filename, "wb")
        name = self.filename if self.filename is not None else getattr(self.file, "name", "")
        if str(name).endswith(".gz"):
            self._out = gzip.GzipFile(fileobj=self.file, mode="wb")
        else:
            self._out = self.file
        return self

    def __exit__(self, exception_type, exception_value, traceback):
        if self._out is not None and self._out is not self.file:
            self._out.close()
        if self.filename is not None and self.file is not None:
            self.file.close()

    def write(self, read):
        if isinstance(read, FastQFile):
            for line in read.raw_lines():
                self._out.write(line)
            return True
        raise Exception("writing {} not implemented".format(type(read)))
