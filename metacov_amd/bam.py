"""BAM input through the library's C++ decoder (mc_bam_*).

`BamFile(path)` decodes the whole file once (multi-threaded BGZF inflate)
into coordinate-sorted pileup intervals and keeps the header.  It offers the
parts of `pysam.AlignmentFile` the reference's pileup path touches:
`references` / `lengths` (metacov/cli.py:80, metacov/util.py:64-69),
`mapped` / `unmapped` (cli.py:67-76) and `filename`.
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check

FLAG_FILTER = 0x704   # pysam pileup stepper "all": UNMAP|SECONDARY|QCFAIL|DUP


class BamFile:
    def __init__(self, path, n_threads=0, flag_filter=FLAG_FILTER, keep_cigar=False):
        if hasattr(path, "filename"):          # pysam.AlignmentFile
            path = path.filename
        if isinstance(path, bytes):
            path = path.decode()
        self.filename = os.fspath(path)
        lib = _lib.load()
        h = ctypes.c_void_p()
        check(lib.mc_bam_open(self.filename.encode(), int(n_threads), int(flag_filter),
                              1 if keep_cigar else 0, ctypes.byref(h)))
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

    def engine(self, device=0, compute=True):
        """A CoverageEngine holding this file's reads (cached per device);
        with compute=True its depth is computed (once)."""
        eng = self._engines.get(device)
        if eng is None:
            from .engine import CoverageEngine
            eng = CoverageEngine(device)
            eng.set_contigs(np.asarray(self.lengths, dtype=np.int64))
            eng.add_reads(self.tid, self.pos, self.span)
            eng.prepare()
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
