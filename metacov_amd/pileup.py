"""Drop-in for the reference's `metacov.pileup.classic` (metacov/pileup.py:9-26).

    classic(bam, ref, start, end) -> {min, max, med, std, avg, q23, sum}

`bam` may be a path, a `metacov_amd.bam.BamFile` / `GpuBamFile`, or a `pysam.AlignmentFile`
(its `.filename` is decoded by this library, on the GPU: `GpuBamFile`).  The
depth of every contig is computed once per file on the GPU (K2) and each
call reduces one region (K3); `classic_batch` reduces many regions in one
launch.  Semantics match
classic(): positions are 0-based half-open [start, end); positions the reads
do not cover (or past the contig end) count as 0 (pileup.py:11-16); an empty
region raises ValueError (pileup.py:19 on a zero-size vector); an unknown
`ref` raises KeyError.

Like pysam's pileup, the depth is capped: `max_depth` (default 8000, pysam's)
reproduces htslib's read-pool cap per region query (metacov_amd.depthcap);
`max_depth=None` gives exact depths.  A mapped read without a
reference-consuming CIGAR op adds nothing (current htslib `bam_plp_push`);
`legacy_endpos=True` counts it on one column (htslib <= 1.9).

`experimental` and `load_kmerhist` (pileup.py:29-173) are re-exported from
`metacov_amd.experimental`, so `pileup.<name>` resolves as in the reference.
"""
import collections
import os

import numpy as np

from . import depthcap
from .bam import BamFile, GpuBamFile
from .engine import classic_stats, numpy_std
from .experimental import experimental, load_kmerhist  # noqa: F401  (pileup.py:29-173)

HTSLIB_MAX_DEPTH = depthcap.HTSLIB_MAX_DEPTH
_OPEN_MAX = 2                              # decoded files kept between calls
_open_files = collections.OrderedDict()    # (path, size, mtime_ns, legacy, device) -> GpuBamFile


def _as_bamfile(bam, legacy_endpos=False, device=0):
    """An open decoded file for `bam`: the library's own handles as given; a
    path (or a pysam.AlignmentFile's .filename) is decoded on the GPU
    (GpuBamFile: BGZF inflate and record parse in HBM, the reads handed to
    the engine by a device copy) and kept for later calls."""
    if isinstance(bam, BamFile) or hasattr(bam, "engine"):   # BamFile, GpuBamFile, StreamedBam
        return bam
    path = getattr(bam, "filename", bam)
    if isinstance(path, bytes):
        path = path.decode()
    path = os.fspath(path)
    st = os.stat(path)
    key = (os.path.abspath(path), st.st_size, st.st_mtime_ns, bool(legacy_endpos), int(device))
    f = _open_files.pop(key, None)
    if f is None:
        f = GpuBamFile(path, device=device, legacy_endpos=legacy_endpos)
        f.trim()                           # kept between calls: only its results stay in HBM
    _open_files[key] = f                   # most recently used last
    while len(_open_files) > _OPEN_MAX:
        _open_files.popitem(last=False)[1].close()
    return f


def close_all():
    """Releases the decoded files (and their GPU engines) kept for path
    arguments."""
    while _open_files:
        _open_files.popitem()[1].close()


def _resolve(bf, ref):
    try:
        return bf.references.index(ref)
    except ValueError:
        raise KeyError(ref)


def classic(bam, ref, start, end, device=0, max_depth=HTSLIB_MAX_DEPTH, legacy_endpos=False):
    return classic_batch(bam, [(ref, start, end)], device=device, max_depth=max_depth,
                         legacy_endpos=legacy_endpos)[0]


def classic_batch(bam, regions, device=0, max_depth=HTSLIB_MAX_DEPTH, legacy_endpos=False):
    """[(ref, start, end), ...] -> [dict, ...] in input order.  Each dict is
    classic()'s; an empty region raises ValueError like classic().
    max_depth (default 8000 = pysam's): htslib's pileup read cap per region
    query, applied where it can act (metacov_amd.depthcap); None: exact.
    legacy_endpos applies when `bam` is a path (an open file keeps the rule
    it was decoded with)."""
    bf = _as_bamfile(bam, legacy_endpos, device)
    regions = list(regions)
    if not regions:
        return []
    tids = np.empty(len(regions), dtype=np.int32)
    starts = np.empty(len(regions), dtype=np.int64)
    ends = np.empty(len(regions), dtype=np.int64)
    for i, (ref, s, e) in enumerate(regions):
        tids[i] = _resolve(bf, ref)
        s, e = int(s), int(e)
        if e < s:
            raise ValueError("negative dimensions are not allowed")
        if s < 0:
            raise ValueError("region start %d < 0" % s)
        starts[i], ends[i] = s, e
    eng = bf.engine(device)
    local = bf.local_tid(tids)
    rows = eng.region_stats(local, starts, ends)
    std = numpy_std(eng, rows, local, starts, ends)   # numpy's own std near rounding ties
    if max_depth:
        rows, _, _ = depthcap.apply_cap(bf, rows, tids, starts, ends, bf.lengths, int(max_depth),
                                        device, std=std)
    return [classic_stats(r, s) for r, s in zip(rows, std)]


def depth(bam, ref, start=0, end=None, device=0):
    """The exact (uncapped) per-position depth vector (int32) of [start, end)
    of `ref`."""
    bf = _as_bamfile(bam, device=device)
    t = _resolve(bf, ref)
    return bf.engine(device).depth(t, start, bf.lengths[t] if end is None else end)
