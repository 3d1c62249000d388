"""Drop-in for the reference's `metacov.pileup.classic` (metacov/pileup.py:9-26).

    classic(bam, ref, start, end) -> {min, max, med, std, avg, q23, sum}

`bam` may be a path, a `metacov_amd.bam.BamFile` / `GpuBamFile`, or a `pysam.AlignmentFile`
(its `.filename` is decoded by this library).  The depth of every contig is
computed once per file on the GPU (K2) and each call reduces one region
(K3); `classic_batch` reduces many regions in one launch.  Semantics match
classic(): positions are 0-based half-open [start, end); positions the reads
do not cover (or past the contig end) count as 0 (pileup.py:11-16); an empty
region raises ValueError (pileup.py:19 on a zero-size vector); an unknown
`ref` raises KeyError.

`experimental` and `load_kmerhist` (pileup.py:29-173) are re-exported from
`metacov_amd.experimental`, so `pileup.<name>` resolves as in the reference.
"""
import numpy as np

from . import depthcap
from .bam import BamFile
from .engine import classic_stats
from .experimental import experimental, load_kmerhist  # noqa: F401  (pileup.py:29-173)

_open_files = {}


def _as_bamfile(bam):
    if isinstance(bam, BamFile) or hasattr(bam, "engine"):   # BamFile, GpuBamFile, StreamedBam
        return bam
    key = getattr(bam, "filename", bam)
    if isinstance(key, bytes):
        key = key.decode()
    f = _open_files.get(key)
    if f is None:
        f = BamFile(key)
        _open_files[key] = f
    return f


def _resolve(bf, ref):
    try:
        return bf.references.index(ref)
    except ValueError:
        raise KeyError(ref)


def classic(bam, ref, start, end, device=0, max_depth=None):
    return classic_batch(bam, [(ref, start, end)], device=device, max_depth=max_depth)[0]


def classic_batch(bam, regions, device=0, max_depth=None):
    """[(ref, start, end), ...] -> [dict, ...] in input order.  Each dict is
    classic()'s; an empty region raises ValueError like classic().
    max_depth (opt-in, e.g. 8000 = pysam's default): reproduce htslib's
    pileup read cap per region query (metacov_amd.depthcap); None: exact."""
    bf = _as_bamfile(bam)
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
    if max_depth is not None:
        rows, _ = depthcap.capped_rows(bf, tids, starts, ends, int(max_depth), device)
    else:
        rows = bf.engine(device).region_stats(tids, starts, ends)
    return [classic_stats(r) for r in rows]


def depth(bam, ref, start=0, end=None, device=0):
    """The per-position depth vector (int32) of [start, end) of `ref`."""
    bf = _as_bamfile(bam)
    t = _resolve(bf, ref)
    return bf.engine(device).depth(t, start, bf.lengths[t] if end is None else end)
