"""Full-size parity: BASELINE.json configs[2] (C3: 1000 contigs, ~1 Gbp,
100 M x ~150 bp reads) and configs[4] on one GPU (C5: 10 000 contigs of
50-150 kbp, 50 M lognormal ~10 kbp reads), generated exactly as bench.py
generates them, against the O(N + G) interval oracle (oracle/oracle.c
orc_depth_interval + orc_region_stats: the restated htslib column count and
the exact classic() statistics, metacov/pileup.py:13-26).

Every position of every contig is compared bit for bit, and every
whole-contig row of the fused statistics call (depth + stats in one K2 pass)
field by field.  C5 also runs the raw-CIGAR path (K1 turns BAM CIGAR words
into the same spans on the GPU).
"""
import os
import sys

import numpy as np
import pytest

from oracle import coracle
from metacov_amd.engine import CoverageEngine

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _workload(cfg, seed=1):
    import torch
    import bench
    reads, contigs, _ = bench.CONFIGS[cfg]
    lengths, weights = bench.config_contigs(cfg, reads, contigs)
    dev = torch.device("cuda", 0)
    tid, pos, span, _ = bench.device_workload(torch, lengths, weights, reads, seed, dev,
                                              long_reads=cfg == "c5")
    torch.cuda.synchronize()
    return lengths, (tid, pos, span)


def _paths(eng):
    t = eng.timings()
    return t["direct_batches"], t["full_prepares"]


def _compare(eng, lengths, h, rows):
    d, ext, coff = coracle.depth(lengths, *h)
    assert eng.aligned_bases() == int(h[2].astype(np.int64).sum()) == int(d.sum(dtype=np.int64))
    for t in range(len(lengths)):
        assert eng.contig_offset(t)[1] == ext[t]
        got = eng.depth(t, 0, int(ext[t]))
        if not np.array_equal(got, d[coff[t]:coff[t] + ext[t]]):
            bad = np.nonzero(got != d[coff[t]:coff[t] + ext[t]])[0]
            raise AssertionError("contig %d: %d positions differ, first %s" % (t, len(bad), bad[:5]))
    rt = np.arange(len(lengths), dtype=np.int32)
    want = coracle.region_stats(d, ext, coff, rt, np.zeros(len(lengths), np.int64), lengths)
    for f in want.dtype.names:
        assert np.array_equal(rows[f], want[f]), f
    return d


def test_c3_full_size():
    """C3 at its stated 100 M reads: the per-batch direct path (probe +
    validating K2) with fused whole-contig statistics, bit-exact."""
    lengths, dev_reads = _workload("c3")
    h = [x.cpu().numpy() for x in dev_reads]
    eng = CoverageEngine(0)
    try:
        eng.set_contigs(lengths)
        eng.add_reads(*dev_reads)
        del dev_reads
        rows = eng.compute_depth_stats(np.arange(len(lengths), dtype=np.int32),
                                       np.zeros(len(lengths), np.int64), lengths)
        assert _paths(eng) == (1, 0)
        assert eng.fused_fallbacks() == 0 and eng.fused_recomputes() == 0
        _compare(eng, lengths, h, rows)
        # the reused-index path (explicit full prepare, packed read words) on the same batch
        eng.invalidate()
        eng.prepare()
        rows2 = eng.compute_depth_stats(np.arange(len(lengths), dtype=np.int32),
                                        np.zeros(len(lengths), np.int64), lengths)
        for f in rows.dtype.names:
            assert np.array_equal(rows2[f], rows[f]), f
    finally:
        eng.close()


def test_c5_full_size_and_cigar_path():
    """C5 on one GPU at full size (10 000 contigs, 50 M ~10 kbp reads): the
    long-read path (bucketed end events, per-chunk carries) with fused
    statistics and their K3 fallback rows, bit-exact; then the same spans
    through K1 from BAM CIGAR words (~20 ops per read, 1 G words)."""
    import torch
    from metacov_amd import synth
    lengths, dev_reads = _workload("c5")
    h = [x.cpu().numpy() for x in dev_reads]
    eng = CoverageEngine(0)
    try:
        eng.set_contigs(lengths)
        eng.add_reads(*dev_reads)
        rt = np.arange(len(lengths), dtype=np.int32)
        rows = eng.compute_depth_stats(rt, np.zeros(len(lengths), np.int64), lengths)
        assert _paths(eng)[1] >= 1            # long reads: the full prepare
        print("C5 out-of-window regions: %d recomputed on the device, %d by the host"
              % (eng.fused_recomputes(), eng.fused_fallbacks()))
        assert eng.fused_fallbacks() == 0
        d = _compare(eng, lengths, h, rows)
        # K1: CIGAR words -> the same spans
        tid, pos, span = dev_reads
        cig_off, cigar = synth.device_cigars(torch, span, mean_ops=20, seed=9)
        torch.cuda.synchronize()
        eng.clear_reads()
        eng.add_reads_cigar_device(tid, pos, cig_off, cigar)
        eng.compute_depth()
        assert eng.aligned_bases() == int(h[2].astype(np.int64).sum())
        off = 0
        for t in range(len(lengths)):
            e_t = eng.contig_offset(t)[1]
            assert np.array_equal(eng.depth(t, 0, e_t), d[off:off + e_t]), t
            off += e_t
        del cig_off, cigar
    finally:
        eng.close()
