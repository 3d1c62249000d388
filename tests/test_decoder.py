"""The product's C++ BAM decoder (host code, no GPU) against the goldens."""
import os

import numpy as np
import pytest

from metacov_amd import synth
from metacov_amd._lib import MetacovError
from metacov_amd.bam import BamFile


def _iv(g):
    return [np.array(g["intervals"][k], np.int32) for k in ("tid", "pos", "span")]


@pytest.mark.parametrize("threads", [1, 3, 0])
def test_fixture(lib_built, fixture_golden, golden_dir, threads):
    bf = BamFile(os.path.join(golden_dir, "bbmap.sorted.bam"), n_threads=threads)
    assert list(bf.references) == fixture_golden["names"]
    assert list(bf.lengths) == fixture_golden["lengths"]
    assert bf.n_records == 4112
    # 133 FUNMAP records (129 placed at a mate, 4 with tid -1)
    assert bf.mapped == 4112 - 133 and bf.unmapped == 133
    for got, want in zip((bf.tid, bf.pos, bf.span), _iv(fixture_golden)):
        assert np.array_equal(got, want)
    assert bf.aligned_bases() == 340526


@pytest.mark.parametrize("tag", ["synth_edge", "synth_multi", "synth_longcigar"])
@pytest.mark.parametrize("legacy", [False, True])
def test_synth(lib_built, synth_golden, golden_dir, tag, legacy):
    """Both end rules: current htslib's raw rlen (span 0 for a mapped read
    without reference-consuming ops) and the htslib <= 1.9 bam_endpos one."""
    bf = BamFile(os.path.join(golden_dir, tag + ".bam"), n_threads=2, legacy_endpos=legacy)
    g = synth_golden[tag]
    if legacy and "legacy" in g:
        g = g["legacy"]
    assert list(bf.references) == g["names"]
    for got, want in zip((bf.tid, bf.pos, bf.span), _iv(g)):
        assert np.array_equal(got, want)
    if tag != "synth_longcigar":
        assert (bf.span == 0).any() != legacy      # the edge mix holds zero-length alignments


def test_keep_cigar_spans(lib_built, golden_dir):
    bf = BamFile(os.path.join(golden_dir, "synth_longcigar.bam"), keep_cigar=True)
    assert bf.cig_off[0] == 0 and len(bf.cig_off) == len(bf.tid) + 1
    assert bf.cig_off[1] == 140_000          # CG:B,I tag resolved
    for i in range(len(bf.tid)):
        w = bf.cigar[bf.cig_off[i]:bf.cig_off[i + 1]]
        rl = sum(int(x >> 4) for x in w if (0x18D >> int(x & 0xF)) & 1)
        assert rl == bf.span[i]


def test_flag_filter_override(lib_built, golden_dir):
    bf = BamFile(os.path.join(golden_dir, "synth_edge.bam"), flag_filter=0)
    bf2 = BamFile(os.path.join(golden_dir, "synth_edge.bam"))
    assert len(bf.tid) > len(bf2.tid)


def test_many_blocks_and_threads(lib_built, tmp_path):
    lengths = [200_000, 3_000]
    recs = synth.edge_mix_records(lengths, 30_000, readlen=100, seed=3)
    p = str(tmp_path / "m.bam")
    synth.write_bam(p, ["a", "b"], lengths, recs)
    a = BamFile(p, n_threads=1)
    b = BamFile(p, n_threads=8)
    for x, y in zip((a.tid, a.pos, a.span), (b.tid, b.pos, b.span)):
        assert np.array_equal(x, y)
    kept = [r for r in recs if r.tid >= 0 and not (r.flag & 0x704)]
    assert len(a.tid) == len(kept)
    assert a.span.tolist() == [synth.ref_len(r.cigar) for r in kept]
    c = BamFile(p, n_threads=4, legacy_endpos=True)
    assert c.span.tolist() == [max(synth.ref_len(r.cigar), 1) for r in kept]


def test_errors(lib_built, tmp_path, golden_dir):
    with pytest.raises(MetacovError):
        BamFile(str(tmp_path / "missing.bam"))
    p = tmp_path / "plain.gz"
    import gzip
    with gzip.open(p, "wb") as fh:
        fh.write(b"BAM\1" + b"\0" * 100)
    with pytest.raises(MetacovError, match="BGZF"):
        BamFile(str(p))
    raw = open(os.path.join(golden_dir, "bbmap.sorted.bam"), "rb").read()
    t = tmp_path / "trunc.bam"
    t.write_bytes(raw[: len(raw) // 2])
    with pytest.raises(MetacovError):
        BamFile(str(t))


def test_parallel_boundaries_large(lib_built, tmp_path):
    """2M records through the C++ writer: every thread count decodes the same
    intervals (parallel record-boundary sync + two-pass parse)."""
    lengths = [3_000_000, 1_000, 900_000]
    arrs = synth.edge_mix_arrays(lengths, 2_000_000, seed=11)
    p = str(tmp_path / "big.bam")
    synth.write_bam_fast(p, ["x", "y", "z"], lengths, *arrs, level=1, n_threads=4)
    ref = BamFile(p, n_threads=1)
    assert ref.n_records == 2_000_000
    tid, pos, flag, cig_off, cigar = arrs
    keep = (flag & 0x704) == 0
    assert np.array_equal(ref.tid, tid[keep]) and np.array_equal(ref.pos, pos[keep])
    for th in (2, 7, 16):
        b = BamFile(p, n_threads=th)
        assert b.n_records == ref.n_records and b.mapped == ref.mapped
        for x, y in zip((ref.tid, ref.pos, ref.span), (b.tid, b.pos, b.span)):
            assert np.array_equal(x, y)


# ---- BAI index (mc_bam_index_build) and indexed contig decode ------------

def _parse_bai(path):
    """Test-side reader: {bin: chunks} (sorted; the pseudo-bin as stored),
    the linear index per reference, and the no-coordinate count."""
    import struct
    d = open(path, "rb").read()
    assert d[:4] == b"BAI\1"
    o = 8
    refs = []
    for _ in range(struct.unpack_from("<i", d, 4)[0]):
        n_bin, = struct.unpack_from("<i", d, o)
        o += 4
        bins = {}
        for _ in range(n_bin):
            b, nc = struct.unpack_from("<Ii", d, o)
            o += 8
            ch = [struct.unpack_from("<QQ", d, o + 16 * k) for k in range(nc)]
            o += 16 * nc
            bins[b] = ch if b == 37450 else sorted(ch)
        n_intv, = struct.unpack_from("<i", d, o)
        o += 4
        refs.append((bins, list(struct.unpack_from("<%dQ" % n_intv, d, o))))
        o += 8 * n_intv
    return refs, struct.unpack_from("<Q", d, o)[0]


def test_index_matches_reference_fixture(lib_built, golden_dir, tmp_path):
    """Our index of the reference's test BAM equals the .bai its authors
    shipped beside it (tests/data/bbmap.sorted.bam.bai, made by samtools)."""
    import shutil
    from metacov_amd.bam import build_index, index_stats
    p = tmp_path / "f.bam"
    shutil.copy(os.path.join(golden_dir, "bbmap.sorted.bam"), p)
    ours = build_index(str(p))
    assert _parse_bai(ours) == _parse_bai(os.path.join(golden_dir, "bbmap.sorted.bam.bai"))
    m, u, nc = index_stats(os.path.join(golden_dir, "bbmap.sorted.bam.bai"), 2)
    assert m.tolist() == [1694, 2285] and u.tolist() == [38, 91] and nc == 4


def test_indexed_contig_decode(lib_built, tmp_path):
    """BamFile(contigs=...) through the index == the full decode restricted to
    those contigs; counts come from the index (pysam .mapped / .unmapped)."""
    from metacov_amd.bam import build_index, index_stats
    lengths = [3_000_000, 1_000, 900_000, 50_000, 2_000_000, 7]
    arrs = synth.edge_mix_arrays(lengths, 600_000, seed=5)
    p = str(tmp_path / "m.bam")
    synth.write_bam_fast(p, ["c%d" % i for i in range(len(lengths))], lengths, *arrs, level=1,
                         n_threads=4)
    build_index(p)
    full = BamFile(p, keep_cigar=True)
    m, u, nc = index_stats(p + ".bai", len(lengths))
    assert m.sum() == full.mapped and u.sum() + nc == full.unmapped
    for sel in ([0], [4, 2], [5], [1, 3, 5], list(range(6)), []):
        bf = BamFile(p, contigs=sel, n_threads=3, keep_cigar=True)
        keep = np.isin(full.tid, sel)
        for a, b in ((bf.tid, full.tid), (bf.pos, full.pos), (bf.span, full.span)):
            assert np.array_equal(a, b[keep])
        assert (bf.mapped, bf.unmapped, bf.references) == (full.mapped, full.unmapped,
                                                            full.references)
        r = full.restrict(sel)
        assert np.array_equal(r.cigar, bf.cigar) and np.array_equal(r.cig_off, bf.cig_off)
        if len(sel):
            assert bf.local_tid(sorted(sel)[-1]) == len(set(sel)) - 1
    with pytest.raises(KeyError):
        BamFile(p, contigs=[1]).local_tid(0)


def test_index_errors(lib_built, tmp_path, golden_dir):
    with pytest.raises(MetacovError, match="bai"):
        BamFile(os.path.join(golden_dir, "synth_multi.bam"), contigs=[0],
                index=str(tmp_path / "none.bai"))
    lengths = [10_000]
    tid = np.zeros(3, np.int32)
    pos = np.array([500, 100, 900], np.int32)          # not coordinate-sorted
    flag = np.zeros(3, np.uint16)
    cig_off = np.arange(4, dtype=np.int64)
    cigar = np.full(3, (50 << 4) | 0, np.uint32)
    p = str(tmp_path / "u.bam")
    synth.write_bam_fast(p, ["a"], lengths, tid, pos, flag, cig_off, cigar, l_seq=50)
    from metacov_amd.bam import build_index
    with pytest.raises(MetacovError, match="coordinate-sorted"):
        build_index(p)


# ---- streaming decode (mc_bam_stream_*) ------------------------------------

def _drain(st, cap):
    parts = []
    while True:
        k, out = st.read(cap)
        if k == 0:
            break
        parts.append([a[:k].copy() for a in out])
    if not parts:
        return [np.zeros(0, np.int32)] * 3
    return [np.concatenate([x[i] for x in parts]) for i in range(3)]


@pytest.mark.parametrize("window", [1 << 16, 1 << 20, 0])
def test_stream_equals_full_decode(lib_built, golden_dir, tmp_path, window):
    """Windows far smaller than one record (the 140 000-op CG record) and
    batch sizes that cut windows: the same intervals and counts."""
    from metacov_amd.bam import BamStream
    lengths = [2_000_000, 700, 300_000]
    arrs = synth.edge_mix_arrays(lengths, 300_000, seed=4)
    p = str(tmp_path / "s.bam")
    synth.write_bam_fast(p, ["a", "b", "c"], lengths, *arrs, level=1, n_threads=4)
    for path in (p, os.path.join(golden_dir, "bbmap.sorted.bam"),
                 os.path.join(golden_dir, "synth_longcigar.bam")):
        full = BamFile(path)
        with BamStream(path, n_threads=3, window_bytes=window) as st:
            assert st.references == full.references and st.lengths == full.lengths
            got = _drain(st, 12_345)
            assert st.counts() == (full.n_records, full.mapped, full.unmapped)
        for g, w in zip(got, (full.tid, full.pos, full.span)):
            assert np.array_equal(g, w)


def test_stream_truncated(lib_built, golden_dir, tmp_path):
    from metacov_amd.bam import BamStream
    raw = open(os.path.join(golden_dir, "bbmap.sorted.bam"), "rb").read()
    t = tmp_path / "trunc.bam"
    t.write_bytes(raw[: len(raw) // 2])
    with pytest.raises(MetacovError):
        with BamStream(str(t), window_bytes=1 << 16) as st:
            _drain(st, 1000)
