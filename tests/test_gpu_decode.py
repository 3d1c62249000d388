"""GPU BAM decode (csrc/bam_gpu.hip, csrc/inflate.h).

CPU tests: the lane decoder of the inflate kernel (run on the host through
mc_gz_inflate_host) against zlib on raw deflate streams of every block type
and on the BGZF blocks of the fixture and synthetic BAMs; the record parse
against the host decoder's rules.  GPU tests: mc_bam_gpu_open against the
host decoder (mc_bam_open, itself pinned by the goldens in test_decoder.py)
record for record, including windows far smaller than one record, records
spanning many 64 KiB parse segments, and the error classes.
"""
import ctypes
import os
import struct
import zlib

import numpy as np
import pytest

from metacov_amd import synth
from metacov_amd._lib import MetacovError


def _lib():
    from metacov_amd import _lib as L
    return L.load()


def _raw_deflate(data, level, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
    return c.compress(data) + c.flush()


def _inflate_host(comp, isize):
    lib = _lib()
    out = ctypes.create_string_buffer(max(isize, 1))
    rc = lib.mc_gz_inflate_host(comp, len(comp), out, isize)
    return rc, out.raw[:isize]


def _bgzf_blocks(raw):
    """(payload, isize) of every BGZF block of a file's bytes."""
    o, out = 0, []
    while o < len(raw):
        assert raw[o:o + 4] == b"\x1f\x8b\x08\x04"
        xlen, = struct.unpack_from("<H", raw, o + 10)
        x, bsize = o + 12, None
        while x < o + 12 + xlen:
            si1, si2, slen = raw[x], raw[x + 1], struct.unpack_from("<H", raw, x + 2)[0]
            if si1 == 66 and si2 == 67:
                bsize = struct.unpack_from("<H", raw, x + 4)[0] + 1
            x += 4 + slen
        payload = raw[o + 12 + xlen:o + bsize - 8]
        isize, = struct.unpack_from("<I", raw, o + bsize - 4)
        out.append((payload, isize))
        o += bsize
    return out


def _rare_matches(seed, n=65280):
    """Skewed literals with rare copies: the end-of-block and length symbols
    get long codes (10-14 bits, past the primary table), the case of the byte
    symbol lists' kLitHi split."""
    rng = np.random.default_rng(seed)
    out = bytearray(np.minimum(rng.geometric(0.02, n), 255).astype(np.uint8).tobytes())
    i = 300
    while i < n - 300:
        if rng.random() < 0.004:
            ln, d = int(rng.integers(3, 259)), int(rng.integers(1, min(i, 32768)))
            for k in range(min(ln, n - i)):
                out[i + k] = out[i + k - d]
            i += ln
        i += 1
    return bytes(out)


def test_inflate_host_matches_zlib(lib_built):
    rng = np.random.default_rng(0)
    cases = [b"", b"a", b"ab" * 3, _rare_matches(1), _rare_matches(2),
             bytes(rng.integers(0, 256, 65280, dtype=np.uint8)),          # incompressible
             bytes(rng.integers(0, 4, 65280, dtype=np.uint8) + 65),
             b"ACGT" * 16000,                                             # long matches
             bytes(rng.choice(np.frombuffer(b"ACGTN", np.uint8), 60000, p=[.3, .2, .2, .29, .01])),
             bytes(range(256)) * 200]
    for data in cases:
        for level in (0, 1, 6, 9):
            for strat in (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE):
                comp = _raw_deflate(data, level, strat)
                rc, got = _inflate_host(comp, len(data))
                assert rc == 0 and got == data, (len(data), level, strat)
    # wrong ISIZE either way is an error
    comp = _raw_deflate(b"x" * 1000, 6)
    assert _inflate_host(comp, 999)[0] != 0
    assert _inflate_host(comp, 1001)[0] != 0


def test_inflate_host_bgzf_blocks(lib_built, golden_dir, tmp_path):
    """Every BGZF block of the reference's fixture (samtools-written) and of
    synthetic BAMs (zlib levels 1 and 6) decodes to zlib's bytes."""
    paths = [os.path.join(golden_dir, f) for f in ("bbmap.sorted.bam", "synth_longcigar.bam",
                                                   "synth_edge.bam")]
    lengths = [300_000, 900]
    arrs = synth.edge_mix_arrays(lengths, 20_000, seed=9)
    for level in (1, 6):
        p = str(tmp_path / ("l%d.bam" % level))
        synth.write_bam_fast(p, ["a", "b"], lengths, *arrs, level=level, n_threads=2)
        paths.append(p)
    n = 0
    for p in paths:
        for payload, isize in _bgzf_blocks(open(p, "rb").read()):
            want = zlib.decompress(payload, -15)
            assert len(want) == isize
            rc, got = _inflate_host(payload, isize)
            assert rc == 0 and got == want
            n += 1
    assert n > 20


def test_inflate_host_corrupt_streams_fail_cleanly(lib_built, golden_dir):
    """Flipped bytes in real blocks: the lane decoder returns (ok or an
    error) without reading or writing out of bounds; where it reports ok,
    zlib agrees on the bytes."""
    blocks = _bgzf_blocks(open(os.path.join(golden_dir, "bbmap.sorted.bam"), "rb").read())
    rng = np.random.default_rng(3)
    for trial in range(300):
        payload, isize = blocks[trial % (len(blocks) - 1)]
        b = bytearray(payload)
        for _ in range(1 + trial % 4):
            b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
        if trial % 7 == 0:
            b = b[: int(rng.integers(1, len(b)))]
        rc, got = _inflate_host(bytes(b), isize)
        if rc == 0:
            try:
                want = zlib.decompress(bytes(b), -15)
            except zlib.error:
                continue   # zlib is stricter about some incomplete codes
            assert got == want[:isize]


def _parse_host(body, n_ref=3, flag_filter=0x704):
    out = (ctypes.c_int32 * 3)()
    rc = _lib().mc_bam_rec_parse_host(body, len(body), n_ref, flag_filter, out)
    return rc, tuple(out)


def test_rec_parse_host(lib_built):
    R = synth.SynthRecord
    cases = [
        (R("r", 0, 100, 0, [(0, 50), (2, 3), (1, 4), (0, 20)], 74), (1, (0, 100, 73))),   # M D I M
        (R("r", 1, 5, 0, [(4, 10), (7, 30), (8, 2), (3, 1000)], 40), (1, (1, 5, 1032))),  # S = X N
        (R("r", 2, 7, 0, [(4, 20)], 20), (1, (2, 7, 0))),        # no reference op: span 0 (bam_plp_push)
        (R("r", 0, 7, 0x100, [(0, 20)], 20), (0, None)),          # secondary: dropped
        (R("r", 0, 7, 0x800, [(0, 20)], 20), (1, (0, 7, 20))),   # supplementary: kept
        (R("r", -1, -1, 4, [], 20), (0, None)),
        (R("r", 5, 7, 0, [(0, 20)], 20), (2, None)),             # tid beyond n_ref
    ]
    for rec, (rc_want, iv) in cases:
        body = synth.encode_record(rec)[4:]
        rc, out = _parse_host(body)
        assert rc == rc_want, rec.cigar
        if iv:
            assert out == iv
    # htslib <= 1.9 bam_endpos rule (MC_LEGACY_ENDPOS): such a read spans 1
    rc, out = _parse_host(synth.encode_record(R("r", 2, 7, 0, [(4, 20)], 20))[4:],
                          flag_filter=0x704 | 0x10000)
    assert (rc, out) == (1, (2, 7, 1))
    # CG:B,I placeholder resolved (> 65535 ops)
    ops = [(0, 1), (2, 1)] * 40_000
    body = synth.encode_record(R("r", 0, 9, 0, ops, 40_000), long_cigar_threshold=65535)[4:]
    assert _parse_host(body) == (1, (0, 9, 80_000))


# ---------------------------------------------------------------- GPU

def _host_and_gpu(path, **kw):
    from metacov_amd.bam import BamFile, GpuBamFile
    h = BamFile(path)
    g = GpuBamFile(path, **kw)
    return h, g


def _assert_same(h, g):
    assert g.references == h.references and g.lengths == h.lengths
    assert (g.n_records, g.mapped, g.unmapped) == (h.n_records, h.mapped, h.unmapped)
    tid, pos, span = g.intervals()
    assert np.array_equal(tid, h.tid) and np.array_equal(pos, h.pos) and np.array_equal(span, h.span)


def _assert_oracle(path, g):
    """The GPU decode against the oracle's own reader (oracle/bamread.py:
    gzip + struct, the restated 0x704 filter and bam_plp_push span), not
    against the product's host decoder."""
    from oracle import bamread
    names, lengths, counts, tid, pos, span = bamread.scan_intervals(path)
    assert list(g.references) == names and list(g.lengths) == lengths
    assert (g.n_records, g.mapped, g.unmapped) == counts
    gt, gp, gs = g.intervals()
    assert np.array_equal(gt, tid) and np.array_equal(gp, pos) and np.array_equal(gs, span)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["bbmap.sorted.bam", "synth_edge.bam", "synth_multi.bam",
                                  "synth_longcigar.bam"])
@pytest.mark.parametrize("window", [0, 1 << 20])
def test_gpu_decode_goldens(lib_built, golden_dir, name, window):
    h, g = _host_and_gpu(os.path.join(golden_dir, name), window_bytes=window)
    _assert_same(h, g)
    _assert_oracle(os.path.join(golden_dir, name), g)
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("level,window", [(1, 0), (6, 1 << 20), (1, 3 << 20)])
def test_gpu_decode_large(lib_built, tmp_path, level, window):
    """2M records over several windows (records cut by window ends carried),
    ~600 parse segments per window."""
    lengths = [3_000_000, 1_000, 900_000]
    arrs = synth.edge_mix_arrays(lengths, 2_000_000, seed=11)
    p = str(tmp_path / "big.bam")
    synth.write_bam_fast(p, ["x", "y", "z"], lengths, *arrs, level=level, n_threads=8)
    h, g = _host_and_gpu(p, window_bytes=window)
    _assert_same(h, g)
    _assert_oracle(p, g)
    t = g.timings()
    assert t["blocks"] > 100 and t["inflated_bytes"] > 0
    if window:
        assert t["windows"] > 1
    # false syncs are rare and each is fixed once (a stale-walk cascade once
    # made every later segment a "resync" and fell back to a one-lane walk)
    assert t["resyncs"] <= 64, t["resyncs"]
    # trim() drops the decode's staging (compressed file, inflated
    # stream, tables); intervals, extents, the engine and restrict still work
    ext = g.extents()
    freed = g.trim()
    assert freed >= t["inflated_bytes"] if not window else freed > window
    assert g.trim() == 0
    _assert_same(h, g)
    assert np.array_equal(g.extents()[0], ext[0])
    tid, pos, span = g.intervals([2])
    assert np.array_equal(pos, h.pos[h.tid == 2])
    g.restrict([0, 2])
    assert g.n_kept == int(np.sum(h.tid != 1))
    g.close()


@pytest.mark.gpu
def test_gpu_decode_background_upload(lib_built, tmp_path):
    """A file >= 256 MiB decodes resident with the whole upload running in the
    background while its blocks are scanned: equal to the host decoder; a
    truncated copy (the scan fails while the upload runs) and a copy with a
    corrupt block near its end (the inflate fails after the upload) raise
    without hanging."""
    from metacov_amd.bam import GpuBamFile
    lengths = [20_000_000, 30_000_000]
    arrs = synth.edge_mix_arrays(lengths, 2_000_000, seed=5)
    p = str(tmp_path / "bg.bam")
    synth.write_bam_fast(p, ["a", "b"], lengths, *arrs, level=1, n_threads=8)
    size = os.path.getsize(p)
    assert size >= 256 << 20, size
    h, g = _host_and_gpu(p)
    _assert_same(h, g)
    t = g.timings()
    assert t["windows"] >= 2 and t["upload_ms"] > 0
    g.close()
    raw = open(p, "rb").read()
    tr = tmp_path / "bg_trunc.bam"
    tr.write_bytes(raw[: len(raw) * 2 // 3])
    with pytest.raises(MetacovError):
        GpuBamFile(str(tr))
    b = bytearray(raw)
    off = len(raw) - (1 << 20)
    while raw[off:off + 4] != b"\x1f\x8b\x08\x04":
        off += 1
    for k in range(40, 400):
        b[off + k] ^= 0x5a
    cr = tmp_path / "bg_corrupt.bam"
    cr.write_bytes(bytes(b))
    del raw, b
    with pytest.raises(MetacovError, match="inflate|record|CIGAR|BGZF"):
        GpuBamFile(str(cr))


@pytest.mark.gpu
def test_gpu_decode_long_records(lib_built, tmp_path):
    """Records of 30-200 KB (long reads with their sequence): most 64 KiB
    parse segments hold no record start."""
    rng = np.random.default_rng(2)
    lengths = [5_000_000, 2_000_000]
    recs = []
    for t, L in enumerate(lengths):
        for p in np.sort(rng.integers(0, L - 150_000, 60)):
            rl = int(rng.integers(10_000, 120_000))
            recs.append(synth.SynthRecord("long%d" % len(recs), t, int(p), 0, [(4, 50), (0, rl), (2, 7)], rl + 50))
    path = str(tmp_path / "long.bam")
    synth.write_bam(path, ["a", "b"], lengths, recs)
    for window in (0, 1 << 20):
        h, g = _host_and_gpu(path, window_bytes=window)
        _assert_same(h, g)
        _assert_oracle(path, g)
        g.close()


@pytest.mark.gpu
def test_gpu_decode_header_only_and_tiny(lib_built, tmp_path):
    p = str(tmp_path / "empty.bam")
    synth.write_bam(p, ["a", "b"], [100, 200], [])
    h, g = _host_and_gpu(p)
    _assert_same(h, g)
    assert g.n_kept == 0
    g.close()
    p = str(tmp_path / "one.bam")
    synth.write_bam(p, ["a"], [1000], [synth.SynthRecord("r", 0, 10, 0, [(0, 30)], 30)])
    h, g = _host_and_gpu(p)
    _assert_same(h, g)
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("window", [0, 1 << 18])
def test_gpu_decode_errors(lib_built, tmp_path, golden_dir, window):
    """Truncated and corrupted files raise, resident (window 0) and windowed
    (the next window's upload is in flight on the uploader thread when the
    current window fails)."""
    from metacov_amd.bam import GpuBamFile
    with pytest.raises(MetacovError):
        GpuBamFile(str(tmp_path / "missing.bam"), window_bytes=window)
    raw = open(os.path.join(golden_dir, "bbmap.sorted.bam"), "rb").read()
    t = tmp_path / "trunc.bam"
    t.write_bytes(raw[: len(raw) // 2])
    with pytest.raises(MetacovError):
        GpuBamFile(str(t), window_bytes=window)
    # a corrupted deflate payload in a whole block
    blocks = _bgzf_blocks(raw)
    b = bytearray(raw)
    off = len(raw) // 3
    while raw[off:off + 4] != b"\x1f\x8b\x08\x04":
        off += 1
    for k in range(40, 200):
        b[off + k] ^= 0x5a
    c = tmp_path / "corrupt.bam"
    c.write_bytes(bytes(b))
    with pytest.raises(MetacovError, match="inflate|record|CIGAR|BGZF"):
        GpuBamFile(str(c), window_bytes=window)
    assert len(blocks) > 3


@pytest.mark.gpu
def test_gpu_decode_feeds_engine(lib_built, golden_dir, fixture_golden):
    """The decoded intervals go into a ctx by a device copy: classic() rows
    equal the host-decoded file's."""
    from metacov_amd.bam import BamFile, GpuBamFile
    from metacov_amd import pileup
    path = os.path.join(golden_dir, "bbmap.sorted.bam")
    h = BamFile(path)
    g = GpuBamFile(path)
    for ref, L in zip(h.references, h.lengths):
        assert pileup.classic(g, ref, 0, L) == pileup.classic(h, ref, 0, L)
    g.close()


@pytest.mark.gpu
def test_cli_gpu_decode_windows_vs_oracle(lib_built, tmp_path):
    """`metacov pileup --decode gpu --window-bytes 1 MiB` over a 200k-record
    BAM (~60 windows, records cut by window ends): the CSV equals the one
    built from the oracle alone (bamread intervals -> coracle depth + exact
    region rows -> classic()'s formatting), for whole contigs and tilings."""
    import csv
    import io
    from click.testing import CliRunner
    from metacov_amd.cli import pileup as cli_pileup
    from metacov_amd.engine import classic_stats
    from oracle import bamread, coracle
    lengths = [3_000_000, 1_000, 900_000]
    arrs = synth.edge_mix_arrays(lengths, 200_000, seed=17)
    p = str(tmp_path / "w.bam")
    synth.write_bam_fast(p, ["x", "y", "z"], lengths, *arrs, level=1, n_threads=8)
    names, lens, _c, tid, pos, span = bamread.scan_intervals(p)
    d, ext, coff = coracle.depth(lens, tid, pos, span)
    rng = np.random.default_rng(3)
    regs = [("x", 0, 3_000_000), ("y", 0, 1_000), ("z", 0, 900_000)]
    for _ in range(12):
        t = int(rng.integers(0, 3))
        a = int(rng.integers(0, lens[t]))
        regs.append((names[t], a, int(rng.integers(a + 1, lens[t] + 500))))
    rows = coracle.region_stats(d, ext, coff, np.array([names.index(r[0]) for r in regs], np.int32),
                                np.array([r[1] for r in regs], np.int64),
                                np.array([r[2] for r in regs], np.int64))
    out = io.StringIO()
    w = None
    for r, row in zip(regs, rows):
        res = classic_stats(row)
        if w is None:
            w = csv.DictWriter(out, fieldnames=["sacc", "start", "end"] + sorted(res))
            w.writeheader()
        res.update({"sacc": r[0], "start": str(r[1]), "end": str(r[2])})
        w.writerow(res)
    rc = tmp_path / "r.csv"
    rc.write_text("sacc,sstart,send\n" + "".join("%s,%d,%d\n" % r for r in regs))
    o = tmp_path / "o.csv"
    res = CliRunner().invoke(cli_pileup, ["-b", p, "-rc", str(rc), "-o", str(o), "--decode", "gpu",
                                          "--window-bytes", str(1 << 20)])
    assert res.exit_code == 0, res.output
    assert open(o, newline="").read() == out.getvalue()


def test_bgzf_scan_host(lib_built, golden_dir, tmp_path):
    """The GPU decode's pread block scan (no GPU) finds every BGZF block of
    the golden and synthetic BAMs, with its range split on (many threads on
    a multi-range file) or off, and fails on a truncated file."""
    import numpy as np
    from metacov_amd import synth
    lib = _lib()
    paths = [os.path.join(golden_dir, f) for f in sorted(os.listdir(golden_dir)) if f.endswith(".bam")]
    big = str(tmp_path / "big.bam")
    lengths = np.full(4, 2_000_000, np.int64)
    arrs = synth.edge_mix_arrays(lengths, 1_200_000, seed=3)
    synth.write_bam_fast(big, ["c%d" % i for i in range(4)], lengths, *arrs, level=1, n_threads=8)
    assert os.path.getsize(big) > 64 << 20     # several scan ranges
    paths.append(big)
    for p in paths:
        raw = open(p, "rb").read()
        want, o = [], 0
        for payload, isize in _bgzf_blocks(raw):
            want.append(isize)
        offs, o = [], 0
        while o < len(raw):
            offs.append(o)
            o += struct.unpack_from("<H", raw, o + 16)[0] + 1
        for nt in (1, 3, 16):
            nb, tot = ctypes.c_int64(), ctypes.c_int64()
            got = (ctypes.c_int64 * len(offs))()
            assert lib.mc_bgzf_scan_host(p.encode(), nt, ctypes.byref(nb), ctypes.byref(tot), got, len(offs)) == 0
            assert nb.value == len(offs) and tot.value == sum(want)
            assert list(got) == offs, (p, nt)
    t = tmp_path / "trunc.bam"
    raw = open(big, "rb").read()
    t.write_bytes(raw[: len(raw) // 2 + 1000])
    nb, tot = ctypes.c_int64(), ctypes.c_int64()
    assert lib.mc_bgzf_scan_host(str(t).encode(), 16, ctypes.byref(nb), ctypes.byref(tot), None, 0) != 0


# ------------------------------------------------ record sync: bins and order

def _inflated(path):
    """The BAM's inflated stream, its first record offset and n_ref."""
    data = b"".join(zlib.decompress(p, -15) for p, _ in _bgzf_blocks(open(path, "rb").read()))
    l_text, = struct.unpack_from("<i", data, 4)
    o = 8 + l_text
    n_ref, = struct.unpack_from("<i", data, o)
    o += 4
    for _ in range(n_ref):
        ln, = struct.unpack_from("<i", data, o)
        o += 8 + ln
    return data, o, n_ref


def _record_starts(data, o):
    out = []
    while o < len(data):
        out.append(o)
        o += 4 + struct.unpack_from("<i", data, o)[0]
    return out


def _chain(data, q, n_ref, chain=8):
    return _lib().mc_bam_rec_chain_host(data, len(data), q, n_ref, chain)


def test_rec_chain_accepts_every_record_start(lib_built, golden_dir):
    """The GPU record sync's rule (structure, the bin field of mapped
    records, sort order along the chain) holds at every record of the
    samtools-written fixture and of the synthetic BAMs, whose mapped
    records' bins were computed by their writers."""
    for name in ("bbmap.sorted.bam", "synth_edge.bam", "synth_multi.bam", "synth_longcigar.bam"):
        data, o, n_ref = _inflated(os.path.join(golden_dir, name))
        starts = _record_starts(data, o)
        assert len(starts) >= 2
        for q in starts:
            assert _chain(data, q, n_ref) == 1, (name, q)


FAKE = 38   # bytes per fake record


def _fake_records(k, tid, pos0, good_bins, ascending=True):
    """k back-to-back minimal records (38 bytes each: no CIGAR, no bases, a
    1-character name) that pass the old structural sync test."""
    out = b""
    for j in range(k):
        pos = pos0 + (j if ascending else k - j)
        bin_ = synth._reg2bin(pos, pos + 1) if good_bins else 1234
        out += struct.pack("<i", 34) + struct.pack("<iiBBHHHiiii", tid, pos, 2, 0, bin_, 0, 0, 0, tid,
                                                   pos, 0) + b"f\0"
    return out


def _near_valid_bam(path, n, good_bins, ascending, fakes=12, seed=4):
    """Records whose aux data (an XB:B:C byte array) holds a chain of fake
    records: a sync landing in a record's bytes meets them first."""
    rng = np.random.default_rng(seed)
    names, lengths = ["a", "b"], [4_000_000, 3_000_000]
    recs = []
    for t, L in enumerate(lengths):
        for p in np.sort(rng.integers(0, L - 200, n // 2)):
            r = synth.SynthRecord("r%d" % len(recs), t, int(p), 0, [(0, 100)], 100)
            body = synth.encode_record(r)[4:]
            payload = _fake_records(fakes, t, int(p), good_bins, ascending)
            body += b"XBBC" + struct.pack("<i", len(payload)) + payload
            recs.append(struct.pack("<i", len(body)) + body)
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join("@SQ\tSN:%s\tLN:%d\n" % x for x in zip(names, lengths))
    hdr = bytearray(b"BAM\x01") + struct.pack("<i", len(text)) + text.encode() + struct.pack("<i", 2)
    for nm, L in zip(names, lengths):
        hdr += struct.pack("<i", len(nm) + 1) + nm.encode() + b"\0" + struct.pack("<i", L)
    with open(path, "wb") as fh:
        fh.write(synth._bgzf(bytes(hdr) + b"".join(recs)))


def test_rec_chain_rejects_near_valid_fakes(lib_built, tmp_path):
    """Fake record chains inside aux bytes: wrong bins, or right bins in
    descending order, never start a sync chain; the real records do.  (The
    last of the descending fakes does chain into the real records after it:
    a walk from it lands on the next real record, and the previous
    segment's walk corrects it.)"""
    for good_bins, ascending in ((False, True), (True, False)):
        p = str(tmp_path / "nv.bam")
        _near_valid_bam(p, 200, good_bins, ascending)
        data, o, n_ref = _inflated(p)
        starts = _record_starts(data, o)
        for q in starts:
            assert _chain(data, q, n_ref) == 1
            fake0 = q + 4 + struct.unpack_from("<i", data, q)[0] - 12 * FAKE
            for f in range(fake0, fake0 + (12 if not good_bins else 11) * FAKE, FAKE):
                assert _chain(data, f, n_ref) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("good_bins,ascending", [(False, True), (True, False), (True, True)])
def test_gpu_decode_near_valid_records(lib_built, tmp_path, good_bins, ascending):
    """40k records of ~500 B, most of each a chain of fake records: the
    decode equals the oracle's reader.  Fakes the bin check rejects cost no
    resync at all; fakes that pass the checks (right bins: the last of a
    descending run, or a whole ascending run) are corrected from the
    verified prefix, re-synced with long chains if they persist, in a few
    rounds, never by one lane walking the rest."""
    p = str(tmp_path / "nv.bam")
    _near_valid_bam(p, 40_000, good_bins, ascending, fakes=12)
    from metacov_amd.bam import GpuBamFile
    with GpuBamFile(p) as g:
        _assert_oracle(p, g)
        t = g.timings()
    if not good_bins:
        assert t["resyncs"] == 0 and t["parse_rounds"] == 1, t
    else:
        assert t["parse_rounds"] < 4, t


# ------------------------------------------------ contig shards

def _multi_contig_bam(tmp_path, n_reads=300_000, seed=21):
    rng = np.random.default_rng(seed)
    lengths = rng.integers(20_000, 400_000, 40).astype(np.int64)
    lengths[[3, 17]] = [1, 64]                      # tiny contigs (few or no reads)
    arrs = synth.edge_mix_arrays(lengths, n_reads, seed=seed)
    p = str(tmp_path / "mc.bam")
    synth.write_bam_fast(p, ["c%d" % i for i in range(len(lengths))], lengths, *arrs, level=1, n_threads=8)
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("window", [0, 1 << 20])
def test_gpu_extents_equal_the_index(lib_built, tmp_path, golden_dir, window):
    """A whole-file GPU decode's extents table (computed in the record walk)
    is the BAI's pseudo-bin data: the same first / end virtual offsets and
    mapped / unmapped counts as mc_bam_index_build writes, resident and
    windowed; its kept counts are the decoded records per contig."""
    from metacov_amd.bam import BamFile, GpuBamFile, build_index, index_extents
    import shutil
    paths = [_multi_contig_bam(tmp_path)]
    for name in ("bbmap.sorted.bam", "synth_multi.bam", "synth_edge.bam"):
        q = str(tmp_path / name)
        shutil.copy(os.path.join(golden_dir, name), q)
        paths.append(q)
    for p in paths:
        build_index(p)
        with GpuBamFile(p, window_bytes=window) as g:
            ext, nc = g.extents()
            want, wnc = index_extents(p + ".bai", len(g.references))
            for f in ("beg_voff", "end_voff", "n_mapped", "n_unmapped"):
                assert np.array_equal(ext[f], want[f]), (p, f)
            assert nc == wnc
            h = BamFile(p)
            assert np.array_equal(ext["n_kept"], np.bincount(h.tid, minlength=len(h.lengths)))


@pytest.mark.gpu
def test_gpu_decode_contig_shards(lib_built, tmp_path, golden_dir):
    """One rank's contigs decoded on the GPU, only their BGZF blocks read:
    through the BAI and through the extents of a whole-file decode, equal to
    the host's indexed decode (BamFile(contigs=...)) and to the oracle's
    reader restricted to those contigs, for first / last / scattered /
    neighbouring / empty / tiny selections; the engine holds just those
    contigs and reproduces the oracle's rows."""
    from metacov_amd.bam import BamFile, GpuBamFile, build_index
    from oracle import bamread, coracle
    import shutil
    p = _multi_contig_bam(tmp_path)
    q = str(tmp_path / "sm.bam")
    shutil.copy(os.path.join(golden_dir, "synth_multi.bam"), q)
    for path in (p, q):
        build_index(path)
        names, lens, counts, otid, opos, ospan = bamread.scan_intervals(path)
        n = len(names)
        with GpuBamFile(path) as whole:
            ext = whole.extents()
            sels = [[0], [n - 1], [0, n - 1], list(range(0, n, 3)), [1, 2], list(range(n)), [],
                    [3] if n > 3 else [0], [17 % n, 18 % n]]
            for sel in sels:
                h = BamFile(path, contigs=sel)
                keep = np.isin(otid, sel)
                for g in (GpuBamFile(path, contigs=sel), GpuBamFile(path, contigs=sel, extents=ext)):
                    with g:
                        t, ps, sp = g.intervals()
                        assert np.array_equal(t, otid[keep]) and np.array_equal(ps, opos[keep])
                        assert np.array_equal(sp, ospan[keep])
                        assert np.array_equal(t, h.tid) and np.array_equal(ps, h.pos)
                        assert (g.n_records, g.mapped, g.unmapped) == (h.n_records, h.mapped, h.unmapped)
                        assert g.references == h.references and g.lengths == h.lengths
                        if not len(sel):
                            continue
                        # the shard's engine against the oracle's exact rows
                        su = np.unique(sel)
                        rt = su.astype(np.int32)
                        rs = np.zeros(len(su), np.int64)
                        re_ = np.asarray(lens, np.int64)[su] + 5
                        d, e, c = coracle.depth(lens, otid, opos, ospan)
                        want = coracle.region_stats(d, e, c, rt, rs, re_)
                        got = g.engine(0, compute=False).compute_depth_stats(g.local_tid(rt), rs, re_)
                        for f in want.dtype.names:
                            assert np.array_equal(got[f], want[f]), f
            # bounded copies of chosen contigs from the whole-file decode
            sel = [1, n - 1]
            t, ps, sp = whole.intervals(sel)
            keep = np.isin(otid, sel)
            assert np.array_equal(t, otid[keep]) and np.array_equal(ps, opos[keep])
        # a whole-file decode restricted in place (rank 0 without an index)
        for sel in ([n - 1, 0], list(range(1, n, 2)), []):
            with GpuBamFile(path) as g:
                ext_before = g.extents()
                g.restrict(sel)
                keep = np.isin(otid, sel)
                t, ps, sp = g.intervals()
                assert np.array_equal(t, otid[keep]) and np.array_equal(ps, opos[keep])
                assert np.array_equal(sp, ospan[keep])
                ext_after, _ = g.extents()
                assert np.array_equal(ext_after["beg_voff"], ext_before[0]["beg_voff"])
                assert int(ext_after["n_kept"].sum()) == int(keep.sum()) == g.n_kept
                if len(sel):
                    su = np.unique(sel).astype(np.int32)
                    d, e, c = coracle.depth(lens, otid, opos, ospan)
                    rs = np.zeros(len(su), np.int64)
                    re_ = np.asarray(lens, np.int64)[su]
                    want = coracle.region_stats(d, e, c, su, rs, re_)
                    got = g.engine(0, compute=False).compute_depth_stats(g.local_tid(su), rs, re_)
                    assert all(np.array_equal(got[f], want[f]) for f in want.dtype.names)


@pytest.mark.gpu
def test_classic_path_decodes_on_the_gpu(lib_built, golden_dir, fixture_golden):
    """pileup.classic(path) — INTEGRATION.md's drop-in — opens the BAM with
    the GPU decoder and returns the real classic()'s goldens."""
    from metacov_amd import pileup
    from metacov_amd.bam import GpuBamFile
    path = os.path.join(golden_dir, "bbmap.sorted.bam")
    pileup.close_all()
    try:
        got = pileup.classic(path, "ref1", 1, 425)
        assert all(isinstance(f, GpuBamFile) for f in pileup._open_files.values())
        assert len(pileup._open_files) == 1
    finally:
        pileup.close_all()
    assert got == {"min": 7, "max": 526, "med": 344, "std": 134.03, "avg": 342.53, "q23": 353.25,
                   "sum": 145231}
