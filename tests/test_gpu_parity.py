"""GPU parity: the HIP path (through the C ABI) against the oracle and the
goldens.  Integer outputs must be bit-exact; region statistics are compared
as exact integer rows and as the classic() dicts of the real reference.

Run on an MI355X:  python -m pytest tests -m gpu
"""
import hashlib
import io
import os

import numpy as np
import pytest

from oracle import coracle
from metacov_amd import synth
from metacov_amd._lib import MetacovError, MC_E_INVALID
from metacov_amd.bam import BamFile
from metacov_amd.engine import CoverageEngine, classic_stats

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(lib_built):
    e = CoverageEngine(0)
    yield e
    e.close()


def _iv(g):
    return [np.array(g["intervals"][k], np.int32) for k in ("tid", "pos", "span")]


def run_engine(eng, lengths, tid, pos, span):
    eng.set_contigs(np.asarray(lengths, np.int64))
    eng.add_reads(tid, pos, span)
    eng.compute_depth()


def check_depth_vs_oracle(eng, lengths, tid, pos, span):
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    for t in range(len(lengths)):
        got = eng.depth(t, 0, int(ext[t]))
        assert np.array_equal(got, d[coff[t]:coff[t] + ext[t]]), "contig %d" % t
        assert eng.contig_offset(t)[1] == ext[t]
    return d, ext, coff


def check_regions_vs_oracle(eng, d, ext, coff, rtid, rs, re_):
    got = eng.region_stats(rtid, rs, re_)
    want = coracle.region_stats(d, ext, coff, rtid, rs, re_)
    for f in want.dtype.names:
        assert np.array_equal(got[f], want[f]), f
    return got


def random_regions(rng, lengths, k):
    rtid = rng.integers(0, len(lengths), size=k).astype(np.int32)
    rs = np.array([rng.integers(0, max(1, lengths[t] + 5)) for t in rtid], np.int64)
    re_ = rs + rng.integers(0, 3000, size=k)
    return rtid, rs, re_


# ------------------------------------------------------------- goldens

def test_fixture_depth_and_stats(eng, fixture_golden):
    tid, pos, span = _iv(fixture_golden)
    run_engine(eng, fixture_golden["lengths"], tid, pos, span)
    for t, gold in enumerate(fixture_golden["depth"]):
        assert eng.depth(t, 0, len(gold)).tolist() == gold
    assert eng.aligned_bases() == 340526
    regs = fixture_golden["blast7"] + fixture_golden["whole"]
    rows = eng.region_stats([fixture_golden["names"].index(r["sacc"]) for r in regs],
                            [r["start"] for r in regs], [r["end"] for r in regs])
    for row, r in zip(rows, regs):
        assert classic_stats(row) == r["stats"]


def test_stats_cases(eng, stats_golden):
    """Every golden stats vector as a one-contig depth built from reads."""
    for case in stats_golden:
        vec = np.array(case["depth"], np.int64)
        # reads of span 1 reproduce the vector exactly
        pos = np.repeat(np.arange(len(vec)), vec).astype(np.int32)
        tid = np.zeros(len(pos), np.int32)
        span = np.ones(len(pos), np.int32)
        run_engine(eng, [len(vec)], tid, pos, span)
        assert np.array_equal(eng.depth(0, 0, len(vec)), vec)
        row = eng.region_stats([0], [case["start"]], [case["end"]])[0]
        if "error" in case["stats"]:
            with pytest.raises(ValueError):
                classic_stats(row)
        else:
            assert classic_stats(row) == case["stats"], case["tag"]


@pytest.mark.parametrize("tag", ["synth_edge", "synth_multi"])
@pytest.mark.parametrize("legacy", [False, True])
def test_synth_bams(eng, synth_golden, golden_dir, tag, legacy):
    """Depth and the real classic()'s rows under both end rules (current
    htslib: a read without reference-consuming ops adds nothing; legacy
    bam_endpos: one column)."""
    g = synth_golden[tag]["legacy"] if legacy else synth_golden[tag]
    bf = BamFile(os.path.join(golden_dir, tag + ".bam"), legacy_endpos=legacy)
    run_engine(eng, bf.lengths, bf.tid, bf.pos, bf.span)
    for t in range(len(bf.lengths)):
        v = np.ascontiguousarray(eng.depth(t, 0, g["extents"][t]), dtype="<i4")
        assert hashlib.sha256(v.tobytes()).hexdigest() == g["depth_sha"][t]
        assert int(v.sum()) == g["depth_sum"][t]
    regs = g["regions"]
    rows = eng.region_stats([g["names"].index(r["sacc"]) for r in regs],
                            [r["start"] for r in regs], [r["end"] for r in regs])
    for row, r in zip(rows, regs):
        assert classic_stats(row) == r["stats"], r


@pytest.mark.parametrize("tag,legacy", [("synth_edge", False), ("synth_edge", True),
                                        ("synth_longcigar", False)])
def test_cigar_mode(eng, synth_golden, golden_dir, tag, legacy):
    """K1 (raw CIGAR words -> span on the GPU, CG-tag CIGARs included) against
    the oracle: the depth of the golden intervals, which the pure-Python BAM
    reader decoded with its own bam_cigar2rlen rule (oracle/bamread.py)."""
    g = synth_golden[tag]["legacy"] if legacy else synth_golden[tag]
    bf = BamFile(os.path.join(golden_dir, tag + ".bam"), keep_cigar=True)
    lengths = np.asarray(bf.lengths, np.int64)
    eng.set_legacy_endpos(legacy)
    eng.set_contigs(lengths)
    eng.add_reads_cigar(bf.tid, bf.pos, bf.cig_off, bf.cigar)
    eng.compute_depth()
    tid, pos, span = [np.array(g["intervals"][k], np.int32) for k in ("tid", "pos", "span")]
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    for t in range(len(lengths)):
        assert np.array_equal(eng.depth(t, 0, int(ext[t])), d[coff[t]:coff[t] + ext[t]]), t
    assert eng.aligned_bases() == int(span.astype(np.int64).sum())


# ------------------------------------------------------------- oracle parity

CASES = {
    # name: (lengths, n_reads, span range, seed)
    "one_contig": ([300_000], 20_000, (1, 200), 1),
    "tiny_contigs": ([0, 1, 2, 63, 64, 65, 4095, 4096, 4097, 65535, 65536, 65537], 3_000, (1, 30), 2),
    "chunk_edges": ([65536 * 3 + 17, 4096 * 5], 40_000, (1, 9000), 3),
    "long_spans": ([400_000, 90_000], 6_000, (20_000, 28_600), 4),
    "many_contigs": (list(range(1, 2000, 7)), 50_000, (1, 150), 5),
    "mixed_long": ([500_000, 200_000, 70_000, 3], 20_000, (1, 150_000), 6),
    "just_over_ring": ([300_000], 30_000, (4090, 4100), 8),
}


def test_ont_like_long_reads(eng):
    """C5 shape in miniature: lognormal ~10 kbp reads over many contigs."""
    rng = np.random.default_rng(21)
    lengths = rng.integers(50_000, 150_001, size=40).astype(np.int64)
    lengths, tid, pos, span = make_case(lengths, 30_000, (1, 2), 22)
    span = np.minimum(rng.lognormal(np.log(10_000), 0.5, size=len(tid)).astype(np.int64),
                      lengths[tid]).astype(np.int32)
    pos = (rng.random(len(tid)) * (lengths[tid] - span + 1)).astype(np.int32)
    o = np.lexsort((pos, tid))
    tid, pos, span = tid[o], pos[o], span[o]
    run_engine(eng, lengths, tid, pos, span)
    d, ext, coff = check_depth_vs_oracle(eng, lengths, tid, pos, span)
    rtid, rs, re_ = random_regions(np.random.default_rng(8), lengths, 200)
    check_regions_vs_oracle(eng, d, ext, coff, rtid, rs, re_)


def _long_batch(lengths, n, seed, extra_far=False):
    rng = np.random.default_rng(seed)
    tid = np.sort(rng.integers(0, len(lengths), size=n)).astype(np.int32)
    span = np.minimum(rng.lognormal(np.log(10_000), 0.6, size=n).astype(np.int64), lengths[tid]).astype(np.int32)
    if extra_far:   # ends far past their start tile (outside ingest's 64-tile window) and one overhang
        span[:50] = np.minimum(300_000, lengths[tid[:50]]).astype(np.int32)
    pos = (rng.random(n) * (lengths[tid] - span + 1)).astype(np.int32)
    if extra_far:
        k = n // 2
        pos[k] = lengths[tid[k]] - 100
        span[k] = 5000                     # runs 4900 past its contig: the extents grow (second pass)
    o = np.lexsort((pos, tid))
    return tid[o], pos[o], span[o]


def test_long_counts_folded_into_ingest(lib_built):
    """Batches after one with long reads count the end events and chunk
    carries inside ingest (long_count_kernel's pass folded in): exact depth
    and rows for a following long batch (ends outside the LDS window, an
    overhang that re-runs the pass), a short-only batch, and long again."""
    rng = np.random.default_rng(91)
    lengths = rng.integers(60_000, 400_000, size=30).astype(np.int64)
    rt = np.arange(len(lengths), dtype=np.int32)
    rs = np.zeros(len(lengths), np.int64)
    e = CoverageEngine(0)
    try:
        e.set_contigs(lengths)
        batches = [_long_batch(lengths, 40_000, 1), _long_batch(lengths, 30_000, 2, extra_far=True),
                   make_case(lengths, 50_000, (1, 150), 3, overhang=False)[1:],
                   _long_batch(lengths, 20_000, 4)]
        for k, (tid, pos, span) in enumerate(batches):
            e.clear_reads()
            e.add_reads(tid, pos, span)
            d, ext, coff = coracle.depth(lengths, tid, pos, span)
            re_ = np.asarray(ext, np.int64)
            want = coracle.region_stats(d, ext, coff, rt, rs, re_)
            got = e.compute_depth_stats(rt, rs, re_)
            for f in want.dtype.names:
                assert np.array_equal(got[f], want[f]), (k, f)
            check_depth_vs_oracle(e, lengths, tid, pos, span)
    finally:
        e.close()


def make_case(lengths, n, span_rng, seed, overhang=True):
    rng = np.random.default_rng(seed)
    lengths = np.asarray(lengths, np.int64)
    live = np.nonzero(lengths > 0)[0]
    tid = rng.choice(live, size=n).astype(np.int32)
    pos = (rng.random(n) * lengths[tid]).astype(np.int32)
    span = rng.integers(span_rng[0], span_rng[1] + 1, size=n).astype(np.int32)
    if not overhang:
        span = np.minimum(span, (lengths[tid] - pos)).astype(np.int32)
    o = np.lexsort((pos, tid))
    return lengths, tid[o], pos[o], span[o]


@pytest.mark.parametrize("name", sorted(CASES))
def test_random_vs_oracle(eng, name):
    lengths, tid, pos, span = make_case(*CASES[name])
    run_engine(eng, lengths, tid, pos, span)
    d, ext, coff = check_depth_vs_oracle(eng, lengths, tid, pos, span)
    assert eng.aligned_bases() == int(span.astype(np.int64).sum()) == int(d.sum())
    assert eng.max_depth() == int(d.max())
    rtid, rs, re_ = random_regions(np.random.default_rng(7), lengths, 300)
    whole_t = np.arange(len(lengths), dtype=np.int32)
    check_regions_vs_oracle(eng, d, ext, coff, np.concatenate([rtid, whole_t]),
                            np.concatenate([rs, np.zeros(len(lengths), np.int64)]),
                            np.concatenate([re_, lengths]))


def test_empty_and_single(eng):
    run_engine(eng, [1000, 5], np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.int32))
    assert eng.depth(0).sum() == 0 and eng.max_depth() == 0
    row = eng.region_stats([0], [10], [20])[0]
    assert classic_stats(row) == {"min": 0, "max": 0, "med": 0, "std": 0.0, "avg": 0.0,
                                  "q23": 0.0, "sum": 0}
    run_engine(eng, [1000], np.zeros(1, np.int32), np.array([998], np.int32), np.array([5], np.int32))
    d = eng.depth(0, 0, 1005)
    assert d[998:1003].tolist() == [1] * 5 and d.sum() == 5
    assert eng.contig_offset(0)[1] == 1003          # read runs past the end


def test_high_depth_histogram_paths(eng):
    # LDS histogram (<= 16384 bins) and the global-histogram path beyond
    for depth_target in (5_000, 20_000):
        n = depth_target
        tid = np.zeros(n, np.int32)
        pos = np.sort(np.random.default_rng(depth_target).integers(0, 50, size=n)).astype(np.int32)
        span = np.full(n, 100, np.int32)
        lengths = [1000]
        run_engine(eng, lengths, tid, pos, span)
        d, ext, coff = check_depth_vs_oracle(eng, lengths, tid, pos, span)
        check_regions_vs_oracle(eng, d, ext, coff, np.array([0, 0], np.int32),
                                np.array([0, 40], np.int64), np.array([1000, 300], np.int64))


def test_append_equals_single(eng):
    lengths, tid, pos, span = make_case([200_000, 7000], 30_000, (1, 300), 11)
    run_engine(eng, lengths, tid, pos, span)
    a = [eng.depth(t) for t in range(2)]
    eng.set_contigs(lengths)
    for part in np.array_split(np.arange(len(tid)), 3):
        eng.add_reads(tid[part], pos[part], span[part])
    eng.compute_depth()
    eng.compute_depth()          # idempotent
    for t in range(2):
        assert np.array_equal(a[t], eng.depth(t))


def test_device_tensor_input(eng):
    import torch
    lengths, tid, pos, span = make_case([100_000], 10_000, (1, 150), 12)
    eng.set_contigs(lengths)
    eng.add_reads(*(torch.from_numpy(x).cuda() for x in (tid, pos, span)))
    eng.compute_depth()
    d, _, _ = coracle.depth(lengths, tid, pos, span)
    assert np.array_equal(eng.depth(0, 0, len(d)), d)


def test_errors(eng):
    eng.set_contigs([100])
    eng.add_reads(np.array([0, 0], np.int32), np.array([5, 3], np.int32), np.array([1, 1], np.int32))
    with pytest.raises(MetacovError) as ei:
        eng.compute_depth()
    assert ei.value.code == MC_E_INVALID and "sorted" in str(ei.value)
    eng.set_contigs([100])
    eng.add_reads(np.array([1], np.int32), np.array([5], np.int32), np.array([1], np.int32))
    with pytest.raises(MetacovError):
        eng.compute_depth()
    eng.add_reads(np.array([0], np.int32), np.array([-5], np.int32), np.array([4], np.int32))
    with pytest.raises(MetacovError):
        eng.compute_depth()
    eng.set_contigs([100])
    eng.add_reads(np.array([0], np.int32), np.array([5], np.int32), np.array([3], np.int32))
    eng.compute_depth()
    with pytest.raises(MetacovError):
        eng.region_stats([0], [10], [5])
    with pytest.raises(MetacovError):
        eng.region_stats([3], [0], [5])


# ------------------------------------------------------------- full size

def test_c2_full_size(eng):
    """BASELINE config 2: 1 contig x 5 Mbp, 10M x 150 bp: bit-exact depth."""
    tid, pos, span = synth.interval_workload([5_000_000], 10_000_000, seed=1)
    lengths = [5_000_000]
    run_engine(eng, lengths, tid, pos, span)
    d, ext, coff = check_depth_vs_oracle(eng, lengths, tid, pos, span)
    assert eng.aligned_bases() == int(d.sum())
    check_regions_vs_oracle(eng, d, ext, coff, np.zeros(3, np.int32),
                            np.array([0, 1_000_000, 4_999_000], np.int64),
                            np.array([5_000_000, 3_000_001, 5_000_100], np.int64))


def test_c3_shape_properties(eng):
    """C3 shape (1000 contigs, ~1 Gbp, lognormal abundance) at 20M reads:
    depth bit-exact vs the oracle; every whole-contig stat row exact."""
    lengths, weights = synth.c3_workload()
    tid, pos, span = synth.interval_workload(lengths, 20_000_000, seed=3, weights=weights)
    run_engine(eng, lengths, tid, pos, span)
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    ptr_, total = eng.depth_device()
    got = np.concatenate([eng.depth(t, 0, int(ext[t])) for t in range(len(lengths))])
    want = np.concatenate([d[coff[t]:coff[t] + ext[t]] for t in range(len(lengths))])
    assert np.array_equal(got, want)
    check_regions_vs_oracle(eng, d, ext, coff, np.arange(len(lengths), dtype=np.int32),
                            np.zeros(len(lengths), np.int64), lengths)


# ------------------------------------------------------------- drop-in API

def test_classic_api(lib_built, fixture_golden, golden_dir):
    from metacov_amd import pileup
    path = os.path.join(golden_dir, "bbmap.sorted.bam")
    for r in fixture_golden["blast7"] + fixture_golden["whole"]:
        assert pileup.classic(path, r["sacc"], r["start"], r["end"]) == r["stats"]
    with pytest.raises(KeyError):
        pileup.classic(path, "nope", 0, 10)
    with pytest.raises(ValueError):
        pileup.classic(path, "ref1", 5, 5)
    assert pileup.depth(path, "ref1").tolist() == fixture_golden["depth"][0]


@pytest.mark.parametrize("mode", ["blast7", "whole"])
@pytest.mark.parametrize("decode", ["gpu", "host"])
def test_cli_csv_bytes(lib_built, fixture_golden, golden_dir, tmp_path, mode, decode):
    from click.testing import CliRunner
    from metacov_amd.cli import pileup as cli_pileup
    args = ["-b", os.path.join(golden_dir, "bbmap.sorted.bam"), "-o", str(tmp_path / "o.csv"),
            "--decode", decode]
    if mode == "blast7":
        args += ["-rb", os.path.join(golden_dir, "regions.blast7")]
    res = CliRunner().invoke(cli_pileup, args)
    assert res.exit_code == 0, res.output
    with open(tmp_path / "o.csv", newline="") as fh:
        assert fh.read() == fixture_golden["csv_" + mode]


def test_long_read_ends_on_chunk_and_tile_starts(eng):
    lengths = [200_000]
    pos = np.array([100, 5000, 60_000, 61_440], np.int32)
    span = np.array([65436, 60536, 5536, 69632], np.int32)
    o = np.argsort(pos)
    tid = np.zeros(4, np.int32)
    run_engine(eng, lengths, tid, pos[o], span[o])
    check_depth_vs_oracle(eng, lengths, tid, pos[o], span[o])


def test_read_words_alias_masked(eng):
    # K2's read words keep 18 start bits: a read 262,044 positions before a
    # chunk start decodes to chunk position 100.  Each group of 4 reads puts
    # such a read A in the same aligned batch slot as the chunk's first read B
    # (A at an index = 0 mod 4, B right after it), so A is loaded for B's chunk
    # and for every empty chunk between them, and only the mask before the
    # chunk's first read keeps it out.  B sits 50 past a multiple of 32768, so
    # this holds for 2-, 4- and 8-tile chunks.
    pos = []
    for k in range(6):
        b = (k * 12 + 10) * 32768 + 50
        pos += [b - 50 - 262_044, b, b + 10, b + 20]
    pos = np.array(pos, np.int32)
    span = np.full(len(pos), 150, np.int32)
    lengths = [int(pos[-1]) + 10_000]
    tid = np.zeros(len(pos), np.int32)
    run_engine(eng, lengths, tid, pos, span)
    d, ext, coff = check_depth_vs_oracle(eng, lengths, tid, pos, span)
    eng.set_contigs(lengths)
    eng.add_reads(tid, pos, span)
    got = eng.compute_depth_stats(np.zeros(1, np.int32), np.zeros(1, np.int64),
                                  np.asarray(lengths, np.int64))
    want = coracle.region_stats(d, ext, coff, np.zeros(1, np.int32), np.zeros(1, np.int64),
                                np.asarray(lengths, np.int64))
    for f in want.dtype.names:
        assert np.array_equal(got[f], want[f]), f


# ------------------------------------------------------------- fused K2 + stats

def _tiling(rng, lengths, pieces):
    rt, rs, re_ = [], [], []
    for t, L in enumerate(lengths):
        cuts = np.sort(rng.integers(0, L + 1, size=pieces))
        edges = np.concatenate([[0], cuts, [L + 37]])
        for a, b in zip(edges[:-1], edges[1:]):
            rt.append(t)
            rs.append(a)
            re_.append(b)
    o = rng.permutation(len(rt))      # any input order
    return (np.array(rt, np.int32)[o], np.array(rs, np.int64)[o], np.array(re_, np.int64)[o])


@pytest.mark.parametrize("name", ["one_contig", "many_contigs", "mixed_long", "chunk_edges",
                                  "tiny_contigs"])
def test_fused_stats_vs_oracle(eng, name):
    lengths, tid, pos, span = make_case(*CASES[name])
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    rng = np.random.default_rng(31)
    for rt, rs, re_ in [(np.arange(len(lengths), dtype=np.int32), np.zeros(len(lengths), np.int64),
                         np.asarray(lengths, np.int64)),
                        _tiling(rng, lengths, 7)]:
        eng.set_contigs(lengths)
        eng.add_reads(tid, pos, span)
        got = eng.compute_depth_stats(rt, rs, re_)
        want = coracle.region_stats(d, ext, coff, rt, rs, re_)
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), f
        for t in range(len(lengths)):
            assert np.array_equal(eng.depth(t, 0, int(ext[t])), d[coff[t]:coff[t] + ext[t]])


def test_fused_overlapping_and_high_depth(eng):
    # overlapping regions -> K2 + K3 path; depth > 1024 -> exact fallback
    n = 3000
    tid = np.zeros(n, np.int32)
    pos = np.sort(np.random.default_rng(3).integers(0, 40, size=n)).astype(np.int32)
    span = np.full(n, 100, np.int32)
    lengths = [5000]
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    cases = [
        (np.array([0, 0], np.int32), np.array([0, 10], np.int64), np.array([200, 300], np.int64)),
        (np.array([0], np.int32), np.array([0], np.int64), np.array([120], np.int64)),
        (np.array([0, 0], np.int32), np.array([0, 4000], np.int64), np.array([4000, 5000], np.int64)),
    ]
    for k, (rt, rs, re_) in enumerate(cases):
        eng.set_contigs(lengths)
        eng.add_reads(tid, pos, span)
        got = eng.compute_depth_stats(rt, rs, re_)
        want = coracle.region_stats(d, ext, coff, rt, rs, re_)
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), f
        if k == 1:      # median of [0,120) is > 1024: recomputed (device or host K3)
            assert eng.fused_fallbacks() + eng.fused_recomputes() == 1
        if k == 2:
            assert eng.fused_fallbacks() + eng.fused_recomputes() == 0


def test_fused_fixture_goldens(eng, fixture_golden):
    tid, pos, span = _iv(fixture_golden)
    regs = fixture_golden["whole"]
    eng.set_contigs(fixture_golden["lengths"])
    eng.add_reads(tid, pos, span)
    rows = eng.compute_depth_stats([fixture_golden["names"].index(r["sacc"]) for r in regs],
                                   [r["start"] for r in regs], [r["end"] for r in regs])
    for row, r in zip(rows, regs):
        assert classic_stats(row) == r["stats"]


def test_fused_window_follows_mean_depth(eng):
    """Depth ~5000 everywhere: the fused histogram window is centred on the
    contig's mean, so no region needs the fallback and rows stay exact."""
    rng = np.random.default_rng(41)
    L = 120_000
    n = 4_000_000
    pos = np.sort(rng.integers(0, L - 150, size=n)).astype(np.int32)
    tid = np.zeros(n, np.int32)
    span = np.full(n, 150, np.int32)
    d, ext, coff = coracle.depth([L], tid, pos, span)
    rt = np.zeros(3, np.int32)
    rs = np.array([0, 1000, 60_000], np.int64)
    re_ = np.array([1000, 60_000, L + 10], np.int64)
    eng.set_contigs([L])
    eng.add_reads(tid, pos, span)
    got = eng.compute_depth_stats(rt, rs, re_)
    want = coracle.region_stats(d, ext, coff, rt, rs, re_)
    for f in want.dtype.names:
        assert np.array_equal(got[f], want[f]), f
    assert eng.fused_fallbacks() == 0


def test_cli_csv_regions_and_batch_api(lib_built, fixture_golden, golden_dir, tmp_path):
    """-rc CSV regions (values stay strings, util.py:61) and classic_batch."""
    from click.testing import CliRunner
    from metacov_amd.cli import pileup as cli_pileup
    from metacov_amd import pileup
    bam = os.path.join(golden_dir, "bbmap.sorted.bam")
    rc = tmp_path / "r.csv"
    rc.write_text("sequence_id,start,stop\nref1,1,425\nref2,575,1\n")
    res = CliRunner().invoke(cli_pileup, ["-b", bam, "-rc", str(rc), "-o", str(tmp_path / "o.csv")])
    assert res.exit_code == 0, res.output
    lines = open(tmp_path / "o.csv", newline="").read().split("\r\n")
    b7 = {(r["sacc"], r["start"], r["end"]): r["stats"] for r in fixture_golden["blast7"]}
    s = b7[("ref1", 1, 425)]
    assert lines[1] == "ref1,1,425,%r,%d,%d,%d,%r,%r,%d" % (s["avg"], s["max"], s["med"], s["min"],
                                                             s["q23"], s["std"], s["sum"])
    assert lines[2].startswith("ref2,575,1,")          # raw (unsorted) start/end echoed
    regs = [("ref1", 1, 425), ("ref2", 1, 575), ("ref2", 1, 300), ("ref2", 301, 575)]
    got = pileup.classic_batch(bam, regs)
    assert got == [b7[r] for r in regs]
    with pytest.raises(KeyError):
        pileup.classic_batch(bam, [("nope", 0, 5)])


def test_external_stream(lib_built):
    """mc_ctx_set_stream: the ctx runs on torch's current stream."""
    import torch
    eng = CoverageEngine(0)
    s = torch.cuda.Stream()
    eng.set_stream(s.cuda_stream)
    lengths, tid, pos, span = make_case([70_000], 5_000, (1, 150), 13)
    run_engine(eng, lengths, tid, pos, span)
    d, _, _ = coracle.depth(lengths, tid, pos, span)
    assert np.array_equal(eng.depth(0, 0, len(d)), d)
    eng.set_stream(None)
    eng.compute_depth()
    assert np.array_equal(eng.depth(0, 0, len(d)), d)
    eng.close()


@pytest.mark.parametrize("decode,indexed", [("gpu", True), ("gpu", False), ("host", True)])
def test_cli_two_ranks(lib_built, golden_dir, tmp_path, decode, indexed):
    """`metacov pileup` on 2 ranks (torch.distributed.run, contig shards,
    region-table all-gather; gloo so both ranks can share the box's one GPU)
    writes byte-for-byte the CSV built from the oracle alone (bamread +
    coracle) and the CSV of one process.  --decode gpu: each rank decodes
    only its contigs' BGZF blocks on the GPU, located by the BAI, or without
    one by the extents table of rank 0's whole-file GPU decode."""
    import shutil
    import socket
    import subprocess
    import sys
    from click.testing import CliRunner
    from metacov_amd.bam import build_index
    from metacov_amd.cli import pileup as cli_pileup
    from tests.oracle_csv import oracle_csv
    bam = str(tmp_path / "m.bam")
    shutil.copy(os.path.join(golden_dir, "synth_multi.bam"), bam)
    if indexed:
        build_index(bam)
    regs = [("contig_5", "100", "39000"), ("contig_0", "0", "5000"), ("contig_6", "7000", "10"),
            ("contig_2", "5", "6"), ("contig_3", "0", "1"), ("contig_5", "0", "40000"),
            ("contig_1", "0", "300"), ("contig_4", "3", "2000"), ("contig_4", "0", "20000")]
    rc = tmp_path / "r.csv"
    rc.write_text("sequence_id,start,stop\n" + "".join("%s,%s,%s\n" % r for r in regs))
    want = oracle_csv(bam, regs)
    one = tmp_path / "one.csv"
    res = CliRunner().invoke(cli_pileup, ["-b", bam, "-rc", str(rc), "-o", str(one), "--decode", decode])
    assert res.exit_code == 0, res.output
    assert open(one, newline="").read() == want
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    two = tmp_path / "two.csv"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MC_DIST_BACKEND="gloo",
               PYTHONPATH=os.pathsep.join([root, os.environ.get("PYTHONPATH", "")]))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=%d" % port, "-m", "metacov_amd.cli", "pileup",
           "-b", bam, "-rc", str(rc), "-o", str(two), "--decode", decode]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    assert open(two, newline="").read() == want


def test_cigar_device_batches(lib_built):
    """Raw-CIGAR batches from device memory (borrowed cig_off / cigar, K1 in
    prepare), cleared and re-added: depth and region rows equal the
    interval path's and the oracle's."""
    import torch
    lengths, tid, pos, span = make_case([60_000, 7, 25_000, 9_000], 4_000, (1, 12_000), 21)
    dev = torch.device("cuda", 0)
    t_span = torch.from_numpy(span).to(dev)
    cig_off, cigar = synth.device_cigars(torch, t_span, mean_ops=30, seed=3, batch_reads=1_000)
    t_tid, t_pos = torch.from_numpy(tid).to(dev), torch.from_numpy(pos).to(dev)
    a = CoverageEngine(0)
    a.set_contigs(lengths)
    b = CoverageEngine(0)
    b.set_contigs(lengths)
    b.add_reads(tid, pos, span)
    rt = np.array([0, 2, 3, 0], np.int32)
    rs = np.array([0, 100, 0, 59_000], np.int64)
    re_ = np.array([60_000, 24_000, 9_000, 61_000], np.int64)
    want = b.compute_depth_stats(rt, rs, re_)
    for _ in range(2):
        a.clear_reads()
        a.add_reads_cigar_device(t_tid, t_pos, cig_off, cigar)
        got = a.compute_depth_stats(rt, rs, re_)
        assert a.timings()["cigar_ms"] > 0
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), f
        for t in range(len(lengths)):
            assert np.array_equal(a.depth(t), b.depth(t))
    check_depth_vs_oracle(a, lengths, tid, pos, span)
    with pytest.raises(MetacovError):
        a.add_reads_cigar_device(t_tid, t_pos, cig_off, cigar)   # reads already present
    # int64 tid/pos: the int32 casts are temporaries freed when the call
    # returns; the caching allocator hands their memory straight to the
    # scribble below, on torch's stream, so a pending copy would read garbage
    a.clear_reads()
    a.add_reads_cigar_device(t_tid.to(torch.int64), t_pos.to(torch.int64), cig_off, cigar)
    scribble = torch.full((2 * len(tid),), -7, dtype=torch.int32, device=dev)
    got = a.compute_depth_stats(rt, rs, re_)
    for f in want.dtype.names:
        assert np.array_equal(got[f], want[f]), f
    del scribble
    a.close()
    b.close()


def test_streamed_ingest_and_cli(lib_built, golden_dir, tmp_path):
    """StreamedBam (windowed decode, pinned double-buffered async H2D) gives
    the rows of the whole-file decode; the CLI's --stream CSV is identical."""
    from click.testing import CliRunner
    from metacov_amd.bam import StreamedBam
    from metacov_amd.cli import pileup as cli_pileup
    lengths = [1_500_000, 800, 600_000]
    arrs = synth.edge_mix_arrays(lengths, 400_000, seed=8)
    p = str(tmp_path / "s.bam")
    synth.write_bam_fast(p, ["a", "b", "c"], lengths, *arrs, level=1, n_threads=4)
    full = BamFile(p)
    sb = StreamedBam(p, batch_reads=50_000, window_bytes=1 << 20)
    assert (sb.mapped, sb.unmapped) == (full.mapped, full.unmapped)
    rt = np.array([0, 2, 1, 0], np.int32)
    rs = np.array([0, 10, 0, 999_000], np.int64)
    re_ = np.array([1_500_000, 600_000, 900, 1_600_000], np.int64)
    a = full.engine(0, compute=False).compute_depth_stats(rt, rs, re_)
    b = sb.engine(0, compute=False).compute_depth_stats(rt, rs, re_)
    for f in a.dtype.names:
        assert np.array_equal(a[f], b[f]), f
    sb.close()
    full.close()
    outs = []
    for flag in ("--stream", "--no-stream"):
        o = tmp_path / ("o%s.csv" % flag)
        res = CliRunner().invoke(cli_pileup, ["-b", os.path.join(golden_dir, "synth_multi.bam"),
                                              flag, "-o", str(o)])
        assert res.exit_code == 0, res.output
        outs.append(open(o, newline="").read())
    assert outs[0] == outs[1] and outs[0].count("\n") == 8


def test_fused_repeated_calls_reuse_and_invalidate(eng):
    """A repeated fused call with the same regions reuses the staged region
    arrays; other regions, or new reads (a new prepare), restage them."""
    lengths, tid, pos, span = make_case([60_000, 90_000, 30_000], 30_000, (1, 300), 17)
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    whole = (np.arange(3, dtype=np.int32), np.zeros(3, np.int64), np.asarray(lengths, np.int64))
    tiles = _tiling(np.random.default_rng(5), lengths, 9)
    eng.set_contigs(lengths)
    eng.add_reads(tid, pos, span)

    def check(regs, d, ext, coff):
        got = eng.compute_depth_stats(*regs)
        want = coracle.region_stats(d, ext, coff, *regs)
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), f

    for regs in (whole, whole, tiles, tiles, whole):
        check(regs, d, ext, coff)
    # new reads: the staged window bases (per-contig mean depth) change
    lengths2, tid2, pos2, span2 = make_case([60_000, 90_000, 30_000], 90_000, (1, 300), 18)
    d2, ext2, coff2 = coracle.depth(lengths2, tid2, pos2, span2)
    eng.set_contigs(lengths2)
    eng.add_reads(tid2, pos2, span2)
    check(whole, d2, ext2, coff2)
    check(whole, d2, ext2, coff2)


def test_engines_on_two_threads(lib_built):
    """Two contexts driven from two host threads at once (their own streams
    and buffers; the calls release the GIL), each over a different batch
    with the direct step repeated (invalidate + fused call): every row equals
    the oracle's (scripts/bench_streams.py measures what it buys)."""
    import threading
    from metacov_amd.engine import CoverageEngine
    cases = [make_case([80_000, 50_000, 120_000], 60_000, (1, 300), 31),
             make_case([200_000, 7_000], 90_000, (1, 700), 32)]
    engines, wants, regs = [], [], []
    for lengths, tid, pos, span in cases:
        e = CoverageEngine(0)
        e.set_contigs(lengths)
        e.add_reads(tid, pos, span)
        engines.append(e)
        d, ext, coff = coracle.depth(lengths, tid, pos, span)
        r = _tiling(np.random.default_rng(len(lengths)), lengths, 7)
        regs.append(r)
        wants.append(coracle.region_stats(d, ext, coff, *r))
    got = [[], []]
    errors = []

    def loop(i):
        try:
            for _ in range(12):
                engines[i].invalidate()
                got[i].append(engines[i].compute_depth_stats(*regs[i]))
        except Exception as ex:   # noqa: BLE001 (reported below)
            errors.append(ex)

    ths = [threading.Thread(target=loop, args=(i,)) for i in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    for i in range(2):
        assert len(got[i]) == 12
        for g in got[i]:
            for f in wants[i].dtype.names:
                assert np.array_equal(g[f], wants[i][f]), (i, f)


def test_fused_timing_totals(eng):
    """mc_timings.fused_*_total: each fused call adds its K2 and K3b event
    times (what bench.py averages over the timed steps)."""
    lengths, tid, pos, span = make_case([60_000, 90_000], 20_000, (1, 300), 23)
    regs = (np.arange(2, dtype=np.int32), np.zeros(2, np.int64), np.asarray(lengths, np.int64))
    eng.set_contigs(lengths)
    eng.add_reads(tid, pos, span)
    t0 = eng.timings()
    for _ in range(3):
        eng.compute_depth_stats(*regs)
    t1 = eng.timings()
    assert t1["fused_calls"] - t0["fused_calls"] == 3
    dk2 = t1["fused_depth_ms_total"] - t0["fused_depth_ms_total"]
    dk3 = t1["fused_stats_ms_total"] - t0["fused_stats_ms_total"]
    assert dk2 > 0 and dk3 > 0
    assert dk2 >= t1["depth_ms"] * 0.99   # three launches, the last one among them


@pytest.fixture
def eng_checked(lib_built, monkeypatch):
    """An engine that verifies every skipped fused_init on the device
    (MC_CHECK_CLEAN=1, read at mc_ctx_create): a stale buffer is MC_E_STATE."""
    monkeypatch.setenv("MC_CHECK_CLEAN", "1")
    e = CoverageEngine(0)
    yield e
    e.close()


def test_fused_clean_buffers_across_mixed_calls(eng_checked):
    """K3b leaves the fused buffers initialised for the next call on the same
    regions (no init launch); a plain K2, a K3 pass, a fallback or a
    re-prepare in between must not leave stale queue / histogram state.  The
    engine also checks on the device, before each clean call, that every
    buffer the skipped init would write holds its initial value."""
    eng = eng_checked
    lengths, tid, pos, span = make_case([60_000, 90_000, 30_000], 30_000, (1, 300), 31)
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    whole = (np.arange(3, dtype=np.int32), np.zeros(3, np.int64), np.asarray(lengths, np.int64))
    want = coracle.region_stats(d, ext, coff, *whole)
    eng.set_contigs(lengths)
    eng.add_reads(tid, pos, span)

    def fused():
        got = eng.compute_depth_stats(*whole)
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), f

    def plain():
        eng.compute_depth()
        got = eng.region_stats(*whole)
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), f
        assert np.array_equal(eng.depth(1), d[coff[1]:coff[1] + lengths[1]])

    for step in (fused, fused, fused, plain, fused, fused, plain, plain, fused):
        step()
    eng.invalidate()      # re-prepare the same reads: restaged regions, init again
    fused()
    fused()
    # a region set with a fallback (a contig whose depth ramps from 4000 to 0:
    # its quartile ranks span far more values than the histogram window)
    lt = np.zeros(4000, np.int32)
    lp = np.zeros(4000, np.int32)
    ls = np.random.default_rng(3).integers(1, 5001, 4000).astype(np.int32)
    t2 = np.concatenate([tid, lt + 3])
    o = np.lexsort((np.concatenate([pos, lp]), t2))
    lengths2 = np.array(list(lengths) + [5_000], np.int64)
    t2, p2, s2 = t2[o], np.concatenate([pos, lp])[o], np.concatenate([span, ls])[o]
    eng.set_contigs(lengths2)
    eng.add_reads(t2, p2, s2)
    d2, ext2, coff2 = coracle.depth(lengths2, t2, p2, s2)
    regs2 = (np.arange(4, dtype=np.int32), np.zeros(4, np.int64), lengths2)
    want2 = coracle.region_stats(d2, ext2, coff2, *regs2)
    for k in range(3):
        got = eng.compute_depth_stats(*regs2)
        for f in want2.dtype.names:
            assert np.array_equal(got[f], want2[f]), f
        assert eng.fused_fallbacks() + eng.fused_recomputes() >= 1
        if k:           # after a call with out-of-window regions: recomputed on the device
            assert eng.fused_recomputes() >= 1 and eng.fused_fallbacks() == 0


def test_invalidate_reprepares_same_reads(eng):
    """mc_invalidate drops the prepared index; the next compute call
    re-prepares the same device reads and gives the same results."""
    lengths, tid, pos, span = make_case([70_000, 40_000], 20_000, (1, 400), 37)
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    regs = (np.arange(2, dtype=np.int32), np.zeros(2, np.int64), np.asarray(lengths, np.int64))
    want = coracle.region_stats(d, ext, coff, *regs)
    eng.set_contigs(lengths)
    eng.add_reads(tid, pos, span)
    for _ in range(3):
        eng.invalidate()
        got = eng.compute_depth_stats(*regs)
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), f
    assert eng.aligned_bases() == int(span.astype(np.int64).sum())


def test_long_reads_reprepare_end_words(eng):
    """Long reads through the full prepare, three times: the first pass counts
    the end events with long_count_kernel and fills the buckets from the
    tuples; later passes (the contig set had long reads) count inside ingest
    and fill from ingest's per-read end words.  Depth and rows equal the
    oracle's every time, including ends on chunk starts and past the extents."""
    lengths = [500_000, 300_000, 7, 131_072]
    rng = np.random.default_rng(91)
    n = 200_000
    t = np.sort(rng.choice(4, size=n, p=[0.5, 0.3, 0.0, 0.2])).astype(np.int32)
    span = rng.integers(4_000, 30_000, size=n)
    L = np.asarray(lengths)[t]
    pos = (rng.random(n) * (L + 1000)).astype(np.int64)          # some run past their contig
    pos = np.minimum(pos, L - 1)
    span[::97] = (32768 - pos[::97] % 32768)                    # ends exactly on chunk starts
    span = np.maximum(span, 1).astype(np.int32)
    pos = pos.astype(np.int32)
    o = np.lexsort((pos, t))
    t, pos, span = t[o], pos[o], span[o]
    d, ext, coff = coracle.depth(lengths, t, pos, span)
    regs = (np.arange(4, dtype=np.int32), np.zeros(4, np.int64), np.asarray(lengths, np.int64) + 500)
    want = coracle.region_stats(d, ext, coff, *regs)
    eng.set_contigs(lengths)
    eng.add_reads(t, pos, span)
    for k in range(3):
        eng.invalidate()
        got = eng.compute_depth_stats(*regs)
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), (k, f)
        for c in range(4):
            assert np.array_equal(eng.depth(c, 0, int(ext[c])), d[coff[c]:coff[c] + ext[c]]), (k, c)


def test_new_batch_same_layout_moves_windows(eng):
    """A second batch over the same contigs and regions keeps the staged
    region table (same layout) but must move the histogram windows to the
    new depth: a shallow batch, then one ~3000 deep, then shallow again, each
    exact and without fallbacks (a window left at the first batch's depth
    would send every deep region to the K3 fallback)."""
    lengths = [60_000, 45_000]
    regs = (np.array([0, 1, 0], np.int32), np.array([0, 0, 30_000], np.int64),
            np.array([30_000, 45_000, 60_000], np.int64))
    eng.set_contigs(lengths)
    for k, n in enumerate([4_000, 1_000_000, 6_000]):
        rng = np.random.default_rng(70 + k)
        t = np.sort(rng.integers(0, 2, size=n)).astype(np.int32)
        span = rng.integers(100, 200, size=n).astype(np.int32)
        L = np.asarray(lengths)[t]
        pos = rng.integers(0, L - span + 1).astype(np.int32)
        o = np.lexsort((pos, t))
        t, pos, span = t[o], pos[o], span[o]
        d, ext, coff = coracle.depth(lengths, t, pos, span)
        want = coracle.region_stats(d, ext, coff, *regs)
        eng.clear_reads()
        eng.add_reads(t, pos, span)
        got = eng.compute_depth_stats(*regs)
        for f in want.dtype.names:
            assert np.array_equal(got[f], want[f]), (k, f)
        assert eng.fused_fallbacks() == 0, k


def _edge_index_cases():
    """Read layouts aimed at ingest_kernel's chunk index (base chunks of
    16 Ki positions on genomes of >= 2048 chunks, 8 Ki below that)."""
    cases = {}
    # starts exactly on base-chunk boundaries, reads crossing them, reads ending on
    # them: 8 Ki base chunks (a small genome) and 16 Ki ones (>= 2048 full chunks)
    for name, W, length in (("on_boundaries_8k", 8192, 40 * 8192),
                            ("on_boundaries_16k", 16384, 72 * 10**6)):
        lengths = np.array([length], np.int64)
        k = np.arange(1, 40) * (length // 40 // W) * W
        p = np.sort(np.concatenate([k, k - 100, k - 1, k + 1, k - W // 2]))
        s = np.tile(np.array([100, 150, 1, 4096, 5000, W // 2], np.int32), len(p) // 6 + 1)[:len(p)]
        cases[name] = (lengths, np.zeros(len(p), np.int32), p.astype(np.int32), s)
    # sparse reads over long empty stretches, many empty contigs, a read at the very end
    lengths = np.array([3 * 10**6, 5, 0, 2 * 10**6, 7, 1 * 10**6], np.int64)
    t = np.array([0, 0, 0, 3, 3, 5], np.int32)
    p = np.array([17, 1_500_000, 2_999_990, 0, 1_999_999, 999_999], np.int32)
    s = np.array([300, 20_000, 50, 1, 40, 1], np.int32)
    cases["sparse_tail"] = (lengths, t, p, s)
    # 1..3 reads (partial int4 groups)
    for k in (1, 2, 3):
        lengths = np.array([100_000], np.int64)
        cases["n%d" % k] = (lengths, np.zeros(k, np.int32),
                            np.array([5, 16_380, 16_383][:k], np.int32), np.array([10, 9, 4000][:k], np.int32))
    # overhangs (the second ingest pass) together with long reads (the long path)
    rng = np.random.default_rng(11)
    lengths = np.array([50_000, 80_000, 30_000], np.int64)
    t = rng.integers(0, 3, 6000).astype(np.int32)
    p = (rng.random(6000) * lengths[t]).astype(np.int32)
    s = np.where(rng.random(6000) < 0.3, rng.integers(4097, 30_000, 6000),
                 rng.integers(1, 300, 6000)).astype(np.int32)
    o = np.lexsort((p, t))
    cases["overhang_long"] = (lengths, t[o], p[o], s[o])
    return cases


@pytest.mark.parametrize("name", sorted(_edge_index_cases()))
def test_index_edge_layouts(eng, name):
    lengths, tid, pos, span = _edge_index_cases()[name]
    run_engine(eng, lengths, tid, pos, span)
    d, ext, coff = check_depth_vs_oracle(eng, lengths, tid, pos, span)
    assert eng.aligned_bases() == int(span.astype(np.int64).sum())
    whole = (np.arange(len(lengths), dtype=np.int32), np.zeros(len(lengths), np.int64),
             np.maximum(lengths, 1))
    want = coracle.region_stats(d, ext, coff, *whole)
    got = eng.compute_depth_stats(*whole)
    for f in want.dtype.names:
        assert np.array_equal(got[f], want[f]), f


# ------------------------------------------------------------- large coordinates

def _sparse_row(starts, ends, L):
    """Exact stat row of region [0, L) from read intervals (clipped to it),
    without a dense vector: the depth is piecewise constant between events,
    so its value histogram (value -> positions) gives every classic() field
    (test infrastructure: the dense oracle would need L int64s)."""
    s = np.clip(starts, 0, L)
    e = np.clip(ends, 0, L)
    keep = e > s
    ev = np.concatenate([s[keep], e[keep]])
    dv = np.concatenate([np.ones(keep.sum(), np.int64), -np.ones(keep.sum(), np.int64)])
    o = np.argsort(ev, kind="stable")
    ev, dv = ev[o], dv[o]
    pts = np.concatenate([[0], ev, [L]])
    val = np.concatenate([[0], np.cumsum(dv)])          # depth on [pts[k], pts[k+1])
    run = np.diff(pts)
    hist = {}
    for v, r in zip(val.tolist(), run.tolist()):
        if r:
            hist[v] = hist.get(v, 0) + r
    vals = sorted(hist)
    n = L

    def at(rank):
        c = 0
        for v in vals:
            c += hist[v]
            if rank < c:
                return v
        raise AssertionError
    q_lo, q_hi = n // 4, n - n // 4
    q23, c = 0, 0
    for v in vals:
        lo, hi = max(c, q_lo), min(c + hist[v], q_hi)
        if hi > lo:
            q23 += (hi - lo) * v
        c += hist[v]
    return {"n": n, "sum": sum(v * k for v, k in hist.items()),
            "sumsq": sum(v * v * k for v, k in hist.items()), "min": vals[0], "max": vals[-1],
            "med_lo": at((n - 1) // 2), "med_hi": at(n // 2), "q23_sum": q23, "q23_cnt": q_hi - q_lo}


def test_large_coordinates(eng):
    """A 5.2 Gbp genome (20.8 GB depth vector): global offsets past 2^31 and
    2^32, a contig of 2.1 Gbp (positions near the int32 limit), read clusters
    with long reads at those boundaries and at contig ends, and an
    overhanging read (second ingest pass on the grown layout).  Windows
    around every cluster are checked against the oracle on the clipped reads;
    whole contigs against the exact sparse value histogram."""
    rng = np.random.default_rng(2024)
    lengths = np.array([1_900_000_000, 2_100_000_000, 1_200_000_000], np.int64)
    g0 = np.concatenate([[0], np.cumsum(lengths)])
    centers = [(0, 0), (0, 1_000_000_000), (0, int(lengths[0]) - 1),
               (1, 2 ** 31 - int(g0[1])), (1, 2 ** 31 - 1 - 2 ** 15 - int(g0[1]) + 5),
               (1, int(lengths[1]) - 10), (2, 2 ** 32 - int(g0[2])), (2, int(lengths[2]) - 1)]
    T, P, S = [], [], []
    for t, c in centers:
        L = int(lengths[t])
        sp = rng.integers(100, 301, size=3000)
        p = np.clip(c + rng.integers(-2000, 2001, size=3000), 0, L - sp)
        T.append(np.full(3000, t)); P.append(p); S.append(sp)
        lsp = rng.integers(5000, 50_001, size=20)
        lp = np.clip(c - rng.integers(0, 60_001, size=20), 0, L - lsp)
        T.append(np.full(20, t)); P.append(lp); S.append(lsp)
    for t in range(3):   # sparse background
        sp = np.full(50_000, 150)
        T.append(np.full(50_000, t)); P.append(rng.integers(0, int(lengths[t]) - 150, size=50_000)); S.append(sp)
    T.append(np.array([2])); P.append(np.array([int(lengths[2]) - 100])); S.append(np.array([400]))  # overhang
    tid = np.concatenate(T).astype(np.int64)
    pos = np.concatenate(P).astype(np.int64)
    span = np.concatenate(S).astype(np.int64)
    o = np.lexsort((pos, tid))
    tid, pos, span = tid[o].astype(np.int32), pos[o].astype(np.int32), span[o].astype(np.int32)
    ends = pos.astype(np.int64) + span

    # windows around the clusters (non-overlapping: the fused path)
    wt, ws, we = [], [], []
    for t, c in centers:
        L = int(lengths[t])
        wt.append(t); ws.append(max(0, c - 70_000)); we.append(min(L, c + 6000))
    wt, ws, we = np.array(wt, np.int32), np.array(ws, np.int64), np.array(we, np.int64)
    want = []
    for t, a, b in zip(wt, ws, we):
        m = (tid == t) & (pos < b) & (ends > a)
        lp = np.maximum(pos[m], a) - a
        ls = np.minimum(ends[m], b) - np.maximum(pos[m], a)
        o = np.argsort(lp, kind="stable")
        dl, ext_l, coff_l = coracle.depth([b - a], np.zeros(m.sum(), np.int32),
                                          lp[o].astype(np.int32), ls[o].astype(np.int32))
        want.append((dl[:b - a], coracle.region_stats(dl, ext_l, coff_l, np.zeros(1, np.int32),
                                                      np.zeros(1, np.int64), np.array([b - a], np.int64))))
    eng.set_contigs(lengths)
    eng.add_reads(tid, pos, span)
    got = eng.compute_depth_stats(wt, ws, we)
    assert eng.contig_offset(2)[1] == lengths[2] + 300          # grown by the overhang
    assert eng.contig_offset(1)[0] < 2 ** 31 < eng.contig_offset(2)[0] < 2 ** 32 < eng.contig_offset(2)[0] + lengths[2]
    for k, (t, a, b) in enumerate(zip(wt, ws, we)):
        dl, row = want[k]
        for f in row.dtype.names:
            assert got[f][k] == row[f][0], (k, f)
        assert np.array_equal(eng.depth(int(t), int(a), int(b)), dl), k
    # the unfused path (K2 + K3) on the same windows
    got2 = eng.region_stats(wt, ws, we)
    for f in got.dtype.names:
        assert np.array_equal(got2[f], got[f]), f
    # whole contigs, fused
    rows = eng.compute_depth_stats(np.arange(3, dtype=np.int32), np.zeros(3, np.int64), lengths)
    for t in range(3):
        m = tid == t
        exp = _sparse_row(pos[m].astype(np.int64), ends[m], int(lengths[t]))
        for f, v in exp.items():
            assert int(rows[f][t]) == v, (t, f)


def test_assembly_scale_contig_count(eng):
    """A metagenome assembly's contig count: 300,000 contigs of 1-1,000 bp
    (whole-contig regions fused: 300,000 histogram rows) with reads that
    overhang contig ends (the second ingest pass over a grown layout), then
    the same regions plus overlapping ones through the K2 + K3 path."""
    rng = np.random.default_rng(300)
    lengths = rng.integers(1, 1001, size=300_000).astype(np.int64)
    lengths, tid, pos, span = make_case(lengths, 1_000_000, (1, 150), 301)
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    R = len(lengths)
    rt = np.arange(R, dtype=np.int32)
    rs = np.zeros(R, np.int64)
    re_ = lengths.copy()
    eng.set_contigs(lengths)
    eng.add_reads(tid, pos, span)
    got = eng.compute_depth_stats(rt, rs, re_)
    want = coracle.region_stats(d, ext, coff, rt, rs, re_)
    for f in want.dtype.names:
        assert np.array_equal(got[f], want[f]), f
    # overlapping regions (K2 + K3): every contig, plus a second region per 8th contig
    k = np.arange(0, R, 8)
    rt2 = np.concatenate([rt, rt[k]])
    rs2 = np.concatenate([rs, lengths[k] // 3])
    re2 = np.concatenate([re_, lengths[k] + 20])
    got2 = eng.compute_depth_stats(rt2, rs2, re2)
    want2 = coracle.region_stats(d, ext, coff, rt2, rs2, re2)
    for f in want2.dtype.names:
        assert np.array_equal(got2[f], want2[f]), f
    for t in (0, 1, R // 2, R - 1):
        assert np.array_equal(eng.depth(t, 0, int(ext[t])), d[coff[t]:coff[t] + ext[t]])


def test_bench_json_contract(tmp_path):
    """bench.py's one JSON line carries the fields the driver and the judge
    read (metric / value / unit / roofline / cpu_baseline ...), on a short C2
    run with a small CPU baseline sample."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--config", "c2", "--steps", "3",
                          "--warmup", "1", "--prepare-steps", "2", "--cpu-sample-bases", "2e7",
                          "--cpu-threads", "2"],
                         capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert "workload" in d["config"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["value"] > 0 and c["kind"] in ("port", "reference")


@pytest.mark.parametrize("cfg,reads,contigs", [("c3", 2_000_000, 64), ("c5", 2_000_000, 400)])
def test_bench_gpus_two_launches_ranks(tmp_path, cfg, reads, contigs):
    """`bench.py --gpus 2` (no torchrun around it) starts two ranks through a
    child torch.distributed.run and prints rank 0's line: n_gpus == 2, the
    contig-sharded (strong) layout, the all-gather timed apart.  gloo lets
    both ranks share the box's one GPU.  C3's layout and C5's (long reads:
    the full prepare, long-read K2, device recomputes) rehearse C4 / the
    8-GPU C5 run; the gathered rows equal the oracle's."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    rows_path = str(tmp_path / "rows.npy")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--backend", "gloo",
                          "--config", cfg, "--reads", str(reads), "--contigs", str(contigs), "--steps", "2",
                          "--warmup", "1", "--prepare-steps", "1", "--dump-rows", rows_path],
                         capture_output=True, text=True, timeout=600, cwd=str(tmp_path), env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["ranks_seen"] == 2
    assert d["scaling"] == "strong" and d["backend"] == "gloo"
    assert d["allgather_ms"] is not None and d["allgather_ms"] > 0
    assert d["config"]["regions"] == contigs
    assert d["value"] > 0
    # the gathered table, field by field, against the oracle on the same
    # workload (regenerated here: the bench's GPU generator is seeded)
    import torch
    sys.path.insert(0, root)
    import bench
    lengths, weights = bench.config_contigs(cfg, reads, contigs)
    tid, pos, span, _ = bench.device_workload(torch, lengths, weights, reads, 1,
                                              torch.device("cuda", 0), long_reads=cfg == "c5")
    tid, pos, span = (x.cpu().numpy() for x in (tid, pos, span))
    dd, ext, coff = coracle.depth(lengths, tid, pos, span)
    R = len(lengths)
    want = coracle.region_stats(dd, ext, coff, np.arange(R, dtype=np.int32), np.zeros(R, np.int64),
                                lengths.astype(np.int64))
    got = np.load(rows_path)
    for f in want.dtype.names:
        assert np.array_equal(got[f], want[f]), f


def test_bench_rccl_exchange_one_rank(tmp_path):
    """The bench's RCCL path on the one-GPU box: one torchrun rank with
    MC_BENCH_FORCE_EXCHANGE=1 runs the nccl process group, the asynchronous
    device-tensor all-gathers into alternating exchange buffers (with the
    host-side completion wait before a buffer is rewritten) and the timed
    all-gather, then checks the gathered table's bases (bench.py asserts it)."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env["MC_BENCH_FORCE_EXCHANGE"] = "1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(root, "bench.py"), "--backend", "nccl", "--config", "c3",
                          "--reads", "2000000", "--contigs", "64", "--steps", "6", "--warmup", "2",
                          "--prepare-steps", "2", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=600, cwd=str(tmp_path), env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["ranks_seen"] == 1 and d["backend"] == "nccl"
    assert d["allgather_ms"] is not None and d["allgather_ms"] > 0
    assert d["config"]["regions"] == 64 and d["value"] > 0


def test_library_then_torch_same_process():
    """The library first, torch after it, in one fresh process: one HIP
    runtime is shared (metacov_amd._lib preloads PyTorch's), so torch still
    finds the device and both work on the same data.  (Loaded the other way
    round the library's /opt/rocm runtime left torch with hipErrorNoDevice.)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import numpy as np\n"
        "from metacov_amd.engine import CoverageEngine\n"
        "e = CoverageEngine(0)\n"
        "e.set_contigs(np.array([1000], np.int64))\n"
        "e.add_reads(np.zeros(3, np.int32), np.array([1, 5, 9], np.int32), np.array([10, 10, 10], np.int32))\n"
        "e.compute_depth()\n"
        "d = e.depth(0, 0, 20)\n"
        "import torch\n"
        "assert torch.cuda.is_available()\n"
        "t = torch.from_numpy(d).to('cuda:0')\n"
        "assert int(t.sum().item()) == 30, t\n"
        "e.close()\n"
        "print('ok')\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=root)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stderr[-3000:]


# ------------------------------------------------------------- direct prepare

def _paths(eng):
    t = eng.timings()
    return t["direct_batches"], t["full_prepares"]


def _fresh(lib_built):
    return CoverageEngine(0)


def test_direct_path_taken_and_equal_to_full(lib_built):
    """Sorted in-bounds short reads go the direct way (probe + validating
    K2), and give the same depth, rows and aligned bases as the full
    prepare, for the plain and the fused K2."""
    lengths, weights = synth.c3_workload(2_000_000, 300)
    tid, pos, span = synth.interval_workload(lengths, 2_000_000, seed=31, weights=weights)
    rt = np.arange(len(lengths), dtype=np.int32)
    rs = np.zeros(len(lengths), np.int64)
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    want = coracle.region_stats(d, ext, coff, rt, rs, lengths)
    e = _fresh(lib_built)
    try:
        e.set_contigs(lengths)
        e.add_reads(tid, pos, span)
        e.compute_depth()
        assert _paths(e) == (1, 0)
        assert e.aligned_bases() == int(span.astype(np.int64).sum())
        got = np.concatenate([e.depth(t, 0, int(ext[t])) for t in range(len(lengths))])
        assert np.array_equal(got, np.concatenate([d[coff[t]:coff[t] + ext[t]] for t in range(len(lengths))]))
        for direct in (True, False):
            e.set_direct_prepare(direct)
            e.invalidate()
            rows = e.compute_depth_stats(rt, rs, lengths)
            for f in want.dtype.names:
                assert np.array_equal(rows[f], want[f]), (direct, f)
            assert e.fused_fallbacks() == 0
        assert _paths(e) == (2, 1)
    finally:
        e.close()


def _direct_case(lib_built, lengths, tid, pos, span, expect_direct, regions=True):
    e = _fresh(lib_built)
    try:
        e.set_contigs(lengths)
        e.add_reads(tid, pos, span)
        e.compute_depth()
        assert (_paths(e)[0] == 1) == expect_direct, _paths(e)
        check_depth_vs_oracle(e, lengths, tid, pos, span)
        if regions:
            d, ext, coff = coracle.depth(lengths, tid, pos, span)
            rt = np.arange(len(lengths), dtype=np.int32)
            e.invalidate()
            got = e.compute_depth_stats(rt, np.zeros(len(lengths), np.int64), np.asarray(lengths, np.int64))
            want = coracle.region_stats(d, ext, coff, rt, np.zeros(len(lengths), np.int64),
                                        np.asarray(lengths, np.int64))
            for f in want.dtype.names:
                assert np.array_equal(got[f], want[f]), f
        return _paths(e)
    finally:
        e.close()


def test_direct_hands_over_unsampled_long_read(lib_built):
    """A read longer than 4096 at an index the probe does not sample: K2's
    check sends the batch to the full prepare (long-read path), exactly."""
    lengths, tid, pos, span = make_case([400_000, 100_000], 20_000, (1, 150), 41, overhang=False)
    i = 1001                      # not a multiple of 256
    assert i % 256
    span = span.copy()
    span[i] = min(9000, int(lengths[tid[i]] - pos[i]))
    assert span[i] > 4096
    paths = _direct_case(lib_built, lengths, tid, pos, span, expect_direct=False)
    assert paths[1] >= 1


def test_direct_hands_over_unsampled_overhang(lib_built):
    lengths, tid, pos, span = make_case([300_000, 50_000], 20_000, (1, 150), 42, overhang=False)
    last = np.nonzero(tid == 0)[0][-1]
    assert last % 256
    pos = pos.copy()
    pos[last] = lengths[0] - 10
    span = span.copy()
    span[last] = 40               # runs 30 past contig 0's end
    o = np.lexsort((pos, tid))
    tid, pos, span = tid[o], pos[o], span[o]
    _direct_case(lib_built, lengths, tid, pos, span, expect_direct=False)


def test_direct_rejects_unsampled_disorder_and_invalid(lib_built):
    """Unsorted or invalid reads between the samples: the same errors as the
    full prepare (K2's check, then mc_prepare's exact message)."""
    lengths, tid, pos, span = make_case([200_000], 5_000, (1, 150), 43, overhang=False)
    bad_order = pos.copy()
    bad_order[[700, 701]] = bad_order[[701, 700]]
    assert bad_order[700] != bad_order[701]
    e = _fresh(lib_built)
    try:
        e.set_contigs(lengths)
        e.add_reads(tid, bad_order, span)
        with pytest.raises(MetacovError) as ei:
            e.compute_depth()
        assert ei.value.code == MC_E_INVALID and "sorted" in str(ei.value)
        e.set_contigs(lengths)
        bad_tid = tid.copy()
        bad_tid[3001] = 5
        e.add_reads(bad_tid, pos, span)
        with pytest.raises(MetacovError) as ei:
            e.compute_depth_stats([0], [0], [200_000])
        assert ei.value.code == MC_E_INVALID
        # a good batch afterwards on the same ctx goes direct again
        e.set_contigs(lengths)
        e.add_reads(tid, pos, span)
        e.compute_depth()
        assert _paths(e)[0] == 1
        check_depth_vs_oracle(e, lengths, tid, pos, span)
    finally:
        e.close()


def test_direct_sparse_and_empty_contigs(lib_built):
    """Sample blocks spanning empty contigs, huge gaps and contig boundaries
    (chunk ranges from the J counts only), and fewer reads than one sample
    block."""
    rng = np.random.default_rng(44)
    lengths = np.array([5, 0, 1_000_000, 3, 2_000_000, 64, 65, 4096 * 9 + 1, 0, 7_000_000], np.int64)
    for n in (1, 3, 255, 257, 2000):
        live = np.array([0, 2, 4, 6, 7, 9])
        t = rng.choice(live, size=n).astype(np.int32)
        sp = rng.integers(1, 150, size=n).astype(np.int32)
        sp = np.minimum(sp, lengths[t]).astype(np.int32)
        p = (rng.random(n) * (lengths[t] - sp + 1)).astype(np.int32)
        o = np.lexsort((p, t))
        _direct_case(lib_built, lengths, t[o], p[o], sp[o], expect_direct=True)


def test_direct_halo_follows_the_spans(lib_built):
    """The chunk halo of a direct batch is the previous batch's maximum span
    (+1/8): a batch with a longer read than that (3000 bp crossing a chunk
    boundary from 1000 before it) is redone on the direct path with a halo
    that covers it, exactly, for the plain and the fused K2; no full prepare."""
    lengths, tid, pos, span = make_case([400_000], 20_000, (1, 150), 46, overhang=False)
    t2 = np.append(tid, np.int32(0))
    p2 = np.append(pos, np.int32(131_072 - 1000))
    s2 = np.append(span, np.int32(3000))
    o = np.lexsort((p2, t2))
    t2, p2, s2 = t2[o], p2[o], s2[o]
    rt, rs, re_ = np.zeros(1, np.int32), np.zeros(1, np.int64), np.asarray(lengths, np.int64)
    e = _fresh(lib_built)
    try:
        e.set_contigs(lengths)
        for k, fused in enumerate((False, True)):
            e.clear_reads()
            e.add_reads(tid, pos, span)          # max span 150: the next halo is 192
            e.compute_depth()
            assert e.timings()["halo_redos"] == k
            e.clear_reads()
            e.add_reads(t2, p2, s2)
            if fused:
                d, ext, coff = coracle.depth(lengths, t2, p2, s2)
                want = coracle.region_stats(d, ext, coff, rt, rs, re_)
                got = e.compute_depth_stats(rt, rs, re_)
                for f in want.dtype.names:
                    assert np.array_equal(got[f], want[f]), f
            else:
                e.compute_depth()
            check_depth_vs_oracle(e, lengths, t2, p2, s2)
            t = e.timings()
            assert t["halo_redos"] == k + 1 and t["direct_halo"] >= 3000, t
            assert t["full_prepares"] == 0 and t["direct_batches"] == 2 * (k + 1), t
    finally:
        e.close()


def _fuzz_batch(rng):
    """A random batch: contig count / lengths from tiny to 300 kbp (some
    empty), a span mix of zero, short, N-skip-like and (sometimes) long
    spans, deep piles at one start, optional overhangs; sorted."""
    nc = int(rng.integers(1, 40))
    lengths = rng.integers(0, 300_000, size=nc).astype(np.int64)
    lengths[rng.random(nc) < 0.1] = 0
    lengths[rng.random(nc) < 0.1] = rng.integers(1, 100)
    live = np.nonzero(lengths > 0)[0]
    if len(live) == 0:
        lengths[0] = 5000
        live = np.array([0])
    n = int(rng.integers(1, 60_000))
    tid = rng.choice(live, size=n).astype(np.int32)
    span = rng.integers(0, 300, size=n)
    u = rng.random(n)
    span[u < 0.01] = rng.integers(300, 4000, size=int((u < 0.01).sum()))
    if rng.random() < 0.3:
        span[u > 0.9995] = rng.integers(4097, 20_000, size=int((u > 0.9995).sum()))
    pos = (rng.random(n) * lengths[tid]).astype(np.int64)
    if rng.random() < 0.5:   # no overhang
        span = np.minimum(span, lengths[tid] - pos)
    if rng.random() < 0.3:   # a deep pile at one start
        k = int(rng.integers(0, n))
        pos[max(0, k - 500):k] = pos[k]
        tid[max(0, k - 500):k] = tid[k]
    o = np.lexsort((pos, tid))
    return lengths, tid[o], pos[o].astype(np.int32), span[o].astype(np.int32)


def test_direct_and_full_fuzz(lib_built):
    """Random batches through one ctx (the direct path with its halo carried
    from batch to batch, the full prepare for long reads and overhangs):
    depth, whole-contig fused rows and random-region rows equal the oracle."""
    # (MC_FUZZ_ITERS / MC_FUZZ_SEED: longer soak runs, profiles/r06/r06soak_*)
    rng = np.random.default_rng(int(os.environ.get("MC_FUZZ_SEED", "2024")))
    e = _fresh(lib_built)
    try:
        for k in range(int(os.environ.get("MC_FUZZ_ITERS", "24"))):
            lengths, tid, pos, span = _fuzz_batch(rng)
            e.set_contigs(lengths)
            e.add_reads(tid, pos, span)
            d, ext, coff = coracle.depth(lengths, tid, pos, span)
            rt = np.arange(len(lengths), dtype=np.int32)
            rs = np.zeros(len(lengths), np.int64)
            re_ = np.asarray(ext, np.int64)
            want = coracle.region_stats(d, ext, coff, rt, rs, re_)
            got = e.compute_depth_stats(rt, rs, re_)
            for f in want.dtype.names:
                assert np.array_equal(got[f], want[f]), (k, f)
            check_depth_vs_oracle(e, lengths, tid, pos, span)
            check_regions_vs_oracle(e, d, ext, coff, *random_regions(rng, lengths, 50))
            # the same contigs, a second batch: the direct path with the halo the first one set
            e.clear_reads()
            lengths2, tid2, pos2, span2 = lengths, tid, pos, np.maximum(span - 1, 0).astype(np.int32)
            e.add_reads(tid2, pos2, span2)
            d2, ext2, coff2 = coracle.depth(lengths2, tid2, pos2, span2)
            got2 = e.compute_depth_stats(rt, rs, np.asarray(ext2, np.int64))
            want2 = coracle.region_stats(d2, ext2, coff2, rt, rs, np.asarray(ext2, np.int64))
            for f in want2.dtype.names:
                assert np.array_equal(got2[f], want2[f]), (k, "second", f)
    finally:
        e.close()


def test_direct_ctx_sticks_to_full_after_long_reads(lib_built):
    lengths, tid, pos, span = make_case([300_000], 8_000, (1, 150), 45, overhang=False)
    span_long = span.copy()
    span_long[500] = min(6000, int(lengths[0] - pos[500]))
    e = _fresh(lib_built)
    try:
        e.set_contigs(lengths)
        e.add_reads(tid, pos, span_long)
        e.compute_depth()
        assert _paths(e) == (0, 1)
        e.clear_reads()
        e.add_reads(tid, pos, span)
        e.compute_depth()            # same contig set: straight to the full prepare
        assert _paths(e) == (0, 2)
        check_depth_vs_oracle(e, lengths, tid, pos, span)
        e.set_contigs(lengths)       # a new contig set tries the direct path again
        e.add_reads(tid, pos, span)
        e.compute_depth()
        assert _paths(e) == (1, 2)
    finally:
        e.close()


# ------------------------------------------------------------- pysam's defaults: the cap, span-0 reads

def test_max_depth_cap_gpu_rows(lib_built):
    """depthcap.capped_rows (one engine call for all regions) on a >8000x
    synthetic contig (amplicon piles, span-0 reads among them): each row equals
    classic() over the literal htslib restatement's columns
    (oracle/htslib_plp.py).  Parity with htslib itself unpinned."""
    import types
    from metacov_amd import depthcap
    from oracle import htslib_plp
    from oracle.classic_np import classic_from_vector
    rng = np.random.default_rng(12)
    L = 4000
    pos = np.concatenate([np.full(12_000, 700), np.full(9_500, 710), np.full(11_000, 2100),
                          rng.integers(0, 3800, size=6000)])
    span = np.concatenate([np.full(12_000, 150), rng.integers(100, 200, size=9_500),
                           np.full(11_000, 300), rng.integers(0, 200, size=6000)])
    span[rng.random(len(span)) < 0.02] = 0
    o = np.argsort(pos, kind="stable")
    bf = types.SimpleNamespace(tid=np.zeros(len(pos), np.int32), pos=pos[o].astype(np.int32),
                               span=span[o].astype(np.int32), lengths=(L,))
    regions = [(0, L), (650, 900), (705, 2500), (2200, 2300), (0, 1)]
    rows, dropped = depthcap.capped_rows(bf, np.zeros(len(regions), np.int32),
                                         np.array([r[0] for r in regions], np.int64),
                                         np.array([r[1] for r in regions], np.int64), bf.lengths, 8000)
    assert dropped > 0
    for row, (s, e) in zip(rows, regions):
        want, _ = htslib_plp.region_depth(bf.tid, bf.pos, bf.span, 0, s, e, max_depth=8000)
        assert classic_stats(row) == classic_from_vector(want.astype(np.float64)), (s, e)


def _deep_bam(path):
    """Two contigs: "amp" (1200 bp) with amplicon piles of 12,000 and 9,000
    reads and span-0 records (30S: mapped, no reference-consuming op) opening
    and inside the start groups; "bg" (5000 bp) shallow.  Plus filtered
    records (secondary, duplicate, unmapped)."""
    R = synth.SynthRecord
    rng = np.random.default_rng(2024)
    recs = []
    k = [0]

    def add(tid, pos, flag, cigar):
        k[0] += 1
        recs.append(R("r%d" % k[0], tid, pos, flag, cigar, 150))

    for p in sorted(rng.integers(0, 290, size=600).tolist()):
        add(0, p, 0, [(4, 30)] if rng.random() < 0.05 else [(0, 100)])
    add(0, 300, 0, [(4, 30)])                                   # opens the group at 300
    for i in range(12_000):
        add(0, 300, 0x400 if i % 997 == 0 else 0, [(4, 30)] if i % 401 == 7 else [(0, 150)])
    for i in range(9_000):
        add(0, 310, 0x100 if i % 1009 == 0 else 0, [(0, 60), (2, 5), (0, 40)])
    for p in sorted(rng.integers(311, 1150, size=900).tolist()):
        add(0, p, 0, [(4, 30)] if rng.random() < 0.05 else [(0, 100)])
    for p in sorted(rng.integers(0, 4900, size=3000).tolist()):
        add(1, p, 0x4 if rng.random() < 0.01 else 0,
            [(4, 30)] if rng.random() < 0.02 else [(0, 100)])
    synth.write_bam(path, ["amp", "bg"], [1200, 5000], recs)


def _oracle_csv(path, regions, max_depth, legacy=False):
    """The CSV cli.py:85-108 writes, from the oracle: the pure-Python BAM
    reader's intervals, htslib's literal push/next loop per region query
    (max_depth None: a plain interval count), classic()'s numpy restatement."""
    import csv
    import io
    from oracle import bamread, htslib_plp
    from oracle.classic_np import classic_from_vector
    names, lengths, recs = bamread.read_bam(path)
    iv = bamread.pileup_intervals(recs, legacy_endpos=legacy)
    tid = np.array([x[0] for x in iv], np.int32)
    pos = np.array([x[1] for x in iv], np.int32)
    span = np.array([x[2] for x in iv], np.int32)
    out = io.StringIO()
    writer = None
    for sacc, a, b in regions:
        s, e = sorted((int(a), int(b)))
        t = names.index(sacc)
        want, _ = htslib_plp.region_depth(tid, pos, span, t, s, e,
                                          max_depth=max_depth or 10 ** 9)
        res = classic_from_vector(want.astype(np.float64))
        if writer is None:
            writer = csv.DictWriter(out, fieldnames=["sacc", "start", "end"] + sorted(res))
            writer.writeheader()
        res.update({"sacc": sacc, "start": a, "end": b})
        writer.writerow(res)
    return out.getvalue()


@pytest.mark.parametrize("decode", ["gpu", "host", "stream"])
def test_cli_defaults_follow_pysam(lib_built, tmp_path, decode):
    """`metacov pileup` with no options on a contig piled at 12,000x with
    span-0 records: the CSV equals the oracle's (htslib's max_depth=8000 cap
    per region query, current htslib's raw-rlen read end, classic()), for
    whole contigs and for CSV regions; --max-depth 0 gives the exact counts;
    --legacy-endpos the htslib <= 1.9 end."""
    from click.testing import CliRunner
    from metacov_amd.cli import pileup as cli_pileup
    bam = str(tmp_path / "deep.bam")
    _deep_bam(bam)
    mode = {"gpu": ["--decode", "gpu"], "host": ["--decode", "host", "--no-stream"],
            "stream": ["--decode", "host", "--stream"]}[decode]
    rc = tmp_path / "r.csv"
    regs = [("amp", "305", "320"), ("bg", "0", "5000"), ("amp", "0", "1200"), ("amp", "301", "299"),
            ("bg", "100", "101"), ("amp", "455", "470")]
    rc.write_text("sacc,sstart,send\n" + "".join("%s,%s,%s\n" % r for r in regs))
    cases = [([], [("amp", 0, 1200), ("bg", 0, 5000)], 8000, False),
             (["-rc", str(rc)], regs, 8000, False),
             (["-rc", str(rc), "--max-depth", "0"], regs, None, False),
             (["-rc", str(rc), "--legacy-endpos"], regs, 8000, True)]
    for extra, regions, cap, legacy in cases:
        out = tmp_path / "o.csv"
        res = CliRunner().invoke(cli_pileup, ["-b", bam, "-o", str(out)] + mode + extra)
        assert res.exit_code == 0, res.output
        want = _oracle_csv(bam, regions, cap, legacy)
        assert open(out, newline="").read() == want, extra
    # the cap did act, and the exact path differs from it
    capped = _oracle_csv(bam, [("amp", 0, 1200)], 8000)
    assert capped != _oracle_csv(bam, [("amp", 0, 1200)], None)


def test_classic_defaults_and_cache(lib_built, tmp_path):
    """pileup.classic: max_depth=8000 by default on every source (path,
    BamFile, GpuBamFile, StreamedBam), None for exact; a rewritten file at
    the same path is decoded again (the cache keys on size and mtime)."""
    from metacov_amd import pileup
    from metacov_amd.bam import GpuBamFile, StreamedBam
    from oracle import bamread, htslib_plp
    from oracle.classic_np import classic_from_vector
    bam = str(tmp_path / "deep.bam")
    _deep_bam(bam)
    names, lengths, recs = bamread.read_bam(bam)
    iv = bamread.pileup_intervals(recs)
    tid, pos, span = (np.array([x[i] for x in iv], np.int32) for i in range(3))
    want = {}
    for cap in (8000, None):
        v, _ = htslib_plp.region_depth(tid, pos, span, 0, 250, 600, max_depth=cap or 10 ** 9)
        want[cap] = classic_from_vector(v.astype(np.float64))
    assert want[8000] != want[None]
    for src in (bam, BamFile(bam), GpuBamFile(bam), StreamedBam(bam)):
        assert pileup.classic(src, "amp", 250, 600) == want[8000]
        assert pileup.classic(src, "amp", 250, 600, max_depth=None) == want[None]
    # rewrite the path with other contents: no stale depths
    shutil_bam = str(tmp_path / "other.bam")
    synth.write_bam(shutil_bam, ["amp", "bg"], [1200, 5000],
                    [synth.SynthRecord("x", 0, 10, 0, [(0, 50)], 50)])
    os.replace(shutil_bam, bam)
    assert pileup.classic(bam, "amp", 0, 100)["sum"] == 50
    pileup.close_all()


def test_cli_writes_rows_before_a_bad_region(lib_built, golden_dir, tmp_path):
    """As cli.py:85-108: rows are written one region at a time, so an unknown
    name (KeyError, cli.py:86), a non-integer coordinate (cli.py:89) or an
    empty region (classic's ValueError) leaves the rows before it in the CSV
    and raises."""
    from click.testing import CliRunner
    from metacov_amd.cli import pileup as cli_pileup
    bam = os.path.join(golden_dir, "bbmap.sorted.bam")
    good = "ref1,1,425\nref2,1,575\n"
    for bad, exc in [("nope,1,5\n", KeyError), ("ref1,x,5\n", ValueError),
                     ("ref2,7,7\n", ValueError)]:
        rc = tmp_path / "r.csv"
        rc.write_text("sacc,sstart,send\n" + good + bad + "ref1,3,9\n")
        out = tmp_path / "o.csv"
        res = CliRunner().invoke(cli_pileup, ["-b", bam, "-rc", str(rc), "-o", str(out)])
        assert isinstance(res.exception, exc), (bad, res.exception)
        lines = open(out, newline="").read().split("\r\n")
        assert len(lines) == 4 and lines[3] == "", lines            # header + 2 rows
        assert lines[1].startswith("ref1,1,425,") and lines[2].startswith("ref2,1,575,")


def test_fused_device_recompute(lib_built):
    """Out-of-window regions recomputed on the device within the fused call
    (long reads, or after a call that had them): many deep ramped contigs
    (C5 in miniature), rows exact against the oracle, no host fallback; a
    depth beyond the device histogram (16384) hands them to the host K3."""
    rng = np.random.default_rng(77)
    lengths = rng.integers(20_000, 40_000, size=60).astype(np.int64)
    w = np.minimum(rng.lognormal(0, 1.2, size=60), 6.0)   # every depth below 16384
    n = 400_000
    tid = np.sort(rng.choice(60, size=n, p=w / w.sum())).astype(np.int32)
    span = np.minimum(rng.lognormal(np.log(8000), 0.4, size=n).astype(np.int64), lengths[tid]).astype(np.int32)
    pos = (rng.random(n) * (lengths[tid] - span + 1)).astype(np.int32)
    o = np.lexsort((pos, tid))
    tid, pos, span = tid[o], pos[o], span[o]
    d, ext, coff = coracle.depth(lengths, tid, pos, span)
    regs = (np.arange(60, dtype=np.int32), np.zeros(60, np.int64), lengths)
    want = coracle.region_stats(d, ext, coff, *regs)
    e = CoverageEngine(0)
    try:
        e.set_contigs(lengths)
        e.add_reads(tid, pos, span)
        for k in range(3):
            got = e.compute_depth_stats(*regs)
            for f in want.dtype.names:
                assert np.array_equal(got[f], want[f]), (k, f)
            assert e.fused_fallbacks() == 0          # long reads: the device recomputes
        assert e.max_depth() < 16384
        assert e.fused_recomputes() > 0, "the case should have out-of-window regions"
        # depth above 16384 at one spot: the device histogram cannot hold it
        t2 = np.concatenate([tid, np.zeros(17_000, np.int32)])
        p2 = np.concatenate([pos, np.full(17_000, 100, np.int32)])
        s2 = np.concatenate([span, np.full(17_000, 50, np.int32)])
        o = np.lexsort((p2, t2))
        t2, p2, s2 = t2[o], p2[o], s2[o]
        d2, ext2, coff2 = coracle.depth(lengths, t2, p2, s2)
        want2 = coracle.region_stats(d2, ext2, coff2, *regs)
        e.clear_reads()
        e.add_reads(t2, p2, s2)
        got = e.compute_depth_stats(*regs)
        for f in want2.dtype.names:
            assert np.array_equal(got[f], want2[f]), f
        assert e.max_depth() > 16384 and e.fused_recomputes() == 0 and e.fused_fallbacks() > 0
    finally:
        e.close()
