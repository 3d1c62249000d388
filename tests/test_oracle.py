"""The oracle against the golden fixtures (CPU, no GPU).

Goldens: tests/golden/make_golden.py — region statistics from the
reference's real pileup.classic (metacov/pileup.py:9-26), depth from the
htslib pileup-count restatement.  These tests pin the oracle (C and numpy
restatements) and the product's host-side statistics formatting
(`metacov_amd.engine.classic_stats`) before either is trusted.
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import bamread, classic_np, coracle
from metacov_amd.engine import classic_stats


def _iv(g):
    return (np.array(g["intervals"]["tid"], np.int32), np.array(g["intervals"]["pos"], np.int32),
            np.array(g["intervals"]["span"], np.int32))


def test_fixture_decode_matches_golden(fixture_golden, golden_dir):
    names, lengths, recs = bamread.read_bam(os.path.join(golden_dir, "bbmap.sorted.bam"))
    assert names == fixture_golden["names"] and lengths == fixture_golden["lengths"]
    assert len(recs) == fixture_golden["n_records"] == 4112
    iv = bamread.pileup_intervals(recs)
    assert [t for t, _, _ in iv] == fixture_golden["intervals"]["tid"]
    assert [p for _, p, _ in iv] == fixture_golden["intervals"]["pos"]
    assert [s for _, _, s in iv] == fixture_golden["intervals"]["span"]
    assert sum(s for _, _, s in iv) == fixture_golden["aligned_bases"] == 340526


@pytest.mark.parametrize("method", ["interval", "columnwalk"])
def test_c_oracle_depth_fixture(fixture_golden, method):
    tid, pos, span = _iv(fixture_golden)
    d, ext, coff = coracle.depth(fixture_golden["lengths"], tid, pos, span, method=method)
    for t, gold in enumerate(fixture_golden["depth"]):
        assert d[coff[t]:coff[t] + ext[t]].tolist() == gold
    assert int(d.sum()) == fixture_golden["aligned_bases"]


def test_depth_methods_agree_random():
    rng = np.random.default_rng(5)
    lengths = np.array([1, 50, 3000, 0, 999], np.int64)
    tid = np.sort(rng.choice([0, 1, 2, 4], size=4000)).astype(np.int32)
    pos = np.array([rng.integers(0, max(1, lengths[t])) for t in tid], np.int32)
    span = rng.integers(1, 400, size=len(tid)).astype(np.int32)
    order = np.lexsort((pos, tid))
    tid, pos, span = tid[order], pos[order], span[order]
    a = coracle.depth(lengths, tid, pos, span, "interval")[0]
    b = coracle.depth(lengths, tid, pos, span, "columnwalk")[0]
    assert np.array_equal(a, b)
    assert a.sum() == span.sum()


def _check_regions(depth_vec, ext, coff, names, regions):
    rtid = np.array([names.index(r["sacc"]) for r in regions], np.int32)
    rs = np.array([r["start"] for r in regions], np.int64)
    re_ = np.array([r["end"] for r in regions], np.int64)
    rows = coracle.region_stats(depth_vec, ext, coff, rtid, rs, re_)
    for row, r in zip(rows, regions):
        if "error" in r["stats"]:
            with pytest.raises(ValueError):
                classic_stats(row)
        else:
            assert classic_stats(row) == r["stats"], r


def test_c_oracle_stats_fixture(fixture_golden):
    tid, pos, span = _iv(fixture_golden)
    d, ext, coff = coracle.depth(fixture_golden["lengths"], tid, pos, span)
    _check_regions(d, ext, coff, fixture_golden["names"],
                   fixture_golden["blast7"] + fixture_golden["whole"])


def test_stats_cases(stats_golden):
    """Edge cases + 60 random vectors through the real classic()."""
    for case in stats_golden:
        vec = np.array(case["depth"], np.int32)
        ext = np.array([len(vec)], np.int64)
        coff = np.array([0, len(vec)], np.int64)
        row = coracle.region_stats(vec, ext, coff, np.zeros(1, np.int32),
                                   np.array([case["start"]]), np.array([case["end"]]))[0]
        if "error" in case["stats"]:
            with pytest.raises(ValueError):
                classic_stats(row)
            continue
        assert classic_stats(row) == case["stats"], case["tag"]
        cols = classic_np.region_vector(vec, case["start"], case["end"])
        assert classic_np.classic_from_vector(cols) == case["stats"], case["tag"]


@pytest.mark.parametrize("legacy", [False, True])
def test_synth_goldens(synth_golden, golden_dir, legacy):
    for tag in ("synth_edge", "synth_multi"):
        g = synth_golden[tag]["legacy"] if legacy else synth_golden[tag]
        names, lengths, recs = bamread.read_bam(os.path.join(golden_dir, tag + ".bam"))
        assert len(recs) == g["n_records"]
        tid, pos, span = _iv(g)
        iv = bamread.pileup_intervals(recs, legacy_endpos=legacy)
        assert [x[2] for x in iv] == span.tolist()
        d, ext, coff = coracle.depth(lengths, tid, pos, span, method="columnwalk")
        assert ext.tolist() == g["extents"]
        for t in range(len(lengths)):
            v = np.ascontiguousarray(d[coff[t]:coff[t] + ext[t]], dtype="<i4")
            assert hashlib.sha256(v.tobytes()).hexdigest() == g["depth_sha"][t]
        _check_regions(d, ext, coff, names, g["regions"])


def test_pileup_classic_cpu_path(fixture_golden):
    """orc_pileup_classic (the CPU baseline) reproduces classic() end to end."""
    tid, pos, span = _iv(fixture_golden)
    regs = fixture_golden["blast7"] + fixture_golden["whole"]
    rtid = np.array([fixture_golden["names"].index(r["sacc"]) for r in regs], np.int32)
    out, cols = coracle.pileup_classic(tid, pos, span, rtid, [r["start"] for r in regs],
                                       [r["end"] for r in regs])
    assert cols == sum(r["end"] - r["start"] for r in regs)
    for o, r in zip(out, regs):
        s = r["stats"]
        assert (int(o[0]), int(o[1]), int(o[2]), int(o[6])) == (s["min"], s["max"], s["med"], s["sum"])
        for k, key in ((3, "std"), (4, "avg"), (5, "q23")):
            assert round(float(o[k]), 2) == s[key]


def test_parallel_classic_equals_one_core():
    """bench.py's contig-parallel CPU baseline computes the same rows."""
    rng = np.random.default_rng(7)
    lengths = rng.integers(1_000, 20_000, 12).astype(np.int64)
    tid, pos, span = [], [], []
    for t, L in enumerate(lengths):
        n = int(L // 10)
        pos.append(np.sort(rng.integers(0, L, n)).astype(np.int32))
        tid.append(np.full(n, t, np.int32))
        span.append(rng.integers(1, 300, n).astype(np.int32))
    tid, pos, span = map(np.concatenate, (tid, pos, span))
    R = len(lengths)
    args = (tid, pos, span, np.arange(R, dtype=np.int32), np.zeros(R, np.int64), lengths)
    a, ca = coracle.pileup_classic(*args)
    b, cb = coracle.pileup_classic_parallel(*args, threads=5)
    assert np.array_equal(a, b) and ca == cb


@pytest.mark.parametrize("legacy", [False, True])
def test_scan_intervals_equals_record_reader(golden_dir, legacy):
    """bamread.scan_intervals (the large-file form the multi-window GPU
    decode tests use) equals the record reader on every golden BAM."""
    for f in ("bbmap.sorted.bam", "synth_edge.bam", "synth_multi.bam", "synth_longcigar.bam"):
        path = os.path.join(golden_dir, f)
        names, lengths, recs = bamread.read_bam(path)
        iv = bamread.pileup_intervals(recs, legacy_endpos=legacy)
        n, l, counts, t, p, s = bamread.scan_intervals(path, legacy_endpos=legacy)
        assert (n, l, counts[0]) == (names, lengths, len(recs))
        assert counts[1] == sum(1 for r in recs if r.tid >= 0 and not r.flag & 4)
        assert t.tolist() == [x[0] for x in iv] and p.tolist() == [x[1] for x in iv]
        assert s.tolist() == [x[2] for x in iv]
