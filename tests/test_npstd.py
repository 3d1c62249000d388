"""classic()'s std at round(x, 2) ties: numpy's own float64 value
(metacov/pileup.py:22, `round(np.std(columns), 2)`).

The exact variance rounds like numpy's std everywhere except within numpy's
rounding noise of an x.xx5 boundary.  There the engine recomputes numpy's
value on the device in numpy's summation order (mc_region_np_sqdev,
metacov_amd/csrc/npstd.h; engine.numpy_std).  Pinning:
  * oracle/classic_np.np_std_restated (numpy's order restated) equals np.std
    bit for bit on random vectors;
  * tests/golden/std_ties.json holds vectors on exact ties with the real
    reference classic()'s dicts (tests/golden/make_std_ties.py), 39 of 40 of
    them rounding differently from the exact variance;
  * on the GPU, mc_region_np_sqdev equals the restated order bit for bit,
    and the engine / classic_batch / CLI reproduce the reference's dicts.
"""
import json
import math
import os

import numpy as np
import pytest

from metacov_amd import engine as E
from metacov_amd.engine import classic_stats, std_near_tie
from oracle.classic_np import classic_from_vector, np_buffered_sum, np_std_restated
from tests.std_ties import skyline_reads, tie_vector
from tests.test_stats_format import exact_row


@pytest.fixture(scope="module")
def ties(golden_dir):
    with open(os.path.join(golden_dir, "std_ties.json")) as fh:
        return json.load(fh)["cases"]


def _vec(c):
    return tie_vector(c["n"], c["a"], c["b"], c["d1"], c["d2"], c["y"], c["seed"])


def test_restated_order_is_numpys():
    rng = np.random.default_rng(11)
    for _ in range(150):
        n = int(np.exp(rng.uniform(0, np.log(50_000))))
        v = rng.poisson(float(np.exp(rng.uniform(-1, 9))), n).astype(np.float64)
        if rng.random() < 0.3:
            v[rng.integers(0, n + 1):] = 0
        assert np_std_restated(v) == float(np.std(v)), n


def test_tie_fixture(ties):
    """numpy here gives the fixture's values; the restatement and
    classic_stats with numpy's value give the reference's dicts; the exact
    variance alone does not (the gap numpy_std closes)."""
    differs = 0
    for c in ties:
        v = _vec(c)
        npstd = float.fromhex(c["np_std_hex"])
        assert float(np.std(v.astype(np.float64))) == npstd
        assert np_std_restated(v) == npstd
        assert classic_from_vector(v.astype(np.float64)) == c["stats"]
        row = exact_row(v)
        assert v.sum() % len(v) != 0                    # non-integer mean
        assert classic_stats(row, npstd) == c["stats"]
        if c["exact_rounding_differs"]:
            differs += 1
            assert classic_stats(row)["std"] != c["stats"]["std"]
    assert differs >= 30
    # numpy's value on both sides of the tie
    sides = {float.fromhex(c["np_std_hex"]) * 100 % 1 > 0.5 for c in ties if c["exact_rounding_differs"]}
    assert sides == {True, False}


def test_near_tie_mask(ties):
    rows = np.array([tuple(exact_row(_vec(c)).values()) for c in ties], dtype=E.REGION_STAT_DTYPE)
    assert std_near_tie(rows).all()
    rng = np.random.default_rng(3)
    rnd = [exact_row(rng.poisson(40.0, 1000)) for _ in range(300)]
    rows = np.array([tuple(r.values()) for r in rnd], dtype=E.REGION_STAT_DTYPE)
    assert std_near_tie(rows).sum() <= 2
    assert std_near_tie(rows, rel=1.0).all()


def test_classic_stats_nan_means_exact():
    row = exact_row(np.array([1, 2, 3, 7]))
    assert classic_stats(row, float("nan")) == classic_stats(row)


# ------------------------------------------------------------------ GPU

def _engine_for(vectors, pad=0):
    """An engine whose contig k has depth vectors[k] on [pad, pad + n) and 0
    elsewhere (contig length n + 2 pad)."""
    from metacov_amd.engine import CoverageEngine
    tids, poss, spans, lengths = [], [], [], []
    for k, v in enumerate(vectors):
        p, s = skyline_reads(v, start=pad)
        tids.append(np.full(len(p), k, np.int32))
        poss.append(p)
        spans.append(s)
        lengths.append(len(v) + 2 * pad)
    eng = CoverageEngine(0)
    eng.set_contigs(np.array(lengths, np.int64))
    eng.add_reads(np.concatenate(tids), np.concatenate(poss), np.concatenate(spans))
    return eng


@pytest.mark.gpu
def test_np_sqdev_is_numpys_order(lib_built):
    """mc_region_np_sqdev against the restated order, bit for bit: regions of
    1 to 60,000 positions (partial and whole 8192-element buffers), inside
    the contig, overlapping its start, and running past its extent."""
    rng = np.random.default_rng(5)
    vecs = [rng.poisson(lam, n).astype(np.int64)
            for lam, n in ((3.5, 9000), (40.0, 60_000), (0.7, 700), (250.0, 20_000))]
    eng = _engine_for(vecs, pad=100)
    try:
        eng.compute_depth()
        regs = []
        for k, v in enumerate(vecs):
            L = len(v) + 200
            for a, b in ((0, L), (100, 100 + len(v)), (5, 6), (7, 20), (50, 8242), (L - 300, L + 9000),
                         (L + 10, L + 20)):
                regs.append((k, a, b))
        tids = np.array([r[0] for r in regs], np.int32)
        starts = np.array([r[1] for r in regs], np.int64)
        ends = np.array([r[2] for r in regs], np.int64)
        full = [np.concatenate([np.zeros(100, np.int64), v, np.zeros(100, np.int64)]) for v in vecs]
        cols = [np.concatenate([full[t][a:b], np.zeros(max(0, b - max(a, len(full[t]))), np.int64)])
                .astype(np.float64) for t, a, b in regs]
        means = np.array([np.float64(c.sum()) / np.float64(len(c)) for c in cols])
        got = eng.np_sqdev(tids, starts, ends, means)
        for c, m, g in zip(cols, means, got):
            want = np_buffered_sum((c - m) * (c - m))
            assert g == want, (len(c), g, want)
        # every row through numpy_std (window forced open) equals np.std
        rows = eng.region_stats(tids, starts, ends)
        std = E.numpy_std(eng, rows, tids, starts, ends, rel=1.0)
        for c, row, s in zip(cols, rows, std):
            if c.max() != c.min():
                assert s == float(np.std(c))
            assert classic_stats(row, s) == classic_from_vector(c)
        with pytest.raises(Exception):
            eng.np_sqdev(tids[:1], starts[:1], starts[:1], means[:1])   # empty region
    finally:
        eng.close()


@pytest.mark.gpu
def test_engine_ties_match_reference(lib_built, ties):
    """The tie vectors as contigs of one batch: fused rows, then numpy_std
    (default window) reproduces every reference dict."""
    vecs = [_vec(c) for c in ties]
    eng = _engine_for(vecs)
    try:
        R = len(vecs)
        tids = np.arange(R, dtype=np.int32)
        starts = np.zeros(R, np.int64)
        ends = np.array([len(v) for v in vecs], np.int64)
        rows = eng.compute_depth_stats(tids, starts, ends)
        std = E.numpy_std(eng, rows, tids, starts, ends)
        assert not np.isnan(std).any()
        for c, row, s in zip(ties, rows, std):
            assert s == float.fromhex(c["np_std_hex"])
            assert classic_stats(row, s) == c["stats"]
    finally:
        eng.close()


def _tie_bam(path, ties):
    from metacov_amd import synth
    names, lengths, recs = [], [], []
    for k, c in enumerate(ties):
        v = _vec(c)
        names.append("t%d" % k)
        lengths.append(len(v))
        p, s = skyline_reads(v)
        recs += [synth.SynthRecord("r%d_%d" % (k, i), k, int(a), 0, [(0, int(b))], 0)
                 for i, (a, b) in enumerate(zip(p, s))]
    synth.write_bam(path, names, lengths, recs)
    return names


@pytest.mark.gpu
def test_classic_batch_and_cli_ties(lib_built, ties, tmp_path):
    """The product path end to end: a BAM of the tie vectors, decoded on the
    GPU; classic_batch and `metacov pileup` (whole contigs and CSV regions)
    give the reference's dicts / CSV values at every tie."""
    import csv
    from click.testing import CliRunner
    from metacov_amd import pileup
    from metacov_amd.cli import pileup as cli_pileup
    sub = ties[:12] + ties[-6:]
    bam = str(tmp_path / "ties.bam")
    names = _tie_bam(bam, sub)
    got = pileup.classic_batch(bam, [(nm, 0, c["n"]) for nm, c in zip(names, sub)])
    assert got == [c["stats"] for c in sub]
    pileup.close_all()
    rc = tmp_path / "r.csv"
    rc.write_text("sacc,sstart,send\n" + "".join("%s,0,%d\n" % (nm, c["n"]) for nm, c in zip(names, sub)))
    for extra in ([], ["-rc", str(rc)]):
        out = tmp_path / "o.csv"
        res = CliRunner().invoke(cli_pileup, ["-b", bam, "-o", str(out)] + extra)
        assert res.exit_code == 0, res.output
        rows = list(csv.DictReader(open(out, newline="")))
        assert len(rows) == len(sub)
        for r, c in zip(rows, sub):
            assert float(r["std"]) == c["stats"]["std"], (r, c["stats"])
            assert float(r["avg"]) == c["stats"]["avg"]


@pytest.mark.gpu
def test_capped_rows_carry_numpy_std(lib_built, monkeypatch):
    """apply_cap replaces the recomputed regions' numpy std with the capped
    batch's (window forced open so every row is recomputed)."""
    from metacov_amd import depthcap
    monkeypatch.setattr(E, "STD_TIE_REL", 1.0)
    L = 3000
    pos = np.concatenate([np.full(9000, 100, np.int32), np.arange(0, 2800, 7, dtype=np.int32)])
    span = np.concatenate([np.full(9000, 150, np.int32), np.full(400, 90, np.int32)])
    order = np.argsort(pos, kind="stable")
    pos, span = pos[order], span[order]
    tid = np.zeros(len(pos), np.int32)

    class Src:
        pass
    src = Src()
    src.tid, src.pos, src.span = tid, pos, span
    from metacov_amd.engine import CoverageEngine
    eng = CoverageEngine(0)
    try:
        eng.set_contigs([L])
        eng.add_reads(tid, pos, span)
        t, s, e = np.zeros(2, np.int32), np.array([0, 2000], np.int64), np.array([L, L], np.int64)
        rows = eng.compute_depth_stats(t, s, e)
        std = E.numpy_std(eng, rows, t, s, e)
        rows2, n_cap, dropped = depthcap.apply_cap(src, rows, t, s, e, [L], 8000, 0, std=std)
        assert n_cap == 1 and dropped > 0
        keep, _ = depthcap.cap_mask(tid, pos, span, 8000)
        d = np.zeros(L, np.int64)
        for p, q in zip(pos[keep], span[keep]):
            d[p:p + q] += 1
        assert classic_stats(rows2[0], std[0]) == classic_from_vector(d.astype(np.float64))
        assert std[0] == float(np.std(d.astype(np.float64)))
        assert not math.isnan(std[1])
    finally:
        eng.close()
