"""htslib's pileup read cap (pysam's max_depth, on by default): the library's closed form
(mc_depth_cap_mask, host C++) against a literal restatement of htslib's
bam_plp_push / bam_plp_next loop (oracle/htslib_plp.py), per region query
the way pysam's AlignmentFile.pileup(ref, start, end) runs it
(metacov/pileup.py:13).  Parity with htslib itself is unpinned (htslib is
absent here and the cap is version-dependent)."""
import os

import numpy as np
import pytest

from metacov_amd import depthcap
from oracle import htslib_plp


def kept_depth(pos, span, keep, start, end):
    """classic()'s column vector from the kept reads (difference array; a
    span-0 read adds nothing, as current htslib's bam_plp_push)."""
    d = np.zeros(end - start + 1, np.int64)
    for p, s in zip(pos[keep], span[keep]):
        a, b = max(p, start), min(p + s, end)
        if b > a:
            d[a - start] += 1
            d[b - start] -= 1
    return np.cumsum(d)[:-1]


def piles(rng, n_piles, pile_size, bg, L, span_rng):
    starts = [int(x) for x in rng.integers(0, L - 400, size=n_piles)]
    pos = [np.full(pile_size, s) for s in starts]
    pos.append(rng.integers(0, L - 200, size=bg))
    pos = np.concatenate(pos)
    span = rng.integers(span_rng[0], span_rng[1] + 1, size=len(pos))
    span = np.minimum(span, L - pos)
    o = np.argsort(pos, kind="stable")
    return pos[o].astype(np.int32), span[o].astype(np.int32)


@pytest.mark.parametrize("cap,n_piles,pile,bg,seed,smin", [
    (5, 20, 12, 300, 1, 1), (20, 10, 40, 500, 2, 1), (64, 6, 150, 2000, 3, 1), (3, 50, 6, 100, 4, 1),
    (1, 10, 5, 50, 5, 1), (5, 20, 12, 300, 6, 0), (20, 10, 40, 500, 7, 0), (3, 50, 6, 100, 8, 0),
    (2, 30, 9, 200, 9, 0)])
def test_cap_mask_matches_literal_htslib(cap, n_piles, pile, bg, seed, smin):
    """smin = 0: span-0 reads (no reference-consuming op) in the piles and the
    background, which enter the pool only as a start group's first read."""
    rng = np.random.default_rng(seed)
    L = 5000
    pos, span = piles(rng, n_piles, pile, bg, L, (smin, 300))
    if smin == 0:
        span[rng.random(len(span)) < 0.15] = 0
    tid = np.zeros(len(pos), np.int32)
    for (s, e) in [(0, L), (0, 1), (100, 2600), (2500, 4999), (1234, 1300)]:
        want, dropped = htslib_plp.region_depth(tid, pos, span, 0, s, e, max_depth=cap)
        idx = depthcap.region_reads(tid, pos, span, 0, s, e)
        keep, d2 = depthcap.cap_mask(tid[idx], pos[idx], span[idx], cap)
        assert d2 == dropped, (s, e)
        got = kept_depth(pos[idx], span[idx], keep, s, e)
        assert np.array_equal(got, want), (s, e)


def test_cap_8000_amplicon_piles():
    """Amplicon-like piles deeper than pysam's default cap: 3 starts with
    9000-12000 reads each over background coverage (> 8000x columns)."""
    rng = np.random.default_rng(11)
    L = 3000
    pos = np.concatenate([np.full(12_000, 500), np.full(9_000, 520), np.full(10_500, 1400),
                          rng.integers(0, 2800, size=4000)])
    span = np.concatenate([np.full(12_000, 150), rng.integers(100, 200, size=9_000),
                           np.full(10_500, 120), rng.integers(1, 200, size=4000)])
    o = np.argsort(pos, kind="stable")
    pos, span = pos[o].astype(np.int32), span[o].astype(np.int32)
    tid = np.zeros(len(pos), np.int32)
    want, dropped = htslib_plp.region_depth(tid, pos, span, 0, 0, L, max_depth=8000)
    keep, d2 = depthcap.cap_mask(tid, pos, span, 8000)
    assert dropped > 0 and d2 == dropped
    assert np.array_equal(kept_depth(pos, span, keep, 0, L), want)
    full = kept_depth(pos, span, np.ones(len(pos), bool), 0, L)
    assert full.max() > 8000 and want.max() < full.max()


def test_cap_mask_contigs_independent_and_errors():
    rng = np.random.default_rng(5)
    tid = np.repeat(np.arange(4, dtype=np.int32), 300)
    pos = np.concatenate([np.sort(rng.integers(0, 40, size=300)) for _ in range(4)]).astype(np.int32)
    span = rng.integers(1, 50, size=len(pos)).astype(np.int32)
    keep, _ = depthcap.cap_mask(tid, pos, span, 7, n_threads=3)
    for t in range(4):
        m = tid == t
        k1, _ = depthcap.cap_mask(tid[m], pos[m], span[m], 7, n_threads=1)
        assert np.array_equal(keep[m], k1)
    from metacov_amd._lib import MetacovError
    with pytest.raises(MetacovError):
        depthcap.cap_mask(np.zeros(2, np.int32), np.array([5, 3], np.int32), np.ones(2, np.int32), 7)
    with pytest.raises(MetacovError):
        depthcap.cap_mask(tid, pos, span, 0)


@pytest.mark.parametrize("seed", range(12))
def test_gate_never_misses_a_drop(seed):
    """depthcap.may_cap's bound: while 2 + 2 * (exact max depth of the region)
    <= max_depth, htslib's literal push/next loop drops nothing, so the
    exact row is the capped one.  Random piles sized around the bound, with
    span-0 reads and both end rules."""
    rng = np.random.default_rng(100 + seed)
    L = 600
    cap = int(rng.integers(4, 24))
    n = int(rng.integers(50, 400))
    pos = np.sort(np.concatenate([rng.integers(0, L - 50, size=n),
                                  np.full(int(rng.integers(0, cap)), int(rng.integers(0, L - 60)))]))
    span = rng.integers(0, 60, size=len(pos))
    span[rng.random(len(span)) < 0.2] = 0
    if seed % 2:
        span = np.maximum(span, 1)                      # legacy bam_endpos spans
    pos, span = pos.astype(np.int32), span.astype(np.int32)
    tid = np.zeros(len(pos), np.int32)
    checked = 0
    for _ in range(30):
        s = int(rng.integers(0, L - 1))
        e = int(rng.integers(s + 1, L + 20))
        exact = kept_depth(pos, span, np.ones(len(pos), bool), s, e)
        want, dropped = htslib_plp.region_depth(tid, pos, span, 0, s, e, max_depth=cap)
        if 2 + 2 * int(exact.max()) <= cap:
            checked += 1
            assert dropped == 0 and np.array_equal(want, exact), (s, e, cap)
        rows = np.zeros(1, dtype=[("max", np.int64)])
        rows["max"] = exact.max()
        assert depthcap.may_cap(rows, cap)[0] == (2 + 2 * int(exact.max()) > cap)


def test_zero_span_reads_and_the_pool():
    """A span-0 read that opens a start group occupies a pool node until its
    column, so a later read of the same group can be dropped because of it;
    one inside a group never joins the pool (bam_plp_push: tail->end > pos)."""
    pos = np.array([10, 10, 10, 10, 20, 20, 20], np.int32)
    span = np.array([0, 5, 5, 5, 5, 0, 5], np.int32)
    tid = np.zeros(len(pos), np.int32)
    for cap in (1, 2, 3, 4):
        want, dropped = htslib_plp.region_depth(tid, pos, span, 0, 0, 40, max_depth=cap)
        keep, d2 = depthcap.cap_mask(tid, pos, span, cap)
        assert d2 == dropped, cap
        assert np.array_equal(kept_depth(pos, span, keep, 0, 40), want), cap


# ---- the device walk (csrc/capmask.h) --------------------------------------

def _model_case(rng, cap, pile, bg, L, smin, inq_frac=0.0):
    pos, span = piles(rng, int(rng.integers(1, 12)), pile, bg, L, (smin, 300))
    if smin == 0:
        span[rng.random(len(span)) < 0.15] = 0
    inq = np.ones(len(pos), np.uint8)
    if inq_frac:
        inq[rng.random(len(pos)) < inq_frac] = 0
    return pos, span, inq


@pytest.mark.parametrize("seed", range(24))
def test_device_walk_model_matches_host_closed_form(seed):
    """tests/cap_model.py (cap_walk_kernel lane for lane: bulk chunks, groups
    in lane order, the ring of ends) against mc_depth_cap_mask on the reads
    of the query; reads outside the query are invisible to the walk and keep
    0; small rings take the wrap-around and gap paths."""
    from tests import cap_model
    rng = np.random.default_rng(100 + seed)
    cap = int(rng.choice([1, 2, 3, 5, 20, 64, 100, 300]))
    pile = int(rng.choice([3, 12, 40, 70, 150, 400]))
    pos, span, inq = _model_case(rng, cap, pile, int(rng.integers(0, 600)), 5000, int(rng.integers(0, 2)),
                                 inq_frac=0.2 if seed % 3 == 0 else 0.0)
    ring = int(rng.choice([512, 1024, 32768]))
    keep, out_span, dropped = cap_model.cap_walk(list(pos), list(span), list(inq), cap, int(span.max(initial=0)),
                                                 ring=ring)
    sel = np.nonzero(inq)[0]
    want, wd = depthcap.cap_mask(np.zeros(len(sel), np.int32), pos[sel], span[sel], cap)
    assert dropped == wd
    got = np.array(keep, bool)
    assert not got[inq == 0].any()
    assert np.array_equal(got[sel], want)
    assert np.array_equal(np.array(out_span), np.where(got, span, 0))


def test_device_walk_model_deep_pile():
    """A 20,000x pile at the 8000 cap: groups larger than a chunk, bulk
    stretches before and after."""
    from tests import cap_model
    rng = np.random.default_rng(9)
    pos = np.sort(np.concatenate([rng.integers(0, 3000, 600), rng.integers(1000, 1150, 20000)])).astype(np.int32)
    span = rng.integers(0, 200, len(pos)).astype(np.int32)
    keep, _, dropped = cap_model.cap_walk(list(pos), list(span), [1] * len(pos), 8000, 200)
    want, wd = depthcap.cap_mask(np.zeros(len(pos), np.int32), pos, span, 8000)
    assert dropped == wd > 0
    assert np.array_equal(np.array(keep, bool), want)


@pytest.mark.gpu
def test_device_cap_mask_matches_host(lib_built):
    """mc_depth_cap_mask_device against mc_depth_cap_mask and the literal
    htslib restatement: many queries (tids) in one call, span-0 reads,
    8000-cap amplicon piles, unsorted input refused."""
    import torch
    rng = np.random.default_rng(21)
    tids, poss, spans = [], [], []
    for t in range(40):
        cap_case = t % 4
        pos, span = piles(rng, int(rng.integers(1, 8)), [12, 60, 150, 2500][cap_case], int(rng.integers(0, 800)),
                          6000, (0 if t % 2 else 1, 300))
        if t % 2:
            span[rng.random(len(span)) < 0.15] = 0
        tids.append(np.full(len(pos), t, np.int32))
        poss.append(pos)
        spans.append(span)
    tid, pos, span = (np.concatenate(x) for x in (tids, poss, spans))
    for cap in (3, 40, 8000, 1):
        want, wd = depthcap.cap_mask(tid, pos, span, cap)
        got, gd = depthcap.cap_mask_device(*(torch.from_numpy(a).cuda() for a in (tid, pos, span)), cap)
        assert gd == wd
        assert np.array_equal(got.cpu().numpy().astype(bool), want)
    # one query against the literal pileup loop
    t0 = tid == 3
    idx = np.nonzero(t0)[0]
    got, gd = depthcap.cap_mask_device(*(torch.from_numpy(a[idx]).cuda() for a in (tid, pos, span)), 40)
    v, dropped = htslib_plp.region_depth(tid[idx], pos[idx], span[idx], 3, 0, 6000, max_depth=40)
    assert gd == dropped
    assert np.array_equal(kept_depth(pos[idx], span[idx], got.cpu().numpy().astype(bool), 0, 6000), v)
    bad = pos.copy()
    bad[5], bad[6] = bad[6] + 1, bad[5]
    with pytest.raises(Exception, match="sorted"):
        depthcap.cap_mask_device(*(torch.from_numpy(a).cuda() for a in (tid, bad, span)), 40)


@pytest.mark.gpu
def test_device_cap_mask_random_sets(lib_built):
    """Random query sets (1-30 contigs of random piles, background depth,
    span-0 share and cap from 1 to 9000): the device mask and drop count
    equal mc_depth_cap_mask's.  MC_CAP_SOAK_ITERS / MC_CAP_SOAK_SEED: soak
    runs (profiles/r06/r06soak_cap.txt)."""
    import torch
    rng = np.random.default_rng(int(os.environ.get("MC_CAP_SOAK_SEED", "77")))
    for _ in range(int(os.environ.get("MC_CAP_SOAK_ITERS", "4"))):
        tids, poss, spans = [], [], []
        for t in range(int(rng.integers(1, 31))):
            pos, span = piles(rng, int(rng.integers(1, 6)), int(rng.integers(5, 3000)), int(rng.integers(0, 400)),
                              int(rng.integers(800, 9000)), (int(rng.integers(0, 2)), int(rng.integers(2, 400))))
            span[rng.random(len(span)) < rng.random() * 0.3] = 0
            tids.append(np.full(len(pos), t, np.int32))
            poss.append(pos)
            spans.append(span)
        tid, pos, span = (np.concatenate(x) for x in (tids, poss, spans))
        cap = int(rng.choice([1, 2, 7, 50, 300, 2000, 8000, 9000]))
        want, wd = depthcap.cap_mask(tid, pos, span, cap)
        got, gd = depthcap.cap_mask_device(*(torch.from_numpy(a).cuda() for a in (tid, pos, span)), cap)
        assert gd == wd, cap
        assert np.array_equal(got.cpu().numpy().astype(bool), want), cap


@pytest.mark.gpu
def test_capped_rows_device_equals_host(lib_built, tmp_path):
    """capped_rows on a GPU decode (mc_add_reads_capped: gather, cap and
    batch in HBM) equals the host sweep on the same file's host decode, on
    8000-cap piles with span-0 reads, for regions that share a contig, start
    before / inside piles, run past the contig end, and on a contig shard."""
    from metacov_amd import synth
    from metacov_amd.bam import BamFile, GpuBamFile
    rng = np.random.default_rng(5)
    names, lengths, recs = ["a", "b", "c"], [6000, 3000, 9000], []
    for t, L in enumerate(lengths):
        pos, span = piles(rng, 3, [9000, 4100, 12000][t], 3000, L, (0, 300))
        span[rng.random(len(span)) < 0.05] = 0
        recs += [synth.SynthRecord("r%d_%d" % (t, i), t, int(p), 0, [(0, int(s))] if s else [(4, 20)], 0)
                 for i, (p, s) in enumerate(zip(pos, span))]
    bam = str(tmp_path / "deep.bam")
    synth.write_bam(bam, names, lengths, recs)
    regs = [(0, 0, 6000), (0, 1000, 2500), (2, 0, 9500), (1, 100, 2900), (2, 4000, 4100), (0, 5990, 6000)]
    t, s, e = (np.array([r[i] for r in regs], np.int64) for i in range(3))
    want, wd = depthcap.capped_rows(BamFile(bam), t, s, e, lengths)
    g = GpuBamFile(bam)
    got, gd = depthcap.capped_rows(g, t, s, e, lengths)
    assert gd == wd > 0
    assert np.array_equal(got, want)
    g.restrict([0, 2])
    sel = t != 1
    got2, gd2 = depthcap.capped_rows(g, t[sel], s[sel], e[sel], lengths)
    want2, wd2 = depthcap.capped_rows(BamFile(bam), t[sel], s[sel], e[sel], lengths)
    assert gd2 == wd2 and np.array_equal(got2, want2)
    g.close()


def _continuation_pile():
    """Start groups of 70 reads (longer than a 64-read chunk) whose tails are
    1 bp and span-0 reads, 3 positions apart, below the cap, then a pile
    at the cap: a bulk chunk must insert the open group's ends before it
    moves its pointer, or they linger and inflate the later pool count."""
    pos, span = [], []
    for s in range(0, 12000, 3):
        for j in range(70):
            pos.append(s)
            span.append((0 if j % 2 else 1) if j >= 60 else 1 + (j % 3))
    for j in range(400):
        pos.append(12100)
        span.append(50)
    return np.array(pos, np.int32), np.array(span, np.int32)


def test_device_walk_model_continuation_groups():
    from tests import cap_model
    pos, span = _continuation_pile()
    for cap in (120, 75, 300):
        keep, _, dropped = cap_model.cap_walk(list(pos), list(span), [1] * len(pos), cap, 3, ring=1024)
        want, wd = depthcap.cap_mask(np.zeros(len(pos), np.int32), pos, span, cap)
        assert dropped == wd and np.array_equal(np.array(keep, bool), want)


@pytest.mark.gpu
def test_device_cap_mask_continuation_groups(lib_built):
    import torch
    pos, span = _continuation_pile()
    tid = np.zeros(len(pos), np.int32)
    for cap in (120, 75, 300):
        want, wd = depthcap.cap_mask(tid, pos, span, cap)
        got, gd = depthcap.cap_mask_device(*(torch.from_numpy(a).cuda() for a in (tid, pos, span)), cap)
        assert gd == wd
        assert np.array_equal(got.cpu().numpy().astype(bool), want)
