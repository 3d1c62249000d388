"""pileup.experimental / load_kmerhist (reference metacov/pileup.py:29-173,
SURVEY.md §8 f).

Goldens (tests/golden/experimental.json) are the real reference function's
outputs (make_experimental_golden.py).  Bar: every field bit-exact with the
reference's value type (`covc` too: per-position sums in read order and
numpy's pairwise mean), except `ecor` / `cov3` (the reference's np.inner is a BLAS dot; the
GPU correlation sums in another order: the unrounded ecor*L agrees to
relative 1e-12, and the 3-decimal rounded values are equal unless the
reference's value lies within 1e-9 of a rounding tie).

CPU tests: the oracle against the goldens, the host read side (no FASTA) of
the product against the goldens and the oracle, load_kmerhist, the taps.
GPU tests: everything with a FASTA (the ecor kernel), the CLI's -k columns.
"""
import contextlib
import io
import math
import os

import numpy as np
import pytest

from oracle import experimental as ox
from metacov_amd import experimental as mx
from metacov_amd import synth

EXACT_FP = {}   # fields compared with a relative tolerance (none)
NEAR_TIE = ("ecor", "cov3")


@pytest.fixture(scope="module")
def gold(experimental_golden):
    return experimental_golden


def _same(key, want, got, tie_ok=False):
    if isinstance(want, float) and math.isnan(want):
        return isinstance(got, (float, np.floating)) and math.isnan(got)
    if key in EXACT_FP:
        return abs(got - want) <= EXACT_FP[key] * max(1.0, abs(want))
    if want == got:
        return True
    if tie_ok and key in NEAR_TIE:
        # a rounding tie the re-associated sum may fall either side of
        return abs(got - want) <= 1.0001e-3
    return False


def check_result(case, res, tie_ok=False):
    if "error" in case:
        assert res.error is not None, case["region"]
        assert type(res.error).__name__ == case["error"], (case["region"], res.error)
        return
    assert res.error is None, (case["region"], res.error)
    assert set(res.row) == set(case["row"])
    for key, want in case["row"].items():
        got = res.row[key]
        assert _same(key, want, got, tie_ok), (case["bam"], case["kcor"], case["region"], key,
                                               want, got)
        assert type(got).__name__ == case["types"][key], (key, type(got).__name__)
    assert res.zero_lines == case["stdout"].splitlines()


def _kcor(gold, case):
    return gold["kcor"][case["kcor"]] if case["kcor"] else None


# ------------------------------------------------------------------ CPU

def test_oracle_matches_reference_goldens(gold, golden_dir):
    """The restatement, run on duck-typed pysam objects, reproduces every
    golden exactly (values, types, printed lines, errors)."""
    bams, fastas = {}, {}
    for case in gold["cases"]:
        bam = bams.setdefault(case["bam"], ox.DuckBam(os.path.join(golden_dir, case["bam"])))
        fa = None
        if case["fasta"]:
            fa = fastas.setdefault(case["fasta"],
                                   ox.DuckFasta(os.path.join(golden_dir, case["fasta"])))
        buf = io.StringIO()
        try:
            with contextlib.redirect_stdout(buf):
                row = ox.experimental(bam, _kcor(gold, case), case["k"], fa, *case["region"])
            err = None
        except Exception as e:  # noqa: BLE001
            row, err = None, e
        res = mx.RegionResult(row=row, error=err, zero_lines=buf.getvalue().splitlines())
        check_result(case, res)


def test_read_side_matches_goldens(gold, golden_dir, lib_built):
    """Host C++ read pass (mc_experimental_reads) + the Python finish, for the
    cases without a FASTA (no GPU needed)."""
    n = 0
    for case in gold["cases"]:
        if case["fasta"]:
            continue
        res = mx.experimental_batch(os.path.join(golden_dir, case["bam"]), _kcor(gold, case),
                                    case["k"], None, [tuple(case["region"])])[0]
        check_result(case, res)
        n += 1
    assert n >= 10


def test_taps_equal_scipy():
    ref = ox.norm_taps()
    assert np.array_equal(mx.norm_taps(), ref)
    sps = pytest.importorskip("scipy.stats")
    assert np.array_equal(sps.norm(450, 150).pdf(range(0, 901)).ravel(), ref)


def test_load_kmerhist(tmp_path):
    csv = tmp_path / "k.csv"
    csv.write_text(
        "kmer,n0,n1,n2,R,Mapped\n"
        "AAAAAAA,4,2,6,R1,Mapped\n"
        "NNNNNNN,9,9,9,R1,Mapped\n"
        "CCCCCCC,3,1,2,R2,Mapped\n"
        "GGGGGGG,5,5,5,R1,Unmapped\n"
        "TTTTTTT,0,0,0,R2,Mapped\n"
        "ACGTACG,1,0,0,R1,Mapped\n")
    got = mx.load_kmerhist(str(csv))
    want = ox.load_kmerhist(str(csv))
    assert got[0].keys() == want[0].keys() and got[1].keys() == want[1].keys()
    assert got[0]["AAAAAAA"] == 4 / 4 and got[1]["CCCCCCC"] == 3 / 1.5
    assert "NNNNNNN" not in got[0] and "GGGGGGG" not in got[0]
    assert math.isnan(got[1]["TTTTTTT"]) and math.isinf(got[0]["ACGTACG"])
    # file objects, as the CLI passes them (cli.py:81)
    with open(csv) as fh:
        assert mx.load_kmerhist(fh)[1].keys() == got[1].keys()


def test_kmer_tables_drop_foreign_keys(caplog):
    t = mx.KmerTables([{"ACGT": 2.0, "ACG": 1.0, "ACNT": 3.0}, {"TTTT": 0.5}], 4)
    assert t.has.sum() == 2
    assert t.val[0, 0b00011011] == 2.0 and t.val[1, 255] == 0.5
    assert t.decode(0b00011011) == "ACGT"
    assert "dropped" in caplog.text


def _long_bam(path, seed, L=60_000, pairs=2_500):
    """One long contig, paired reads with real bases: regions longer than
    numpy's 8192-element reduction chunk, many starts and mates."""
    rng = np.random.default_rng(seed)
    ref = "".join(rng.choice(list("ACGT"), size=L))
    recs = []
    for q in range(pairs):
        rl = int(rng.integers(50, 150))
        p1 = int(rng.integers(0, L - rl))
        p2 = int(min(L - rl, p1 + rng.integers(0, 600)))
        for mate, (p, rev) in enumerate(((p1, False), (p2, True))):
            seq = ref[p:p + rl]
            if rng.random() < 0.05:
                seq = "N" + seq[1:]
            flag = 0x1 | (0x40 if mate == 0 else 0x80) | (0x10 if rev else 0)
            u = rng.random()
            flag |= 0x2 if u < 0.9 else (0x102 if u < 0.95 else 0)
            recs.append(synth.SynthRecord("p%d" % q, 0, p, flag, [(0, rl)], rl, seq))
    recs.sort(key=lambda r: r.pos)
    synth.write_bam(path, ["chr"], [L], recs)
    return ref


def test_read_side_long_regions_vs_oracle(tmp_path, lib_built):
    path = str(tmp_path / "long.bam")
    _long_bam(path, 5)
    k = 5
    rng = np.random.default_rng(6)
    keys = ["".join(p) for p in __import__("itertools").product("ACGT", repeat=k)]
    kc = [{x: float(rng.uniform(0.3, 3)) for x in keys if rng.random() < 0.8} for _ in range(2)]
    kc[0][keys[7]] = 0.0
    regions = [("chr", 0, 60_000), ("chr", 123, 41_000), ("chr", 8_191, 16_385),
               ("chr", 59_000, 70_000), ("chr", 30_000, 30_017)]
    bam = ox.DuckBam(path)
    with mx.ReadTable(path, k) as table:
        got = mx.experimental_batch(table, kc, k, None, regions)
    for (ref, s, e), res in zip(regions, got):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            want = ox.experimental(bam, kc, k, None, ref, s, e)
        case = {"row": {a: (float(b) if isinstance(b, np.floating) else b) for a, b in want.items()},
                "types": {a: type(b).__name__ for a, b in want.items()},
                "stdout": buf.getvalue(), "bam": "long", "kcor": "k5", "region": [ref, s, e]}
        check_result(case, res)


def test_read_table_threads_agree(tmp_path, lib_built, monkeypatch):
    """The record walk splits a window's placed records over threads (each
    with its own name arena): 1 and 8 threads, and many small windows, give
    the same results."""
    path = str(tmp_path / "many.bam")
    _long_bam(path, 9, L=200_000, pairs=20_000)
    k = 4
    rng = np.random.default_rng(3)
    keys = ["".join(p) for p in __import__("itertools").product("ACGT", repeat=k)]
    kc = [{x: float(rng.uniform(0.3, 3)) for x in keys} for _ in range(2)]
    regions = [("chr", 0, 200_000), ("chr", 50_000, 51_000), ("chr", 123_457, 190_001)]
    outs = []
    for nt, window in ((1, None), (8, None), (8, "65536")):
        # (a 64 KiB window: the file in ~40 windows, records cut at every
        # window end, each window inflated while the previous one is walked)
        if window:
            monkeypatch.setenv("MC_READS_WINDOW", window)
        with mx.ReadTable(path, k, nt) as table:
            res = mx.experimental_batch(table, kc, k, None, regions, n_threads=nt)
            outs.append([repr((r.row, r.error, r.zero_lines)) for r in res])
    assert outs[0] == outs[1] == outs[2]


def test_unsorted_bam_rejected(tmp_path, lib_built):
    from metacov_amd._lib import MetacovError
    path = str(tmp_path / "u.bam")
    synth.write_bam(path, ["c"], [1000], [
        synth.SynthRecord("a", 0, 500, 0x3, [(0, 10)], 10, "ACGTACGTAC"),
        synth.SynthRecord("b", 0, 100, 0x3, [(0, 10)], 10, "ACGTACGTAC")])
    with pytest.raises(MetacovError):
        mx.ReadTable(path, 4)


def _mixed_reads_bam(path, seed=11, n=12_000):
    """Placed records of every kind the read table distinguishes: soft and
    hard clips at both ends (query_alignment_sequence bounds), insertions at
    the end (getQueryEnd stops there), N bases, no SEQ, placed but unmapped
    (no CIGAR: reference_length None), CIGARs over 8 ops stored as CG:B,I
    tags, three contigs, and unplaced records at the end."""
    rng = np.random.default_rng(seed)
    lengths = [40_000, 25_000, 60_000]
    recs = []
    for i in range(n):
        tid = int(rng.integers(0, 3))
        u = rng.random()
        l = int(rng.integers(20, 120))
        if u < 0.04:                                   # placed, unmapped, no CIGAR
            cig, flag = [], 0x4
        elif u < 0.12:                                 # long CIGAR (CG tag)
            parts = [(0, 5)] * 10
            cig, l, flag = [(4, 3)] + parts + [(1, 2), (4, 4)], 3 + 50 + 2 + 4, 0x10
        else:
            a, b = int(rng.integers(0, 6)), int(rng.integers(0, 6))
            m = max(1, l - a - b)
            cig = ([(5, 2)] if rng.random() < 0.2 else []) + ([(4, a)] if a else []) + [(0, m)]
            cig += ([(1, 2)] if rng.random() < 0.1 else []) + ([(4, b)] if b else [])
            cig += [(5, 3)] if rng.random() < 0.2 else []
            l = sum(n_ for op, n_ in cig if op in (0, 1, 4))
            flag = int(rng.choice([0x1 | 0x2 | 0x40, 0x1 | 0x80 | 0x10, 0x100, 0]))
        seq = "".join(rng.choice(list("ACGTN"), size=l, p=[0.24, 0.24, 0.24, 0.24, 0.04]))
        if rng.random() < 0.03:
            l, seq = 0, None                           # no SEQ
        pos = int(rng.integers(0, lengths[tid] - 200))
        recs.append(synth.SynthRecord("q%d%s" % (i, "x" * int(rng.integers(0, 40))), tid, pos, flag, cig, l, seq))
    recs.sort(key=lambda r: (r.tid, r.pos))
    recs += [synth.SynthRecord("u%d" % j, -1, -1, 0x4, [], 30, "ACGT" * 7 + "AC") for j in range(40)]
    synth.write_bam(path, ["c0", "c1", "c2"], lengths, recs, long_cigar_threshold=8)


def test_read_table_fields(tmp_path, lib_built):
    path = str(tmp_path / "mixed.bam")
    _mixed_reads_bam(path, n=3000)
    with mx.ReadTable(path, 6) as t:
        f = t.fields()
        assert t.n_records == 3040 and t.n_placed == 3000
    assert len(f["name"]) == 3000 and all(nm.startswith(b"q") for nm in f["name"])
    assert f["first"][0] == 0 and f["first"][-1] == 3000 and np.all(np.diff(f["first"]) >= 0)
    assert np.all(f["end"] > f["pos"])
    assert np.all((f["bits"] & 2) == ((f["flag"] & 4) != 0) * 2)
    assert np.all(f["max_span"] >= 1)


def test_region_errors_without_gpu(golden_dir, lib_built):
    bam = os.path.join(golden_dir, "bbmap.sorted.bam")
    res = mx.experimental_batch(bam, [{}, {}], 7, None,
                                [("ref1", 5, 5), ("nope", 0, 10), ("ref1", 0, 300),
                                 ("ref1", 0, 10)])
    assert type(res[0].error) is Exception and str(res[0].error) == "Length must be > 0"
    assert isinstance(res[1].error, ValueError)
    assert res[2].error is None
    # every position of ref1[0:10] has a read start: nzef = 0, and without a
    # FASTA (ecor = -1, a Python int) cov3 divides a Python float by 0.0
    assert isinstance(res[3].error, ZeroDivisionError)
    with pytest.raises(ZeroDivisionError):
        ox.experimental(ox.DuckBam(bam), [{}, {}], 7, None, "ref1", 0, 10)
    with pytest.raises(Exception, match="Length must be > 0"):
        mx.experimental(bam, [{}, {}], 7, None, "ref1", 3, 3)


# ------------------------------------------------------------------ GPU

def _same_tables(a, b):
    for key in a:
        if isinstance(a[key], list):
            assert a[key] == b[key], key
        else:
            np.testing.assert_array_equal(a[key], b[key], err_msg=key)


@pytest.mark.gpu
@pytest.mark.parametrize("window", [None, "1048576"])
def test_read_table_gpu_decode_equals_host(golden_dir, tmp_path, lib_built, monkeypatch, window):
    """mc_reads_open_gpu (inflate + record walk on the GPU) gives the host
    walk's table field for field, on every golden BAM and on a mixed BAM
    (clips, CG-tag CIGARs, no SEQ, placed-unmapped, unplaced records), whole
    and in 1 MiB windows (records cut at window ends)."""
    mixed = str(tmp_path / "mixed.bam")
    _mixed_reads_bam(mixed)
    if window:
        monkeypatch.setenv("MC_READS_GPU_WINDOW", window)
    paths = [os.path.join(golden_dir, f) for f in sorted(os.listdir(golden_dir)) if f.endswith(".bam")]
    for path in paths + [mixed]:
        for k in (4, 7):
            with mx.ReadTable(path, k, decode="host") as h, mx.ReadTable(path, k, decode="gpu") as g:
                assert (h.references, h.lengths, h.n_records, h.n_placed) == \
                    (g.references, g.lengths, g.n_records, g.n_placed), path
                _same_tables(h.fields(), g.fields())


@pytest.mark.gpu
def test_read_table_gpu_decode_edge_files(tmp_path, lib_built):
    """Header-only and unplaced-only BAMs give the host walk's (empty) tables;
    a BAM cut inside a record is refused by both decodes."""
    from metacov_amd._lib import MetacovError
    empty, unpl, cut = (str(tmp_path / n) for n in ("empty.bam", "unplaced.bam", "cut.bam"))
    synth.write_bam(empty, ["c0", "c1"], [100, 200], [])
    synth.write_bam(unpl, ["c0"], [100], [synth.SynthRecord("u%d" % j, -1, -1, 0x4, [], 12, "ACGTACGTACGT")
                                          for j in range(50)])
    for path in (empty, unpl):
        with mx.ReadTable(path, 5, decode="host") as h, mx.ReadTable(path, 5, decode="gpu") as g:
            assert (h.references, h.lengths, h.n_records, h.n_placed) == \
                (g.references, g.lengths, g.n_records, g.n_placed)
            _same_tables(h.fields(), g.fields())
    _mixed_reads_bam(cut, n=400)
    import gzip
    raw = gzip.decompress(open(cut, "rb").read())
    with open(cut, "wb") as fh:              # the same stream re-blocked, cut mid-record
        fh.write(synth._bgzf(raw[:len(raw) - 37]))
    for decode in ("host", "gpu"):
        with pytest.raises(MetacovError):
            mx.ReadTable(cut, 5, decode=decode)


@pytest.mark.gpu
def test_read_table_gpu_contig_subset(tmp_path, lib_built, golden_dir):
    """A rank's read table (contigs=[...]): only those contigs' BGZF blocks
    decoded, located by the BAI or by a whole-file decode's extents table;
    its records are the host table's records of those contigs."""
    from metacov_amd.bam import GpuBamFile, build_index
    mixed = str(tmp_path / "mixed.bam")
    _mixed_reads_bam(mixed, n=30_000)
    multi = str(tmp_path / "multi.bam")
    import shutil
    shutil.copy(os.path.join(golden_dir, "synth_multi.bam"), multi)
    for path in (mixed, multi):
        build_index(path)
        with mx.ReadTable(path, 6, decode="host") as h:
            fh, first = h.fields(), None
            n_ref = len(h.references)
        first = fh["first"]
        with GpuBamFile(path) as whole:
            ext = whole.extents()
        for sel in ([0], [n_ref - 1], list(range(0, n_ref, 2)), []):
            for extents in (None, ext):
                with mx.ReadTable(path, 6, decode="gpu", contigs=sel, extents=extents) as g:
                    fg = g.fields()
                keep = np.zeros(len(fh["pos"]), bool)
                for t in sel:
                    keep[first[t]:first[t + 1]] = True
                for key in ("pos", "end", "flag", "bits", "kmer"):
                    np.testing.assert_array_equal(fh[key][keep], fg[key], err_msg=key)
                assert [nm for nm, k in zip(fh["name"], keep) if k] == fg["name"]
                for t in range(n_ref):
                    want = first[t + 1] - first[t] if t in sel else 0
                    assert fg["first"][t + 1] - fg["first"][t] == want
                    if t in sel:
                        assert fg["max_span"][t] == fh["max_span"][t]


@pytest.mark.gpu
def test_read_table_gpu_unsorted_rejected(tmp_path, lib_built):
    from metacov_amd._lib import MetacovError
    path = str(tmp_path / "u.bam")
    synth.write_bam(path, ["c"], [1000], [
        synth.SynthRecord("a", 0, 500, 0x3, [(0, 10)], 10, "ACGTACGTAC"),
        synth.SynthRecord("b", 0, 100, 0x3, [(0, 10)], 10, "ACGTACGTAC")])
    with pytest.raises(MetacovError, match="coordinate-sorted"):
        mx.ReadTable(path, 4, decode="gpu")


@pytest.mark.gpu
def test_goldens_with_fasta_gpu(gold, golden_dir, lib_built):
    """Every golden case through the product, FASTA cases on the GPU kernel."""
    reads = {}
    for case in gold["cases"]:
        key = (case["bam"], case["k"])
        if key not in reads:
            reads[key] = mx.ReadTable(os.path.join(golden_dir, case["bam"]), case["k"])
        fasta = os.path.join(golden_dir, case["fasta"]) if case["fasta"] else None
        res = mx.experimental_batch(reads[key], _kcor(gold, case), case["k"], fasta,
                                    [tuple(case["region"])])[0]
        check_result(case, res, tie_ok=True)
    for r in reads.values():
        r.close()


@pytest.mark.gpu
def test_goldens_batched_gpu(gold, golden_dir, lib_built):
    """All regions of one (bam, fasta, k_cor) in one batch: same rows."""
    groups = {}
    for case in gold["cases"]:
        groups.setdefault((case["bam"], case["fasta"], case["kcor"], case["k"]), []).append(case)
    for (bam, fasta, kc, k), cases in groups.items():
        got = mx.experimental_batch(os.path.join(golden_dir, bam),
                                    gold["kcor"][kc] if kc else None, k,
                                    os.path.join(golden_dir, fasta) if fasta else None,
                                    [tuple(c["region"]) for c in cases])
        for case, res in zip(cases, got):
            check_result(case, res, tie_ok=True)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 4, 7, 11])
def test_ecor_kernel_vs_oracle_gpu(k, lib_built, tmp_path):
    """mc_ecor_run against the oracle's per-position arrays (np.inner) on
    random sequence with lower case and N runs, multi-tile regions, regions
    cut short by the sequence end and a table with zero / inf weights."""
    rng = np.random.default_rng(100 + k)
    seqs = []
    for L in (70_000, 5_000, 900, 3):
        s = rng.choice(list("ACGTacgtN"), size=L, p=[.22, .22, .22, .22, .02, .02, .02, .02, .04])
        seqs.append("".join(s))
    fa = tmp_path / "r.fa"
    fa.write_text("".join(">s%d extra\n%s\n" % (i, s) for i, s in enumerate(seqs)))
    n = 4 ** k
    vals = [rng.uniform(0.2, 3.0, size=n) for _ in range(2)]
    for v in vals:
        v[rng.random(n) < 0.2] = 0.0
    vals[1][rng.integers(0, n)] = np.inf if k == 4 else vals[1][0]
    codes = ["".join(p) for p in __import__("itertools").product("ACGT", repeat=k)] if k <= 7 \
        else None
    if codes is None:    # large k: keep a random subset of keys
        idx = rng.choice(n, size=5000, replace=False)
        to_s = lambda c: "".join("ACGT"[(c >> (2 * (k - 1 - m))) & 3] for m in range(k))  # noqa: E731
        kc = [{to_s(int(c)): float(v[c]) for c in idx} for v in vals]
    else:
        kc = [{codes[c]: float(v[c]) for c in range(n)} for v in vals]
    fasta = mx.FastaFile(str(fa))
    regions = [("s0", 0, 70_000), ("s0", 10, 2058), ("s0", 4095, 4096 + 2048 * 3 + 5),
               ("s0", 69_500, 71_000), ("s1", 0, 5000), ("s1", 4990, 6000), ("s2", 0, 900),
               ("s3", 0, 3), ("s3", 5, 50), ("s0", 3, 4)]
    tables = mx.KmerTables(kc, k)
    eng = mx.EcorEngine(0)
    eng.set_sequence(fasta)
    eng.set_tables(tables)
    spans = [fasta.span(*r) for r in regions]
    inner, gc, at = eng.run([s[0] for s in spans], [s[1] for s in spans],
                            [r[2] - r[1] for r in regions])
    eng.close()
    for q, (ref, s, e) in enumerate(regions):
        region = fasta.fetch(ref, s, e).upper()
        want = ox.raw_ecor(kc, k, region, e - s)
        if np.isnan(want):
            assert np.isnan(inner[q])
        else:
            assert abs(inner[q] - want) <= 1e-12 * max(1.0, abs(want)), (ref, s, e, inner[q], want)
        assert gc[q] == region.count("G") + region.count("C")
        assert at[q] == region.count("A") + region.count("T")


@pytest.mark.gpu
def test_cli_kmer_histogram_gpu(golden_dir, fixture_golden, lib_built, tmp_path):
    """`metacov pileup -k H -f F`: classic + experimental columns per region
    (cli.py:81, :93-108), against the reference's classic goldens and the
    oracle's experimental on the same k_cor."""
    import csv as _csv
    from click.testing import CliRunner
    from metacov_amd.cli import pileup as cli_pileup
    rng = np.random.default_rng(11)
    keys = ["".join(p) for p in __import__("itertools").product("ACGT", repeat=7)]
    rows = ["kmer,n0,n1,n2,R,Mapped"]
    for r in ("R1", "R2"):
        for x in keys:
            if rng.random() < 0.7:
                rows.append("%s,%d,%d,%d,%s,Mapped" % (x, rng.integers(1, 50), rng.integers(1, 50),
                                                       rng.integers(1, 50), r))
    rows.append("NNNNNNN,1,1,1,R1,Mapped")
    hist = tmp_path / "k.csv"
    hist.write_text("\n".join(rows) + "\n")
    fasta = _indexable_fasta(golden_dir, tmp_path)
    bam = os.path.join(golden_dir, "bbmap.sorted.bam")
    out = tmp_path / "o.csv"
    res = CliRunner().invoke(cli_pileup, ["-b", bam, "-rb", os.path.join(golden_dir, "regions.blast7"),
                                          "-k", str(hist), "-f", fasta, "-o", str(out)])
    assert res.exit_code == 0, res.output
    got = list(_csv.DictReader(open(out, newline="")))
    kc = ox.load_kmerhist(str(hist))
    obam, ofa = ox.DuckBam(bam), ox.DuckFasta(fasta)
    b7 = fixture_golden["blast7"]
    assert len(got) == len(b7)
    assert list(got[0].keys()) == ["sacc", "start", "end"] + sorted(
        list(b7[0]["stats"]) + ["cov", "covc", "den", "denc", "cov2", "cf", "ambig", "improper",
                                "nzef", "gc", "ecor", "wnf", "cov3"])
    for g, w in zip(got, b7):
        for key, v in w["stats"].items():
            assert g[key] == str(v), key
        s, e = sorted((int(w["start"]), int(w["end"])))
        want = ox.experimental(obam, kc, 7, ofa, w["sacc"], s, e)
        for key, v in want.items():
            if key in ("covc", "ecor", "cov3"):
                assert abs(float(g[key]) - float(v)) <= 1.0001e-3 * max(1.0, abs(float(v))), key
            else:
                assert g[key] == str(v), (key, g[key], v)


def _indexable_fasta(golden_dir, tmp_path):
    """The reference's FASTA fixture as pysam.FastaFile (cli.py:59) can open
    it: the fixture is plain gzip and its ref2 starts with a 65-base line
    (faidx refuses both), so the same sequences go in re-wrapped at 70."""
    fasta = str(tmp_path / "reference_1K.fa")
    src = mx.FastaFile(os.path.join(golden_dir, "reference_1K.fa.gz"))
    with open(fasta, "w") as fh:
        for name, L in zip(src.references, src.lengths):
            seq = src.fetch(name, 0, L)
            fh.write(">%s\n" % name + "".join(seq[i:i + 70] + "\n" for i in range(0, L, 70)))
    mx.check_faidx(fasta)
    return fasta


@pytest.mark.gpu
@pytest.mark.parametrize("indexed", [True, False])
def test_cli_kmer_histogram_two_ranks(golden_dir, lib_built, tmp_path, indexed):
    """`metacov pileup -k` under torch.distributed.run with 2 ranks: each rank
    computes the experimental columns of the regions on its own contigs (its
    read table decoded from those contigs' BGZF blocks, found by the BAI or
    by rank 0's extents table) and rank 0 gathers them with the region table;
    the CSV equals one process's byte for byte (gloo: both ranks share the
    box's one GPU)."""
    import socket
    import subprocess
    import sys
    from click.testing import CliRunner
    from metacov_amd.cli import pileup as cli_pileup
    rng = np.random.default_rng(12)
    keys = ["".join(p) for p in __import__("itertools").product("ACGT", repeat=7)]
    rows = ["kmer,n0,n1,n2,R,Mapped"]
    for r in ("R1", "R2"):
        for x in keys:
            if rng.random() < 0.7:
                rows.append("%s,%d,%d,%d,%s,Mapped" % (x, rng.integers(1, 50), rng.integers(1, 50),
                                                       rng.integers(1, 50), r))
    hist = tmp_path / "k.csv"
    hist.write_text("\n".join(rows) + "\n")
    fasta = _indexable_fasta(golden_dir, tmp_path)
    bam = os.path.join(golden_dir, "bbmap.sorted.bam")
    if not indexed:
        import shutil
        bam = shutil.copy(bam, str(tmp_path / "noindex.bam"))
    args = ["-b", bam, "-rb", os.path.join(golden_dir, "regions.blast7"), "-k", str(hist), "-f", fasta]
    one = tmp_path / "one.csv"
    res = CliRunner().invoke(cli_pileup, args + ["-o", str(one)])
    assert res.exit_code == 0, res.output
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    two = tmp_path / "two.csv"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MC_DIST_BACKEND="gloo",
               PYTHONPATH=os.pathsep.join([root, os.environ.get("PYTHONPATH", "")]))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=%d" % port, "-m", "metacov_amd.cli", "pileup",
           *args, "-o", str(two)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    assert open(two, newline="").read() == open(one, newline="").read()


def test_check_faidx_follows_pysam_open(tmp_path):
    """`pileup -f` opens the reference like pysam.FastaFile (cli.py:59):
    plain and BGZF FASTA with equal-length lines open; plain gzip, ragged
    lines inside a sequence and text before the first header fail."""
    import gzip as _gz
    import subprocess
    ok = tmp_path / "ok.fa"
    ok.write_text(">a desc\nACGTACGT\nACGTACGT\nACG\n>b\nAC\n")
    mx.check_faidx(str(ok))
    crlf = tmp_path / "crlf.fa"
    crlf.write_bytes(b">a\r\nACGT\r\nAC\r\n")
    mx.check_faidx(str(crlf))
    gz = tmp_path / "plain.fa.gz"
    gz.write_bytes(_gz.compress(ok.read_bytes()))
    with pytest.raises(OSError, match="bgzip"):
        mx.check_faidx(str(gz))
    from metacov_amd import synth
    bg = tmp_path / "bg.fa.gz"
    bg.write_bytes(synth._bgzf(ok.read_bytes()))
    mx.check_faidx(str(bg))
    for bad in (">a\nACGT\nAC\nACGT\n", ">a\nACG\nACGTA\n", "ACGT\n>a\nAC\n", ">a\nACGT\n\nACGT\n"):
        f = tmp_path / "bad.fa"
        f.write_text(bad)
        with pytest.raises(OSError):
            mx.check_faidx(str(f))
    # an existing index is taken as it is (htslib fai_load), whatever the lines
    (tmp_path / "bad.fa.fai").write_text("a\t6\t3\t4\t5\n")
    mx.check_faidx(str(tmp_path / "bad.fa"))


def _faidx_lines(data):
    """The per-line form of faidx's build checks (the first failing line's
    message, or None), against which check_faidx's array form is fuzzed."""
    name, width, short = None, None, False
    for no, line in enumerate(data.split(b"\n"), 1):
        line = line.rstrip(b"\r")
        if line.startswith(b">"):
            name, width, short = line[1:].split()[0].decode() if line[1:].split() else "", None, False
            continue
        if not line:
            if name is not None:
                short = short or width is not None
            continue
        if name is None:
            return "Format error, unexpected \"%s\" at line %d" % (chr(line[0]), no)
        if short or (width is not None and len(line) > width):
            return "Different line length in sequence '%s'" % name
        if width is None:
            width = len(line)
        elif len(line) < width:
            short = True
    return None


def test_check_faidx_fuzz(tmp_path):
    rng = np.random.default_rng(4)
    f = tmp_path / "r.fa"
    kinds = 0
    for it in range(400):
        parts = []
        if rng.random() < 0.1:
            parts.append(b"AC")
        for s in range(int(rng.integers(0, 4))):
            parts.append(b">s%d x" % s if rng.random() < 0.9 else b">")
            w = int(rng.integers(1, 9))
            for k in range(int(rng.integers(0, 5))):
                r = rng.random()
                ln = w if r < 0.7 else int(rng.integers(0, 2 * w + 1))
                parts.append(b"A" * ln + (b"\r" if rng.random() < 0.1 else b""))
        data = b"\n".join(parts) + (b"\n" if rng.random() < 0.7 else b"")
        f.write_bytes(data)
        want = _faidx_lines(data)
        if want is None:
            mx.check_faidx(str(f))
        else:
            kinds += 1
            with pytest.raises(OSError) as e:
                mx.check_faidx(str(f))
            assert str(e.value).endswith(want), (data, want, str(e.value))
    assert 50 < kinds < 350


def test_cli_rejects_unopenable_fasta_without_k(lib_built, golden_dir, tmp_path):
    """Without -k the reference still opens -f (cli.py:59): a plain-gzip
    FASTA fails before any row is written."""
    from click.testing import CliRunner
    from metacov_amd.cli import pileup as cli_pileup
    out = tmp_path / "o.csv"
    res = CliRunner().invoke(cli_pileup, ["-b", os.path.join(golden_dir, "bbmap.sorted.bam"),
                                          "-f", os.path.join(golden_dir, "reference_1K.fa.gz"),
                                          "-o", str(out)])
    assert res.exit_code != 0 and isinstance(res.exception, OSError)
    assert not out.exists() or out.read_text() == ""


def _dup_names_bam(path, seed=13, L=30_000, n=6_000):
    """Names repeated 1-5 times (supplementary-like copies), some across
    strands and contigs: the reference's dict pairs occurrences 1-2, 3-4,
    ... of a name in read order, and a region query sees only its reads."""
    rng = np.random.default_rng(seed)
    ref = "".join(rng.choice(list("ACGT"), size=L))
    recs = []
    for q in range(n // 3):
        for c in range(int(rng.integers(1, 6))):
            tid = int(rng.integers(0, 2))
            rl = int(rng.integers(30, 120))
            p = int(rng.integers(0, L - rl))
            flag = 0x1 | 0x2 | (0x40 if c % 2 == 0 else 0x80) | (0x10 if rng.random() < 0.5 else 0)
            if rng.random() < 0.05:
                flag |= 0x100
            recs.append(synth.SynthRecord("d%d" % q, tid, p, flag, [(0, rl)], rl, ref[p:p + rl]))
    recs.sort(key=lambda r: (r.tid, r.pos))
    synth.write_bam(path, ["a", "b"], [L, L], recs)


@pytest.mark.gpu
def test_device_read_pass_equals_host_pass(tmp_path, lib_built, monkeypatch):
    """The read pass on the device (exp_gpu.hip, the GPU decode's table in
    HBM) against the host pass over the same table (MC_EXP_READS=host):
    rows, errors and "RCOR is ZERO" lines identical, for k_cor with zeros,
    NaN and missing keys, k_cor None (the pair error), reads without SEQ or
    reference length (errors after and before events), duplicate names,
    regions past the contig end, one position long, and whole contigs."""
    import itertools
    paths = {"long": str(tmp_path / "long.bam"), "mixed": str(tmp_path / "mixed.bam"),
             "dup": str(tmp_path / "dup.bam")}
    _long_bam(paths["long"], 21, L=70_000, pairs=8_000)
    _mixed_reads_bam(paths["mixed"], n=8_000)
    _dup_names_bam(paths["dup"])
    rng = np.random.default_rng(8)
    for k in (4, 6):
        keys = ["".join(p) for p in itertools.product("ACGT", repeat=k)]
        kc = [{x: float(rng.uniform(0.3, 3)) for x in keys if rng.random() < 0.85} for _ in range(2)]
        kc[0][keys[5]] = 0.0
        kc[1][keys[9]] = 0.0
        kc[1][keys[11]] = float("nan")
        ones = [{x: 1.0 for x in keys}, {x: 1.0 for x in keys}]
        for name, path in paths.items():
            with mx.ReadTable(path, k, decode="gpu") as t:
                refs, lens = t.references, t.lengths
                regions = []
                for ref, L in zip(refs, lens):
                    regions += [(ref, 0, L), (ref, 1234, 9000), (ref, 8191, 8192 * 3 + 5), (ref, L - 500, L + 800),
                                (ref, 17, 18), (ref, 5000, 5001 + 8192)]
                for kcor in (kc, ones, None):
                    outs = []
                    for mode in ("gpu", "host"):
                        if mode == "host":
                            monkeypatch.setenv("MC_EXP_READS", "host")
                        else:
                            monkeypatch.delenv("MC_EXP_READS", raising=False)
                        res = mx.experimental_batch(t, kcor, k, None, regions)
                        outs.append([(r.row, repr(r.error), r.zero_lines) for r in res])
                    monkeypatch.delenv("MC_EXP_READS", raising=False)
                    for a, b, reg in zip(outs[0], outs[1], regions):
                        assert repr(a) == repr(b), (name, k, kcor is None, reg)
                # the device pass keeps its buffers with the table: region sets
                # that shrink and grow between calls on it
                for sub in (regions[:2], regions, regions[3:5], regions[::-1]):
                    outs = []
                    for mode in ("gpu", "host"):
                        if mode == "host":
                            monkeypatch.setenv("MC_EXP_READS", "host")
                        else:
                            monkeypatch.delenv("MC_EXP_READS", raising=False)
                        res = mx.experimental_batch(t, kc, k, None, sub)
                        outs.append([(r.row, repr(r.error), r.zero_lines) for r in res])
                    monkeypatch.delenv("MC_EXP_READS", raising=False)
                    assert repr(outs[0]) == repr(outs[1]), (name, k, len(sub))
