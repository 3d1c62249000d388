"""`metacov scan` (reference metacov/cli.py:112-285, metacov/scan.pyx,
metacov/pyfq.pyx; SURVEY.md §8 f ranks 3-4).

Pinned: the FASTQ readers (the oracle's, the product's Python pyfq mirror
and the C++ batch source the GPU path reads through) against the known
answers of the reference's tests/test_pyfq.py (tests/golden/pyfq.json).
Histograms: parity unpinned beyond oracle/scan.py, the line-by-line
restatement of scan.pyx (the Cython cannot be built here: SURVEY.md §8 c);
the GPU path must reproduce its CSV files byte for byte.  Bar: bit-exact
(integer histograms).
"""
import ctypes
import gzip
import os

import numpy as np
import pytest
from click.testing import CliRunner

from oracle import bamread
from oracle import scan as oscan
from metacov_amd import synth


@pytest.fixture(scope="module")
def pyfq_golden(golden_dir):
    import json
    with open(os.path.join(golden_dir, "pyfq.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def mix(tmp_path_factory):
    d = tmp_path_factory.mktemp("scanmix")
    names, lengths, recs, fasta = synth.scan_mix()
    bam = str(d / "mix.bam")
    synth.write_bam(bam, names, lengths, recs)
    fa = str(d / "mix.fa")
    synth.write_fasta(fa, fasta)
    return bam, fa


def _paths(golden_dir, files):
    return [os.path.join(golden_dir, f) for f in files]


# ------------------------------------------------------------ FASTQ (pinned)

def _hist(reads):
    lengths, freq, n = [0] * 11, [0] * 5, 0
    for rlen, seq in reads:
        lengths[int(rlen / 10)] += 1
        for b in seq:
            freq[b] += 1
        n += 1
    return lengths, freq, n


def test_oracle_fastq_matches_reference_known_answers(pyfq_golden, golden_dir):
    for case in pyfq_golden["cases"]:
        paths = _paths(golden_dir, case["files"])
        f = oscan.FastQFile(*paths) if len(paths) == 1 else oscan.FastQFilePair(*paths)
        assert f.size == case["size_kb"]
        lengths, freq, _ = _hist((r.rlen, r.seq) for r in f.reads())
        assert lengths == case["lengths_by_10"]
        assert freq == case["base_freq"]


def test_pyfq_matches_reference_known_answers(pyfq_golden, golden_dir):
    """reference tests/test_pyfq.py:12-45 against metacov_amd.pyfq."""
    from metacov_amd import pyfq
    for case in pyfq_golden["cases"]:
        paths = _paths(golden_dir, case["files"])
        fq = pyfq.FastQFile(*paths) if len(paths) == 1 else pyfq.FastQFilePair(*paths)
        with fq as infile:
            assert infile.size == case["size_kb"]
            assert infile.pos == 0
            lengths, freq = [0] * 11, [0] * 5
            for read in infile:
                lengths[int(read.rlen / 10)] += 1
                assert read.pos <= infile.size
                for base in read.seq:
                    assert 0 <= base < 5
                    freq[base] += 1
        assert freq == case["base_freq"]
        assert lengths == case["lengths_by_10"]


def test_pyfq_writer_round_trip(pyfq_golden, golden_dir, tmp_path):
    """reference tests/test_pyfq.py:48-64."""
    from metacov_amd import pyfq
    src = os.path.join(golden_dir, "ecoli_1K_1.fq.gz")
    out = str(tmp_path / "out.fq.gz")
    n1 = 0
    with pyfq.FastQFile(src) as infile, pyfq.FastQWriter(out) as outfile:
        for read in infile:
            outfile.write(read)
            n1 += 1
    n2 = 0
    with pyfq.FastQFile(out) as a, pyfq.FastQFile(src) as b:
        for r1, r2 in zip(a, b):
            assert r1.rlen == r2.rlen and r1.seq == r2.seq
            n2 += 1
    assert n1 == n2 == pyfq_golden["writer_records"]


def _src_batches(lib, h, cap=997):
    from metacov_amd import _lib
    P = ctypes.c_void_p
    while True:
        n = ctypes.c_int64()
        _lib.check(lib.mc_scan_src_next(h, cap, 1 << 20, ctypes.byref(n)), lib)
        if n.value == 0:
            return
        ptrs = [P() for _ in range(7)]
        nb = ctypes.c_int64()
        _lib.check(lib.mc_scan_src_batch(h, *[ctypes.byref(p) for p in ptrs], ctypes.byref(nb)), lib)
        k = n.value

        def arr(p, dt, m):
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(dt)), shape=(m,)).copy() \
                if m else np.zeros(0, np.dtype(dt))
        cols = [arr(ptrs[i], ctypes.c_int32, k) for i in range(5)]
        off = arr(ptrs[5], ctypes.c_int64, k + 1)
        seq = arr(ptrs[6], ctypes.c_uint8, nb.value)
        yield cols, off, seq


def _unpack(seq, off, rlen):
    nib = np.empty(2 * len(seq), np.uint8)
    nib[0::2] = seq >> 4
    nib[1::2] = seq & 15
    t = np.array(oscan.NT16_NT4, np.uint8)
    return [t[nib[2 * off[i]:2 * off[i] + rlen[i]]] for i in range(len(rlen))]


def test_cpp_fastq_source_matches_reference_known_answers(pyfq_golden, golden_dir, lib_built):
    from metacov_amd import _lib
    lib = _lib.load()
    for case in pyfq_golden["cases"]:
        paths = _paths(golden_dir, case["files"])
        h = ctypes.c_void_p()
        _lib.check(lib.mc_scan_src_open_fastq(paths[0].encode(),
                                              paths[1].encode() if len(paths) > 1 else None,
                                              ctypes.byref(h)), lib)
        try:
            reads, flags = [], []
            for (rlen, flag, gpos, gisize, tid), off, seq in _src_batches(lib, h):
                assert (gpos == -1).all() and (gisize == -1).all() and (tid == -1).all()
                flags += flag.tolist()
                reads += list(zip(rlen.tolist(), _unpack(seq, off, rlen)))
        finally:
            lib.mc_scan_src_close(h)
        lengths, freq, n = _hist(reads)
        assert lengths == case["lengths_by_10"]
        assert freq == case["base_freq"]
        if len(paths) == 2:   # FastQFilePair: second file first
            assert flags[:4] == [0x81, 0x41, 0x81, 0x41]
        else:
            assert set(flags) == {0}
        # record by record against the oracle iterator
        want = list(oscan.fastq_reads(*paths))
        assert [(r.rlen, list(r.seq), r.flags) for r in want] == \
               [(a, list(s), f) for (a, s), f in zip(reads, flags)]


def test_cpp_fastq_source_truncated_and_plain(tmp_path, lib_built):
    """A file ending inside a record ends the stream (pyfq.pyx:166-175); the
    last quality line may lack its newline; plain files read as-is."""
    from metacov_amd import _lib
    lib = _lib.load()
    text = b"@a\nACGTN\n+\nIIIII\n@b\nacgtx\n+\nIIIII"   # no final newline
    for name, data in (("t.fq", text), ("t2.fq", text + b"\n@c\nAC\n+\n")):
        p = tmp_path / name
        p.write_bytes(data)
        h = ctypes.c_void_p()
        _lib.check(lib.mc_scan_src_open_fastq(str(p).encode(), None, ctypes.byref(h)), lib)
        got = []
        for (rlen, *_), off, seq in _src_batches(lib, h):
            got += [(int(a), s.tolist()) for a, s in zip(rlen, _unpack(seq, off, rlen))]
        lib.mc_scan_src_close(h)
        assert got == [(6, [0, 1, 2, 3, 4, 4]), (6, [0, 1, 2, 3, 4, 4])]
        want = [(r.rlen, r.seq) for r in oscan.fastq_reads(str(p))]
        assert got == want


@pytest.mark.parametrize("window", [None, "4096", "65536"])
def test_cpp_bam_source_matches_oracle(mix, golden_dir, lib_built, window, monkeypatch):
    """Every record in file order, with the ReadIterator accessor values; with
    small windows (MC_SCAN_WINDOW) records straddle windows, each window is
    inflated while the previous one is walked, and a 4 KiB window is smaller
    than some headers (the unfinished header carried over)."""
    from metacov_amd import _lib
    if window:
        monkeypatch.setenv("MC_SCAN_WINDOW", window)
    lib = _lib.load()
    for path in (mix[0], os.path.join(golden_dir, "bbmap.sorted.bam"),
                 os.path.join(golden_dir, "synth_edge.bam")):
        _names, _lengths, recs = bamread.read_bam(path)
        h = ctypes.c_void_p()
        _lib.check(lib.mc_scan_src_open_bam(path.encode(), 2, ctypes.byref(h)), lib)
        rows = []
        for (rlen, flag, gpos, gisize, tid), off, seq in _src_batches(lib, h, cap=301):
            codes = []
            for i in range(len(rlen)):
                b = seq[off[i]:off[i + 1]]
                nib = np.empty(2 * len(b), np.uint8)
                nib[0::2], nib[1::2] = b >> 4, b & 15
                codes.append("".join(bamread.NT16[c] for c in nib[:rlen[i]]))
            rows += list(zip(rlen.tolist(), flag.tolist(), gpos.tolist(), gisize.tolist(),
                             tid.tolist(), codes))
        n = ctypes.c_int64()
        lib.mc_scan_src_records(h, ctypes.byref(n))
        lib.mc_scan_src_close(h)
        assert n.value == len(recs)
        want = [(r.l_seq, r.flag, r.pos + r.l_seq if r.flag & 0x10 else r.pos,
                 r.tlen if r.flag & 2 else 0, r.tid, r.seq) for r in recs]
        assert rows == want


def _source_rows(lib, h):
    rows = []
    for (rlen, flag, gpos, gisize, tid), off, seq in _src_batches(lib, h, cap=301):
        codes = []
        for i in range(len(rlen)):
            b = seq[off[i]:off[i + 1]]
            nib = np.empty(2 * len(b), np.uint8)
            nib[0::2], nib[1::2] = b >> 4, b & 15
            codes.append("".join(bamread.NT16[c] for c in nib[:rlen[i]]))
        rows += list(zip(rlen.tolist(), flag.tolist(), gpos.tolist(), gisize.tolist(),
                         tid.tolist(), codes))
    return rows


def test_cpp_sam_source_matches_bam_source(mix, golden_dir, lib_built, tmp_path):
    """SAM text (`metacov scan x.sam`, cli.py:171-173: pysam reads it like a
    BAM) gives the records of the BAM it was converted from: the same
    accessor values and bases, plain and gzip-compressed; pysam's content
    detection picks SAM or BAM whatever the file name."""
    from metacov_amd import _lib, scan as mscan
    from tests.sam_convert import bam_to_sam
    lib = _lib.load()
    for k, path in enumerate((mix[0], os.path.join(golden_dir, "bbmap.sorted.bam"),
                              os.path.join(golden_dir, "synth_edge.bam"))):
        names, lengths, recs = bamread.read_bam(path)
        want = [(r.l_seq, r.flag, r.pos + r.l_seq if r.flag & 0x10 else r.pos,
                 r.tlen if r.flag & 2 else 0, r.tid, r.seq) for r in recs]
        for gz in (False, True):
            sam = bam_to_sam(path, str(tmp_path / ("s%d%s.sam" % (k, ".gz" if gz else ""))), gz)
            assert mscan.is_sam(sam) and not mscan.is_sam(path)
            h = ctypes.c_void_p()
            _lib.check(lib.mc_scan_src_open_sam(sam.encode(), ctypes.byref(h)), lib)
            nt = ctypes.c_int32()
            lib.mc_scan_src_n_targets(h, ctypes.byref(nt))
            assert nt.value == len(names)
            rows = _source_rows(lib, h)
            n = ctypes.c_int64()
            lib.mc_scan_src_records(h, ctypes.byref(n))
            lib.mc_scan_src_close(h)
            assert n.value == len(recs) and rows == want


def test_cpp_sam_source_errors(tmp_path, lib_built):
    from metacov_amd import _lib
    lib = _lib.load()
    head = "@SQ\tSN:a\tLN:100\n"
    good = "r1\t0\ta\t5\t60\t4M\t*\t0\t0\tACGT\t*\n"
    for body, msg in ((good.replace("\ta\t", "\tzz\t"), "not in the header"),
                      ("r1\t0\ta\t5\n", "11 fields"),
                      (good.replace("\t5\t", "\tx5\t"), "bad number"),
                      (good + "@SQ\tSN:b\tLN:5\n", "header line after")):
        p = tmp_path / "bad.sam"
        p.write_text(head + body)
        h = ctypes.c_void_p()
        _lib.check(lib.mc_scan_src_open_sam(str(p).encode(), ctypes.byref(h)), lib)
        n = ctypes.c_int64()
        rc = lib.mc_scan_src_next(h, 100, 1 << 20, ctypes.byref(n))
        lib.mc_scan_src_close(h)
        assert rc != 0 and msg in lib.mc_last_error().decode()


# ----------------------------------------------------- processors (no GPU)

def test_byflag_rows_layout():
    """ByFlag.get_rows: header + group columns in reverse -g order, groups
    in bit order (scan.pyx:395-405) -- same rows as the oracle's."""
    from metacov_amd import scan as mscan
    pf = [mscan.Flags["Mapped"], mscan.Flags["Readdir"]]
    of = [oscan.Flags["Mapped"], oscan.Flags["Readdir"]]
    m = mscan.ByFlag([mscan.MirrorHist(4, 3), mscan.IsizeHist()], pf)
    o = oscan.ByFlag([oscan.MirrorHist(4, 3), oscan.IsizeHist()], of)
    rng = np.random.default_rng(0)
    for g in range(4):
        c = rng.integers(0, 9, (4, 2)).astype(np.uint32)
        m.processors[g].processors[0]._add(c)
        o.processors[g].processors[0].counts = c.tolist()
        isz = rng.integers(0, 5, 9).astype(np.uint32)
        m.processors[g].processors[1]._add(isz, 3 + g)
        o.processors[g].processors[1].counts = dict(enumerate(isz.tolist()))
        o.processors[g].processors[1].max_isize = 3 + g
    for i in range(2):
        got = [[str(v) for v in row] for row in m.get_rows(i)]
        want = [[str(v) for v in row] for row in o.get_rows(i)]
        assert got == want
    assert got[0] == ["n", "count", "Readdir", "Mapped"]
    assert got[1][-2:] == ["Forward", "Mapped"]


@pytest.mark.parametrize("args,msg", [
    (["x.txt", "-o", "o.csv"], "Couldn't guess input format"),
    (["a.bam", "b.bam", "-o", "o.csv"], "Multiple input files only supported for fastq"),
    (["a.fq", "b.fq", "c.fq", "-o", "o.csv"], "At most two fastq files allowed"),
])
def test_cli_scan_usage_errors(tmp_path, args, msg):
    from metacov_amd.cli import scan
    with CliRunner().isolated_filesystem(temp_dir=tmp_path):
        r = CliRunner().invoke(scan, args)
    assert r.exit_code == 2 and msg in r.output


def test_cli_scan_fasta_with_fastq_rejected(tmp_path, golden_dir):
    from metacov_amd.cli import scan
    fq = os.path.join(golden_dir, "ecoli_1K_1.fq.gz")
    fa = tmp_path / "r.fa"
    fa.write_text(">x\nACGT\n")
    r = CliRunner().invoke(scan, [fq, "-f", str(fa), "-o", str(tmp_path / "o.csv")])
    assert r.exit_code == 2
    assert "Reference fasta can only be used with mapped (bam/sam) reads" in r.output


# ----------------------------------------------------------- GPU parity

def _cli_scan(tmp_path, readfile, out, extra=()):
    from metacov_amd.cli import scan
    files = {"base": "-b", "kmer": "-o", "mirror": "-M", "isize": "-I"}
    args = list(readfile)
    for name in out:
        args += [files[name], str(tmp_path / (name + ".csv"))]
    r = CliRunner().invoke(scan, args + list(extra))
    assert r.exit_code == 0, (r.output, r.exception)
    texts = {}
    for name in out:
        with open(tmp_path / (name + ".csv"), newline="") as fh:
            texts[name] = fh.read()
    return texts


def _oracle_kwargs(extra):
    kw, it = {}, iter(extra)
    keys = {"-f": "fasta", "-bo": "boffset", "-k": "k", "-n": "number", "-s": "step",
            "-O": "offset", "-MO": "mirror_offset", "-Ml": "mirror_length", "-m": "max_reads"}
    groups = []
    for a in it:
        v = next(it)
        if a == "-g":
            groups.append(v)
        else:
            kw[keys[a]] = v if a == "-f" else int(v)
    kw["group_by"] = groups
    return kw


ALL = ("base", "kmer", "mirror", "isize")

BAM_CASES = [
    ("bbmap", ALL, ("-f", "@fa")),
    ("bbmap", ("base", "kmer"), ()),                                   # no FASTA
    ("bbmap", ALL, ("-f", "@fa", "-g", "Mapped", "-g", "Readdir", "-bo", "5")),
    ("mix", ALL, ("-f", "@mixfa")),
    ("mix", ALL, ("-f", "@mixfa", "-g", "IsRead1", "-g", "PairedProperly", "-g", "Readdir",
                  "-bo", "7", "-k", "3", "-n", "5", "-s", "2", "-O", "-3", "-MO", "-2",
                  "-Ml", "6")),
    ("mix", ("kmer", "isize"), ("-k", "9", "-n", "3", "-s", "40", "-O", "2")),
    ("mix", ("mirror", "base"), ("-f", "@mixfa", "-MO", "30", "-Ml", "3", "-m", "300")),
    # 6 flags -> 64 groups: BaseHist no longer fits in LDS (global atomics)
    ("mix", ("base", "isize"), ("-f", "@mixfa", "-g", "Paired", "-g", "PairedProperly",
                                "-g", "Mapped", "-g", "Readdir", "-g", "IsRead1",
                                "-g", "MateReaddir")),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(BAM_CASES)))
def test_scan_bam_cli_vs_oracle_gpu(case, mix, golden_dir, lib_built, tmp_path):
    which, out, extra = BAM_CASES[case]
    bam = mix[0] if which == "mix" else os.path.join(golden_dir, "bbmap.sorted.bam")
    subst = {"@fa": os.path.join(golden_dir, "reference_1K.fa.gz"), "@mixfa": mix[1]}
    extra = [subst.get(a, a) for a in extra]
    got = _cli_scan(tmp_path, [bam], out, extra)
    want = oscan.scan_csv([bam], out, **_oracle_kwargs(extra))
    for name in out:
        assert got[name] == want[name], name


@pytest.mark.gpu
@pytest.mark.parametrize("case", [0, 3, 4])
def test_scan_sam_cli_vs_bam_and_oracle_gpu(case, mix, golden_dir, lib_built, tmp_path):
    """`metacov scan x.sam` (the SAM conversion of the BAM) writes the CSV
    bytes of the BAM run and of the oracle (oracle/scan.py on the BAM)."""
    from tests.sam_convert import bam_to_sam
    which, out, extra = BAM_CASES[case]
    bam = mix[0] if which == "mix" else os.path.join(golden_dir, "bbmap.sorted.bam")
    subst = {"@fa": os.path.join(golden_dir, "reference_1K.fa.gz"), "@mixfa": mix[1]}
    extra = [subst.get(a, a) for a in extra]
    sam = bam_to_sam(bam, str(tmp_path / "x.sam"))
    (tmp_path / "sam").mkdir()
    (tmp_path / "bam").mkdir()
    got = _cli_scan(tmp_path / "sam", [sam], out, extra)
    from_bam = _cli_scan(tmp_path / "bam", [bam], out, extra)
    want = oscan.scan_csv([bam], out, **_oracle_kwargs(extra))
    for name in out:
        assert got[name] == from_bam[name] == want[name], name


FQ_CASES = [
    (["ecoli_1K_1.fq.gz"], ("kmer", "base"), ()),                       # reference test_scan
    (["ecoli_1K_2.fq.gz"], ALL, ("-k", "5", "-n", "12", "-s", "8", "-O", "1")),
    (["ecoli_1K_1.fq.gz", "ecoli_1K_2.fq.gz"], ("kmer", "isize"), ("-g", "IsRead1")),
    (["ecoli_1K_1.fq.gz", "ecoli_1K_2.fq.gz"], ("kmer", "mirror"), ("-m", "777", "-g", "IsRead2",
                                                                    "-g", "Paired")),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(FQ_CASES)))
def test_scan_fastq_cli_vs_oracle_gpu(case, golden_dir, lib_built, tmp_path):
    files, out, extra = FQ_CASES[case]
    paths = _paths(golden_dir, files)
    got = _cli_scan(tmp_path, paths, out, extra)
    want = oscan.scan_csv(paths, out, **_oracle_kwargs(extra))
    for name in out:
        assert got[name] == want[name], name


@pytest.mark.gpu
def test_scan_reads_api_accumulates_gpu(mix, lib_built):
    """scan_reads twice into the same counters: counts add up, BaseHist is
    cut back to 50 + start_pos rows at each call's set_max_readlen(50)."""
    from metacov_amd import scan as mscan
    bam, fa = mix
    m = mscan.ByFlag([mscan.BaseHist(2), mscan.KmerHist(4, 3, 5, 1), mscan.IsizeHist()],
                     [mscan.Flags["Readdir"]])
    o = oscan.ByFlag([oscan.BaseHist(2), oscan.KmerHist(4, 3, 5, 1), oscan.IsizeHist()],
                     [oscan.Flags["Readdir"]])
    fasta = oscan.read_fasta(fa)
    for maxreads in (0, 50):
        assert mscan.scan_reads(bam, fa, m, maxreads=maxreads) == \
               oscan.scan_reads(oscan.bam_reads(bam, fasta), o, maxreads)
    for i in range(3):
        assert [[str(v) for v in r] for r in m.get_rows(i)] == \
               [[str(v) for v in r] for r in o.get_rows(i)]


@pytest.mark.gpu
def test_scan_large_isize_and_long_reads_gpu(tmp_path, lib_built):
    """Insert sizes beyond the LDS arena (global IsizeHist) and 20 kbp reads
    (BaseHist rows beyond the arena), against the oracle."""
    rng = np.random.default_rng(3)
    L = 60000
    ref = "".join(np.array(list("ACGT"))[rng.integers(0, 4, L)])
    recs = []
    for i in range(40):
        rl = int(rng.integers(15000, 20000)) if i < 6 else 120
        pos = int(rng.integers(0, L - rl))
        recs.append(synth.SynthRecord("q%d" % i, 0, pos, 0x3 | (0x10 if i % 3 else 0),
                                      [(0, rl)], rl, seq=ref[pos:pos + rl],
                                      tlen=int(rng.integers(-90000, 90000))))
    recs.sort(key=lambda r: r.pos)
    bam = str(tmp_path / "long.bam")
    synth.write_bam(bam, ["big"], [L], recs)
    fa = str(tmp_path / "big.fa")
    synth.write_fasta(fa, {"big": ref})
    got = _cli_scan(tmp_path, [bam], ("base", "isize", "mirror"), ["-f", fa, "-bo", "3"])
    want = oscan.scan_csv([bam], ("base", "isize", "mirror"), fasta=fa, boffset=3)
    assert got == want


@pytest.mark.gpu
def test_scan_kernel_device_batch_gpu(lib_built):
    """mc_scan_add_batch_device (the bench path, 4-byte aligned read starts)
    equals mc_scan_add_batch on a tightly packed batch (repacked on the
    host)."""
    import torch
    from metacov_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(5)
    n = 5000
    rlen = rng.integers(0, 200, n).astype(np.int32)
    nbytes = (rlen + 1) // 2
    off = np.zeros(n + 1, np.int64)            # tight: the host path repacks it
    off[1:] = np.cumsum(nbytes)
    seq = rng.integers(0, 256, int(off[-1])).astype(np.uint8)
    aoff = np.zeros(n + 1, np.int64)           # 4-byte aligned starts (device path contract)
    aoff[1:] = np.cumsum((nbytes + 3) // 4 * 4)
    aseq = np.zeros(int(aoff[-1]), np.uint8)
    for i in range(n):
        aseq[aoff[i]:aoff[i] + nbytes[i]] = seq[off[i]:off[i + 1]]
    flag = rng.integers(0, 0x800, n).astype(np.int32)
    gpos = rng.integers(-5, 3000, n).astype(np.int32)
    gis = rng.integers(-900, 900, n).astype(np.int32)
    rid = rng.integers(-1, 2, n).astype(np.int32)
    refs = rng.choice(list(b"ACGTNacgt"), 5000).astype(np.uint8)
    roff = np.array([0, 2500], np.int64)
    rlen_ref = np.array([2500, 2500], np.int64)
    cfg = _lib.ScanConfig()
    cfg.n_flags = 2
    cfg.flags[0], cfg.flags[1] = 0x10, 0x40
    cfg.base_on, cfg.base_start = 1, 4
    cfg.kmer_on, cfg.kmer_k, cfg.kmer_nk, cfg.kmer_step, cfg.kmer_offset = 1, 6, 9, 5, 2
    cfg.mirror_on, cfg.mirror_offset, cfg.mirror_n = 1, 4, 10
    cfg.isize_on = 1
    outs = []
    for mode in ("host", "device"):
        h = ctypes.c_void_p()
        _lib.check(lib.mc_scan_create(0, ctypes.byref(cfg), ctypes.byref(h)), lib)
        _lib.check(lib.mc_scan_set_reference(h, 2, _lib.ptr(roff), _lib.ptr(rlen_ref), refs.size,
                                             _lib.ptr(refs)), lib)
        arrs = [rlen, flag, gpos, gis, rid, off, seq] if mode == "host" else \
            [rlen, flag, gpos, gis, rid, aoff, aseq]
        if mode == "host":
            _lib.check(lib.mc_scan_add_batch(h, n, *[_lib.ptr(a) for a in arrs]), lib)
        else:
            dev = [torch.from_numpy(a).cuda() for a in arrs]
            ms = ctypes.c_float()
            _lib.check(lib.mc_scan_add_batch_device(h, n, *[ctypes.c_void_p(t.data_ptr()) for t in dev],
                                                    int(rlen.max()), int(np.abs(gis).max()),
                                                    ctypes.byref(ms)), lib)
            assert ms.value > 0
        G, rows, cap = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
        lib.mc_scan_dims(h, ctypes.byref(G), ctypes.byref(rows), ctypes.byref(cap), None, None)
        base = np.zeros((4, rows.value, 5), np.uint32)
        kmer = np.zeros((4, 4 ** 6 + 1, 9), np.uint32)
        mir = np.zeros((4, 11, 2), np.uint32)
        isz = np.zeros((4, cap.value), np.uint32)
        mx = np.zeros(4, np.int32)
        _lib.check(lib.mc_scan_results(h, *[_lib.ptr(a) for a in (base, kmer, mir, isz, mx)]), lib)
        lib.mc_scan_destroy(h)
        outs.append((base, kmer, mir, isz, mx))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    assert outs[0][0].sum() > 0 and outs[0][1].sum() > 0 and outs[0][3].sum() == n


def _mix_batch(lib, bam, fasta_path):
    """The whole BAM as one SoA batch through the C++ source, with ref_id
    forward-filled as mc_scan_run does; plus the FASTA as nt4."""
    from metacov_amd import _lib
    from metacov_amd.experimental import FastaFile
    fa = FastaFile(fasta_path)
    h = ctypes.c_void_p()
    _lib.check(lib.mc_scan_src_open_bam(bam.encode(), 1, ctypes.byref(h)), lib)
    names = []
    nt = ctypes.c_int32()
    lib.mc_scan_src_n_targets(h, ctypes.byref(nt))
    for t in range(nt.value):
        nm = ctypes.c_char_p()
        lib.mc_scan_src_target(h, t, ctypes.byref(nm), None)
        names.append(nm.value.decode())
    parts = list(_src_batches(lib, h, cap=10 ** 7))
    lib.mc_scan_src_close(h)
    (rlen, flag, gpos, gisize, tid), off, seq = parts[0]
    tmap = np.array([fa._index.get(n, -1) for n in names], np.int32)
    rid, last = np.empty_like(tid), -1
    for i, t in enumerate(tid):
        if t >= 0 and tmap[t] >= 0:
            last = tmap[t]
        rid[i] = last
    t4 = np.full(256, 4, np.uint8)
    for ch, v in zip(b"ACGTacgt", (0, 1, 2, 3, 0, 1, 2, 3)):
        t4[ch] = v
    ref = t4[np.asarray(fa.buffer)]
    return [rlen, flag, gpos, gisize, rid, off, seq], ref, np.asarray(fa._off, np.int64), \
        np.asarray(fa.lengths, np.int64)


def test_c_port_matches_python_oracle(mix, lib_built):
    """The two restatements (oracle/scan.py per read, oracle/scan_oracle.c
    over the C++ source's batch) agree: the C port is the bench's CPU
    baseline and the GPU check at scale."""
    from metacov_amd import _lib
    from oracle import coracle
    lib = _lib.load()
    bam, fa = mix
    batch, ref, roff, rlen_ref = _mix_batch(lib, bam, fa)
    cfg = _lib.ScanConfig()
    cfg.n_flags = 2
    cfg.flags[0], cfg.flags[1] = 0x40, 0x10
    cfg.base_on, cfg.base_start = 1, 3
    cfg.kmer_on, cfg.kmer_k, cfg.kmer_nk, cfg.kmer_step, cfg.kmer_offset = 1, 4, 6, 3, -2
    cfg.mirror_on, cfg.mirror_offset, cfg.mirror_n = 1, 4, 10
    cfg.isize_on = 1
    rows = max(50, int(batch[0].max())) + 3
    (base, kmer, mirror, isize, isize_max), done = coracle.scan(cfg, batch, ref, roff, rlen_ref,
                                                               rows, 1024)
    o = oscan.ByFlag([oscan.BaseHist(3), oscan.KmerHist(4, 6, 3, -2), oscan.MirrorHist(4, 10),
                      oscan.IsizeHist()], [oscan.Flags["IsRead1"], oscan.Flags["Readdir"]])
    assert oscan.scan_reads(oscan.bam_reads(bam, oscan.read_fasta(fa)), o) == done
    for g in range(4):
        b, k, m, i = o.processors[g].processors
        assert np.array_equal(base[g], np.array(b.counts, np.uint32))
        assert np.array_equal(kmer[g], np.array(k.counts, np.uint32))
        assert np.array_equal(mirror[g], np.array(m.counts, np.uint32))
        assert isize_max[g] == i.max_isize
        assert all(isize[g][a] == c for a, c in i.counts.items())
        assert isize[g].sum() == sum(i.counts.values())


@pytest.mark.gpu
def test_scan_kernel_vs_c_port_gpu(mix, lib_built):
    """mc_scan_add_batch on the mix BAM's batch equals the C port."""
    from metacov_amd import _lib
    from oracle import coracle
    lib = _lib.load()
    bam, fa = mix
    batch, ref, roff, rlen_ref = _mix_batch(lib, bam, fa)
    for nflags, flags in ((0, ()), (3, (0x2, 0x10, 0x80))):
        cfg = _lib.ScanConfig()
        cfg.n_flags = nflags
        for i, f in enumerate(flags):
            cfg.flags[i] = f
        cfg.base_on, cfg.base_start = 1, 11
        cfg.kmer_on, cfg.kmer_k, cfg.kmer_nk, cfg.kmer_step, cfg.kmer_offset = 1, 7, 8, 7, 0
        cfg.mirror_on, cfg.mirror_offset, cfg.mirror_n = 1, -3, 25
        cfg.isize_on = 1
        h = ctypes.c_void_p()
        _lib.check(lib.mc_scan_create(0, ctypes.byref(cfg), ctypes.byref(h)), lib)
        from metacov_amd.experimental import FastaFile
        f = FastaFile(fa)
        buf = np.ascontiguousarray(f.buffer)
        _lib.check(lib.mc_scan_set_reference(h, len(rlen_ref), _lib.ptr(roff), _lib.ptr(rlen_ref),
                                             buf.size, _lib.ptr(buf)), lib)
        _lib.check(lib.mc_scan_add_batch(h, len(batch[0]), *[_lib.ptr(a) for a in batch]), lib)
        G, rows, cap = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
        lib.mc_scan_dims(h, ctypes.byref(G), ctypes.byref(rows), ctypes.byref(cap), None, None)
        got = (np.zeros((G.value, rows.value, 5), np.uint32),
               np.zeros((G.value, 4 ** 7 + 1, 8), np.uint32),
               np.zeros((G.value, 26, 2), np.uint32), np.zeros((G.value, cap.value), np.uint32),
               np.zeros(G.value, np.int32))
        _lib.check(lib.mc_scan_results(h, *[_lib.ptr(x) for x in got]), lib)
        lib.mc_scan_destroy(h)
        want, _ = coracle.scan(cfg, batch, ref, roff, rlen_ref, rows.value, cap.value)
        for a, b in zip(got, want):
            assert np.array_equal(a, b)


@pytest.mark.gpu
def test_scan_kernel_queue_and_cuts_vs_c_port_gpu(lib_built):
    """A batch large enough for the slice queue, sorted like a coordinate-
    sorted BAM, on a dense and a sparse contig (batches cut at the reference
    window), with odd / even / > 256-base reads on both strands and two
    groups: equal to the C port."""
    from metacov_amd import _lib
    from oracle import coracle
    lib = _lib.load()
    rng = np.random.default_rng(17)
    lens_ref = np.array([300_000, 2_000_000, 40_000], np.int64)
    counts = [250_000, 45_000, 60_000]
    roff = np.zeros(3, np.int64)
    roff[1:] = np.cumsum(lens_ref)[:-1]
    ref_ascii = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(lens_ref.sum()))].copy()
    ref_ascii[rng.random(ref_ascii.size) < 0.001] = ord("N")
    choices = np.array([36, 75, 100, 101, 150, 151, 251, 300], np.int32)
    p = np.array([0.05, 0.1, 0.1, 0.1, 0.3, 0.3, 0.04, 0.01])
    rlen, flag, gpos, rid = [], [], [], []
    for t, (L, c) in enumerate(zip(lens_ref, counts)):
        rl = rng.choice(choices, size=c, p=p)
        pos = np.sort(rng.integers(0, int(L) - 301, c))
        rev = rng.random(c) < 0.5
        rlen.append(rl)
        flag.append((0x1 | np.where(rng.random(c) < 0.5, 0x40, 0x80) | (rng.random(c) < 0.9) * 0x2 |
                     rev * 0x10).astype(np.int32))
        gpos.append((pos + rev * rl).astype(np.int32))
        rid.append(np.full(c, t, np.int32))
    rlen, flag, gpos, rid = (np.concatenate(x) for x in (rlen, flag, gpos, rid))
    n = rlen.size
    gisize = np.where(flag & 0x2, rng.integers(-900, 900, n), 0).astype(np.int32)
    code = np.zeros(256, np.uint8)
    for ch, v in zip(b"ACGTN", (1, 2, 4, 8, 15)):
        code[ch] = v
    nbytes = (rlen + 1) // 2
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(nbytes)
    seq = np.zeros(int(off[-1]), np.uint8)
    start = roff[rid] + np.where(flag & 0x10, gpos - rlen, gpos)
    for i in range(0, n, 50_000):   # bases from the reference, 1 % substitutions, some random reads
        j = np.arange(i, min(n, i + 50_000))
        for L in np.unique(rlen[j]):
            sel = j[rlen[j] == L]
            b = code[ref_ascii[start[sel, None] + np.arange(L)[None, :]]]
            mut = rng.random(b.shape) < 0.01
            b = np.where(mut, np.array([1, 2, 4, 8, 3], np.uint8)[rng.integers(0, 5, b.shape)], b)
            junk = rng.random(sel.size) < 0.05
            b[junk] = np.array([1, 2, 4, 8], np.uint8)[rng.integers(0, 4, (int(junk.sum()), int(L)))]
            if L % 2:
                b = np.concatenate([b, np.zeros((b.shape[0], 1), np.uint8)], axis=1)
            packed = (b[:, 0::2] << 4) | b[:, 1::2]
            for k, r in enumerate(sel):
                seq[off[r]:off[r + 1]] = packed[k]
    t4 = np.full(256, 4, np.uint8)
    for ch, v in zip(b"ACGT", (0, 1, 2, 3)):
        t4[ch] = v
    batch = [rlen, flag, gpos, gisize, rid, off, seq]
    cfg = _lib.ScanConfig()
    cfg.n_flags = 1
    cfg.flags[0] = 0x80
    cfg.base_on, cfg.base_start = 1, 3
    cfg.kmer_on, cfg.kmer_k, cfg.kmer_nk, cfg.kmer_step, cfg.kmer_offset = 1, 7, 8, 7, 0
    cfg.mirror_on, cfg.mirror_offset, cfg.mirror_n = 1, 4, 10
    cfg.isize_on = 1
    h = ctypes.c_void_p()
    _lib.check(lib.mc_scan_create(0, ctypes.byref(cfg), ctypes.byref(h)), lib)
    _lib.check(lib.mc_scan_set_reference(h, 3, _lib.ptr(roff), _lib.ptr(lens_ref), ref_ascii.size,
                                         _lib.ptr(ref_ascii)), lib)
    _lib.check(lib.mc_scan_add_batch(h, n, *[_lib.ptr(a) for a in batch]), lib)
    G, rows, cap = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
    lib.mc_scan_dims(h, ctypes.byref(G), ctypes.byref(rows), ctypes.byref(cap), None, None)
    got = (np.zeros((G.value, rows.value, 5), np.uint32), np.zeros((G.value, 4 ** 7 + 1, 8), np.uint32),
           np.zeros((G.value, 11, 2), np.uint32), np.zeros((G.value, cap.value), np.uint32),
           np.zeros(G.value, np.int32))
    _lib.check(lib.mc_scan_results(h, *[_lib.ptr(x) for x in got]), lib)
    lib.mc_scan_destroy(h)
    want, done = coracle.scan(cfg, batch, t4[ref_ascii], roff, lens_ref, rows.value, cap.value)
    assert done == n
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    assert got[0][:, :, :4].sum() > 0.5 * (rlen.sum())   # most reads passed BaseHist's test


@pytest.mark.gpu
def test_kmer_codes_vs_c_port_gpu(lib_built):
    """KmerHist alone over reads of random nt16 nibbles (mostly A/C/G/T, some
    N and invalid codes), both strands, 1-300 bases plus two reads longer
    than the LDS stage (the global-memory path), under k-mer geometries that
    take the 8-base-window codes (K <= 8, every base inside the read: odd and
    even first bases, windows ending in the read's last dword) and the
    base-by-base loop (K > 8, a negative offset, K > STEP running past the
    read): equal to the C port in every bin."""
    from metacov_amd import _lib
    from oracle import coracle
    lib = _lib.load()
    rng = np.random.default_rng(29)
    rlen = np.concatenate([rng.integers(1, 301, 6000), [12001, 15000]]).astype(np.int32)
    n = rlen.size
    flag = np.where(rng.random(n) < 0.5, 0x10, 0).astype(np.int32) | np.where(rng.random(n) < 0.5, 0x40, 0x80)
    gpos = rng.integers(0, 1000, n).astype(np.int32)
    nbytes = (rlen + 1) // 2
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum((nbytes + 3) // 4 * 4)
    nib = np.array([1, 2, 4, 8], np.uint8)[rng.integers(0, 4, int(2 * off[-1]))]
    odd = rng.random(nib.size)
    nib[odd < 0.01] = 15
    nib[(odd >= 0.01) & (odd < 0.015)] = rng.integers(0, 16, int(((odd >= 0.01) & (odd < 0.015)).sum()))
    seq = ((nib[0::2] << 4) | nib[1::2]).astype(np.uint8)
    batch = [rlen, flag, gpos, np.zeros(n, np.int32), np.full(n, -1, np.int32), off, seq]
    for K, NK, STEP, OFF in ((7, 8, 7, 0), (8, 5, 3, 4), (1, 20, 1, 0), (5, 10, 2, 3), (3, 4, 9, 1),
                             (8, 1, 1, 0), (2, 30, 9, 7), (12, 3, 12, 0), (6, 9, 5, -2), (8, 6, 4, 0)):
        cfg = _lib.ScanConfig()
        cfg.n_flags = 1
        cfg.flags[0] = 0x40
        cfg.kmer_on, cfg.kmer_k, cfg.kmer_nk, cfg.kmer_step, cfg.kmer_offset = 1, K, NK, STEP, OFF
        h = ctypes.c_void_p()
        _lib.check(lib.mc_scan_create(0, ctypes.byref(cfg), ctypes.byref(h)), lib)
        _lib.check(lib.mc_scan_add_batch(h, n, *[_lib.ptr(a) for a in batch]), lib)
        G, rows, cap = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
        lib.mc_scan_dims(h, ctypes.byref(G), ctypes.byref(rows), ctypes.byref(cap), None, None)
        kmer = np.zeros((G.value, 4 ** K + 1, NK), np.uint32)
        _lib.check(lib.mc_scan_results(h, None, _lib.ptr(kmer), None, None, None), lib)
        lib.mc_scan_destroy(h)
        want, done = coracle.scan(cfg, batch, None, None, None, 0, 128)
        assert done == n
        assert np.array_equal(kmer, want[1]), (K, NK, STEP, OFF)
        assert kmer[:, :4 ** K].sum() > 0 and kmer[:, 4 ** K].sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("window, chunk", [(None, None), ("65536", None), (None, "9999")])
def test_scan_gpu_decode_equals_host_source_gpu(mix, golden_dir, lib_built, tmp_path, window, chunk, monkeypatch):
    """scan_reads with the BAM decoded on the GPU (mc_bam_gpu_open_scan +
    mc_scan_run_gpu: every record, the reference ids forward-filled on the
    device) gives the host source's tables; a 64 KiB decode window takes the
    windowed path (records cut at every window end).  The BAMs: the mix (with
    a FASTA), the reference's bbmap BAM, the edge-case BAM, and a 355 K-read
    sorted BAM on three contigs."""
    from metacov_amd import scan as mscan
    if window:
        monkeypatch.setenv("MC_SCAN_GPU_WINDOW", window)
    if chunk:   # the device run in chunks of 9999 reads (the reference id carried across them)
        monkeypatch.setenv("MC_SCAN_RUN_CHUNK", chunk)
    bam, fa = mix
    big = str(tmp_path / "big.bam")
    rng = np.random.default_rng(8)
    lens = [300_000, 2_000_000, 40_000]
    arrs = synth.edge_mix_arrays(np.array(lens, np.int64), 120_000, seed=8,
                                 weights=np.array([5.0, 1.0, 2.0]))
    synth.write_bam_fast(big, ["a", "b", "c"], np.array(lens, np.int64), *arrs, level=1, n_threads=4)
    big_fa = str(tmp_path / "big.fa")
    acgt = np.frombuffer(b"ACGT", np.uint8)
    synth.write_fasta(big_fa, {n: acgt[rng.integers(0, 4, L)].tobytes().decode() for n, L in zip("ab", lens)})
    cases = [(bam, fa), (os.path.join(golden_dir, "bbmap.sorted.bam"), None),
             (os.path.join(golden_dir, "synth_edge.bam"), None), (big, big_fa)]
    for path, fasta in cases:
        outs = []
        for decode in ("host", "gpu"):
            c = mscan.ByFlag([mscan.BaseHist(2), mscan.KmerHist(5, 6, 4, 1), mscan.MirrorHist(4, 10),
                              mscan.IsizeHist()], [mscan.Flags["IsRead1"], mscan.Flags["Readdir"]])
            n = mscan.scan_reads(path, fasta, c, decode=decode)
            rows = [[list(map(str, r)) for r in q.get_rows()] for g in c.processors for q in g.processors]
            outs.append((n, rows))
        assert outs[0][0] == outs[1][0] and outs[0][0] > 0, path
        assert outs[0][1] == outs[1][1], path


@pytest.mark.gpu
def test_scan_gpu_decode_bounded(mix, lib_built, monkeypatch):
    """`scan --max-reads N` streams from the host source (the
    GPU decode would inflate the whole file first), and a GPU decode that
    runs out of device memory falls back to the host source; the tables are
    the host source's either way."""
    from metacov_amd import _lib
    from metacov_amd import scan as mscan
    bam, fa = mix

    def tables(**kw):
        c = mscan.ByFlag([mscan.BaseHist(2), mscan.KmerHist(5, 6, 4, 1), mscan.IsizeHist()], [])
        n = mscan.scan_reads(bam, fa, c, **kw)
        return n, [[list(map(str, r)) for r in q.get_rows()] for g in c.processors for q in g.processors]

    seen = []
    real = mscan._run_layer_on

    def spy(lib, infile, fa_, flags, per_group, maxreads, device, n_threads, batch_reads, decode):
        seen.append(decode)
        return real(lib, infile, fa_, flags, per_group, maxreads, device, n_threads, batch_reads, decode)
    monkeypatch.setattr(mscan, "_run_layer_on", spy)
    assert tables(maxreads=57, decode="gpu") == tables(maxreads=57, decode="host")
    assert seen == ["host", "host"]
    want = tables(decode="host")
    seen.clear()

    def oom(lib, infile, fa_, flags, per_group, maxreads, device, n_threads, batch_reads, decode):
        seen.append(decode)
        if decode == "gpu":
            raise _lib.MetacovError(_lib.MC_E_HIP, "hipMalloc failed: out of memory")
        return real(lib, infile, fa_, flags, per_group, maxreads, device, n_threads, batch_reads, decode)
    monkeypatch.setattr(mscan, "_run_layer_on", oom)
    assert tables(decode="gpu") == want
    assert seen == ["gpu", "host"]
