"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

CPU restatement of the reference's experimental estimator and its inputs:

* `experimental(bam, k_cor, k_len, fasta, ref, start, end)` restates
  `metacov/pileup.py:38-173` with per-position numpy arrays, exactly as the
  reference builds them (cov, cov2, cov_cor, cor, starts, cor_fwd, cor_rev,
  cor_revsum);
* `DuckBam` / `AlignedView` restate the pysam objects it reads:
  `AlignmentFile.fetch(ref, start, end)` (htslib: records of `ref` with
  pos < end and bam_endpos > start, file order) and the AlignedSegment
  attributes is_secondary / is_proper_pair / is_reverse / is_read1 /
  query_name / reference_start / reference_length /
  query_alignment_sequence (pysam getQueryStart / getQueryEnd; None for a
  read without SEQ, reference_length None when unmapped or without CIGAR);
* `DuckFasta` restates `pysam.FastaFile.fetch(ref, start, end)` (0-based,
  half-open, clipped to the sequence; names = first word of the '>' line);
* `load_kmerhist(f, k_len)` restates `metacov/pileup.py:29-35` with the
  pandas < 2.0 behaviour the reference relied on (`DataFrame.mean(axis=1)`
  skipping non-numeric columns).  Under the pandas installed here (2.x) the
  reference function raises TypeError on any histogram that carries the
  R / Mapped columns it filters on, so its behaviour is pinned only by this
  restatement ("parity unpinned" for load_kmerhist).

pysam and htslib are not installed; their semantics are restated here from
their published behaviour (versions unpinned by the reference,
requirements.txt:2).  Small inputs only (fixture BAM, synthetic edge cases).
"""
import gzip
import math

import numpy as np

from . import bamread

INSERT, SD = 450, 150          # pileup.py:55-56
ISTART, IEND = 0, 2 * INSERT   # pileup.py:59-60


def norm_taps():
    """sps.norm(450, 150).pdf(range(0, 901)) (pileup.py:61), as scipy
    evaluates it: exp(-x^2/2) / sqrt(2 pi) at x = (v - loc) / scale, / scale."""
    x = (np.arange(ISTART, IEND + 1, dtype=np.float64) - INSERT) / SD
    return np.exp(-x ** 2 / 2.0) / np.sqrt(2 * np.pi) / SD


class AlignedView:
    """The pysam.AlignedSegment attributes pileup.experimental reads."""

    def __init__(self, rec):
        self._r = rec

    is_secondary = property(lambda self: bool(self._r.flag & 0x100))
    is_proper_pair = property(lambda self: bool(self._r.flag & 0x2))
    is_reverse = property(lambda self: bool(self._r.flag & 0x10))
    is_read1 = property(lambda self: bool(self._r.flag & 0x40))
    query_name = property(lambda self: self._r.name)
    reference_start = property(lambda self: self._r.pos)

    @property
    def reference_length(self):
        r = self._r
        if (r.flag & 0x4) or not r.cigar:
            return None
        return end_pos(r) - r.pos

    @property
    def query_alignment_sequence(self):
        r = self._r
        if r.l_seq == 0:
            return None
        qs = 0
        for op, ln in r.cigar:            # getQueryStart
            if op == 5:
                continue
            if op == 4:
                qs += ln
                continue
            break
        qe = r.l_seq
        for op, ln in reversed(r.cigar[1:]):   # getQueryEnd: op 0 never looked at
            if op == 5:
                continue
            if op == 4:
                qe -= ln
                continue
            break
        return r.seq[qs:qe]


def end_pos(r):
    """htslib bam_endpos."""
    rl = 0 if (r.flag & 0x4) else r.ref_len()
    return r.pos + (rl if rl > 0 else 1)


class DuckBam:
    """pysam.AlignmentFile.fetch over a decoded (sorted) BAM."""

    def __init__(self, path):
        self.references, self.lengths, recs = bamread.read_bam(path)
        self.references = tuple(self.references)
        self._by_tid = {}
        for r in recs:
            if r.tid >= 0:
                self._by_tid.setdefault(r.tid, []).append(r)

    def fetch(self, ref, start, end):
        tid = self.references.index(ref)
        for r in self._by_tid.get(tid, ()):
            if r.pos >= end:
                break
            if end_pos(r) > start:
                yield AlignedView(r)


class DuckFasta:
    """pysam.FastaFile.fetch over a plain or gzip FASTA."""

    def __init__(self, path):
        opener = gzip.open if open(path, "rb").read(2) == b"\x1f\x8b" else open
        self.seqs = {}
        name, parts = None, []
        with opener(path, "rt") as fh:
            for line in fh:
                line = line.rstrip("\r\n")
                if line.startswith(">"):
                    if name is not None:
                        self.seqs[name] = "".join(parts)
                    name, parts = line[1:].split()[0], []
                elif name is not None:
                    parts.append(line.strip())
        if name is not None:
            self.seqs[name] = "".join(parts)

    def fetch(self, ref, start, end):
        return self.seqs[ref][start:end]


def load_kmerhist(f, k_len=7):
    """pileup.py:29-35 with pandas < 2.0 numeric-only row means."""
    import pandas as pd
    df = pd.read_csv(f)
    keep = (df["Mapped"] != "Unmapped") & (df["kmer"] != "N" * k_len)
    df = df[keep].set_index("kmer")
    first = df[df.columns[0]]
    rest = df[df.columns[1:]].select_dtypes(include="number")
    ratio = first / rest.mean(axis=1)
    return [ratio[(df["R"] == name).to_numpy()].to_dict() for name in ("R1", "R2")]


def experimental(bam, k_cor, k_len, fasta, ref, start, end, on_zero=None):
    """Restates pileup.py:38-173.  `on_zero(readno, kmer)` replaces the
    print of pileup.py:134-136 (None: print the same line)."""
    L = end - start
    if L == 0:
        raise Exception("Length must be > 0")
    cov = np.zeros(L)
    cov2 = np.zeros(L)
    cov_cor = np.zeros(L)
    cor = np.zeros(L)
    starts = np.zeros(L)
    wnf = 0.0
    nreads = secondary = improper = 0

    if fasta:
        region = fasta.fetch(ref, start, end).upper()
        gc = region.count("G") + region.count("C")
        gc = gc / (gc + region.count("A") + region.count("T"))
        if k_cor:
            ecor = raw_ecor(k_cor, k_len, region, L) / L
    else:
        gc = -1
        ecor = -1

    mates = {}
    for read in bam.fetch(ref, start, end):
        if read.is_secondary:
            secondary += 1
            continue
        if not read.is_proper_pair:
            improper += 1
            continue
        name = read.query_name
        if name in mates:
            mate = mates.pop(name)
            lo = min(read.reference_start, mate.reference_start) - start
            hi = max(read.reference_start, mate.reference_start) - start
            cov2[lo - 1:hi + 1] += 1
            try:
                a = k_cor[int(read.is_reverse)][read.query_alignment_sequence[:k_len]]
                b = k_cor[int(mate.is_reverse)][mate.query_alignment_sequence[:k_len]]
                wnf += 1 / (a * b)
            except (KeyError, ZeroDivisionError):
                wnf += 1
        else:
            mates[name] = read
        readno = 0 if read.is_read1 else 1
        kmer = read.query_alignment_sequence[:k_len]
        try:
            rcor = k_cor[readno][kmer]
        except Exception:
            rcor = 1
        if rcor == 0:
            if on_zero is None:
                print("RCOR is ZERO: {} {}".format(("R1", "R2")[readno], kmer))
            else:
                on_zero(readno, kmer)
            rcor = 1
        ln = read.reference_length
        if read.is_reverse:
            re_ = read.reference_start - start
            rs = re_ - ln
        else:
            rs = read.reference_start - start
            re_ = rs + ln
        a, b = max(0, rs), min(L, re_)
        if b > a:
            cov[a:b] += 1
            for i in range(a, b):
                cov_cor[i] += 1 / rcor
        if 0 <= rs < L:
            cor[rs] = 1 / rcor
            starts[rs] = 1
            nreads += 1

    nz = int(np.count_nonzero(starts == 0))
    nz_e = L * (1 - 1 / L) ** nreads
    nzef = nz / nz_e
    total = secondary + nreads + improper
    return {
        'cov': np.mean(cov),
        'covc': np.mean(cov_cor),
        'den': round(np.mean(starts), 3),
        'denc': round(np.mean(cor), 3),
        'cov2': round(np.mean(cov2)),
        'cf': round(sum(cor) / sum(starts), 3),
        'ambig': round(secondary / total, 3) if total > 0 else 0,
        'improper': round(improper / total, 3) if total > 0 else 0,
        'nzef': round(nzef, 3),
        'gc': round(gc, 3),
        'ecor': round(ecor, 3),
        'wnf': round(wnf / L, 3),
        'cov3': round(200 * (wnf / ecor) / nzef / L, 3),
    }


def raw_ecor(k_cor, k_len, region, L):
    """inner(fwd, revsum) of pileup.py:67-84 (ecor * L) for the upper-cased
    region string: k-mer weights per window, then the 900-tap correlation."""
    norm = norm_taps()
    fwd = np.zeros(L)
    rev = np.zeros(L)
    for i in range(0, L - k_len):
        fwd[i] = k_cor[0].get(region[i:i + k_len], 0)
    for p in range(k_len - 1, L):
        i = p - L                      # the reference's negative index
        rev[p] = k_cor[1].get(region[i:i - k_len:-1], 0)
    taps = IEND - ISTART
    revsum = np.zeros(L)
    for i in range(L):
        m = min(L - i, taps)
        revsum[i] = np.inner(norm[:m], rev[i:i + m])
    return np.inner(fwd, revsum)


def is_finite(x):
    return isinstance(x, (int, float, np.floating, np.integer)) and math.isfinite(x)
