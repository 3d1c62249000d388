"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

Pure-Python BAM reader (gzip + struct) restating what the reference gets from
pysam/htslib on the pileup path:

* the BAM header (targets, lengths) that `pysam.AlignmentFile` exposes as
  `bam.references` / `bam.lengths`  (used at reference `metacov/cli.py:80`,
  `metacov/util.py:64-69`);
* one record at a time, like the reference's only hand-written read iterator
  `scan.AlignmentFileIterator` (`metacov/scan.pyx:188-294`: `get_tid`
  :282-283, `get_flags` :264-265, `get_len` :261-262) — but emitting the
  *pileup interval* `(tid, pos, span)` that htslib's `bam_plp` uses, not the
  `(pos, l_qseq)` of scan.pyx.

Third-party algorithm restated here: htslib (bundled in pysam, version
unpinned by the reference: `requirements.txt:2`, `setup.py:45,53`) —
`bam_cigar2rlen` (reference-consuming ops M, D, N, =, X; op-type mask 0x18D)
and the end `bam_plp_push` gives a pileup read: current htslib sets
`tail->end = pos + bam_cigar2rlen(...)` ("raw rlen rather than bam_endpos()
which adjusts rlen=0 to rlen=1"), so a mapped read without reference-consuming
ops has span 0 and adds nothing; htslib <= 1.9 used `bam_endpos` (pos + 1),
kept here as `legacy_endpos=True`.  The pileup stepper "all" (pysam's default, the one
`metacov/pileup.py:13` uses) drops records with any of
UNMAP|SECONDARY|QCFAIL|DUP = 0x704.

Small inputs only (fixture / synthetic edge-case BAMs); it is a checker.
"""
import gzip
import struct

FLAG_FILTER = 0x704          # BAM_FUNMAP | BAM_FSECONDARY | BAM_FQCFAIL | BAM_FDUP
REF_CONSUMING_MASK = 0x18D   # bits for M(0) D(2) N(3) =(7) X(8)


NT16 = "=ACMGRSVTWYHKDBN"   # BAM 4-bit base codes (SAMv1 §4.2.3)


class Record:
    __slots__ = ("tid", "pos", "flag", "cigar", "l_seq", "name", "seq", "tlen")

    def __init__(self, tid, pos, flag, cigar, l_seq, name, seq="", tlen=0):
        self.tid, self.pos, self.flag = tid, pos, flag
        self.cigar, self.l_seq, self.name, self.seq = cigar, l_seq, name, seq
        self.tlen = tlen

    def ref_len(self):
        """htslib bam_cigar2rlen: sum of lengths of reference-consuming ops."""
        return sum(ln for op, ln in self.cigar if (REF_CONSUMING_MASK >> op) & 1)

    def pileup_span(self, legacy_endpos=False):
        """Span of the read on the reference as the pileup engine sees it:
        bam_plp_push's tail->end - pos = bam_cigar2rlen (0 without a
        reference-consuming op); legacy_endpos: bam_endpos() - pos, which
        treats a zero-length alignment as 1 bp.
        """
        rl = self.ref_len() if self.cigar else 0
        return 1 if (rl <= 0 and legacy_endpos) else rl

    def endpos(self):
        """htslib bam_endpos(): what the region iterator (hts_itr_next) tests
        overlap with, in every htslib version."""
        rl = self.ref_len() if (self.cigar and not self.flag & 4) else 0
        return self.pos + (rl if rl > 0 else 1)


def read_bam(path):
    """Returns (names, lengths, records). Whole file in memory (small files)."""
    with gzip.open(path, "rb") as fh:
        data = fh.read()
    if data[:4] != b"BAM\x01":
        raise ValueError("not a BAM file: %s" % path)
    off = 4
    (l_text,) = struct.unpack_from("<i", data, off)
    off += 4 + l_text
    (n_ref,) = struct.unpack_from("<i", data, off)
    off += 4
    names, lengths = [], []
    for _ in range(n_ref):
        (l_name,) = struct.unpack_from("<i", data, off)
        off += 4
        names.append(data[off:off + l_name - 1].decode())
        off += l_name
        (l_ref,) = struct.unpack_from("<i", data, off)
        off += 4
        lengths.append(l_ref)
    recs = []
    while off < len(data):
        (block_size,) = struct.unpack_from("<i", data, off)
        rec_end = off + 4 + block_size
        (tid, pos, l_read_name, _mapq, _bin, n_cigar, flag, l_seq,
         _ntid, _npos, tlen) = struct.unpack_from("<iiBBHHHiiii", data, off + 4)
        p = off + 36
        name = data[p:p + l_read_name - 1].decode()
        p += l_read_name
        cig = struct.unpack_from("<%dI" % n_cigar, data, p)
        cigar = [(c & 0xF, c >> 4) for c in cig]
        p += 4 * n_cigar
        packed = data[p:p + (l_seq + 1) // 2]
        seq = "".join(NT16[(packed[i >> 1] >> (4 * (1 - (i & 1)))) & 0xF] for i in range(l_seq))
        # CG:B,I long-CIGAR convention (SAMv1 §4.2.2): placeholder kSmN
        if (n_cigar == 2 and cigar[0] == (4, l_seq) and cigar[1][0] == 3):
            aux = p + (l_seq + 1) // 2 + l_seq
            cigar = _find_cg(data, aux, rec_end) or cigar
        recs.append(Record(tid, pos, flag, cigar, l_seq, name, seq, tlen))
        off = rec_end
    return names, lengths, recs


_AUX_SIZE = {"A": 1, "c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}


def _find_cg(data, p, end):
    while p + 3 <= end:
        tag = data[p:p + 2].decode()
        t = chr(data[p + 2])
        p += 3
        if t in _AUX_SIZE:
            p += _AUX_SIZE[t]
        elif t in "ZH":
            while data[p] != 0:
                p += 1
            p += 1
        elif t == "B":
            sub = chr(data[p])
            (cnt,) = struct.unpack_from("<i", data, p + 1)
            p += 5
            if tag == "CG" and sub == "I":
                raw = struct.unpack_from("<%dI" % cnt, data, p)
                return [(c & 0xF, c >> 4) for c in raw]
            p += cnt * _AUX_SIZE[sub]
        else:
            raise ValueError("bad aux type %r" % t)
    return None


def pileup_intervals(records, flag_filter=FLAG_FILTER, legacy_endpos=False):
    """(tid, pos, span) of every record the "all" pileup stepper keeps."""
    out = []
    for r in records:
        if r.tid < 0 or (r.flag & flag_filter):
            continue
        out.append((r.tid, r.pos, r.pileup_span(legacy_endpos)))
    return out


def depth_vectors(lengths, intervals):
    """Interval count restatement of htslib PileupColumn.n: depth[tid][p] is
    the number of kept records with pos <= p < pos + span.  Positions past
    the contig length are dropped ("contig end")."""
    import numpy as np
    depth = [np.zeros(L + 1, dtype=np.int64) for L in lengths]
    for tid, pos, span in intervals:
        L = lengths[tid]
        a, b = min(pos, L), min(pos + span, L)
        depth[tid][a] += 1
        depth[tid][b] -= 1
    return [np.cumsum(d)[:-1] for d in depth]


def scan_intervals(path, flag_filter=FLAG_FILTER, legacy_endpos=False):
    """The same restatement over a whole (large) file without building Record
    objects or decoding bases: returns (names, lengths, (n_records, mapped,
    unmapped), tid, pos, span) with int32 numpy arrays of the kept records in
    file order.  Mapped = tid >= 0 and not 0x4 (pysam's mapped count of the
    index pseudo-bins, as the product reports it).  For the parity tests of
    multi-window decodes (tests/test_gpu_decode.py): ~2 us per record."""
    import numpy as np
    with gzip.open(path, "rb") as fh:
        data = fh.read()
    if data[:4] != b"BAM\x01":
        raise ValueError("not a BAM file: %s" % path)
    off = 4
    (l_text,) = struct.unpack_from("<i", data, off)
    off += 4 + l_text
    (n_ref,) = struct.unpack_from("<i", data, off)
    off += 4
    names, lengths = [], []
    for _ in range(n_ref):
        (l_name,) = struct.unpack_from("<i", data, off)
        off += 4
        names.append(data[off:off + l_name - 1].decode())
        off += l_name
        (l_ref,) = struct.unpack_from("<i", data, off)
        off += 4
        lengths.append(l_ref)
    tid_l, pos_l, span_l = [], [], []
    n_rec = mapped = 0
    hdr = struct.Struct("<iiiBBHHHi")
    end = len(data)
    while off < end:
        block_size, tid, pos, l_read_name, _mapq, _bin, n_cigar, flag, l_seq = \
            hdr.unpack_from(data, off)
        rec_end = off + 4 + block_size
        n_rec += 1
        if tid >= 0 and not flag & 4:
            mapped += 1
        if tid >= 0 and not flag & flag_filter:
            p = off + 36 + l_read_name
            cig = struct.unpack_from("<%dI" % n_cigar, data, p)
            if (n_cigar == 2 and cig[0] == ((l_seq << 4) | 4) and cig[1] & 0xF == 3):
                cg = _find_cg(data, p + 4 * n_cigar + (l_seq + 1) // 2 + l_seq, rec_end)
                if cg is not None:
                    cig = [(ln << 4) | op for op, ln in cg]
            rl = 0
            for c in cig:
                if (REF_CONSUMING_MASK >> (c & 0xF)) & 1:
                    rl += c >> 4
            tid_l.append(tid)
            pos_l.append(pos)
            span_l.append(1 if (rl <= 0 and legacy_endpos) else rl)
        off = rec_end
    arr = lambda x: np.array(x, dtype=np.int32)
    return names, lengths, (n_rec, mapped, n_rec - mapped), arr(tid_l), arr(pos_l), arr(span_l)
