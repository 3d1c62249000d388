"""Synthetic coverage workloads and a minimal BAM/BGZF writer.

Stands in for the reference's `metacov simulate` (`metacov/cli.py:288-414`,
`metacov/simulate.py:31-50`), which needs the absent `art_illumina` binary.
Configurations follow SURVEY.md §8(d) / BASELINE.json `configs`:

  C1  1 contig x 100,000 bp; 10,000 x 100 bp paired reads, seed 1234
  C2  1 contig x 5,000,000 bp; 10M x 150 bp, seed 1
  C3  1000 contigs, lengths rng(42).integers(200_000, 1_800_001),
      weight = length x lognormal(0,1) abundance; 100M x 150 bp
  C5  10k contigs (50-150 kbp); 50M long reads, lognormal length (mean 10 kbp)

Every config carries the SURVEY edge mix: 95% plain `150M`, 3% soft clips,
1% I/D, 0.1% N, 0.5% =/X, 2% placed-unmapped (flag 0x4, no CIGAR) and the
flag bits 0x100 (1%), 0x400 (0.5%), 0x200 (0.2%), 0x800 (0.5%, kept).

Two forms are produced:
* records with CIGARs (small sizes) -> `write_bam` -> BAM file, for the
  decoder and end-to-end parity tests;
* pileup intervals only (`interval_workload`): coordinate-sorted int32
  (tid, pos, span) after the 0x704 filter, vectorised numpy, for the
  device benchmark (the spans follow the same edge mix).
"""
import os
import struct
import zlib

import numpy as np

# CIGAR op codes (SAMv1 §4.2)
M, I, D, N, S, H, P, EQ, X = range(9)
REF_CONSUMING_MASK = 0x18D
FLAG_FILTER = 0x704

# category probabilities of the edge mix (SURVEY.md §8 d)
_CATS = np.array([0.9290, 0.03, 0.005, 0.005, 0.001, 0.005, 0.02, 0.005])
_CAT_PLAIN, _CAT_SOFT, _CAT_INS, _CAT_DEL, _CAT_SKIP, _CAT_EQX, _CAT_UNMAP, _CAT_ZERO = range(8)


def c3_contig_lengths(n=1000, seed=42):
    rng = np.random.default_rng(seed)
    return rng.integers(200_000, 1_800_001, size=n).astype(np.int64)


def _cigar_for(cat, readlen, rng):
    """One CIGAR (list of (op, len)) for an edge-mix category."""
    if cat == _CAT_PLAIN:
        return [(M, readlen)]
    if cat == _CAT_SOFT:
        s = int(rng.integers(1, max(2, readlen // 5)))
        return [(S, s), (M, readlen - s)] if rng.random() < 0.5 else [(M, readlen - s), (S, s)]
    if cat == _CAT_INS:
        a = int(rng.integers(1, readlen - 10))
        i = int(rng.integers(1, 6))
        return [(M, a), (I, i), (M, readlen - a - i)]
    if cat == _CAT_DEL:
        a = int(rng.integers(1, readlen - 1))
        return [(M, a), (D, int(rng.integers(1, 10))), (M, readlen - a)]
    if cat == _CAT_SKIP:
        a = int(rng.integers(1, readlen - 1))
        return [(M, a), (N, int(rng.integers(50, 2000))), (M, readlen - a)]
    if cat == _CAT_EQX:
        a = int(rng.integers(1, readlen - 1))
        return [(EQ, a), (X, 1), (EQ, readlen - a - 1)]
    if cat == _CAT_ZERO:
        # mapped, but no reference-consuming op (htslib: treated as 1 bp)
        return [(S, readlen)] if rng.random() < 0.5 else []
    return []   # unmapped


def ref_len(cigar):
    return sum(ln for op, ln in cigar if (REF_CONSUMING_MASK >> op) & 1)


class SynthRecord:
    __slots__ = ("name", "tid", "pos", "flag", "cigar", "l_seq", "seq", "tlen")

    def __init__(self, name, tid, pos, flag, cigar, l_seq, seq=None, tlen=0):
        self.name, self.tid, self.pos, self.flag = name, tid, pos, flag
        self.cigar, self.l_seq, self.seq, self.tlen = cigar, l_seq, seq, tlen


def edge_mix_records(lengths, n_reads, readlen=150, seed=1, weights=None,
                     overhang=False, zero_span=False, unplaced=0):
    """Coordinate-sorted records with CIGARs and flags (small sizes).

    `overhang` lets a few reads run past the end of their contig; `zero_span`
    adds mapped reads without reference-consuming ops; `unplaced` appends
    that many tid=-1 unmapped records at the end of the file.
    """
    rng = np.random.default_rng(seed)
    lengths = np.asarray(lengths, dtype=np.int64)
    w = lengths.astype(np.float64) if weights is None else np.asarray(weights, np.float64)
    tids = rng.choice(len(lengths), size=n_reads, p=w / w.sum())
    probs = _CATS.copy()
    if not zero_span:
        probs[_CAT_PLAIN] += probs[_CAT_ZERO]
        probs[_CAT_ZERO] = 0
    cats = rng.choice(len(probs), size=n_reads, p=probs / probs.sum())
    recs = []
    for i in range(n_reads):
        tid = int(tids[i])
        L = int(lengths[tid])
        cat = int(cats[i])
        cigar = _cigar_for(cat, readlen, rng)
        rl = ref_len(cigar)
        hi = L - max(rl, 1) if not overhang else L - 1
        pos = int(rng.integers(0, max(1, hi + 1)))
        flag = 0x1 | (0x40 if i % 2 == 0 else 0x80)
        if cat == _CAT_UNMAP:
            flag |= 0x4
        u = rng.random()
        if u < 0.01:
            flag |= 0x100
        elif u < 0.015:
            flag |= 0x400
        elif u < 0.017:
            flag |= 0x200
        elif u < 0.022:
            flag |= 0x800
        if rng.random() < 0.5:
            flag |= 0x10
        recs.append(SynthRecord("r%d" % i, tid, pos, flag, cigar, readlen))
    recs.sort(key=lambda r: (r.tid, r.pos))
    for j in range(unplaced):
        recs.append(SynthRecord("u%d" % j, -1, -1, 0x4, [], readlen))
    return recs


def scan_mix(n_reads=800, n_contigs=4, contig_len=3000, seed=7, long_reads=4):
    """(names, lengths, records, fasta) for `scan` tests: reads whose bases
    come from their contig (BaseHist's match test passes for most), a few
    percent mutated, N bases, lower-case and IUPAC letters in the FASTA, a
    contig the FASTA lacks, reads running off either contig end, reverse
    strand, proper pairs with +/- insert sizes, unmapped-but-placed and
    unplaced records, empty SEQ, and `long_reads` reads of 1-3 kbp."""
    rng = np.random.default_rng(seed)
    names = ["c%d" % i for i in range(n_contigs)]
    lengths = [contig_len + 37 * i for i in range(n_contigs)]
    alphabet = np.array(list("ACGT"))
    contigs = []
    for L in lengths:
        s = alphabet[rng.integers(0, 4, L)]
        s[rng.random(L) < 0.01] = "N"
        low = rng.random(L) < 0.05
        s[low] = np.char.lower(s[low])
        s[rng.random(L) < 0.002] = "R"
        contigs.append("".join(s))
    fasta = {n: c for n, c in zip(names[:-1], contigs[:-1])}   # the last contig is missing
    recs = []
    for i in range(n_reads):
        tid = int(rng.integers(0, n_contigs))
        L = lengths[tid]
        rlen = int(rng.integers(20, 160)) if i >= long_reads else int(rng.integers(1000, 3000))
        pos = int(rng.integers(-20, L - rlen + 40))
        pos = max(pos, 0)
        ref = contigs[tid].upper()
        bases = list(ref[pos:pos + rlen].ljust(rlen, "A"))
        for j in np.nonzero(rng.random(rlen) < (0.2 if i % 17 == 0 else 0.01))[0]:
            bases[j] = "ACGTN"[int(rng.integers(0, 5))]
        bases = ["N" if b not in "ACGT" else b for b in bases]
        flag = 0
        if rng.random() < 0.8:
            flag |= 0x1 | (0x40 if i % 2 == 0 else 0x80)
            if rng.random() < 0.7:
                flag |= 0x2
            if rng.random() < 0.5:
                flag |= 0x20
            if rng.random() < 0.05:
                flag |= 0x8
        if rng.random() < 0.5:
            flag |= 0x10
        if rng.random() < 0.03:
            flag |= 0x4
        if rng.random() < 0.03:
            flag |= 0x100
        if rng.random() < 0.02:
            flag |= 0x400
        tlen = int(rng.integers(100, 700)) * (1 if rng.random() < 0.5 else -1)
        if rng.random() < 0.1:
            tlen = 0
        seq = "" if i % 97 == 5 else "".join(bases)
        recs.append(SynthRecord("s%d" % i, tid, pos, flag, [(0, max(len(seq), 1))], len(seq),
                                seq=seq, tlen=tlen))
    recs.sort(key=lambda r: (r.tid, r.pos))
    for j in range(6):
        seq = "".join(alphabet[rng.integers(0, 4, 60)])
        recs.append(SynthRecord("u%d" % j, -1, -1, 0x4 | 0x1 | 0x2, [], 60, seq=seq,
                                tlen=int(rng.integers(-500, 500))))
    return names, lengths, recs, fasta


def write_fasta(path, seqs, width=60):
    with open(path, "w") as fh:
        for name, s in seqs.items():
            fh.write(">%s description\n" % name)
            for i in range(0, len(s), width):
                fh.write(s[i:i + width] + "\n")


# ---------------------------------------------------------------- BGZF / BAM

NT16 = "=ACMGRSVTWYHKDBN"

_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _bgzf_block(payload):
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    cdata = c.compress(payload) + c.flush()
    bsize = len(cdata) + 25  # 18 header + 8 trailer - 1
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
    tail = struct.pack("<II", zlib.crc32(payload) & 0xFFFFFFFF, len(payload))
    return hdr + cdata + tail


def _bgzf(data, block=0xff00):
    out = bytearray()
    for i in range(0, len(data), block):
        out += _bgzf_block(data[i:i + block])
    out += _BGZF_EOF
    return bytes(out)


def _reg2bin(beg, end):
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def encode_record(r, long_cigar_threshold=65535):
    """One BAM record (bytes).  CIGARs longer than the threshold are stored
    in a CG:B,I tag behind a `<l_seq>S<rlen>N` placeholder (SAMv1 §4.2.2)."""
    name = r.name.encode() + b"\0"
    cig = [(ln << 4) | op for op, ln in r.cigar]
    aux = b""
    if len(cig) > long_cigar_threshold:
        aux = b"CGBI" + struct.pack("<i", len(cig)) + struct.pack("<%dI" % len(cig), *cig)
        cig = [(r.l_seq << 4) | S, (max(ref_len(r.cigar), 1) << 4) | N]
    if r.seq is None:
        l_seq = r.l_seq
        seq = bytes([0x11] * ((l_seq + 1) // 2))   # "AA..." in nt16
    else:                                          # given bases (SAMv1 §4.2.3)
        l_seq = len(r.seq)
        codes = [NT16.index(c) for c in r.seq.upper()] + [0]
        seq = bytes((codes[i] << 4) | codes[i + 1] for i in range(0, l_seq, 2))
    qual = bytes([30] * l_seq)
    end = r.pos + max(ref_len(r.cigar), 1)
    bin_ = _reg2bin(max(r.pos, 0), max(end, 1)) if r.tid >= 0 else 4680
    core = struct.pack("<iiBBHHHiiii", r.tid, r.pos, len(name), 60, bin_, len(cig),
                       r.flag, l_seq, r.tid, r.pos, getattr(r, "tlen", 0))
    body = core + name + struct.pack("<%dI" % len(cig), *cig) + seq + qual + aux
    return struct.pack("<i", len(body)) + body


def write_bam(path, names, lengths, records, long_cigar_threshold=65535):
    text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join(
        "@SQ\tSN:%s\tLN:%d\n" % (n, L) for n, L in zip(names, lengths))
    hdr = bytearray(b"BAM\x01")
    hdr += struct.pack("<i", len(text)) + text.encode()
    hdr += struct.pack("<i", len(names))
    for n, L in zip(names, lengths):
        nb = n.encode() + b"\0"
        hdr += struct.pack("<i", len(nb)) + nb + struct.pack("<i", int(L))
    body = bytearray(hdr)
    for r in records:
        body += encode_record(r, long_cigar_threshold)
    with open(path, "wb") as fh:
        fh.write(_bgzf(bytes(body)))


# ------------------------------------------------------- interval workloads

def interval_workload(lengths, n_reads, readlen=150, seed=1, weights=None,
                      long_reads=False):
    """Coordinate-sorted pileup intervals (int32 tid, pos, span) after the
    0x704 filter, vectorised.  Spans follow the edge mix: soft clips shorten,
    deletions / N lengthen.  `long_reads` draws lognormal lengths with mean
    ~10 kbp clipped to the contig (config C5)."""
    rng = np.random.default_rng(seed)
    lengths = np.asarray(lengths, dtype=np.int64)
    w = lengths.astype(np.float64) if weights is None else np.asarray(weights, np.float64)
    counts = rng.multinomial(n_reads, w / w.sum())
    tid = np.repeat(np.arange(len(lengths), dtype=np.int32), counts)
    if long_reads:
        span = rng.lognormal(np.log(10_000) - 0.5 * 0.5 ** 2, 0.5, size=n_reads)
        span = np.maximum(span.astype(np.int64), 1)
    else:
        u = rng.random(n_reads)
        span = np.full(n_reads, readlen, dtype=np.int64)
        soft = u < 0.03
        span[soft] -= rng.integers(1, readlen // 5, size=int(soft.sum()))
        ins = (u >= 0.03) & (u < 0.035)
        span[ins] -= rng.integers(1, 6, size=int(ins.sum()))
        dele = (u >= 0.035) & (u < 0.04)
        span[dele] += rng.integers(1, 10, size=int(dele.sum()))
        skip = (u >= 0.04) & (u < 0.041)
        span[skip] += rng.integers(50, 2000, size=int(skip.sum()))
    L = lengths[tid]
    span = np.minimum(span, L)
    pos = (rng.random(n_reads) * (L - span + 1)).astype(np.int64)
    order = np.lexsort((pos, tid))
    return (tid[order].astype(np.int32), pos[order].astype(np.int32),
            span[order].astype(np.int32))


def c3_workload(n_reads=100_000_000, n_contigs=1000, seed=42):
    lengths = c3_contig_lengths(n_contigs, seed)
    rng = np.random.default_rng(seed + 1)
    weights = lengths * rng.lognormal(0.0, 1.0, size=n_contigs)
    return lengths, weights


# --------------------------------------------------- vectorised large BAMs

def edge_mix_arrays(lengths, n_reads, readlen=150, seed=1, weights=None):
    """Coordinate-sorted records as arrays (tid, pos, flag, cig_off, cigar)
    with the SURVEY §8(d) edge mix — vectorised, for BAMs of millions of
    records written by `write_bam_fast`."""
    rng = np.random.default_rng(seed)
    lengths = np.asarray(lengths, dtype=np.int64)
    w = lengths.astype(np.float64) if weights is None else np.asarray(weights, np.float64)
    counts = rng.multinomial(n_reads, w / w.sum())
    tid = np.repeat(np.arange(len(lengths), dtype=np.int32), counts)
    probs = _CATS.copy()
    probs[_CAT_PLAIN] += probs[_CAT_ZERO]
    probs[_CAT_ZERO] = 0
    cat = rng.choice(len(probs), size=n_reads, p=probs / probs.sum())
    nw = np.select([cat == _CAT_PLAIN, cat == _CAT_SOFT, cat == _CAT_UNMAP], [1, 2, 0], 3)
    cig_off = np.zeros(n_reads + 1, np.int64)
    np.cumsum(nw, out=cig_off[1:])
    cigar = np.zeros(int(cig_off[-1]), np.uint32)
    a = rng.integers(1, readlen - 10, size=n_reads)
    x = rng.integers(1, 6, size=n_reads)
    big = rng.integers(50, 2000, size=n_reads)
    o = cig_off[:-1]

    def put(mask, k, op, ln):
        cigar[o[mask] + k] = (np.asarray(ln)[mask] if np.ndim(ln) else ln) << 4 | op

    rl = np.full(n_reads, readlen, np.int64)
    m = cat == _CAT_PLAIN
    put(m, 0, M, readlen)
    m = cat == _CAT_SOFT
    put(m, 0, S, x)
    put(m, 1, M, readlen - x)
    rl[m] = readlen - x[m]
    m = cat == _CAT_INS
    put(m, 0, M, a)
    put(m, 1, I, x)
    put(m, 2, M, readlen - a - x)
    rl[m] = readlen - x[m]
    m = cat == _CAT_DEL
    put(m, 0, M, a)
    put(m, 1, D, x)
    put(m, 2, M, readlen - a)
    rl[m] = readlen + x[m]
    m = cat == _CAT_SKIP
    put(m, 0, M, a)
    put(m, 1, N, big)
    put(m, 2, M, readlen - a)
    rl[m] = readlen + big[m]
    m = cat == _CAT_EQX
    put(m, 0, EQ, a)
    put(m, 1, X, 1)
    put(m, 2, EQ, readlen - a - 1)
    L = lengths[tid]
    pos = (rng.random(n_reads) * np.maximum(L - rl + 1, 1)).astype(np.int64)
    flag = (0x1 | np.where(np.arange(n_reads) % 2 == 0, 0x40, 0x80)).astype(np.uint16)
    flag[cat == _CAT_UNMAP] |= 0x4
    u = rng.random(n_reads)
    flag[u < 0.01] |= 0x100
    flag[(u >= 0.01) & (u < 0.015)] |= 0x400
    flag[(u >= 0.015) & (u < 0.017)] |= 0x200
    flag[(u >= 0.017) & (u < 0.022)] |= 0x800
    flag[rng.random(n_reads) < 0.5] |= 0x10
    order = np.lexsort((pos, tid))
    new_nw = nw[order]
    new_off = np.zeros(n_reads + 1, np.int64)
    np.cumsum(new_nw, out=new_off[1:])
    # gather each read's words in the new order
    src = np.repeat(cig_off[:-1][order], new_nw) + (np.arange(int(new_off[-1])) -
                                                    np.repeat(new_off[:-1], new_nw))
    return (tid[order], pos[order].astype(np.int32), flag[order], new_off, cigar[src])


def write_bam_fast(path, names, lengths, tid, pos, flag, cig_off, cigar, l_seq=150, level=1,
                   n_threads=0):
    """BAM from record arrays through the library's C++ writer (mc_bam_write)."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    enc = [n.encode() for n in names]
    arr = (ctypes.c_char_p * len(enc))(*enc)
    lengths = np.ascontiguousarray(lengths, np.int64)
    tid = np.ascontiguousarray(tid, np.int32)
    pos = np.ascontiguousarray(pos, np.int32)
    flag = np.ascontiguousarray(flag, np.uint16)
    cig_off = np.ascontiguousarray(cig_off, np.int64)
    cigar = np.ascontiguousarray(cigar, np.uint32)
    _lib.check(lib.mc_bam_write(os.fspath(path).encode(), len(enc), ctypes.cast(arr, ctypes.c_void_p),
                                _lib.ptr(lengths), len(tid), _lib.ptr(tid), _lib.ptr(pos),
                                _lib.ptr(flag), _lib.ptr(cig_off), _lib.ptr(cigar), int(l_seq),
                                int(level), int(n_threads)))


def device_cigars(torch, span, mean_ops=200, seed=1, batch_reads=2_000_000):
    """BAM-packed CIGAR words on the GPU whose reference-consuming lengths sum
    to `span` (int32 device tensor): read i gets m_i ~ Poisson(mean_ops / 2)
    reference blocks (M mostly; D, N, =, X mixed in) separated by 1-3 bp
    insertions, i.e. 2 m_i - 1 ops (SURVEY §8 d C5: ~Poisson(200) ops per
    read).  Built in read batches; returns (cig_off int64 [n + 1], cigar
    int32 [W])."""
    dev = span.device
    n = span.numel()
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    m = torch.poisson(torch.full((n,), mean_ops / 2.0, device=dev), generator=g).to(torch.int64)
    m.clamp_(min=1)
    ops = 2 * m - 1
    cig_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    cig_off[1:] = torch.cumsum(ops, 0)
    total = int(cig_off[-1])
    cigar = torch.empty(total, dtype=torch.int32, device=dev)
    lut = torch.tensor([0] * 12 + [2, 3, 7, 8], dtype=torch.int64, device=dev)   # M x12, D, N, =, X
    for r0 in range(0, n, batch_reads):
        r1 = min(n, r0 + batch_reads)
        w0, w1 = int(cig_off[r0]), int(cig_off[r1])
        rid = torch.repeat_interleave(torch.arange(r0, r1, device=dev), ops[r0:r1])
        k = torch.arange(w0, w1, device=dev) - cig_off[rid]
        is_ref = (k & 1) == 0
        j = k >> 1
        s = span[rid].to(torch.int64)
        mm = m[rid]
        ref_len = (s * (j + 1)) // mm - (s * j) // mm
        del s, mm, j, k
        ins_len = torch.randint(1, 4, (w1 - w0,), generator=g, device=dev)
        code = torch.randint(0, 16, (w1 - w0,), generator=g, device=dev)
        op = torch.where(is_ref, lut[code], torch.ones_like(code))          # I = 1
        length = torch.where(is_ref, ref_len, ins_len)
        cigar[w0:w1] = ((length << 4) | op).to(torch.int32)
        del rid, is_ref, ref_len, ins_len, code, op, length
    return cig_off, cigar
