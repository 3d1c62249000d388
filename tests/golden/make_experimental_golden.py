"""Generates the golden fixtures of `pileup.experimental` (SURVEY.md §8 f).

Run ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It loads the reference's real `metacov/pileup.py`
(`experimental`, :38-173) and calls it with duck-typed `bam` / `fasta`
objects (`oracle/experimental.py`: DuckBam.fetch yields objects with the
AlignedSegment attributes experimental() reads; DuckFasta.fetch slices the
FASTA) and k_cor dictionaries made here.  pysam is not installed, so the
fetch / AlignedSegment semantics are the oracle's restatement of htslib and
pysam; every number in the expected rows is the reference's own arithmetic.
Its "RCOR is ZERO" prints (:134-136) are captured per region.

Outputs:
  synth_exp.bam / synth_exp.fa   edge-case pairs (secondary / improper /
      unmapped-placed reads, reverse mates before the region start, soft and
      hard clips, N and lower-case bases, a name seen three times, reads
      past the contig end, a region past the FASTA sequence)
  synth_exp_noseq.bam            one proper read without SEQ (TypeError)
  reference_1K.fa.gz             copied fixture (the reference's test FASTA)
  experimental.json              k_cor tables, cases, expected rows / errors
"""
import contextlib
import importlib.util
import io
import itertools
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import experimental as ox  # noqa: E402
from metacov_amd import synth  # noqa: E402

_spec = importlib.util.spec_from_file_location("ref_pileup", "/root/reference/metacov/pileup.py")
ref_pileup = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(ref_pileup)


def _py(v):
    if isinstance(v, (float, np.floating)):
        return float(v)
    return int(v)


def run_case(bam, k_cor, k, fasta, ref, start, end):
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            r = ref_pileup.experimental(bam, k_cor, k, fasta, ref, start, end)
        out = {"row": {key: _py(v) for key, v in r.items()},
               "types": {key: type(v).__name__ for key, v in r.items()}}
    except Exception as e:  # noqa: BLE001 - the error type is the expected value
        out = {"error": type(e).__name__}
    out["stdout"] = buf.getvalue()
    return out


def kcor_tables(rng, k, p_missing=0.1, p_zero=0.0):
    keys = ["".join(p) for p in itertools.product("ACGT", repeat=k)]
    tabs = []
    for _ in range(2):
        d = {}
        for key in keys:
            u = rng.random()
            if u < p_missing:
                continue
            d[key] = 0.0 if u < p_missing + p_zero else float(rng.uniform(0.4, 2.5))
        tabs.append(d)
    return tabs


def rand_seq(rng, n):
    return "".join(rng.choice(list("ACGT"), size=n))


def synth_exp(rng, path_bam, path_fa):
    """Two contigs, paired reads drawn from the sequence, edge cases mixed in."""
    names, lengths = ["c0", "c1"], [3000, 1500]
    seqs = [rand_seq(rng, L) for L in lengths]
    # lower-case and N runs in the FASTA (experimental upper-cases, N breaks k-mers)
    s0 = list(seqs[0])
    for i in range(100, 160):
        s0[i] = s0[i].lower()
    for i in range(700, 712):
        s0[i] = "N"
    seqs[0] = "".join(s0)
    with open(path_fa, "w") as fh:
        for n, sq in zip(names, seqs):
            fh.write(">%s%s\n" % (n, " description words" if n == "c1" else ""))
            for i in range(0, len(sq), 60):
                fh.write(sq[i:i + 60] + "\n")
    M, I, D, S, H = 0, 1, 2, 4, 5
    recs = []
    qn = 0
    for tid, L in enumerate(lengths):
        ref = seqs[tid].upper()
        for _ in range(260 if tid == 0 else 120):
            rl = int(rng.integers(40, 120))
            p1 = int(rng.integers(0, L - 20))
            ins = int(rng.integers(rl, 500))
            p2 = min(L - 10, p1 + ins - rl)
            name = "q%d" % qn
            qn += 1
            for mate, (p, rev) in enumerate(((p1, False), (p2, True))):
                seq = ref[p:p + rl]
                if len(seq) < 10:
                    seq = seq + rand_seq(rng, 10 - len(seq))
                seq = list(seq)
                for _m in range(int(rng.integers(0, 3))):
                    j = int(rng.integers(0, len(seq)))
                    seq[j] = str(rng.choice(list("ACGTN")))
                seq = "".join(seq)
                u = rng.random()
                if u < 0.15:
                    cig = [(S, 3), (M, len(seq) - 3)]
                elif u < 0.22:
                    cig = [(H, 5), (S, 2), (M, len(seq) - 6), (S, 4)]
                elif u < 0.3:
                    a = len(seq) // 2
                    cig = [(M, a), (D, 7), (M, len(seq) - a - 2), (I, 2)]
                else:
                    cig = [(M, len(seq))]
                flag = 0x1 | (0x40 if mate == 0 else 0x80) | (0x10 if rev else 0) | \
                    (0x20 if not rev else 0)
                v = rng.random()
                if v < 0.8:
                    flag |= 0x2
                elif v < 0.85:
                    flag |= 0x100 | 0x2
                recs.append(synth.SynthRecord(name, tid, p, flag, cig, len(seq), seq))
        # a name seen three times (pairs 1-2, then a dangling third)
        for j in range(3):
            sq = ref[200 + 30 * j:260 + 30 * j]
            recs.append(synth.SynthRecord("triple", tid, 200 + 30 * j, 0x3 | (0x10 if j == 1 else 0),
                                          [(M, len(sq))], len(sq), sq))
        # unmapped placed read (no CIGAR, not proper): improper, no TypeError
        recs.append(synth.SynthRecord("unm%d" % tid, tid, 50, 0x1 | 0x4 | 0x8, [], 20, "A" * 20))
        # reads running past the contig end
        sq = ref[L - 30:] + "ACGTACGTAC"
        recs.append(synth.SynthRecord("tail%d" % tid, tid, L - 30, 0x3 | 0x40, [(M, len(sq))],
                                      len(sq), sq))
    recs.sort(key=lambda r: (r.tid, r.pos))
    synth.write_bam(path_bam, names, lengths, recs)
    return names, lengths


def main():
    rng = np.random.default_rng(2024)
    shutil.copyfile("/root/reference/tests/data/reference_1K.fa.gz",
                    os.path.join(HERE, "reference_1K.fa.gz"))
    names, lengths = synth_exp(rng, os.path.join(HERE, "synth_exp.bam"),
                               os.path.join(HERE, "synth_exp.fa"))
    # a BAM whose one proper read has no SEQ
    synth.write_bam(os.path.join(HERE, "synth_exp_noseq.bam"), ["c0"], [500], [
        synth.SynthRecord("a", 0, 10, 0x3 | 0x40, [(0, 50)], 50, "ACGT" * 12 + "AC"),
        synth.SynthRecord("b", 0, 20, 0x3 | 0x40, [(0, 50)], 0, ""),
    ])

    kcor = {
        "k4": kcor_tables(rng, 4, 0.1),
        "k4zero": kcor_tables(rng, 4, 0.05, 0.15),
        "k5": kcor_tables(rng, 5, 0.3),
        "k7sparse": kcor_tables(np.random.default_rng(7), 7, 0.85),
    }
    fixture_regions = [["ref1", 1, 425], ["ref2", 1, 575], ["ref2", 1, 300], ["ref2", 301, 575],
                       ["ref1", 0, 425], ["ref2", 0, 575], ["ref1", 0, 50], ["ref1", 400, 425],
                       ["ref2", 550, 600], ["ref1", 212, 213], ["ref2", 574, 575]]
    c1 = names[1]
    synth_regions = [["c0", 0, 3000], [c1, 0, 1500], ["c0", 0, 1000], ["c0", 1000, 2990],
                     ["c0", 90, 180], ["c0", 650, 800], [c1, 1400, 1600], [c1, 1499, 1500],
                     ["c0", 2500, 4000], ["c0", 5000, 5100], ["c0", 1, 2], ["c0", 190, 330]]
    cases = []

    def add(bam_name, fasta_name, kc, k, regs, bam, fasta):
        for ref, s, e in regs:
            exp = run_case(bam, kcor[kc] if kc else None, k, fasta, ref, s, e)
            cases.append({"bam": bam_name, "fasta": fasta_name, "kcor": kc, "k": k,
                          "region": [ref, s, e], **exp})

    fbam = ox.DuckBam(os.path.join(HERE, "bbmap.sorted.bam"))
    ffa = ox.DuckFasta(os.path.join(HERE, "reference_1K.fa.gz"))
    sbam = ox.DuckBam(os.path.join(HERE, "synth_exp.bam"))
    sfa = ox.DuckFasta(os.path.join(HERE, "synth_exp.fa"))
    nbam = ox.DuckBam(os.path.join(HERE, "synth_exp_noseq.bam"))
    add("bbmap.sorted.bam", "reference_1K.fa.gz", "k4", 4, fixture_regions, fbam, ffa)
    add("bbmap.sorted.bam", "reference_1K.fa.gz", "k7sparse", 7, fixture_regions[:6], fbam, ffa)
    add("bbmap.sorted.bam", None, "k4zero", 4, fixture_regions[:6], fbam, None)
    add("synth_exp.bam", "synth_exp.fa", "k4", 4, synth_regions, sbam, sfa)
    add("synth_exp.bam", "synth_exp.fa", "k4zero", 4, synth_regions, sbam, sfa)
    add("synth_exp.bam", "synth_exp.fa", "k5", 5, synth_regions[:8], sbam, sfa)
    add("synth_exp.bam", None, "k5", 5, synth_regions[:4], sbam, None)
    add("synth_exp.bam", None, None, 4, synth_regions[:2], sbam, None)          # k_cor None
    add("synth_exp.bam", "synth_exp.fa", None, 4, synth_regions[:1], sbam, sfa)  # ecor unbound
    add("synth_exp_noseq.bam", None, "k4", 4, [["c0", 0, 500], ["c0", 0, 15]], nbam, None)
    with open(os.path.join(HERE, "experimental.json"), "w") as fh:
        json.dump({"kcor": kcor, "cases": cases}, fh, indent=0, sort_keys=True)
    errs = {}
    for c in cases:
        if "error" in c:
            errs[c["error"]] = errs.get(c["error"], 0) + 1
    print("%d cases, errors %s, zero-event cases %d" % (
        len(cases), errs, sum(1 for c in cases if c["stdout"])))


if __name__ == "__main__":
    main()
