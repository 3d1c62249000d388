"""Generates the committed golden fixtures under tests/golden/.

Run ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It imports the reference's real `metacov.pileup.classic`
(`/root/reference/metacov/pileup.py:9-26`) and feeds it depth columns through
a duck-typed `bam` object whose `pileup(ref, start, end)` yields objects with
`.pos` / `.n` — the interface `classic` uses at `pileup.py:13-16`.  pysam and
htslib are not installed, so the column depths come from the oracle's
restatement of htslib's pileup count (`oracle/bamread.py`); the region
statistics are the reference's own arithmetic.

Outputs (JSON, plus synthetic BAMs written by `metacov_amd.synth`):
  fixture.json  bbmap.sorted.bam: header, decoded intervals, depth vectors,
                classic() for the regions.blast7 regions (cli.py:89 sort) and
                for whole contigs (util.py:64-69), and the expected CSV text
                of `metacov pileup` for both (cli.py:97-108)
  stats.json    classic() on edge-case and random depth vectors
  synth_*.bam + synth.json  edge-mix synthetic BAMs and their goldens; the
                synth_edge / synth_multi entries follow current htslib's
                bam_plp_push (a mapped read without reference-consuming ops
                has span 0), their "legacy" sub-entries the htslib <= 1.9
                bam_endpos rule (span 1)
"""
import csv
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")

from oracle import bamread  # noqa: E402
from metacov_amd import synth  # noqa: E402
from metacov.pileup import classic as ref_classic  # noqa: E402  (the real reference)
from metacov import blast as ref_blast  # noqa: E402


class _Col:
    __slots__ = ("pos", "n")

    def __init__(self, pos, n):
        self.pos, self.n = pos, n


class DuckBam:
    """Just enough of pysam.AlignmentFile for pileup.classic."""

    def __init__(self, names, depth):
        self.references = tuple(names)
        self._depth = dict(zip(names, depth))

    def pileup(self, ref, start, end):
        d = self._depth[ref]
        nz = np.nonzero(d)[0]
        for p in nz:
            yield _Col(int(p), int(d[p]))


def _py(v):
    return float(v) if isinstance(v, (float, np.floating)) else int(v)


def run_classic(bam, ref, start, end):
    try:
        r = ref_classic(bam, ref, start, end)
    except ValueError as e:
        return {"error": "ValueError", "msg": str(e)}
    return {k: _py(v) for k, v in r.items()}


def cli_csv(bam, regions):
    """Restates cli.py:85-108's CSV writing around the real classic()."""
    out = io.StringIO()
    writer = None
    name2ref = {w.split()[0]: w for w in bam.references}
    for hit in regions:
        ref = name2ref[hit[0]]
        start, end = sorted((int(hit[1]), int(hit[2])))
        result = ref_classic(bam, ref, start, end)
        if writer is None:
            writer = csv.DictWriter(out, fieldnames=["sacc", "start", "end"] + sorted(result))
            writer.writeheader()
        result.update({"sacc": hit[0], "start": hit[1], "end": hit[2]})
        writer.writerow(result)
    return out.getvalue()


def depth_with_extent(lengths, intervals):
    """Depth vectors over max(contig length, furthest read end): htslib emits
    pileup columns past the contig end when a read runs over it."""
    ext = list(lengths)
    for t, p, s in intervals:
        ext[t] = max(ext[t], p + s)
    return bamread.depth_vectors(ext, intervals), ext


def golden_fixture():
    path = os.path.join(HERE, "bbmap.sorted.bam")
    names, lengths, recs = bamread.read_bam(path)
    iv = bamread.pileup_intervals(recs)
    depth, ext = depth_with_extent(lengths, iv)
    bam = DuckBam(names, depth)
    with open(os.path.join(HERE, "regions.blast7")) as fh:
        hits = [(h.sacc, h.sstart, h.send) for h in ref_blast.reader(fh)]
    blast_stats = []
    for sacc, s, e in hits:
        a, b = sorted((int(s), int(e)))
        blast_stats.append({"sacc": sacc, "start": a, "end": b,
                            "stats": run_classic(bam, sacc, a, b)})
    whole = [{"sacc": n, "start": 0, "end": L, "stats": run_classic(bam, n, 0, L)}
             for n, L in zip(names, lengths)]
    out = {
        "names": names, "lengths": lengths, "extents": ext,
        "n_records": len(recs),
        "intervals": {"tid": [t for t, _, _ in iv], "pos": [p for _, p, _ in iv],
                      "span": [s for _, _, s in iv]},
        "aligned_bases": int(sum(s for _, _, s in iv)),
        "depth": [d.tolist() for d in depth],
        "blast7": blast_stats,
        "whole": whole,
        "csv_blast7": cli_csv(bam, hits),
        "csv_whole": cli_csv(bam, [(n, 0, L) for n, L in zip(names, lengths)]),
    }
    with open(os.path.join(HERE, "fixture.json"), "w") as fh:
        json.dump(out, fh)
    return out


def golden_stats():
    cases = []

    def add(vec, start, end, tag):
        names = ["c"]
        bam = DuckBam(names, [np.asarray(vec, dtype=np.int64)])
        cases.append({"tag": tag, "depth": [int(v) for v in vec], "start": start, "end": end,
                      "stats": run_classic(bam, "c", start, end)})

    add([1, 2], 0, 2, "even-median-trunc")
    add([1, 2, 4, 7], 0, 4, "q23-small")
    add([1, 2, 3, 2, 1], 3, 9, "past-end")
    add([5, 5, 5], 1, 1, "empty-region")
    add([0, 0, 0, 0], 0, 4, "all-zero")
    add([7], 0, 1, "single")
    add([3, 0, 9, 9, 1, 0, 2], 0, 7, "odd")
    rng = np.random.default_rng(20261015)
    for i in range(60):
        n = int(rng.integers(1, 3000))
        kind = i % 4
        if kind == 0:
            v = rng.poisson(rng.uniform(0.5, 400), size=n)
        elif kind == 1:
            v = rng.integers(0, 9000, size=n)
        elif kind == 2:
            v = rng.poisson(3, size=n) * (rng.random(n) < 0.3)
        else:
            v = np.repeat(rng.integers(0, 50, size=max(1, n // 50)), 50)[:n]
        a = int(rng.integers(0, max(1, n // 3)))
        b = int(rng.integers(a + 1, n + 40))
        add(v.tolist(), a, b, "random-%d" % i)
    with open(os.path.join(HERE, "stats.json"), "w") as fh:
        json.dump(cases, fh)
    return cases


def golden_synth():
    out = {}
    specs = [
        ("synth_edge", dict(lengths=[100_000], n_reads=10_000, readlen=100, seed=1234,
                            overhang=True, zero_span=True, unplaced=25)),
        ("synth_multi", dict(lengths=[5_000, 300, 12_000, 1, 64, 40_000, 7_777], n_reads=6_000,
                             readlen=150, seed=7, overhang=True, zero_span=True, unplaced=3)),
    ]
    for tag, kw in specs:
        lengths = kw.pop("lengths")
        names = ["contig_%d" % i for i in range(len(lengths))]
        recs = synth.edge_mix_records(lengths, **kw)
        path = os.path.join(HERE, tag + ".bam")
        synth.write_bam(path, names, lengths, recs)
        _n, _l, recs2 = bamread.read_bam(path)
        rng = np.random.default_rng(99)
        regions = [(n, 0, L) for n, L in zip(names, lengths)]
        for _ in range(20):
            t = int(rng.integers(0, len(lengths)))
            a = int(rng.integers(0, lengths[t]))
            b = int(rng.integers(a + 1, lengths[t] + 200))
            regions.append((names[t], a, b))
        entry = {}
        for legacy in (False, True):
            iv = bamread.pileup_intervals(recs2, legacy_endpos=legacy)
            depth, ext = depth_with_extent(lengths, iv)
            bam = DuckBam(names, depth)
            e = {
                "names": names, "lengths": [int(x) for x in lengths], "extents": ext,
                "n_records": len(recs2),
                "intervals": {"tid": [t for t, _, _ in iv], "pos": [p for _, p, _ in iv],
                              "span": [s for _, _, s in iv]},
                "depth_sha": [_sha(d) for d in depth],
                "depth_sum": [int(d.sum()) for d in depth],
                "regions": [{"sacc": s, "start": a, "end": b, "stats": run_classic(bam, s, a, b)}
                            for s, a, b in regions],
            }
            if legacy:
                entry["legacy"] = e
            else:
                entry.update(e)
        out[tag] = entry
    # long-CIGAR record through the CG:B,I tag (> 65535 ops)
    names, lengths = ["long"], [400_000]
    cig = []
    for k in range(70_000):
        cig += [(M, 2), (I, 1)] if k % 2 else [(M, 2), (D, 1)]
    rec = synth.SynthRecord("longcig", 0, 1000, 0, cig, sum(l for o, l in cig if o in (M, I)))
    short = synth.SynthRecord("short", 0, 2000, 0, [(M, 50)], 50)
    path = os.path.join(HERE, "synth_longcigar.bam")
    synth.write_bam(path, names, lengths, [rec, short], long_cigar_threshold=65535)
    _n, _l, recs2 = bamread.read_bam(path)
    iv = bamread.pileup_intervals(recs2)
    out["synth_longcigar"] = {"names": names, "lengths": lengths,
                              "intervals": {"tid": [t for t, _, _ in iv], "pos": [p for _, p, _ in iv],
                                            "span": [s for _, _, s in iv]}}
    with open(os.path.join(HERE, "synth.json"), "w") as fh:
        json.dump(out, fh)
    return out


def _sha(d):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(d, dtype="<i4").tobytes()).hexdigest()


M, I, D = synth.M, synth.I, synth.D

if __name__ == "__main__":
    f = golden_fixture()
    print("fixture aligned bases", f["aligned_bases"])
    for r in f["blast7"] + f["whole"]:
        print(r["sacc"], r["start"], r["end"], r["stats"])
    print(f["csv_blast7"])
    s = golden_stats()
    print("stats cases", len(s), s[:4])
    y = golden_synth()
    print("synth", {k: len(v["intervals"]["tid"]) for k, v in y.items()})
