"""Benchmark of the `scan` histogram kernel (SURVEY.md §8 f rank 3).

    python scripts/bench_scan.py [--reads N] [--steps K] [--warmup W] [--group-by FLAG ...]

Workload (C3-shaped, per GPU): 1000 contigs with the C3 lengths (~1.0 Gbp,
random A/C/G/T in HBM), 100M x 150 bp reads sampled from them by lognormal
abundance, 1% substitutions, half on the reverse strand, 90% proper pairs
with N(450, 150) insert sizes; every read's packed nt16 bases (75 B), its
5 int32 accessor values and int64 base offset resident in HBM (~11 GB).
The processors are the CLI's defaults with every table on: BaseHist(0),
KmerHist(7, 8, 7, 0), MirrorHist(4, 10), IsizeHist.

One step = one mc_scan_add_batch_device launch over all reads (histograms
accumulate across steps).  HIP events on the library's stream time it.
Algorithmic bytes per launch = 28 B per read (5 int32 + int64 offset) +
the packed bases (ceil(rlen/2) B per read; stored 4-byte aligned, 76 B) +
the reference once (1 B/base).
The CPU baseline is the C port of the reference's read loop
(oracle/scan_oracle.c) on one host core over a sample of the same reads.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--group-by", action="append", default=[])
    ap.add_argument("--procs", default="base,kmer,mirror,isize",
                    help="processors to run (comma list of base, kmer, mirror, isize)")
    ap.add_argument("--cpu-sample", type=int, default=5_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", type=int, default=2_000_000,
                    help="reads checked bit-exact against the C port before timing (0: off)")
    return ap.parse_args(argv)


def workload(torch, n_reads, dev, seed=11, chunk=2_000_000):
    from metacov_amd import synth
    lengths, weights = synth.c3_workload(n_reads, 1000)
    rng = np.random.default_rng(seed)
    counts = rng.multinomial(n_reads, weights / weights.sum())
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    coff = np.zeros(len(lengths) + 1, np.int64)
    coff[1:] = np.cumsum(lengths)
    ref = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)[
        torch.randint(0, 4, (int(coff[-1]),), device=dev, generator=g)]
    tid = torch.repeat_interleave(torch.arange(len(lengths), device=dev, dtype=torch.int32),
                                  torch.from_numpy(counts).to(dev))
    L = torch.from_numpy(lengths).to(dev)[tid.long()]
    rl = 150
    pos = (torch.rand(n_reads, device=dev, generator=g, dtype=torch.float64) *
           (L - rl + 1).double()).long()
    order = torch.argsort(torch.from_numpy(coff[:-1]).to(dev)[tid.long()] + pos)
    tid, pos = tid[order].contiguous(), pos[order].contiguous()
    u = torch.rand(n_reads, device=dev, generator=g)
    rev = torch.rand(n_reads, device=dev, generator=g) < 0.5
    flag = (0x1 | torch.where(torch.arange(n_reads, device=dev) % 2 == 0, 0x40, 0x80)).int()
    flag |= (u < 0.9).int() * 0x2 | rev.int() * 0x10
    rlen = torch.full((n_reads,), rl, dtype=torch.int32, device=dev)
    gpos = (pos + rev.long() * rl).int()
    isz = (torch.randn(n_reads, device=dev, generator=g) * 150 + 450).clamp(min=1).int()
    isz = torch.where(torch.rand(n_reads, device=dev, generator=g) < 0.5, isz, -isz)
    gisize = torch.where((flag & 0x2) != 0, isz, torch.zeros_like(isz))
    ref_id = tid.clone()
    nb = ((rl + 1) // 2 + 3) & ~3          # 4-byte aligned starts (75 -> 76 B)
    seq_off = torch.arange(n_reads + 1, device=dev, dtype=torch.int64) * nb
    seq = torch.zeros(n_reads * nb, dtype=torch.uint8, device=dev)
    seq2 = seq.view(n_reads, nb)
    code = torch.zeros(256, dtype=torch.uint8, device=dev)
    for ch, v in zip(b"ACGT", (1, 2, 4, 8)):
        code[ch] = v
    cof = torch.from_numpy(coff[:-1]).to(dev)
    ar = torch.arange(rl, device=dev)
    for a in range(0, n_reads, chunk):
        b = min(n_reads, a + chunk)
        start = cof[tid[a:b].long()] + pos[a:b]
        bases = code[ref[start[:, None] + ar[None, :]].long()]
        mut = torch.rand(bases.shape, device=dev, generator=g) < 0.01
        rnd = torch.tensor([1, 2, 4, 8, 15], dtype=torch.uint8, device=dev)[
            torch.randint(0, 5, bases.shape, device=dev, generator=g)]
        bases = torch.where(mut, rnd, bases)
        seq2[a:b, :rl // 2] = (bases[:, 0::2] << 4) | bases[:, 1::2]
    del order, u, rev, L, isz
    return dict(rlen=rlen, flag=flag, gpos=gpos, gisize=gisize, ref_id=ref_id, seq_off=seq_off,
                seq=seq, ref=ref, coff=coff, lengths=lengths,
                max_isize=int(gisize.abs().max().item()), seq_bytes=(rl + 1) // 2 * n_reads)


def config(group_by, procs=("base", "kmer", "mirror", "isize")):
    from metacov_amd import _lib, scan as mscan
    cfg = _lib.ScanConfig()
    cfg.n_flags = len(group_by)
    for i, f in enumerate(group_by):
        cfg.flags[i] = mscan.Flags[f].flag
    cfg.base_on, cfg.base_start = int("base" in procs), 0
    cfg.kmer_on, cfg.kmer_k, cfg.kmer_nk, cfg.kmer_step, cfg.kmer_offset = \
        int("kmer" in procs), 7, 8, 7, 0
    cfg.mirror_on, cfg.mirror_offset, cfg.mirror_n = int("mirror" in procs), 4, 10
    cfg.isize_on = int("isize" in procs)
    return cfg


def make_scan(lib, cfg, w):
    from metacov_amd import _lib
    h = ctypes.c_void_p()
    _lib.check(lib.mc_scan_create(0, ctypes.byref(cfg), ctypes.byref(h)), lib)
    ref = w["ref"].cpu().numpy()
    off = np.ascontiguousarray(w["coff"][:-1], np.int64)
    ln = np.ascontiguousarray(w["lengths"], np.int64)
    _lib.check(lib.mc_scan_set_reference(h, len(ln), _lib.ptr(off), _lib.ptr(ln), ref.size,
                                         _lib.ptr(ref)), lib)
    return h


def launch(lib, h, w, a, b, ms=None):
    from metacov_amd import _lib
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
    n = b - a
    cols = [w[k][a:b] for k in ("rlen", "flag", "gpos", "gisize", "ref_id")]
    off = w["seq_off"][a:b + 1]
    seq = w["seq"]
    _lib.check(lib.mc_scan_add_batch_device(h, n, *[P(c) for c in cols], P(off), P(seq), 150,
                                            w["max_isize"],
                                            ctypes.byref(ms) if ms is not None else None), lib)


def results(lib, h, cfg):
    from metacov_amd import _lib
    G, rows, cap = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
    lib.mc_scan_dims(h, ctypes.byref(G), ctypes.byref(rows), ctypes.byref(cap), None, None)
    G = G.value
    out = (np.zeros((G, rows.value, 5), np.uint32), np.zeros((G, 4 ** 7 + 1, 8), np.uint32),
           np.zeros((G, 11, 2), np.uint32), np.zeros((G, cap.value), np.uint32),
           np.zeros(G, np.int32))
    _lib.check(lib.mc_scan_results(h, *[_lib.ptr(x) for x in out]), lib)
    return out, rows.value, cap.value


def host_batch(w, a, b):
    cols = [w[k][a:b].cpu().numpy() for k in ("rlen", "flag", "gpos", "gisize", "ref_id")]
    off = w["seq_off"][a:b + 1].cpu().numpy()
    seq = w["seq"][int(off[0]):int(off[-1])].cpu().numpy()
    return cols + [off - off[0], seq]


def ref_nt4(w):
    t = np.full(256, 4, np.uint8)
    for ch, v in zip(b"ACGTacgt", (0, 1, 2, 3, 0, 1, 2, 3)):
        t[ch] = v
    return t[w["ref"].cpu().numpy()]


# MI355X issue peaks (MI355X_MICROARCH.md): a wave64 VALU instruction issues
# over 2 cycles on a SIMD-32 (4 SIMDs per CU); the LDS array takes one
# 64-lane dword instruction per 2 cycles per CU; 256 CUs at 2.4 GHz.
VALU_PEAK = 256 * 4 * 0.5 * 2.4e9      # wave-instructions / s
LDS_PEAK = 256 * 0.5 * 2.4e9


def issue_roofline(kern_ms):
    """The launch's VALU and LDS issue rates against the chip's, from the SQ
    counters of profiles/sq_scan_kernel.json (scripts/sq_scan_summary.py)
    when they were taken on the current csrc/scan.hip, else None."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from sq_scan_summary import scan_source_id
    p = os.path.join(ROOT, "profiles", "sq_scan_kernel.json")
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        d = json.load(fh)
    if d.get("source_id") != scan_source_id(ROOT):
        return None
    k = d["kernels"]
    valu = sum(v.get("SQ_INSTS_VALU", 0) for v in k.values())
    lds = sum(v.get("SQ_INSTS_LDS", 0) for v in k.values())
    t = kern_ms * 1e-3
    return {"bound": "issue", "unit": "wave-instructions/s",
            "valu": {"achieved": valu / t, "peak": VALU_PEAK, "frac": valu / t / VALU_PEAK, "insts": valu},
            "lds": {"achieved": lds / t, "peak": LDS_PEAK, "frac": lds / t / LDS_PEAK, "insts": lds},
            "per_kernel": k, "record": "profiles/sq_scan_kernel.json (%s)" % d.get("tag")}


def main(argv=None):
    args = parse(argv)
    import torch
    torch.zeros(1, device="cuda")          # torch's HIP runtime first (tests/conftest.py)
    from metacov_amd import _lib
    from oracle import coracle
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    w = workload(torch, args.reads, dev)
    torch.cuda.synchronize()
    gen_s = time.time() - t0
    cfg = config(args.group_by, args.procs.split(","))
    n = args.reads
    nt4 = None
    check = None
    if args.check:
        m = min(args.check, n)
        h = make_scan(lib, cfg, w)
        launch(lib, h, w, 0, m)
        got, rows, cap = results(lib, h, cfg)
        lib.mc_scan_destroy(h)
        nt4 = ref_nt4(w)
        want, _ = coracle.scan(cfg, host_batch(w, 0, m), nt4, np.ascontiguousarray(w["coff"][:-1]),
                               np.ascontiguousarray(w["lengths"]), rows, cap)
        # (a table that is off: the C port returns it empty, the kernel's stays zero)
        same = lambda x, y: np.array_equal(x, y) or (y.size == 0 and not x.any())   # noqa: E731
        check = all(same(x, y) for x, y in zip(got, want))
        if not check:
            names = ("base", "kmer", "mirror", "isize", "isize_max")
            bad = ["%s: %d cells differ (got sum %d, want sum %d)" % (nm, int((x != y).sum()), int(x.sum()), int(y.sum()))
                   if x.shape == y.shape else "%s: shape %s vs %s" % (nm, x.shape, y.shape)
                   for nm, x, y in zip(names, got, want) if not same(x, y)]
            raise SystemExit("scan kernel differs from the C port on the first %d reads: %s" % (m, "; ".join(bad)))
    h = make_scan(lib, cfg, w)
    ms = ctypes.c_float()
    for _ in range(args.warmup):
        launch(lib, h, w, 0, n, ms)
    torch.cuda.synchronize()
    times = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        launch(lib, h, w, 0, n, ms)
        times.append(ms.value)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    lib.mc_scan_destroy(h)
    kern_ms = float(np.mean(times))
    seq_bytes = w["seq_bytes"]     # 75 B of bases per read (the padding byte is layout)
    ref_bytes = int(w["coff"][-1])
    alg = 28 * n + seq_bytes + ref_bytes
    bases = 150 * n
    line = {
        "metric": "reads/sec through the metacov scan histograms (BaseHist+KmerHist+MirrorHist+"
                  "IsizeHist), 1 MI355X",
        "value": n * args.steps / wall, "unit": "reads/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8/int32",
        "data": "synthetic (GPU-generated C3-shaped reads with bases from a random reference)",
        "config": {"workload": "C3-shaped scan: 1000 contigs (~1.0 Gbp), %d x 150 bp reads, "
                               "CLI-default parameters, processors %s, group-by %s"
                               % (n, args.procs, args.group_by or "none"),
                   "bases_per_step": bases, "input": "SoA accessor columns + packed nt16 bases "
                                                     "in HBM", "generate_s": round(gen_s, 2)},
        "bases_per_s": bases * args.steps / wall,
        "kernels_ms": {"scan_kernel+kmer_count_kernel": kern_ms},
        "roofline": {"bound": "hbm", "achieved": alg / (kern_ms * 1e-3) / 1e9, "peak": 8000.0,
                     "unit": "GB/s", "frac": alg / (kern_ms * 1e-3) / 8e12, "traffic": None,
                     "kernel": "scan_kernel + kmer_count_kernel (one mc_scan_add_batch_device)",
                     "algorithmic_bytes_per_launch": alg,
                     "note": "HBM bytes are the floor; the launch is VALU/LDS-issue bound "
                             "(BaseHist: ~10 VALU ops per base)"},
        "checked_reads_vs_c_port": args.check if check else 0,
    }
    issue = issue_roofline(kern_ms)
    if issue is not None:
        line["roofline_issue"] = issue
    if not args.no_cpu_baseline:
        m = min(args.cpu_sample, n)
        if nt4 is None:
            nt4 = ref_nt4(w)
        hb = host_batch(w, 0, m)
        t0 = time.perf_counter()
        coracle.scan(cfg, hb, nt4, np.ascontiguousarray(w["coff"][:-1]),
                     np.ascontiguousarray(w["lengths"]), 150, 4096)
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": m / dt, "unit": "reads/s", "cores": 1, "kind": "port",
                                "sample": "first %d reads of the workload, %.2f s; "
                                          "oracle/scan_oracle.c orc_scan (the reference's "
                                          "scan_reads loop restated in C)" % (m, dt)}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
