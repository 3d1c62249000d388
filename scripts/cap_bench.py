"""htslib's max_depth cap (pysam's 8000, on by default) on deep contigs:
the capped recompute timed on the device path and on the host path.

    python scripts/cap_bench.py [--body 200 --deep 5000,10000,15000,20000]

A C3-shaped file: `--body` contigs of 200 kbp at 30x plus 50 kbp contigs at
the `--deep` depths (plasmid / phage-like), edge-mix records, written once.
Decoded on the GPU (GpuBamFile); every contig is one whole-contig region.
Timed: the exact fused rows (cli.compute_rows without the cap), then
depthcap.apply_cap on those rows — the regions whose exact max depth could
reach the cap recomputed (a) on the device (mc_add_reads_capped: gather,
cap walk and batch in HBM) and (b) on the host path (the intervals of those
contigs copied back, the per-region index lists, the C++ heap sweep on all
host threads, the batch uploaded).  Both must give the same rows.  Also the
mask alone: mc_depth_cap_mask_device vs mc_depth_cap_mask on the deep
contigs' reads.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _HostOnly:
    """A GpuBamFile seen without its device intervals: capped_rows takes the
    host path (intervals copied back from HBM)."""

    def __init__(self, g):
        self._g = g

    def intervals(self, contigs=None):
        return self._g.intervals(contigs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--body", type=int, default=200)
    ap.add_argument("--deep", default="5000,10000,15000,20000")
    ap.add_argument("--dir", default="/tmp/cap_bench")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    from metacov_amd import depthcap, synth
    from metacov_amd.bam import GpuBamFile
    from metacov_amd.cli import compute_rows
    deep = [int(x) for x in a.deep.split(",") if x]
    lengths = np.array([200_000] * a.body + [50_000] * len(deep), np.int64)
    depth = np.array([30.0] * a.body + deep, np.float64)
    n_reads = int((depth * lengths).sum() / 150)
    names = ["body_%d" % i for i in range(a.body)] + ["deep_%d" % d for d in deep]
    os.makedirs(a.dir, exist_ok=True)
    path = os.path.join(a.dir, "cap_%d_%s.bam" % (a.body, "_".join(map(str, deep))))
    t_gen = None
    if not os.path.exists(path):
        t0 = time.perf_counter()
        arrs = synth.edge_mix_arrays(lengths, n_reads, seed=3, weights=depth * lengths)
        synth.write_bam_fast(path + ".tmp", names, lengths, *arrs, l_seq=0, level=1, n_threads=16)
        os.replace(path + ".tmp", path)
        t_gen = time.perf_counter() - t0
    g = GpuBamFile(path)
    R = len(lengths)
    tids = np.arange(R, dtype=np.int32)
    starts = np.zeros(R, np.int64)
    ends = lengths.copy()
    out = {"bam": path, "bam_bytes": os.path.getsize(path), "reads": n_reads, "kept": g.n_kept,
           "contigs": R, "deep_depths": deep, "generate_s": t_gen}
    times = {"exact_rows_s": [], "cap_device_s": [], "cap_host_s": []}
    for _ in range(a.reps):
        t0 = time.perf_counter()
        rows, _ = compute_rows(g, tids, starts, ends, max_depth=0)
        times["exact_rows_s"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        dev_rows, n_cap, dropped = depthcap.apply_cap(g, rows, tids, starts, ends, lengths, 8000)
        times["cap_device_s"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        host_rows, n_cap_h, dropped_h = depthcap.apply_cap(_HostOnly(g), rows, tids, starts, ends, lengths, 8000)
        times["cap_host_s"].append(time.perf_counter() - t0)
        assert np.array_equal(dev_rows, host_rows) and dropped == dropped_h and n_cap == n_cap_h
    out.update({k: min(v) for k, v in times.items()})
    out["all_times"] = times
    out["regions_recomputed"] = int(n_cap)
    out["reads_dropped"] = int(dropped)
    out["max_depth_exact"] = [int(x) for x in rows["max"][-len(deep):]] if deep else []
    out["max_depth_capped"] = [int(x) for x in dev_rows["max"][-len(deep):]] if deep else []
    # the mask alone on the deep contigs' reads (one query per contig)
    deep_ids = np.arange(a.body, R)
    tid, pos, span = g.intervals(deep_ids)
    t0 = time.perf_counter()
    keep_h, dh = depthcap.cap_mask(tid, pos, span, 8000)
    out["mask_host_s"] = time.perf_counter() - t0
    out["mask_host_threads"] = os.cpu_count()
    import torch
    tt, pp, ss = (torch.from_numpy(x).cuda() for x in (tid, pos, span))
    best = None
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        keep_d, dd = depthcap.cap_mask_device(tt, pp, ss, 8000)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    assert dd == dh and np.array_equal(keep_d.cpu().numpy().astype(bool), keep_h)
    out["mask_device_s"] = best
    out["mask_reads"] = int(len(tid))
    g.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
