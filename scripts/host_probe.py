"""Host-side latency of the fused call and of a re-prepare (C3, device-
resident reads): wall-clock per C call against the HIP-event kernel times,
so the gaps between launches (host work, stream syncs, small copies) show.

    python scripts/host_probe.py [--config c3|c5] [--reps 20] [--libs A.so B.so]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--libs", nargs="*", default=[None])
    a = ap.parse_args()
    import torch
    from bench import CONFIGS, config_contigs, device_workload
    from metacov_amd.engine import CoverageEngine

    dev = torch.device("cuda", 0)
    reads, contigs, _ = CONFIGS[a.config]
    lengths, weights = config_contigs(a.config, reads, contigs)
    tid, pos, span, _ = device_workload(torch, lengths, weights, reads, 1, dev,
                                        long_reads=a.config == "c5")
    torch.cuda.synchronize()
    for lib in a.libs:
        e = CoverageEngine(0, lib_path=os.path.abspath(lib) if lib else None)
        e.set_contigs(lengths)
        e.add_reads(tid, pos, span)
        R = len(lengths)
        rt = np.arange(R, dtype=np.int32)
        rs = np.zeros(R, np.int64)
        re_ = lengths.astype(np.int64)
        table = torch.empty((R, 9), dtype=torch.int64, device=dev)
        for _ in range(3):
            e.compute_depth_stats_device(rt, rs, re_, table.data_ptr())
        keys = ["call (cached regions)", "invalidate+prepare", "call after prepare", "direct fresh call"]
        rows = {k: [] for k in keys}
        kern = {k: [] for k in keys}
        for _ in range(a.reps):
            t0 = e.timings()
            w0 = time.perf_counter()
            e.compute_depth_stats_device(rt, rs, re_, table.data_ptr())
            w1 = time.perf_counter()
            t1 = e.timings()
            rows["call (cached regions)"].append((w1 - w0) * 1e3)
            kern["call (cached regions)"].append((t1["fused_depth_ms_total"] - t0["fused_depth_ms_total"]) +
                                                 (t1["fused_stats_ms_total"] - t0["fused_stats_ms_total"]))
            w0 = time.perf_counter()
            e.invalidate()
            e.prepare()
            w1 = time.perf_counter()
            rows["invalidate+prepare"].append((w1 - w0) * 1e3)
            kern["invalidate+prepare"].append(e.timings()["prepare_ms"])
            t0 = e.timings()
            w0 = time.perf_counter()
            e.compute_depth_stats_device(rt, rs, re_, table.data_ptr())
            w1 = time.perf_counter()
            t1 = e.timings()
            rows["call after prepare"].append((w1 - w0) * 1e3)
            kern["call after prepare"].append((t1["fused_depth_ms_total"] - t0["fused_depth_ms_total"]) +
                                              (t1["fused_stats_ms_total"] - t0["fused_stats_ms_total"]))
            # a fresh batch on the direct path: probe + window + validating K2 + K3b
            t0 = e.timings()
            w0 = time.perf_counter()
            e.invalidate()
            e.compute_depth_stats_device(rt, rs, re_, table.data_ptr())
            w1 = time.perf_counter()
            t1 = e.timings()
            assert t1["direct_batches"] == t0["direct_batches"] + 1
            rows["direct fresh call"].append((w1 - w0) * 1e3)
            kern["direct fresh call"].append(sum(t1[k] - t0[k] for k in (
                "fused_depth_ms_total", "fused_stats_ms_total", "prepare_ms_total")))
        for k in rows:
            w, g = np.median(rows[k]), np.median(kern[k])
            name = os.path.basename(lib or "libmetacov_amd.so")
            print("%s %s %-24s wall %.4f ms  events %.4f ms  host/gaps %.4f ms"
                  % (a.config, name, k, w, g, w - g), flush=True)
        e.close()


if __name__ == "__main__":
    main()
