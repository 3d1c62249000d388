"""In-process A/B of library builds (same GPU, same data, interleaved rounds).

    python scripts/ab_inproc.py --libs A.so B.so ... [--mode plain|fused]
                                [--rounds 5 --steps 10 --reads 100000000]

Each build gets its own mc_ctx over identical device-resident C3 reads; the
builds run alternately, round after round (cdna_hip_programming.md rule 24),
and their K2 times (HIP events) are reported as median / min.  Outputs are
cross-checked: every build must produce the same region rows as the first.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--mode", default="plain", choices=["plain", "fused", "both", "direct", "all"],
                    help="plain / fused: K2 on one explicit prepare's index; direct: every call a "
                         "fresh batch (mc_invalidate first: the direct prepare + validating fused K2)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--contigs", type=int, default=None, help="(c3) contigs, e.g. a strong-scaling shard")
    ap.add_argument("--nocheck", action="store_true", help="deliberately-wrong experiment builds")
    ap.add_argument("--loop", action="store_true", help="direct mode: also time back-to-back calls into a device table")
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    a = ap.parse_args()
    import torch
    from bench import CONFIGS, config_contigs, device_workload
    from metacov_amd.engine import CoverageEngine

    dev = torch.device("cuda", 0)
    reads = a.reads if a.config == "c3" else CONFIGS[a.config][0]
    lengths, weights = config_contigs(a.config, reads, a.contigs or CONFIGS[a.config][1])
    tid, pos, span, _ = device_workload(torch, lengths, weights, reads, 1, dev,
                                        long_reads=a.config == "c5")
    R = len(lengths)
    rt, rs, re_ = np.arange(R, dtype=np.int32), np.zeros(R, np.int64), lengths.astype(np.int64)
    engines = []
    for lib in a.libs:
        e = CoverageEngine(0, lib_path=os.path.abspath(lib))
        e.set_contigs(lengths)
        e.add_reads(tid, pos, span)
        engines.append(e)
    modes = {"both": ["plain", "fused"], "all": ["plain", "fused", "direct"]}.get(a.mode, [a.mode])
    for mode in modes:
        times = {lib: [] for lib in a.libs}
        walls = {lib: [] for lib in a.libs}
        ref_rows = None
        import time
        for _ in range(a.rounds):
            for lib, e in zip(a.libs, engines):
                if mode != "direct":
                    e.prepare()
                for _ in range(a.steps):
                    t0 = time.perf_counter()
                    if mode == "plain":
                        e.compute_depth()
                    else:
                        if mode == "direct":
                            e.invalidate()
                        rows = e.compute_depth_stats(rt, rs, re_)
                    e.synchronize()
                    walls[lib].append((time.perf_counter() - t0) * 1e3)
                    times[lib].append(e.timings()["depth_ms"])
                if mode == "plain":
                    rows = e.region_stats(rt, rs, re_)
                if ref_rows is None:
                    ref_rows = rows
                elif not a.nocheck:
                    for f in rows.dtype.names:
                        assert np.array_equal(rows[f], ref_rows[f]), (lib, f)
        if mode == "direct" and a.loop:
            # bench-like: back-to-back fresh-batch calls into a device table,
            # one synchronize per round (host gaps between calls included)
            import torch
            tbl = torch.empty((len(rt), 9), dtype=torch.int64, device="cuda")
            loops = {lib: [] for lib in a.libs}
            for _ in range(a.rounds):
                for lib, e in zip(a.libs, engines):
                    e.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(a.steps):
                        e.invalidate()
                        e.compute_depth_stats_device(rt, rs, re_, tbl.data_ptr())
                    e.synchronize()
                    loops[lib].append((time.perf_counter() - t0) * 1e3 / a.steps)
            for lib in a.libs:
                l = np.array(loops[lib])
                print("loop   %-48s per call median %.4f ms  min %.4f ms  (rounds %d x %d calls)"
                      % (os.path.basename(lib), np.median(l), l.min(), len(l), a.steps), flush=True)
        for lib in a.libs:
            t = np.array(times[lib])
            w = np.array(walls[lib])
            fb = engines[a.libs.index(lib)].fused_fallbacks() if mode != "plain" else 0
            print("%-6s %-48s K2 median %.4f ms  min %.4f ms  call median %.4f ms  fallbacks %d  (n=%d)"
                  % (mode, os.path.basename(lib), np.median(t), t.min(), np.median(w), fb, len(t)), flush=True)


if __name__ == "__main__":
    main()
