"""Batches in flight on two engines (two ctx, two HIP streams, two host
threads) against one engine, on the bench's workloads.

    python scripts/bench_streams.py [--configs c2,c3,s8] [--steps 40]

Each engine holds its own copy of the same device-resident batch and runs
the headline step (mc_invalidate, then the fused call: probe + K2 + K3b) in
a loop; the library's calls release the GIL, so the two threads' calls
overlap on the GPU: one batch's launch gaps and host turnaround, and the
workgroup slots a small batch leaves idle (C2: 610 chunks for 1024
resident workgroups), go to the other.  Reported: batches/s and aligned
bases/s for one engine and for two, and both engines' rows checked equal to
the one engine's.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,s8,c3")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import torch
    from bench import CONFIGS, config_contigs, device_workload
    from metacov_amd.engine import CoverageEngine, REGION_STAT_DTYPE  # noqa: F401

    dev = torch.device("cuda", 0)
    out = {"note": __doc__.strip().splitlines()[0], "runs": []}
    for cfg in a.configs.split(","):
        name, reads, contigs = cfg, None, None
        if cfg == "s8":   # one rank's share of C3 at N = 8
            cfg, reads, contigs = "c3", 12_500_000, 125
        reads = reads or CONFIGS[cfg][0]
        contigs = contigs or CONFIGS[cfg][1]
        lengths, weights = config_contigs(cfg, reads, contigs)
        tid, pos, span, _ = device_workload(torch, lengths, weights, reads, 1, dev, long_reads=cfg == "c5")
        R = len(lengths)
        rt, rs, re_ = np.arange(R, dtype=np.int32), np.zeros(R, np.int64), lengths.astype(np.int64)
        engines, tables = [], []
        for _ in range(2):
            e = CoverageEngine(0)
            e.set_contigs(lengths)
            e.add_reads(tid, pos, span)
            engines.append(e)
            tables.append(torch.empty((R, 9), dtype=torch.int64, device=dev))
        bases = None

        def loop(e, tbl, n):
            for _ in range(n):
                e.invalidate()
                e.compute_depth_stats_device(rt, rs, re_, tbl.data_ptr())

        for e, t in zip(engines, tables):
            loop(e, t, a.warmup)
        torch.cuda.synchronize()
        bases = engines[0].aligned_bases()
        ref = tables[0].cpu().clone()
        # one engine
        t0 = time.perf_counter()
        loop(engines[0], tables[0], a.steps)
        torch.cuda.synchronize()
        one = time.perf_counter() - t0
        # two engines, two threads, the same number of batches each
        ths = [threading.Thread(target=loop, args=(e, t, a.steps)) for e, t in zip(engines, tables)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        torch.cuda.synchronize()
        two = time.perf_counter() - t0
        same = all(torch.equal(t.cpu(), ref) for t in tables)
        run = {"config": name, "reads": reads, "contigs": contigs, "steps_per_engine": a.steps,
               "one_engine": {"ms_per_batch": one / a.steps * 1e3,
                              "aligned_bases_per_s": bases * a.steps / one},
               "two_engines": {"ms_per_batch": two / (2 * a.steps) * 1e3,
                               "aligned_bases_per_s": bases * 2 * a.steps / two},
               "speedup": (one / a.steps) / (two / (2 * a.steps)), "rows_equal": bool(same)}
        out["runs"].append(run)
        print(json.dumps(run), file=sys.stderr, flush=True)
        del engines, tables
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
