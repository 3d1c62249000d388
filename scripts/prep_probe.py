"""Steady-state cost of mc_prepare (ingest + chunk index [+ long-read
buckets]) on device-resident reads: the first prepare of a ctx also
allocates the depth vector, so the batch is re-added and re-prepared
--reps times and the HIP-event prepare times of the repeats are reported.

    python scripts/prep_probe.py [--config c3|c5] [--reps 10] [--libs A.so B.so]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    ap.add_argument("--reps", type=int, default=10)
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
        first = None
        times = []
        for r in range(a.reps + 1):
            e.clear_reads()
            e.add_reads(tid, pos, span)
            e.prepare()
            t = e.timings()["prepare_ms"]
            if r == 0:
                first = t
            else:
                times.append(t)
        t = np.array(times)
        print("%s %-28s prepare first %.3f ms, repeat median %.4f ms min %.4f ms (n=%d)"
              % (a.config, os.path.basename(lib) if lib else "libmetacov_amd.so", first,
                 np.median(t), t.min(), len(t)), flush=True)
        e.close()


if __name__ == "__main__":
    main()
