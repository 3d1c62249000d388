"""How wide a fused-histogram window each C5 region needs (CPU analysis).

Regenerates the C5 workload with bench.py's generator on the CPU (torch's CPU
generator: the same distributions, not the same numbers as on the GPU), builds
each contig's exact depth, and reports how many whole-contig regions fall
outside the window the engine places ([body - 648, body + 216), engine.hip
depth_stats_impl) and how wide a window their quartile ranks would need.

    python scripts/c5_window_need.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import config_contigs, device_workload

    t0 = time.time()
    lengths, weights = config_contigs("c5", 50_000_000, 10_000)
    tid, pos, span, _ = device_workload(torch, lengths, weights, 50_000_000, 1, torch.device("cpu"),
                                        long_reads=True)
    tid, pos, span = tid.numpy(), pos.numpy(), span.numpy()
    print("generated in %.1f s" % (time.time() - t0), flush=True)
    nc = len(lengths)
    span_mean = span.astype(np.float64).mean()
    cbases = np.bincount(tid, weights=span.astype(np.float64), minlength=nc)
    first = np.concatenate([[0], np.cumsum(np.bincount(tid, minlength=nc))])
    qlo, qhi, mlo, mhi, body_depth = (np.zeros(nc) for _ in range(5))
    for c in range(nc):
        L = int(lengths[c])
        a, b = first[c], first[c + 1]
        d = np.zeros(L + 1, np.int64)
        np.add.at(d, pos[a:b], 1)
        np.add.at(d, pos[a:b] + span[a:b], -1)
        dep = np.sort(np.cumsum(d[:L]))
        qlo[c], qhi[c] = dep[L // 4], dep[L - L // 4 - 1]
        mlo[c], mhi[c] = dep[(L - 1) // 2], dep[L // 2]
        body = L - span_mean if L > 2 * span_mean else L
        body_depth[c] = cbases[c] / body
    base = np.maximum(0, np.round(body_depth) - 648)
    fb = (qlo < base) | (mlo < base) | (qhi >= base + 864) | (mhi >= base + 864)
    need = qhi - qlo
    print("fallback regions with the engine's window: %d (mean span %.0f)" % (fb.sum(), span_mean))
    for t in [864, 1024, 1296, 1728, 2048, 3456]:
        print("regions needing a window of at least %d values: %d" % (t, (need >= t).sum()))


if __name__ == "__main__":
    main()
