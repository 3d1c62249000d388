"""GPU decode A/B of library builds on one BAM (each build in its own
process: METACOV_AMD_LIB selects it).

    python scripts/gz_pipeline_ab.py --make /tmp/e2e/ab.bam     # write the e2e BAM once
    python scripts/gz_pipeline_ab.py --bam /tmp/e2e/ab.bam --libs A.so B.so [--rounds 3]

Rounds interleave the builds; each prints the open time and the library's
decode timings (mc_bam_gpu_stats), and every build must keep the same records.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(bam):
    from metacov_amd.bam import GpuBamFile
    GpuBamFile(bam, device=0, n_threads=16).close()   # warm: device init, page cache
    t0 = time.perf_counter()
    g = GpuBamFile(bam, device=0, n_threads=16)
    dt = time.perf_counter() - t0
    out = {"open_s": dt, "kept": g.n_kept, **g.timings()}
    g.close()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--make")
    ap.add_argument("--bam")
    ap.add_argument("--libs", nargs="*", default=[])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--one", action="store_true")
    a = ap.parse_args()
    if a.make:
        import numpy as np
        from metacov_amd import synth
        lengths = np.full(1000, 1_000_000, np.int64)
        arrs = synth.edge_mix_arrays(lengths, 30_000_000, seed=1)
        synth.write_bam_fast(a.make, ["contig_%d" % i for i in range(1000)], lengths, *arrs, level=6,
                             n_threads=16)
        return
    if a.one:
        one(a.bam)
        return
    kept = None
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, METACOV_AMD_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", "--bam", a.bam],
                               env=env, capture_output=True, text=True, timeout=300)
            if p.returncode:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(p.returncode)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            assert kept is None or d["kept"] == kept, (lib, d["kept"], kept)
            kept = d["kept"]
            print("round %d %-14s open %.3f s  read %.1f  inflate %.1f  parse %.1f  scan %.1f  total %.1f ms  "
                  "windows %d" % (r, os.path.basename(lib), d["open_s"], d["read_ms"], d["inflate_ms"],
                                  d["parse_ms"], d["scan_ms"], d["total_ms"], d["windows"]), flush=True)


if __name__ == "__main__":
    main()
