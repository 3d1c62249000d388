"""Cold `metacov pileup` wall time: a fresh `python -m metacov_amd.cli pileup`
process per run, from process start to the CSV on disk.

    python scripts/cold_cli.py [--reads 30000000 --contigs 1000 --length 1000000] [--runs 3]

Writes (once) the same edge-mix BAM as scripts/e2e.py (30 M records, 1000
contigs of 1 Mbp, ~5.2 GB), then runs the CLI `--runs` times as a child
process with MC_CLI_TIMES set: the child reports its phases (interpreter
and imports, CLI parse, library load, HIP init, decode, regions, rows,
write; metacov_amd.cli._PhaseTimes) and this script the wall clock around
the whole child.  The BAM is in the page cache (it was just written or
read); the first run also pays the first-`import` disk reads of a fresh
box.  Every run's CSV must be identical.  Prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=30_000_000)
    ap.add_argument("--contigs", type=int, default=1000)
    ap.add_argument("--length", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/cold_cli")
    ap.add_argument("--extra", default="", help="extra CLI arguments")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    path = os.path.join(a.dir, "e2e_%d_%d_%d.bam" % (a.reads, a.contigs, a.length))
    t_gen = None
    if not os.path.exists(path):
        import numpy as np
        from metacov_amd import synth
        t0 = time.perf_counter()
        lengths = np.full(a.contigs, a.length, np.int64)
        arrs = synth.edge_mix_arrays(lengths, a.reads, seed=1)
        synth.write_bam_fast(path + ".tmp", ["contig_%d" % i for i in range(a.contigs)], lengths, *arrs,
                             level=6, n_threads=a.threads)
        os.replace(path + ".tmp", path)
        t_gen = time.perf_counter() - t0
    runs, csv0 = [], None
    for k in range(a.runs):
        out = os.path.join(a.dir, "out_%d.csv" % k)
        tj = os.path.join(tempfile.mkdtemp(), "times.json")
        env = dict(os.environ, MC_CLI_TIMES=tj)
        cmd = [sys.executable, "-m", "metacov_amd.cli", "pileup", "-b", path, "-o", out] + a.extra.split()
        t0 = time.time()
        env["MC_CLI_T0"] = repr(t0)
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True)
        wall = time.time() - t0
        if p.returncode != 0:
            print(p.stderr[-3000:], file=sys.stderr)
            sys.exit(p.returncode)
        with open(tj) as fh:
            phases = json.load(fh)
        phases["wall_s"] = wall
        phases["exit_after_csv_s"] = wall - phases["total_s"]
        runs.append(phases)
        data = open(out, "rb").read()
        if csv0 is None:
            csv0 = data
        assert data == csv0, "run %d's CSV differs" % k
    best = min(runs, key=lambda r: r["wall_s"])
    print(json.dumps({"bam": path, "bam_bytes": os.path.getsize(path), "records": a.reads, "contigs": a.contigs,
                      "generate_s": t_gen, "csv_rows": csv0.count(b"\n") - 1, "runs": runs,
                      "best_wall_s": best["wall_s"],
                      "note": "wall = launcher clock around the child; phases from the child (MC_CLI_TIMES)"}))


if __name__ == "__main__":
    main()
