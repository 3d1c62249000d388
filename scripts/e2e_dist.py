"""End-to-end `metacov pileup` over N ranks (torch.distributed.run, gloo for
the table so the ranks can share one GPU box) on the e2e BAM, with and
without a BAI: each rank GPU-decodes only its contigs' BGZF blocks.

    python scripts/e2e_dist.py [--reads 30000000 --contigs 1000 --length 1000000 --ranks 2]

Prints one JSON line: the 1-rank in-process GPU decode path for reference,
then per launch the wall time and every rank's phases (head = index read or
rank 0's whole-file decode + broadcast, decode = the shard's GPU decode,
rows, gather, total) parsed from the ranks' logs; all CSVs must be equal.
"""
import argparse
import io
import json
import os
import re
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def launch(path, out, ranks, extra=()):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MC_DIST_BACKEND="gloo",
               PYTHONPATH=os.pathsep.join([ROOT, os.environ.get("PYTHONPATH", "")]))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % ranks,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, "-m", "metacov_amd.cli", "pileup",
           "-b", path, "-o", out, *extra]
    t0 = time.perf_counter()
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    wall = time.perf_counter() - t0
    if p.returncode:
        sys.stderr.write(p.stderr[-4000:])
        raise SystemExit("launch failed")
    phases = [json.loads(m.group(2)) for m in re.finditer(r"rank (\d+)/\d+ phases: (\{.*\})", p.stderr)]
    return {"wall_s": wall, "ranks": phases}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=30_000_000)
    ap.add_argument("--contigs", type=int, default=1000)
    ap.add_argument("--length", type=int, default=1_000_000)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    import numpy as np
    from metacov_amd import synth, regions as mreg
    from metacov_amd.bam import GpuBamFile, build_index
    from metacov_amd.cli import write_rows
    lengths = np.full(a.contigs, a.length, np.int64)
    names = ["contig_%d" % i for i in range(a.contigs)]
    d = a.dir or tempfile.mkdtemp()
    path = os.path.join(d, "e2e.bam")
    arrs = synth.edge_mix_arrays(lengths, a.reads, seed=1)
    synth.write_bam_fast(path, names, lengths, *arrs, level=6, n_threads=a.threads)
    del arrs
    res = {"bam_bytes": os.path.getsize(path), "ranks": a.ranks}
    # one process, in-process timing (the single-GPU default path)
    t0 = time.perf_counter()
    gb = GpuBamFile(path, device=0, n_threads=a.threads)
    regs = list(mreg.get_regions_from_bam(gb))
    buf = io.StringIO()
    write_rows(gb, regs, buf)
    res["one_rank_in_process_s"] = time.perf_counter() - t0
    res["one_rank_decode"] = {k: gb.timings()[k] for k in ("total_ms", "open_ms", "blocks", "resyncs",
                                                             "parse_rounds")}
    gb.close()
    want = buf.getvalue()
    one = os.path.join(d, "one.csv")
    res["one_rank_cli"] = launch(path, one, 1)
    assert open(one, newline="").read() == want, "1-rank CSV differs"
    for tag in ("no_index", "index"):
        if tag == "index":
            t0 = time.perf_counter()
            build_index(path)
            res["index_build_s"] = time.perf_counter() - t0
        out = os.path.join(d, "%s.csv" % tag)
        res[tag] = launch(path, out, a.ranks)
        assert open(out, newline="").read() == want, "%s CSV differs" % tag
        print(json.dumps({tag: res[tag]}), file=sys.stderr, flush=True)
    res["csv_identical"] = True
    print(json.dumps(res))
    for f in (path, path + ".bai"):
        if os.path.exists(f):
            os.remove(f)


if __name__ == "__main__":
    main()
