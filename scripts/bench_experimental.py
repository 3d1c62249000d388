"""`pileup.experimental` (the -k columns, reference metacov/pileup.py:38-173)
on a C3-shaped subset: the first --contigs contigs of the C3 workload
(lengths and lognormal abundances as bench.py's C3) at C3 read density, a
random reference FASTA, a random 7-mer correction table.

    python scripts/bench_experimental.py [--contigs 40 --reps 3]

Times, per whole-contig region set: the read table opened with the host
decode (mc_reads_open) and with the GPU decode (mc_reads_open_gpu; the two
tables compared field for field), the batch's host read pass
(mc_experimental_reads), the GPU k-mer correlation (ecor_kernel, HIP events)
against the MI355X FP64 vector peak, the whole experimental_batch call, and
the CPU restatement of the reference's sequence side (oracle/experimental.py
raw_ecor: the reference's per-position np.inner loop, pileup.py:63-88) on a
bounded sample, scaled per position.  Prints one JSON line.
"""
import argparse
import itertools
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (AMD spec; 1/2 of the 157.3 TF FP32 vector peak)
TAPS = 900                       # 2 * INSERT taps of the normal pdf (pileup.py:55-60)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contigs", type=int, default=40)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--oracle-positions", type=int, default=40_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    import numpy as np
    from metacov_amd import synth
    from metacov_amd import experimental as mx
    lengths_all, weights_all = synth.c3_workload(100_000_000, 1000)
    k = a.contigs
    lengths, weights = lengths_all[:k], weights_all[:k]
    n_reads = int(100_000_000 * weights.sum() / weights_all.sum())
    names = ["contig_%d" % i for i in range(k)]
    d = a.dir or tempfile.mkdtemp()
    bam, fasta = os.path.join(d, "exp.bam"), os.path.join(d, "exp.fa")
    arrs = synth.edge_mix_arrays(lengths, n_reads, seed=3, weights=weights)
    synth.write_bam_fast(bam, names, lengths, *arrs, level=1, n_threads=a.threads)
    del arrs
    rng = np.random.default_rng(4)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    seqs = {n: acgt[rng.integers(0, 4, int(L))].tobytes().decode() for n, L in zip(names, lengths)}
    synth.write_fasta(fasta, seqs)
    keys = ["".join(p) for p in itertools.product("ACGT", repeat=7)]
    k_cor = [{x: float(rng.uniform(0.5, 1.5)) for x in keys if rng.random() < 0.9} for _ in range(2)]
    regions = [(n, 0, int(L)) for n, L in zip(names, lengths)]
    positions = int(lengths.sum())
    runs = []
    for rep in range(a.reps):
        t0 = time.perf_counter()
        reads_h = mx.ReadTable(bam, 7, a.threads, decode="host")
        t_open = time.perf_counter() - t0
        t0 = time.perf_counter()
        reads = mx.ReadTable(bam, 7, a.threads, decode="gpu", device=0)
        t_open_gpu = time.perf_counter() - t0
        if rep == 0:   # the two decodes' tables, field for field
            fh, fg = reads_h.fields(), reads.fields()
            for key in fh:
                same = fh[key] == fg[key] if isinstance(fh[key], list) else np.array_equal(fh[key], fg[key])
                assert same, "GPU-decoded read table differs from the host's in " + key
        reads_h.close()
        fa = mx.FastaFile(fasta)
        tm = {}
        t0 = time.perf_counter()
        res = mx.experimental_batch(reads, k_cor, 7, fa, regions, device=0, n_threads=a.threads,
                                    timings=tm)
        t_batch = time.perf_counter() - t0
        # the same batch with the read pass on the host (the table copied back)
        tm_h = {}
        os.environ["MC_EXP_READS"] = "host"
        try:
            res_h = mx.experimental_batch(reads, k_cor, 7, fa, regions, device=0, n_threads=a.threads,
                                          timings=tm_h)
        finally:
            del os.environ["MC_EXP_READS"]
        assert [repr((r.row, r.zero_lines)) for r in res] == [repr((r.row, r.zero_lines)) for r in res_h], \
            "device read pass differs from the host pass"
        reads.close()
        assert all(r.error is None for r in res)
        ecor_ms = tm["ecor_kernel_ms"]
        flop = 2.0 * TAPS * positions
        runs.append({"reads_open_s": t_open, "reads_open_gpu_s": t_open_gpu, "batch_s": t_batch,
                     "reads_pass_device_ms": tm["reads_pass_ms"], "reads_pass_host_ms": tm_h["reads_pass_ms"],
                     "host_threads": a.threads, "ecor_kernel_ms": ecor_ms,
                     "ecor_tflops": flop / (ecor_ms * 1e-3) / 1e12,
                     "ecor_frac_fp64_peak": flop / (ecor_ms * 1e-3) / 1e12 / FP64_VECTOR_PEAK_TFLOPS})
        print(json.dumps(runs[-1]), file=sys.stderr, flush=True)
    # the CPU restatement of the reference's sequence side on a bounded sample
    from oracle import experimental as ox
    n0 = min(a.oracle_positions, int(lengths[0]))
    region = seqs[names[0]][:n0]
    t0 = time.perf_counter()
    ox.raw_ecor(k_cor, 7, region, n0)
    t_or = time.perf_counter() - t0
    best = min(runs, key=lambda r: r["batch_s"])
    print(json.dumps({
        "workload": "C3 subset: first %d C3 contigs (%.3g bp), %d reads at C3 density, whole-contig "
                    "regions, random FASTA, 7-mer table" % (k, positions, n_reads),
        "regions": len(regions), "positions": positions, "reads": n_reads,
        "best": best, "runs": runs,
        "note": "batch_s: experimental_batch with the read pass on the device over the GPU-decoded table "
                "(reads_pass_device_ms); reads_pass_host_ms: the same pass on the host (MC_EXP_READS=host), "
                "results compared",
        "fp64_vector_peak_tflops": FP64_VECTOR_PEAK_TFLOPS,
        "cpu_reference_sequence_side": {"positions": n0, "seconds": t_or,
                                        "positions_per_s": n0 / t_or,
                                        "kind": "port (oracle/experimental.py raw_ecor: the "
                                                "reference's per-position np.inner loop), 1 core",
                                        "projected_s_for_workload": positions / (n0 / t_or)},
    }))
    os.remove(bam)
    os.remove(fasta)


if __name__ == "__main__":
    main()
