"""End-to-end `metacov pileup` timing on a synthetic BAM (host decode + GPU).

    python scripts/e2e.py [--reads 10000000 --contigs 1 --length 5000000]

Writes an edge-mix BAM with the library's writer, then times the phases of
the CLI path: C++ decode (BGZF inflate + parse, all host threads), ingest
(H2D + prepare), fused depth + statistics on the GPU, CSV formatting.
Then the same file through the GPU decode (GpuBamFile: BGZF inflate and
record parse on the device); every path's CSV must equal the first.
Prints one JSON line.
"""
import argparse
import io
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--contigs", type=int, default=1)
    ap.add_argument("--length", type=int, default=5_000_000, help="bp per contig")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--gpu-windows", default="",
                    help="comma-separated inflated window sizes in MiB: extra GPU decodes of the same file, "
                         "timed (window_sweep in the JSON)")
    ap.add_argument("--env-sweep", default="",
                    help="';'-separated settings 'K=V[,K=V]' of the decode's environment knobs: extra resident GPU "
                         "decodes per setting, in rounds (env_sweep in the JSON)")
    ap.add_argument("--sweep-rounds", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    from metacov_amd import synth, regions as mreg
    from metacov_amd.bam import BamFile
    from metacov_amd.cli import write_rows

    lengths = np.full(a.contigs, a.length, np.int64)
    names = ["contig_%d" % i for i in range(a.contigs)]
    d = a.dir or tempfile.mkdtemp()
    path = os.path.join(d, "e2e.bam")
    t0 = time.perf_counter()
    arrs = synth.edge_mix_arrays(lengths, a.reads, seed=1)
    synth.write_bam_fast(path, names, lengths, *arrs, level=6, n_threads=a.threads)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    bam = BamFile(path, n_threads=a.threads)
    t_dec = time.perf_counter() - t0
    t0 = time.perf_counter()
    eng = bam.engine(0, compute=False)
    t_ing = time.perf_counter() - t0
    regs = list(mreg.get_regions_from_bam(bam))
    t0 = time.perf_counter()
    out = io.StringIO()
    write_rows(bam, regs, out)
    t_cmp = time.perf_counter() - t0
    bases = bam.aligned_bases()
    tot = t_dec + t_ing + t_cmp
    csv_full = out.getvalue()
    tm = eng.timings()
    n_rec, n_kept = bam.n_records, len(bam.tid)
    bam.close()
    # the bounded-memory path: windowed decode + pinned double-buffered H2D
    from metacov_amd.bam import StreamedBam
    t0 = time.perf_counter()
    sb = StreamedBam(path, device=0, n_threads=a.threads)
    t_stream = time.perf_counter() - t0
    t0 = time.perf_counter()
    out2 = io.StringIO()
    write_rows(sb, regs, out2)
    t_cmp2 = time.perf_counter() - t0
    assert out2.getvalue() == csv_full, "streamed CSV differs"
    sb.close()
    # the GPU decode path: compressed windows up, inflate + record parse in HBM
    from metacov_amd.bam import GpuBamFile
    t0 = time.perf_counter()
    gb = GpuBamFile(path, device=0, n_threads=a.threads)
    t_gdec = time.perf_counter() - t0
    t0 = time.perf_counter()
    gb.engine(0, compute=False)
    t_ging = time.perf_counter() - t0
    t0 = time.perf_counter()
    out3 = io.StringIO()
    write_rows(gb, regs, out3)
    t_cmp3 = time.perf_counter() - t0
    assert out3.getvalue() == csv_full, "GPU-decoded CSV differs"
    gtm = gb.timings()
    gb.close()
    sweep = []
    for mib in [int(x) for x in a.gpu_windows.split(",") if x]:
        t0 = time.perf_counter()
        gw = GpuBamFile(path, device=0, n_threads=a.threads, window_bytes=mib << 20)
        dt = time.perf_counter() - t0
        wt = gw.timings()
        assert gw.n_kept == n_kept
        gw.close()
        sweep.append({"window_mib": mib, "decode_s": dt, **{k: wt[k] for k in
                      ("read_ms", "inflate_ms", "parse_ms", "scan_ms", "total_ms", "windows", "upload_ms", "kernel_ms", "open_ms")}})
        print(json.dumps(sweep[-1]), file=sys.stderr, flush=True)
    advice = []
    settings = [x for x in a.env_sweep.split(";") if x]
    for r in range(a.sweep_rounds if settings else 0):
        for st in settings:
            kv = dict(x.split("=", 1) for x in st.split(","))
            saved = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            t0 = time.perf_counter()
            gw = GpuBamFile(path, device=0, n_threads=a.threads)
            dt = time.perf_counter() - t0
            wt = gw.timings()
            assert gw.n_kept == n_kept
            gw.close()
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            advice.append({"env": st, "round": r, "decode_s": dt, **wt})
            print(json.dumps(advice[-1]), file=sys.stderr, flush=True)
    print(json.dumps({
        "bam_bytes": os.path.getsize(path), "records": n_rec, "kept": n_kept,
        "aligned_bases": bases, "host_threads": a.threads,
        "decode_s": t_dec, "ingest_h2d_prepare_s": t_ing, "gpu_stats_csv_s": t_cmp,
        "end_to_end_s": tot, "end_to_end_aligned_bases_per_s": bases / tot,
        "decode_records_per_s": n_rec / t_dec, "generate_write_s": t_gen,
        "timings": tm,
        "stream_decode_ingest_prepare_s": t_stream, "stream_gpu_stats_csv_s": t_cmp2,
        "stream_end_to_end_s": t_stream + t_cmp2,
        "stream_end_to_end_aligned_bases_per_s": bases / (t_stream + t_cmp2),
        "gpu_decode_s": t_gdec, "gpu_decode_timings": gtm, "gpu_ingest_s": t_ging,
        "gpudec_stats_csv_s": t_cmp3, "gpu_end_to_end_s": t_gdec + t_ging + t_cmp3,
        "gpu_end_to_end_aligned_bases_per_s": bases / (t_gdec + t_ging + t_cmp3),
        "window_sweep": sweep, "env_sweep": advice}))
    os.remove(path)


if __name__ == "__main__":
    main()
