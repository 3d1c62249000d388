"""`metacov pileup` on the MI355X engine — same options and CSV as the
reference command (metacov/cli.py:35-108).

    python -m metacov_amd.cli pileup -b X.bam [-rb R.blast7 | -rc R.csv] [-o out.csv]

Differences from the reference, all outside the CSV: the BAM need not be
indexed (it is decoded whole, on the GPU by default); all regions are
reduced in one batched GPU call.  Defaults follow pysam: the pileup read cap
of 8000 (`--max-depth`, 0 = exact depths; metacov_amd.depthcap) and current
htslib's end of a read without reference-consuming ops (`--legacy-endpos`
for htslib <= 1.9).  Rows are written in input order up to the first region
the reference would fail on (unknown name, bad coordinate, empty region),
and that error is raised after them, as cli.py:85-108 does.  With `-k/--kmer-histogram` every row also
carries pileup.experimental's 13 columns (cli.py:81, :93-95; SURVEY.md §8 f):
the read side runs on host threads, the k-mer correlation against `-f` on
the GPU (metacov_amd/experimental.py).

Multi-GPU (one process per GPU, SURVEY.md §8 e):

    python -m torch.distributed.run --nproc-per-node 8 -m metacov_amd.cli pileup -b X.bam ...

Contigs are split across ranks by LPT on reads and length; with `X.bam.bai`
each rank decodes only its contigs' BGZF blocks (otherwise it decodes all and
keeps its shard).  Each rank reduces the regions on its contigs; one
all-gather of the region table (RCCL; MC_DIST_BACKEND=gloo for a CPU
rehearsal) brings the rows to rank 0, which writes the same CSV.
"""
import os
import sys
import time


def _prewarm_hip():
    """`python -m metacov_amd.cli` (one process): the HIP runtime and the
    device context are initialised on a thread while the imports below run
    (the library's calls release the GIL); mc_ctx_create then finds them
    done.  MC_CLI_PREWARM=0 turns it off."""
    if os.environ.get("MC_CLI_PREWARM", "1") == "0" or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return
    argv = sys.argv[1:]
    device = 0
    if "--device" in argv[:-1]:
        try:
            device = int(argv[argv.index("--device") + 1])
        except ValueError:
            pass

    def run():
        try:
            from metacov_amd import _lib
            _lib.load().mc_runtime_init(device)
        except Exception:   # noqa: BLE001 (the real calls report it)
            pass

    import threading
    threading.Thread(target=run, name="hip-prewarm", daemon=True).start()


if __name__ == "__main__":
    _prewarm_hip()

import csv  # noqa: E402
import json  # noqa: E402
import logging  # noqa: E402

import click  # noqa: E402
import numpy as np  # noqa: E402

from . import depthcap as _depthcap  # noqa: E402
from . import experimental as _experimental
from . import regions as _regions
from . import scan as _scan
from .bam import BamFile, GpuBamFile, StreamedBam, index_stats
from .engine import REGION_STAT_DTYPE, classic_stats, numpy_std

_T_IMPORTED = time.time()    # (MC_CLI_TIMES: the end of the module imports)

logging.basicConfig(level=logging.INFO,
                    format="[%(relativeCreated)6.1f %(funcName)s]  %(message)s",
                    datefmt="%I:%M:%S")
log = logging.getLogger(__name__)


@click.group()
def main():
    """
    MetaCov estimates abundance values from the stacking depth of
    reads mapped to a reference.
    """


@main.command()
@click.option('--bamfile', '-b', type=click.File('rb'), required=True,
              help="Input BAM file. Must be coordinate-sorted.")
@click.option('--reference-fasta', '-f', type=click.File('rb'))
@click.option('--regionfile-blast7', '-rb', type=click.File('r'),
              help="Input Region file in BLAST7 format")
@click.option('--regionfile-csv', '-rc', type=click.File('r'),
              help="Input Region file in CSV format")
@click.option('--kmer-histogram', '-k', type=click.File('r'),
              help="Kmer Histogram produced with metacov scan")
@click.option('--kmer-length', '-K', type=int, default=7,
              help="Length of k-mer")
@click.option('--outfile', '-o', type=click.File('w'), default="-",
              help="Output CSV (default STDOUT)")
@click.option('--device', type=int, default=0, help="HIP device ordinal")
@click.option('--stream/--no-stream', default=True,
              help="Decode in bounded-memory windows, feeding the GPU through pinned double "
                   "buffers (default; --no-stream decodes the whole file into host memory first)")
@click.option('--max-depth', type=click.IntRange(0), default=_depthcap.HTSLIB_MAX_DEPTH,
              metavar="N", show_default=True,
              help="htslib's pileup read cap per region query, as pysam's pileup applies it "
                   "(its default is 8000); 0: exact depths, no cap")
@click.option('--legacy-endpos', is_flag=True, default=False,
              help="Count a mapped read without reference-consuming CIGAR ops on one column "
                   "(htslib <= 1.9 bam_endpos); default: it adds nothing (current htslib)")
@click.option('--window-bytes', type=click.IntRange(0), default=0, metavar="B",
              help="Decode in windows of B inflated bytes (bounded memory); 0: --decode gpu keeps "
                   "the file resident when it fits in HBM, --stream uses 256 MiB")
@click.option('--decode', type=click.Choice(['gpu', 'host']), default='gpu',
              help="gpu (default): BGZF inflate and record parse on the device (csrc/bam_gpu.hip); "
                   "host: the C++ decoder on host threads (--stream / --no-stream)")
def pileup(bamfile, reference_fasta, regionfile_blast7, regionfile_csv,
           kmer_histogram, kmer_length, outfile, device, stream, max_depth, legacy_endpos,
           window_bytes, decode):
    """
    Compute fold coverage values
    """
    fasta = reference_fasta.name if reference_fasta else None
    if fasta:            # cli.py:59: pysam.FastaFile(...) for every run with -f
        _experimental.check_faidx(fasta)
    # cli.py:81: the histogram is read with load_kmerhist's default k_len (7)
    k_cor = _experimental.load_kmerhist(kmer_histogram) if kmer_histogram else None
    exp = (k_cor, kmer_length, fasta) if k_cor is not None else None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return pileup_distributed(bamfile.name, regionfile_blast7, regionfile_csv, outfile, exp,
                                  max_depth=max_depth, legacy_endpos=legacy_endpos, decode=decode)
    times = _PhaseTimes.start(device)
    if decode == 'gpu':
        bam = GpuBamFile(bamfile.name, device=device, window_bytes=window_bytes,
                         legacy_endpos=legacy_endpos)
    elif stream:
        bam = StreamedBam(bamfile.name, device=device, window_bytes=window_bytes,
                          legacy_endpos=legacy_endpos)
    else:
        bam = BamFile(bamfile.name, legacy_endpos=legacy_endpos)
    times.mark("decode")
    regions = _regions.make_region_iterator(regionfile_blast7, regionfile_csv, bam)
    log_counts(bam)
    write_rows(bam, regions, outfile, device=device, exp=exp, max_depth=max_depth, times=times)
    times.finish(outfile, bam)


class _PhaseTimes:
    """MC_CLI_TIMES=<path>: the single-process `pileup`'s wall-clock phases as
    JSON (scripts/cold_cli.py): process start (MC_CLI_T0, the launcher's
    clock, else the OS's process start) to the end of the imports, HIP
    runtime and device init (one ctx created and destroyed up front, so the
    decode phase holds the decode alone), decode, rows (depth, statistics,
    cap), write.  Without the variable every call is a no-op."""

    def __init__(self, path):
        self.path = path
        self.t = {}
        self.last = time.time()

    @classmethod
    def start(cls, device=0):
        path = os.environ.get("MC_CLI_TIMES")
        if not path:
            return _NoTimes()
        t0 = os.environ.get("MC_CLI_T0")
        if t0:
            t0 = float(t0)
        else:
            import psutil
            t0 = psutil.Process().create_time()
        self = cls(path)
        self.t["interpreter_and_imports_s"] = _T_IMPORTED - t0
        self.t["cli_parse_s"] = time.time() - _T_IMPORTED
        self.t0 = t0
        self.last = time.time()
        from . import _lib as L
        import ctypes
        lib = L.load()
        self.mark("library_load")
        h = ctypes.c_void_p()
        L.check(lib.mc_ctx_create(int(device), ctypes.byref(h)), lib)
        lib.mc_ctx_destroy(h)
        self.mark("hip_init")
        return self

    def mark(self, name):
        now = time.time()
        self.t[name + "_s"] = now - self.last
        self.last = now

    def finish(self, outfile, bam):
        outfile.flush()
        self.mark("write")
        self.t["total_s"] = time.time() - self.t0
        tm = getattr(bam, "timings", None)
        if tm is not None:
            self.t["decode_timings"] = {k: round(v, 3) if isinstance(v, float) else v for k, v in tm().items()}
        with open(self.path, "w") as fh:
            json.dump(self.t, fh, indent=1)


class _NoTimes:
    def mark(self, name):
        pass

    def finish(self, outfile, bam):
        pass


def log_counts(bam):
    total = bam.mapped + bam.unmapped
    log.info("Number of reads:\n  total:    {total}\n  mapped:   {mapped} ({pct}%)\n"
             "  unmapped: {unmapped}\n".format(total=total, mapped=bam.mapped,
                                                unmapped=bam.unmapped,
                                                pct=bam.mapped / total * 100 if total else 0))


def resolve_regions(bam, regions):
    """Header contig id and sorted 0-based half-open range per region, as
    cli.py:80-91, for the regions before the first one the reference fails
    on: returns (hits, tids, starts, ends, error).  The error is what the
    reference raises at that region, in its order: the region file's own
    parse error, KeyError for an unknown name (cli.py:86), ValueError from
    int() (cli.py:89), then classic()'s ValueError for a negative start or an
    empty region (pileup.py:19, a zero-size reduction).  None when every
    region resolves."""
    name2ref = {w.split()[0]: w for w in bam.references}
    ref2tid = {}
    for t, w in enumerate(bam.references):
        ref2tid.setdefault(w, t)      # first header entry, as list.index
    hits, tids, starts, ends = [], [], [], []
    err = None
    it = iter(regions)
    while True:
        try:
            hit = next(it)
        except StopIteration:
            break
        except Exception as e:        # a malformed line of the region file
            err = e
            break
        try:
            ref = name2ref[hit.sacc]
            start, end = sorted((int(hit.sstart), int(hit.send)))
            if start < 0:
                raise ValueError("start out of range (%d)" % start)
            if start == end:
                raise ValueError("zero-size array to reduction operation minimum which has "
                                 "no identity")
        except Exception as e:
            err = e
            break
        hits.append(hit)
        tids.append(ref2tid[ref])
        starts.append(start)
        ends.append(end)
    return (hits, np.array(tids, np.int32), np.array(starts, np.int64),
            np.array(ends, np.int64), err)


def compute_rows(bam, tids, starts, ends, device=0, max_depth=_depthcap.HTSLIB_MAX_DEPTH):
    """Stat rows of the regions (header contig ids) on `bam`'s engine: depth
    and statistics in one pass (fused K2) when the regions do not overlap;
    the library falls back to K2 + K3 otherwise.  max_depth: htslib's read
    cap per region query; only regions whose exact maximum could reach it
    are recomputed, together in one more engine call (metacov_amd.depthcap);
    0 / None: exact depths.  Returns (rows, std): std is numpy's own np.std
    value for the rows near a rounding tie, NaN elsewhere (engine.numpy_std)."""
    if len(tids) == 0:
        return np.zeros(0, dtype=REGION_STAT_DTYPE), np.zeros(0)
    eng = bam.engine(device, compute=False)
    local = np.asarray(bam.local_tid(tids), np.int32)
    rows = eng.compute_depth_stats(local, starts, ends)
    eng._depth_ready = True
    std = numpy_std(eng, rows, local, starts, ends)
    if max_depth:
        rows, n_cap, dropped = _depthcap.apply_cap(bam, rows, tids, starts, ends, bam.lengths,
                                                   max_depth, device, std=std)
        if n_cap:
            log.info("max_depth %d: %d regions deep enough for the pileup cap, %d reads dropped",
                     max_depth, n_cap, dropped)
    return rows, std


def experimental_results(path, exp, references, tids, starts, ends, device=0, contigs=None, extents=None):
    """pileup.experimental for every region (cli.py:93-95), or None without -k.
    contigs / extents: a distributed rank's shard, whose read table is decoded
    from those contigs' BGZF blocks only (experimental_batch)."""
    if exp is None:
        return None
    k_cor, k_len, fasta = exp
    regs = [(references[t], int(a), int(b)) for t, a, b in zip(tids, starts, ends)]
    if not regs:
        return []
    return _experimental.experimental_batch(path, k_cor, k_len, fasta, regs, device=device, contigs=contigs,
                                            extents=extents)


def write_csv(regions, rows, outfile, extra=None, std=None):
    """Rows in input order exactly as cli.py:97-108 writes them; `extra`
    (experimental_batch results) adds the -k columns, its "RCOR is ZERO"
    lines and its errors at the region where the reference meets them.
    std: numpy's std per row where given (engine.numpy_std; NaN: none)."""
    writer = None
    for i, (hit, row) in enumerate(zip(regions, rows)):
        result = classic_stats(row, None if std is None else std[i])
        if extra is not None:
            result.update(extra[i].emit(out=sys.stdout))
        if writer is None:
            writer = csv.DictWriter(outfile, fieldnames=['sacc', 'start', 'end'] + sorted(result))
            writer.writeheader()
        result.update({'sacc': hit.sacc, 'start': hit.sstart, 'end': hit.send})
        writer.writerow(result)


def write_rows(bam, regions, outfile, device=0, exp=None, max_depth=_depthcap.HTSLIB_MAX_DEPTH, times=None):
    """Resolves names like cli.py:80-91, reduces the regions in one GPU call,
    then writes rows in input order exactly as cli.py:97-108 does; the rows
    before a failing region are written before its error is raised."""
    times = times or _NoTimes()
    hits, tids, starts, ends, err = resolve_regions(bam, regions)
    times.mark("regions")
    rows, std = compute_rows(bam, tids, starts, ends, device, max_depth)
    times.mark("rows")
    extra = experimental_results(bam.filename, exp, bam.references, tids, starts, ends, device)
    if exp is not None:
        times.mark("experimental")
    write_csv(hits, rows, outfile, extra, std)
    if err is not None:
        raise err


def pileup_distributed(path, regionfile_blast7, regionfile_csv, outfile, exp=None,
                       max_depth=_depthcap.HTSLIB_MAX_DEPTH, legacy_endpos=False, decode="gpu"):
    """One rank of a multi-GPU `pileup` (launched by torch.distributed.run).
    With -k, each rank also computes the experimental columns of the regions
    on its contigs (cli.py:93-95 per region), and rank 0 gathers them with
    the table."""
    import torch
    import torch.distributed as dist
    from . import dist as mdist
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MC_DIST_BACKEND", "nccl")
    device = local % max(1, torch.cuda.device_count())
    if backend == "nccl":
        torch.cuda.set_device(device)
    dist.init_process_group(backend)
    coll_dev = torch.device("cuda", device) if backend == "nccl" else None
    times = {}
    t_start = time.perf_counter()
    try:
        err = region_err = None
        try:
            table_args = _pileup_shard(path, regionfile_blast7, regionfile_csv, rank, world, device,
                                       max_depth, legacy_endpos, decode, coll_dev, times)
            head, regions, tids, starts, ends, rows, std, mine, r_max, region_err, shard = table_args
            # -k: the read table of this rank's contigs only (their BGZF blocks, by
            # the BAI or rank 0's extents table), when the GPU decodes
            mine_extra = experimental_results(path, exp, head.references, tids[mine], starts[mine],
                                              ends[mine], device, *shard)
        except BaseException as e:   # every rank learns of it before the table gather
            err = e
        mdist.agree_on_error(err, device=coll_dev)
        t0 = time.perf_counter()
        table = mdist.all_gather_table(mdist.pack_rows(rows, mine, std), r_max, device=coll_dev)
        times["gather_s"] = time.perf_counter() - t0
        extra = None
        if exp is not None:          # each rank's experimental results (our own objects) to rank 0
            parts = [None] * world if rank == 0 else None
            dist.gather_object((mine.tolist(), mine_extra), parts, dst=0)
            if rank == 0:
                extra = [None] * len(regions)
                for idx, res in parts:
                    for i, r in zip(idx, res):
                        extra[i] = r
        if rank == 0:
            log_counts(head)
            write_csv(regions, mdist.unpack_rows(table, len(regions), REGION_STAT_DTYPE), outfile,
                      extra, mdist.unpack_std(table, len(regions)))
        times["total_s"] = time.perf_counter() - t_start
        log.info("rank %d/%d phases: %s", rank, world, json.dumps(times))
    finally:
        dist.destroy_process_group()
    if region_err is not None:       # every rank resolved the same regions
        raise region_err


class _Header:
    """What the ranks of a distributed pileup use of an opened BAM besides
    its reads: names, lengths and the whole file's record counts."""

    def __init__(self, references, lengths, counts):
        self.references, self.lengths = tuple(references), tuple(lengths)
        self.n_records, self.mapped, self.unmapped = counts


def _pileup_shard(path, regionfile_blast7, regionfile_csv, rank, world, device,
                  max_depth=_depthcap.HTSLIB_MAX_DEPTH, legacy_endpos=False, decode="gpu",
                  coll_dev=None, times=None):
    """This rank's part of a distributed pileup: header and regions (every
    rank; those before the first failing one, and its error), LPT contig
    shards, the rows of the regions on its contigs, and (contigs, extents)
    for its -k read table.

    Each rank decodes only its own contigs' BGZF blocks, on
    its GPU by default, located by the BAI's extents.  Without a .bai, rank 0
    decodes the whole file on its GPU, which yields the same extents table
    (mc_bam_gpu_extents: what the index would hold), and broadcasts it; the
    other ranks then decode their contigs from it.  --decode host: the C++
    host decoder (whole file without an index)."""
    from . import dist as mdist
    full = None          # rank 0 without an index: the whole-file GPU decode
    times = {} if times is None else times
    t0 = time.perf_counter()
    index = path + ".bai"
    have_index = os.path.exists(index)
    ext = None
    if have_index:       # header + per-contig counts from the index, no decode
        head = BamFile(path, contigs=[])
        reads_per, _, _ = index_stats(index, len(head.lengths))
    elif decode == "gpu":
        def whole_file():
            nonlocal full
            full = GpuBamFile(path, device=device, legacy_endpos=legacy_endpos)
            return (full.references, full.lengths, (full.n_records, full.mapped, full.unmapped),
                    full.extents())
        try:
            refs, lens, counts, ext = mdist.broadcast_result(whole_file, rank, device=coll_dev)
        except BaseException:
            if full is not None:
                full.close()
            raise
        head = _Header(refs, lens, counts)
        reads_per = ext[0]["n_mapped"]
    else:
        head = BamFile(path, legacy_endpos=legacy_endpos)
        reads_per = np.bincount(head.tid, minlength=len(head.lengths))
    times["head_s"] = time.perf_counter() - t0
    regions, tids, starts, ends, region_err = resolve_regions(
        head, _regions.make_region_iterator(regionfile_blast7, regionfile_csv, head))
    shards = mdist.lpt_shard(mdist.contig_costs(head.lengths, reads_per), world)
    owner = np.zeros(len(head.lengths), np.int64)
    for r, sh in enumerate(shards):
        owner[sh] = r
    region_rank = owner[tids] if len(tids) else np.zeros(0, np.int64)
    mine = np.nonzero(region_rank == rank)[0]
    r_max = max(1, int(np.bincount(region_rank, minlength=world).max()) if len(tids) else 1)
    rows, std = np.zeros(0, dtype=REGION_STAT_DTYPE), np.zeros(0)
    if len(mine):
        t0 = time.perf_counter()
        if full is not None:      # rank 0 keeps its shard of the whole file
            bam, full = full.restrict(shards[rank]), None
            times["decode_timings"] = {}
        elif decode == "gpu":
            bam = GpuBamFile(path, device=device, contigs=shards[rank], extents=ext,
                             legacy_endpos=legacy_endpos)
            times["decode_timings"] = {k: round(v, 3) if isinstance(v, float) else v
                                       for k, v in bam.timings().items()}
        elif have_index:
            bam = BamFile(path, contigs=shards[rank], legacy_endpos=legacy_endpos)
        else:
            bam = head.restrict(shards[rank])
        times["decode_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        try:
            rows, std = compute_rows(bam, tids[mine], starts[mine], ends[mine], device, max_depth)
        finally:
            if decode == "gpu":
                bam.close()
        times["rows_s"] = time.perf_counter() - t0
    if full is not None:
        full.close()
    # (contigs, extents) for this rank's -k read table: a contig-subset GPU decode
    shard = (shards[rank], ext) if decode == "gpu" and (have_index or ext is not None) else (None, None)
    return head, regions, tids, starts, ends, rows, std, mine, r_max, region_err, shard


@main.command()
@click.option("--readfile-type", "-t",
              type=click.Choice(['bam', 'fq']),
              help="Override filename based detection of readfile type.")
@click.option("--max-reads", "-m",
              type=click.IntRange(1), metavar="N",
              help="Only consider the first N reads.")
@click.option("--group-by", "-g",
              type=click.Choice(_scan.Flags.keys()), multiple=True, metavar="FLAG",
              help="Group output by BAM flag. May be specified multiple times. "
              "FLAG can be one of {}".format(list(_scan.Flags.keys())))
@click.option('--reference-fasta', '-f',
              type=click.File('rb'), metavar="FILE",
              help="Fasta file reads where mapped to. Required for boffset."
              " File may be bgzip'ed, but not gzip'ed.")
@click.option("--out-basehist", "-b",
              type=click.File("w", lazy=False), metavar="FILE",
              help="Compute histogram of base counts by position in read.")
@click.option('--boffset', '-bo',
              type=click.IntRange(0, 200), default=0, metavar="N", show_default=True,
              help="Include N bases prior to read start in base histogram. "
              "Requires reference fasta file.")
@click.option("--out-kmerhist", "-o",
              type=click.File("w", lazy=False), metavar="FILE",
              help="Compute histogram of kmers in reads")
@click.option("-k",
              type=click.IntRange(2, 12), default=7, metavar="N", show_default=True,
              help="Length of kmers")
@click.option("--step", "-s",
              type=click.IntRange(1, 100), default=7, metavar="N", show_default=True,
              help="Step between sampled kmers")
@click.option("--offset", "-O",
              type=click.IntRange(-100, 100), default=0, metavar="N", show_default=True,
              help="Offset of first sampled kmer")
@click.option("--number", "-n",
              type=click.IntRange(1, 100), default=8, metavar="N", show_default=True,
              help="Numer of sampled kmers")
@click.option('--out-mirrorhist', '-M',
              type=click.File('w', lazy=False), metavar="FILE",
              help="Compute histogram of mismatches against palindrome")
@click.option('--mirror-offset', '-MO',
              type=click.IntRange(-100, 100), default=4, metavar="N", show_default=True,
              help="Offset of palindrome center from read start")
@click.option('--mirror-length', '-Ml',
              type=click.IntRange(1, 50), default=10, metavar="N", show_default=True,
              help="Palindrome length is 2N+1")
@click.option('--out-isizehist', '-I',
              type=click.File('w', lazy=False), metavar="FILE",
              help="Compute histogram of insert sizes.")
@click.option('--device', type=int, default=0, help="HIP device ordinal")
@click.argument("readfile", nargs=-1, required=True)
def scan(readfile, readfile_type, out_basehist, boffset, out_kmerhist,
         k, number, step, offset, max_reads, reference_fasta,
         out_mirrorhist, mirror_offset, mirror_length,
         out_isizehist, group_by, device):
    """
    Gather read statistics
    """
    # reference metacov/cli.py:162-285: same options, checks and CSV files;
    # the histograms run on the GPU (metacov_amd/scan.py)
    if not readfile_type:
        for ext, ft in {'.bam': 'bam', '.sam': 'bam', '.fq': 'fq', '.fq.gz': 'fq',
                        '.fastq': 'fq', '.fastq.gz': 'fq'}.items():
            if readfile[0].endswith(ext):
                readfile_type = ft
                break
    if not readfile_type:
        raise click.UsageError("Couldn't guess input format. Please supply -t")
    if readfile_type != 'fq' and len(readfile) > 1:
        raise click.UsageError("Multiple input files only supported for fastq")
    if len(readfile) > 2:
        raise click.UsageError("At most two fastq files allowed (fwd and rev)")
    if readfile_type != 'bam' and reference_fasta:
        raise click.UsageError("Reference fasta can only be used with mapped (bam/sam) reads")

    from . import pyfq
    fasta = None
    if readfile_type == 'bam':
        infile = readfile[0]
        if os.path.exists(infile + ".bai"):
            head = BamFile(infile, contigs=[])
            mapped, unmapped, nocoor = index_stats(infile + ".bai", len(head.lengths))
            mapped, unmapped = int(mapped.sum()), int(unmapped.sum()) + nocoor
            log.info("mapped = {}, unmapped = {}, total = {}".format(
                mapped, unmapped, mapped + unmapped))
        if reference_fasta:
            fasta = reference_fasta.name
    else:
        infile = (pyfq.FastQFilePair(readfile[0], readfile[1]) if len(readfile) > 1
                  else pyfq.FastQFile(readfile[0]))

    counters = []
    if out_basehist:
        counters.append(_scan.BaseHist(boffset))
    if out_kmerhist:
        counters.append(_scan.KmerHist(k, number, step, offset))
    if out_mirrorhist:
        counters.append(_scan.MirrorHist(mirror_offset, mirror_length))
    if out_isizehist:
        counters.append(_scan.IsizeHist())
    counters = _scan.ByFlag(counters, [_scan.Flags[flag] for flag in group_by])

    nreads = _scan.scan_reads(infile, fasta, counters, maxreads=max_reads or 0, device=device)
    log.info("Processed {} reads".format(nreads))

    # the reference's output index sequence, including the missing
    # `n = n + 1` after the k-mer table (cli.py:266-285)
    n = 0
    if out_basehist:
        csv.writer(out_basehist).writerows(counters.get_rows(n))
        n = n + 1
    if out_kmerhist:
        csv.writer(out_kmerhist).writerows(counters.get_rows(n))
    if out_mirrorhist:
        csv.writer(out_mirrorhist).writerows(counters.get_rows(n))
        n = n + 1
    if out_isizehist:
        csv.writer(out_isizehist).writerows(counters.get_rows(n))
        n = n + 1


def run_and_exit():
    """`python -m metacov_amd.cli ...`: the command, then the process ends
    without tearing down what it leaves in HBM.  The outputs are closed and
    the standard streams flushed first; then os._exit skips Python's object
    teardown and the HIP runtime's destructors (the decode's buffers, ~0.13 s
    after a 5.2 GB BAM: profiles/r06/r06d_cold_cli.json) — the driver
    reclaims the device memory of an exiting process.  MC_FAST_EXIT=0: the
    ordinary exit."""
    if os.environ.get("MC_FAST_EXIT", "1") == "0":
        sys.exit(main())
    import traceback
    try:
        rc = main(standalone_mode=False)
        rc = rc if isinstance(rc, int) else 0
    except click.exceptions.ClickException as e:
        e.show()
        rc = e.exit_code
    except click.exceptions.Abort:
        print("Aborted!", file=sys.stderr)
        rc = 1
    except SystemExit as e:
        rc = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
        if e.code is not None and not isinstance(e.code, int):
            print(e.code, file=sys.stderr)
    except BaseException:   # noqa: BLE001 - printed as the interpreter would, then the same status
        traceback.print_exc()
        rc = 1
    logging.shutdown()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)


if __name__ == "__main__":
    run_and_exit()
