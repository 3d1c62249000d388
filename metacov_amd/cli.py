"""`metacov pileup` on the MI355X engine — same options and CSV as the
reference command (metacov/cli.py:35-108).

    python -m metacov_amd.cli pileup -b X.bam [-rb R.blast7 | -rc R.csv] [-o out.csv]

Differences from the reference, all outside the CSV: the BAM need not be
indexed (it is decoded whole by the library's C++ decoder); all regions are
reduced in one batched GPU call; `-k/--kmer-histogram` (pileup.experimental,
SURVEY.md §8 f rank 2) is not part of this build and is rejected with a
usage error.

Multi-GPU (one process per GPU, SURVEY.md §8 e):

    python -m torch.distributed.run --nproc-per-node 8 -m metacov_amd.cli pileup -b X.bam ...

Contigs are split across ranks by LPT on reads and length; with `X.bam.bai`
each rank decodes only its contigs' BGZF blocks (otherwise it decodes all and
keeps its shard).  Each rank reduces the regions on its contigs; one
all-gather of the region table (RCCL; MC_DIST_BACKEND=gloo for a CPU
rehearsal) brings the rows to rank 0, which writes the same CSV.
"""
import csv
import logging
import os
import sys

import click
import numpy as np

from . import regions as _regions
from .bam import BamFile, StreamedBam, index_stats
from .engine import REGION_STAT_DTYPE, classic_stats

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
              help="Kmer Histogram produced with metacov scan (not supported by this build)")
@click.option('--kmer-length', '-K', type=int, default=7,
              help="Length of k-mer")
@click.option('--outfile', '-o', type=click.File('w'), default="-",
              help="Output CSV (default STDOUT)")
@click.option('--device', type=int, default=0, help="HIP device ordinal")
@click.option('--stream/--no-stream', default=True,
              help="Decode in bounded-memory windows, feeding the GPU through pinned double "
                   "buffers (default; --no-stream decodes the whole file into host memory first)")
def pileup(bamfile, reference_fasta, regionfile_blast7, regionfile_csv,
           kmer_histogram, kmer_length, outfile, device, stream):
    """
    Compute fold coverage values
    """
    if kmer_histogram is not None:
        raise click.UsageError("--kmer-histogram (pileup.experimental) is not supported by "
                               "the metacov_amd engine")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return pileup_distributed(bamfile.name, regionfile_blast7, regionfile_csv, outfile)
    bam = StreamedBam(bamfile.name, device=device) if stream else BamFile(bamfile.name)
    regions = list(_regions.make_region_iterator(regionfile_blast7, regionfile_csv, bam))
    log_counts(bam)
    write_rows(bam, regions, outfile, device=device)


def log_counts(bam):
    total = bam.mapped + bam.unmapped
    log.info("Number of reads:\n  total:    {total}\n  mapped:   {mapped} ({pct}%)\n"
             "  unmapped: {unmapped}\n".format(total=total, mapped=bam.mapped,
                                                unmapped=bam.unmapped,
                                                pct=bam.mapped / total * 100 if total else 0))


def resolve_regions(bam, regions):
    """Header contig id and sorted 0-based half-open range per region, as
    cli.py:80-91 (KeyError for an unknown name, as cli.py:86)."""
    name2ref = {w.split()[0]: w for w in bam.references}
    tids, starts, ends = [], [], []
    for hit in regions:
        ref = name2ref[hit.sacc]
        start, end = sorted((int(hit.sstart), int(hit.send)))
        if start < 0:
            raise ValueError("region start %d < 0" % start)
        tids.append(bam.references.index(ref))
        starts.append(start)
        ends.append(end)
    return (np.array(tids, np.int32), np.array(starts, np.int64), np.array(ends, np.int64))


def compute_rows(bam, tids, starts, ends, device=0):
    """Exact stat rows of the regions (header contig ids) on `bam`'s engine:
    depth and statistics in one pass (fused K2) when the regions do not
    overlap; the library falls back to K2 + K3 otherwise."""
    if len(tids) == 0:
        return np.zeros(0, dtype=REGION_STAT_DTYPE)
    eng = bam.engine(device, compute=False)
    rows = eng.compute_depth_stats(np.asarray(bam.local_tid(tids), np.int32), starts, ends)
    eng._depth_ready = True
    warn_depth_cap(eng.max_depth())
    return rows


HTSLIB_MAX_DEPTH = 8000   # pysam pileup's default max_depth (the htslib read-pool cap)


def warn_depth_cap(max_depth):
    """The reference's pysam pileup stops adding reads to a column's pool past
    max_depth=8000 (version-dependent); this engine never caps.
    Above the cap the two disagree, so say so."""
    if max_depth > HTSLIB_MAX_DEPTH:
        log.warning("maximum depth %d exceeds pysam's pileup cap of %d: the reference would "
                    "report capped depths there; these values are exact", max_depth,
                    HTSLIB_MAX_DEPTH)


def write_csv(regions, rows, outfile):
    """Rows in input order exactly as cli.py:97-108 writes them."""
    writer = None
    for hit, row in zip(regions, rows):
        result = classic_stats(row)
        if writer is None:
            writer = csv.DictWriter(outfile, fieldnames=['sacc', 'start', 'end'] + sorted(result))
            writer.writeheader()
        result.update({'sacc': hit.sacc, 'start': hit.sstart, 'end': hit.send})
        writer.writerow(result)


def write_rows(bam, regions, outfile, device=0):
    """Resolves names like cli.py:80-91, reduces all regions in one GPU call,
    then writes rows in input order exactly as cli.py:97-108 does."""
    tids, starts, ends = resolve_regions(bam, regions)
    write_csv(regions, compute_rows(bam, tids, starts, ends, device), outfile)


def pileup_distributed(path, regionfile_blast7, regionfile_csv, outfile):
    """One rank of a multi-GPU `pileup` (launched by torch.distributed.run)."""
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
    try:
        index = path + ".bai"
        have_index = os.path.exists(index)
        if have_index:       # header + per-contig counts from the index, no decode
            head = BamFile(path, contigs=[])
            reads_per, _, _ = index_stats(index, len(head.lengths))
        else:
            head = BamFile(path)
            reads_per = np.bincount(head.tid, minlength=len(head.lengths))
        regions = list(_regions.make_region_iterator(regionfile_blast7, regionfile_csv, head))
        tids, starts, ends = resolve_regions(head, regions)
        shards = mdist.lpt_shard(mdist.contig_costs(head.lengths, reads_per), world)
        owner = np.zeros(len(head.lengths), np.int64)
        for r, sh in enumerate(shards):
            owner[sh] = r
        region_rank = owner[tids] if len(tids) else np.zeros(0, np.int64)
        mine = np.nonzero(region_rank == rank)[0]
        r_max = max(1, int(np.bincount(region_rank, minlength=world).max()) if len(tids) else 1)
        rows = np.zeros(0, dtype=REGION_STAT_DTYPE)
        if len(mine):
            bam = BamFile(path, contigs=shards[rank]) if have_index else head.restrict(shards[rank])
            rows = compute_rows(bam, tids[mine], starts[mine], ends[mine], device)
        coll_dev = torch.device("cuda", device) if backend == "nccl" else None
        table = mdist.all_gather_table(mdist.pack_rows(rows, mine), r_max, device=coll_dev)
        if rank == 0:
            log_counts(head)
            write_csv(regions, mdist.unpack_rows(table, len(regions), REGION_STAT_DTYPE), outfile)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
