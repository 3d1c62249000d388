"""`metacov pileup` on the MI355X engine — same options and CSV as the
reference command (metacov/cli.py:35-108).

    python -m metacov_amd.cli pileup -b X.bam [-rb R.blast7 | -rc R.csv] [-o out.csv]

Differences from the reference, all outside the CSV: the BAM need not be
indexed (it is decoded whole by the library's C++ decoder); all regions are
reduced in one batched GPU call; `-k/--kmer-histogram` (pileup.experimental,
SURVEY.md §8 f rank 2) is not part of this build and is rejected with a
usage error.
"""
import csv
import logging
import sys

import click
import numpy as np

from . import regions as _regions
from .bam import BamFile
from .engine import classic_stats

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
def pileup(bamfile, reference_fasta, regionfile_blast7, regionfile_csv,
           kmer_histogram, kmer_length, outfile, device):
    """
    Compute fold coverage values
    """
    if kmer_histogram is not None:
        raise click.UsageError("--kmer-histogram (pileup.experimental) is not supported by "
                               "the metacov_amd engine")
    bam = BamFile(bamfile.name)
    regions = list(_regions.make_region_iterator(regionfile_blast7, regionfile_csv, bam))
    total = bam.mapped + bam.unmapped
    log.info("Number of reads:\n  total:    {total}\n  mapped:   {mapped} ({pct}%)\n"
             "  unmapped: {unmapped}\n".format(total=total, mapped=bam.mapped,
                                                unmapped=bam.unmapped,
                                                pct=bam.mapped / total * 100 if total else 0))
    write_rows(bam, regions, outfile, device=device)


def write_rows(bam, regions, outfile, device=0):
    """Resolves names like cli.py:80-91, reduces all regions in one GPU call,
    then writes rows in input order exactly as cli.py:97-108 does."""
    name2ref = {w.split()[0]: w for w in bam.references}
    tids, starts, ends = [], [], []
    for hit in regions:
        ref = name2ref[hit.sacc]                       # KeyError as cli.py:86
        start, end = sorted((int(hit.sstart), int(hit.send)))
        if start < 0:
            raise ValueError("region start %d < 0" % start)
        tids.append(bam.references.index(ref))
        starts.append(start)
        ends.append(end)
    # depth and statistics in one pass (fused K2) when the regions do not
    # overlap; the library falls back to K2 + K3 otherwise
    rows = []
    if regions:
        eng = bam.engine(device, compute=False)
        rows = eng.compute_depth_stats(np.array(tids, np.int32), np.array(starts, np.int64),
                                       np.array(ends, np.int64))
        eng._depth_ready = True
    writer = None
    for hit, row in zip(regions, rows):
        result = classic_stats(row)
        if writer is None:
            writer = csv.DictWriter(outfile, fieldnames=['sacc', 'start', 'end'] + sorted(result))
            writer.writeheader()
        result.update({'sacc': hit.sacc, 'start': hit.sstart, 'end': hit.send})
        writer.writerow(result)


if __name__ == "__main__":
    sys.exit(main())
