"""Region table sources of `metacov pileup`.

Behaviour follows the reference's region I/O:
  * BLAST -outfmt 7 parser: metacov/blast.py:48-94 (first line must contain
    "BLAST"; "# Fields:" names mapped to short names by the table at
    blast.py:13-29; typed per blast.py:32-45, so sstart/send are ints);
  * CSV regions: metacov/util.py:36-61 (column aliases sacc|sequence_id,
    sstart|start, send|end|stop; values stay strings);
  * whole contigs from the BAM header: metacov/util.py:64-69
    (Region(n, name, 0, length));
  * make_region_iterator: metacov/util.py:72-83 (blast7 and csv exclusive).
"""
import csv
from collections import namedtuple

Region = namedtuple("Region", ["qacc", "sacc", "sstart", "send"])

_LONG_TO_SHORT = {
    "query acc.": "qacc", "subject acc.": "sacc", "% identity": "pident",
    "alignment length": "length", "mismatches": "mismatch", "gap opens": "gapopen",
    "q. start": "qstart", "q. end": "qend", "s. start": "sstart", "s. end": "send",
    "evalue": "evalue", "bit score": "bitscore", "subject strand": "sstrand",
    "sbjct frame": "sframe", "score": "score",
}
_TYPES = {"pident": float, "length": int, "mismatch": int, "gapopen": int, "qstart": int,
          "qend": int, "sstart": int, "send": int, "evalue": float, "bitscore": float,
          "score": float, "sframe": int}


class Blast7Reader:
    """Iterates the hit lines of a BLAST tabular-with-comments file as
    namedtuples whose fields are the file's "# Fields:" columns."""

    def __init__(self, fileobj):
        self.fileobj = fileobj
        self.fields = None
        self.hit = 0
        self.query = None
        if "BLAST" not in fileobj.readline():
            raise ValueError("not a BLAST7 formatted file")

    def __iter__(self):
        Hit = None
        for line in self.fileobj:
            if line.startswith("# Fields: "):
                names = line[len("# Fields: "):].strip().split(", ")
                self.fields = [_LONG_TO_SHORT.get(f, f) for f in names]
                Hit = namedtuple("BlastHit", self.fields)
            elif line.startswith("# Query: ") or line.startswith("# Database: "):
                self.query = line.split(": ", 1)[1].strip()
                self.hit = 0
            elif line.strip().endswith(" hits found"):
                self.hits = int(line.split()[1])
                self.hit = 0
            elif line[0] == "#":
                continue
            else:
                self.hit += 1
                vals = line.strip().split("\t")
                yield Hit(*[_TYPES[k](v) if k in _TYPES else v for k, v in zip(self.fields, vals)])


def get_regions_from_blast7(fileobj):
    return iter(Blast7Reader(fileobj))


def get_regions_from_csv(fileobj):
    reader = csv.reader(fileobj)
    header = next(reader)
    cols = []
    for names in (("sacc", "sequence_id"), ("sstart", "start"), ("send", "end", "stop")):
        col = next((header.index(n) for n in names if n in header), None)
        if col is None:
            raise ValueError("Region file must have a column with a name in {}".format(names))
        cols.append(col)
    for row in reader:
        yield Region("", row[cols[0]], row[cols[1]], row[cols[2]])


def get_regions_from_bam(bam):
    for n, (length, name) in enumerate(zip(bam.lengths, bam.references)):
        yield Region(n, name, 0, length)


def make_region_iterator(regionfile_blast7, regionfile_csv, bam):
    if regionfile_blast7 and regionfile_csv:
        import click
        raise click.BadParameter(
            "Only one of regionfile-blast7 and regionfile-csv may be specified")
    if regionfile_blast7:
        return get_regions_from_blast7(regionfile_blast7)
    if regionfile_csv:
        return get_regions_from_csv(regionfile_csv)
    return get_regions_from_bam(bam)
