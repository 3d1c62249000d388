"""Region-table sources (reference: metacov/util.py:30-83, metacov/blast.py)."""
import io
import os

import pytest

from metacov_amd import regions


def test_blast7_fixture(golden_dir):
    with open(os.path.join(golden_dir, "regions.blast7")) as fh:
        hits = list(regions.get_regions_from_blast7(fh))
    assert [(h.sacc, h.sstart, h.send) for h in hits] == [
        ("ref1", 1, 425), ("ref2", 1, 575), ("ref2", 1, 300), ("ref2", 301, 575)]
    assert all(isinstance(h.sstart, int) for h in hits)


def test_blast7_requires_header():
    with pytest.raises(ValueError):
        regions.Blast7Reader(io.StringIO("nope\n"))


def test_blast7_typed_fields_and_queries():
    txt = ("# BLASTN 2.5.0+\n# Query: q1\n# Database: db\n"
           "# Fields: query acc., subject acc., % identity, s. start, s. end, evalue\n"
           "# 2 hits found\nq1\tc1\t99.5\t10\t5\t1e-5\nq1\tc2\t80.0\t1\t20\t0.1\n")
    hits = list(regions.get_regions_from_blast7(io.StringIO(txt)))
    assert hits[0].qacc == "q1" and hits[0].pident == 99.5 and hits[0].sstart == 10
    assert hits[1].evalue == 0.1 and hits[1].send == 20


def test_csv_aliases():
    txt = "sequence_id,start,stop,x\nc1,5,10,a\nc2,7,3,b\n"
    rs = list(regions.get_regions_from_csv(io.StringIO(txt)))
    assert rs == [regions.Region("", "c1", "5", "10"), regions.Region("", "c2", "7", "3")]
    with pytest.raises(ValueError):
        list(regions.get_regions_from_csv(io.StringIO("a,b\n1,2\n")))


def test_whole_contigs_and_exclusive():
    class B:
        references = ("x", "y")
        lengths = (10, 20)
    assert list(regions.make_region_iterator(None, None, B())) == [
        regions.Region(0, "x", 0, 10), regions.Region(1, "y", 0, 20)]
    import click
    with pytest.raises(click.BadParameter):
        regions.make_region_iterator(io.StringIO(""), io.StringIO(""), B())


def test_cli_kmer_histogram_without_columns(tmp_path, golden_dir):
    """-k with a histogram lacking the Mapped / R columns fails in
    load_kmerhist with the reference's AttributeError (pileup.py:31), before
    any GPU work (runs on CPU)."""
    from click.testing import CliRunner
    from metacov_amd.cli import pileup
    k = tmp_path / "k.csv"
    k.write_text("kmer,n\n")
    res = CliRunner().invoke(pileup, ["-b", os.path.join(golden_dir, "bbmap.sorted.bam"),
                                      "-k", str(k), "-o", str(tmp_path / "o.csv")])
    assert res.exit_code == 1 and isinstance(res.exception, AttributeError)


def test_cli_bad_first_region_writes_nothing(tmp_path, golden_dir, lib_built):
    """No GPU needed: the first region already fails, so the reference
    (cli.py:85-91) raises before any row or header is written."""
    from click.testing import CliRunner
    from metacov_amd.cli import pileup
    rc = tmp_path / "r.csv"
    rc.write_text("sacc,sstart,send\nnope,1,5\nref1,1,425\n")
    out = tmp_path / "o.csv"
    res = CliRunner().invoke(pileup, ["-b", os.path.join(golden_dir, "bbmap.sorted.bam"),
                                      "--decode", "host", "--no-stream", "-rc", str(rc),
                                      "-o", str(out)])
    assert isinstance(res.exception, KeyError)
    # click.File('w') opens lazily, in the reference too: no row, no file
    assert not out.exists() or out.read_text() == ""
