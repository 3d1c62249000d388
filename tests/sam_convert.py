"""BAM -> SAM text for the `scan` SAM-input tests (test infrastructure):
every record of oracle/bamread.py's reader as a SAM line (SAMv1 §1.4), the
@SQ header in reference order.  Fields scan does not read (MAPQ, mate,
QUAL) are written as defaults."""
import gzip

from oracle import bamread

OPS = "MIDNSHP=X"


def bam_to_sam(bam, sam, compress=False):
    names, lengths, recs = bamread.read_bam(bam)
    lines = ["@HD\tVN:1.6\tSO:coordinate"]
    lines += ["@SQ\tSN:%s\tLN:%d" % (n, L) for n, L in zip(names, lengths)]
    lines.append("@PG\tID:sam_convert\tPN:tests")
    for r in recs:
        cigar = "".join("%d%s" % (ln, OPS[op]) for op, ln in r.cigar) or "*"
        lines.append("\t".join([
            r.name or "*", str(r.flag), names[r.tid] if r.tid >= 0 else "*", str(r.pos + 1), "255",
            cigar, "*", "0", str(r.tlen), r.seq if r.l_seq else "*", "*"]))
    text = ("\n".join(lines) + "\n").encode()
    with (gzip.open if compress else open)(sam, "wb") as fh:
        fh.write(text)
    return sam
