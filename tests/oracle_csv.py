"""Expected `metacov pileup` CSV text built from the oracle alone (test
infrastructure): oracle/bamread.py's intervals -> coracle's depth and exact
region rows -> classic()'s formatting (engine.classic_stats, the host half
of metacov/pileup.py:18-26, pinned by the real classic()'s goldens) -> the
csv module as metacov/cli.py:97-108 writes it."""
import csv
import io

import numpy as np

from metacov_amd.engine import classic_stats
from oracle import bamread, coracle


def oracle_csv(path, regs):
    """regs: [(sacc, sstart, send)] as the region file holds them (echoed
    raw; sorted and taken as 0-based half-open, cli.py:89).  sacc is the
    first word of a header name (cli.py:80)."""
    names, lens, _c, tid, pos, span = bamread.scan_intervals(path)
    d, ext, coff = coracle.depth(lens, tid, pos, span)
    first_word = {}
    for t, n in enumerate(names):
        first_word.setdefault(n.split()[0], t)
    rt, rs, re_ = [], [], []
    for sacc, a, b in regs:
        s, e = sorted((int(a), int(b)))
        rt.append(first_word[sacc])
        rs.append(s)
        re_.append(e)
    rows = coracle.region_stats(d, ext, coff, np.array(rt, np.int32), np.array(rs, np.int64),
                                np.array(re_, np.int64))
    out = io.StringIO()
    w = None
    for (sacc, a, b), row in zip(regs, rows):
        res = classic_stats(row)
        if w is None:
            w = csv.DictWriter(out, fieldnames=["sacc", "start", "end"] + sorted(res))
            w.writeheader()
        res.update({"sacc": sacc, "start": a, "end": b})
        w.writerow(res)
    return out.getvalue()
