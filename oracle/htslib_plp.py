"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

A literal, column-by-column restatement of htslib's pileup engine as pysam's
`AlignmentFile.pileup(ref, start, end)` drives it (called at the reference's
`metacov/pileup.py:13`), INCLUDING the read-pool cap `max_depth` (pysam's
default 8000, set through `bam_mplp_set_maxcnt`).  htslib is a third-party
dependency the reference does not vendor and does not pin (`requirements.txt:2`,
`setup.py:45,53`); what is restated is htslib 1.x `sam.c`:

  bam_plp_push(iter, b):
      if (b->core.tid < 0 || b->core.flag & BAM_FUNMAP) return 0   (filtered before here)
      if (iter->tid == b->core.tid && iter->pos == b->core.pos
          && iter->mp->cnt > iter->maxcnt) return 0                  <- the cap: b dropped
      copy b to the tail node; tail->beg = pos;
      tail->end = pos + bam_cigar2rlen(b)   (current htslib: "raw rlen rather
                  than bam_endpos()"; htslib <= 1.9: bam_endpos(b), i.e. the
                  spans passed in are then already >= 1)
      iter->max_tid = tid; iter->max_pos = beg
      if (tail->end > iter->pos || tid > iter->tid) tail->next = mp_alloc()   (cnt + 1)

  bam_plp_next(iter):   (bam_plp_auto returns each column with n_plp > 0)
      while (is_eof || max_tid > tid || (max_tid == tid && max_pos > pos)):
          for each buffered node p:
              if p.tid < tid or (p.tid == tid and p.end <= pos): free p  (cnt - 1)
              elif p.tid == tid and p.beg <= pos: n_plp += 1
          emit (tid, pos, n_plp) if n_plp
          if buffer non-empty: new contig -> (tid, pos) = (head.tid, head.beg);
                               pos < head.beg -> pos = head.beg; else pos += 1
          else pos += 1
          if is_eof and buffer empty: break

mp->cnt starts at 1 (head == tail == one allocated node).  The reads fed in
are the region query's: records of `tid` overlapping [start, end) (htslib's
iterator, hts_itr_next, returns a record when beg < end and bam_endpos > start,
bam_endpos = pos + max(rlen, 1) in every version), after the stepper "all"
filter (flag & 0x704 == 0), in file order.  O(columns x buffered reads): small
inputs only.
"""
import numpy as np


class PileupIter:
    def __init__(self, maxcnt):
        self.maxcnt = maxcnt
        self.buf = []          # [tid, beg, end] of the buffered reads, head first
        self.cnt = 1           # nodes alive in the pool (the tail node)
        self.tid = self.pos = 0
        self.max_tid = self.max_pos = -1
        self.is_eof = False
        self.dropped = 0

    def push(self, tid, beg, end):
        if self.tid == tid and self.pos == beg and self.cnt > self.maxcnt:
            self.dropped += 1
            return False
        self.max_tid, self.max_pos = tid, beg
        if end > self.pos or tid > self.tid:
            self.buf.append([tid, beg, end])
            self.cnt += 1
        return True

    def next_columns(self):
        out = []
        while self.is_eof or self.max_tid > self.tid or (self.max_tid == self.tid and self.max_pos > self.pos):
            n = 0
            keep = []
            for p in self.buf:
                if p[0] < self.tid or (p[0] == self.tid and p[2] <= self.pos):
                    self.cnt -= 1
                else:
                    keep.append(p)
                    if p[0] == self.tid and p[1] <= self.pos:
                        n += 1
            self.buf = keep
            if n:
                out.append((self.tid, self.pos, n))
            if self.buf:
                h = self.buf[0]
                if self.tid < h[0]:
                    self.tid, self.pos = h[0], h[1]
                elif self.pos < h[1]:
                    self.pos = h[1]
                else:
                    self.pos += 1
            else:
                self.pos += 1
            if self.is_eof and not self.buf:
                break
        return out


def region_depth(tid, pos, span, t, start, end, max_depth=8000):
    """classic()'s column vector for [start, end) of contig t as pysam's
    pileup(ref, start, end) with max_depth fills it (pileup.py:11-16), from
    coordinate-sorted (tid, pos, span) records after the 0x704 filter."""
    tid = np.asarray(tid)
    pos = np.asarray(pos, np.int64)
    span = np.asarray(span, np.int64)
    endp = pos + np.maximum(span, 1)                  # bam_endpos: the iterator's overlap test
    sel = np.nonzero((tid == t) & (pos < end) & (endp > start))[0]
    it = PileupIter(max_depth)
    cols = []
    for i in sel:
        it.push(t, int(pos[i]), int(pos[i] + span[i]))   # bam_plp_push: tail->end
        cols += it.next_columns()
    it.is_eof = True
    cols += it.next_columns()
    out = np.zeros(end - start, np.int64)
    for (ct, p, n) in cols:
        if ct == t and start <= p < end:
            out[p - start] += n
    return out, it.dropped
