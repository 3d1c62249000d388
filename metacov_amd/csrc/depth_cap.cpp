// htslib's pileup read-pool cap, opt-in (pysam AlignmentFile.pileup's
// max_depth, 8000 by default, called at metacov/pileup.py:13).
//
// htslib's bam_plp_push (sam.c) drops a read, before it joins the pileup
// buffer, when
//     iter->tid == b->core.tid && iter->pos == b->core.pos && iter->mp->cnt > iter->maxcnt
// where iter->pos is the column the pileup has reached and mp->cnt the nodes
// alive in its buffer pool (the buffered reads + the empty tail node).  When a
// read is pushed, the pileup has produced every column before the previous
// read's start, so iter->pos equals that start: only a read starting at the
// SAME position as its predecessor can be dropped, and the buffered reads are
// then the kept reads whose end (tail->end = pos + span, exclusive) is >= that
// position (bam_plp_next frees a read at the first column at or past its end;
// reads of earlier contigs are all freed when the contig changes, and a
// contig's first read is never dropped).  A kept read joins the buffer only if
// `tail->end > iter->pos`: a group's first read always does (iter->pos is
// still the previous start), a later one only with span > 0 (current htslib
// gives a read without reference-consuming ops span 0; under the legacy
// bam_endpos rule every span is >= 1).  So for a group of reads starting at s:
//   C = kept reads before the group with end >= s;
//   the group's first read is kept; each further read is kept while
//   1 + C + (group reads buffered so far) <= maxcnt.
// One sweep per contig with a min-heap of the kept reads' ends.  The cap is
// version-dependent (parity unpinned: htslib is absent here); the oracle's
// literal restatement of the push / next loop (oracle/htslib_plp.py) pins
// this closed form.
#include <algorithm>
#include <atomic>
#include <functional>
#include <queue>
#include <thread>
#include <vector>

#include "../../include/metacov_amd.h"
#include "common.h"

extern "C" int mc_depth_cap_mask(int64_t n, const int32_t* tid, const int32_t* pos, const int32_t* span,
                                 int32_t max_depth, int n_threads, uint8_t* keep, int64_t* n_dropped) {
    MC_REQUIRE(n >= 0 && (n == 0 || (tid && pos && span && keep)), MC_E_INVALID, "bad read arrays");
    MC_REQUIRE(max_depth >= 1, MC_E_INVALID, "max_depth must be >= 1 (got %d)", max_depth);
    // contig segments of the sorted reads
    std::vector<int64_t> seg{0};
    for (int64_t i = 1; i < n; ++i) {
        MC_REQUIRE(tid[i] > tid[i - 1] || (tid[i] == tid[i - 1] && pos[i] >= pos[i - 1]), MC_E_INVALID,
                   "reads are not coordinate-sorted at %lld", (long long)i);
        if (tid[i] != tid[i - 1]) seg.push_back(i);
    }
    seg.push_back(n);
    const int64_t n_seg = (int64_t)seg.size() - 1;
    std::atomic<int64_t> next{0}, dropped{0};
    auto worker = [&]() {
        std::priority_queue<int64_t, std::vector<int64_t>, std::greater<int64_t>> ends;
        for (int64_t q; (q = next.fetch_add(1)) < n_seg;) {
            while (!ends.empty()) ends.pop();
            int64_t lost = 0;
            for (int64_t i = seg[q]; i < seg[q + 1];) {
                const int32_t s = pos[i];
                int64_t g = i + 1;
                while (g < seg[q + 1] && pos[g] == s) ++g;
                while (!ends.empty() && ends.top() < s) ends.pop();
                const int64_t c = (int64_t)ends.size();
                int64_t kept = 0;
                for (int64_t j = i; j < g; ++j) {
                    const bool k = j == i || 1 + c + kept <= max_depth;
                    keep[j] = k ? 1 : 0;
                    if (k) {
                        if (j == i || span[j] > 0) {
                            ++kept;
                            ends.push((int64_t)pos[j] + span[j]);
                        }
                    } else {
                        ++lost;
                    }
                }
                i = g;
            }
            dropped += lost;
        }
    };
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n_seg));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    if (n_dropped) *n_dropped = dropped.load();
    return MC_OK;
}
