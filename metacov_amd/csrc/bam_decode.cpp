// Host BAM decoder: BGZF (multi-threaded raw-deflate inflate with zlib) ->
// BAM header + records -> coordinate-sorted pileup intervals (tid, pos, span).
//
// Replaces what the reference obtains through pysam/htslib on the pileup
// path: the header (`bam.references`, `bam.lengths`: metacov/cli.py:80,
// metacov/util.py:64-69), the record walk (IteratorRowAll in
// scan.AlignmentFileIterator, metacov/scan.pyx:204-216) and, per record, the
// interval htslib's pileup engine gives the read:
//   kept   iff tid >= 0 and (flag & flag_filter) == 0     (pysam stepper "all":
//          UNMAP|SECONDARY|QCFAIL|DUP = 0x704; supplementary reads kept)
//   span = bam_cigar2rlen (ops M/D/N/=/X, op-type mask 0x18D): what current
//          htslib's bam_plp_push takes as the read's end (tail->end = pos +
//          raw rlen), so a read without a reference-consuming op has span 0;
//          with MC_LEGACY_ENDPOS in flag_filter, 1 (htslib <= 1.9: bam_endpos)
// Records with more than 65535 CIGAR ops carry the real CIGAR in a CG:B,I
// tag behind a `<l_seq>S<rlen>N` placeholder (SAMv1 §4.2.2), as htslib's
// bam_read1 resolves it.
#include <chrono>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <memory>

#include "bgzf.h"

using namespace mc::bgzf;

namespace {

// Parses the BAM records in d[o, n) and appends the kept ones to `bam`.
// partial: d may end inside a record (a streaming window); parsing stops
// before it and *consumed is its offset.  Otherwise the records must tile
// [o, n) exactly.
int parse_records(const uint8_t* d, size_t o, size_t n, bool partial, int32_t n_ref,
                  uint32_t flag_filter, int nt, mc_bam* bam, size_t* consumed, const char* path,
                  const std::function<void(const char*)>& lap) {
    auto fail = [&](const char* msg, size_t at) {
        mc::set_error("%s: %s at byte %zu of the inflated stream", path, msg, at);
        return MC_E_IO;
    };
    // a complete record starts at q
    auto complete = [&](size_t q) -> bool {
        if (q + 4 > n) return false;
        const int32_t bs = rdi32(d + q);
        return bs >= 32 && q + 4 + (size_t)bs <= n;
    };
    // ---- records: the stream is cut into byte ranges; each range finds its
    // first record start in parallel (a candidate offset must begin a chain
    // of structurally valid records), and the ranges' walks must meet exactly
    // (range i ends on range i+1's first record) or the split falls back to
    // one sequential walk.  The ranges are then parsed in parallel twice
    // (count kept records / CIGAR words, then fill exact-size outputs).
    auto plausible = [&](size_t q) -> bool {
        if (q + 36 > n) return false;
        const int32_t bs = rdi32(d + q);
        if (bs < 32 || q + 4 + (size_t)bs > n) return false;
        const int32_t tid = rdi32(d + q + 4), pos = rdi32(d + q + 8);
        const uint8_t lrn = d[q + 12];
        const uint32_t ncig = rd16(d + q + 16);
        const int32_t lseq = rdi32(d + q + 20), ntid = rdi32(d + q + 24);
        if (tid < -1 || tid >= n_ref || ntid < -1 || ntid >= n_ref || pos < -1 || lrn == 0 ||
            lseq < 0)
            return false;
        const uint64_t need = 32 + (uint64_t)lrn + 4ull * ncig + ((uint64_t)lseq + 1) / 2 + (uint64_t)lseq;
        if (need > (uint64_t)bs) return false;
        return d[q + 36 + lrn - 1] == 0;
    };
    auto sync_at = [&](size_t from, size_t limit) -> size_t {   // first chained record start
        for (size_t q = from; q < limit; ++q) {
            size_t z = q;
            int k = 0;
            for (; k < 8 && z < n && plausible(z); ++k) z += 4 + (size_t)rdi32(d + z);
            if (k == 8 || z == n) return q;
        }
        return limit;
    };
    if (o >= n) {
        *consumed = n;
        return MC_OK;
    }
    const size_t nseg_target = std::max<size_t>(1, std::min<size_t>((size_t)nt * 4, (n - o) / (1 << 20) + 1));
    std::vector<size_t> seg_off(nseg_target + 1);
    seg_off[0] = o;
    seg_off[nseg_target] = n;
    {
        std::vector<size_t> cut(nseg_target + 1);
        for (size_t i = 0; i <= nseg_target; ++i) cut[i] = o + (n - o) * i / nseg_target;
        std::vector<std::thread> pool;
        std::atomic<size_t> nx{1};
        auto w = [&]() {
            for (size_t i; (i = nx.fetch_add(1)) < nseg_target;) seg_off[i] = sync_at(cut[i], n);
        };
        for (int i = 1; i < nt; ++i) pool.emplace_back(w);
        w();
        for (auto& t : pool) t.join();
    }
    // verify that consecutive ranges meet; fall back to the sequential walk
    bool chained = true;
    size_t tail_end = n;
    {
        std::vector<char> ok(nseg_target, 1);
        std::vector<std::thread> pool;
        std::atomic<size_t> nx{0};
        auto w = [&]() {
            for (size_t i; (i = nx.fetch_add(1)) < nseg_target;) {
                size_t q = seg_off[i];
                const bool last = i + 1 == nseg_target;
                const size_t end = seg_off[i + 1];
                if (q > end) { ok[i] = 0; continue; }
                while (q < end) {
                    if (!complete(q)) {
                        if (!(last && partial)) ok[i] = 0;
                        break;
                    }
                    q += 4 + (size_t)rdi32(d + q);
                }
                if (last && partial) tail_end = q;     // the window's last complete record ends here
                else if (q != end) ok[i] = 0;
            }
        };
        for (int i = 1; i < nt; ++i) pool.emplace_back(w);
        w();
        for (auto& t : pool) t.join();
        for (char c : ok) chained &= c != 0;
    }
    if (!chained) {
        seg_off.assign(1, o);
        size_t q = o;
        while (q < n) {
            if (!complete(q)) {
                if (partial) break;
                return fail(q + 4 > n ? "truncated record" : "bad record size", q);
            }
            q += 4 + (size_t)rdi32(d + q);
        }
        tail_end = q;
        seg_off.push_back(q);
    } else {
        seg_off.back() = tail_end;
    }
    *consumed = tail_end;
    // drop empty ranges
    seg_off.erase(std::unique(seg_off.begin(), seg_off.end()), seg_off.end());
    if (seg_off.size() < 2) seg_off.push_back(tail_end);
    lap("boundaries");
    const size_t nseg = seg_off.size() - 1;
    // one pass: each range fills its own buffers, then they are concatenated
    // in parallel after what `bam` already holds
    struct Seg {
        int64_t mapped = 0, unmapped = 0, records = 0;
        int err = 0;
        size_t err_at = 0;
        std::vector<int32_t> tid, pos, span;
        std::vector<uint32_t> cigar;
        std::vector<int64_t> nw;
    };
    std::vector<Seg> sg(nseg);
    const bool keep_cigar = bam->keep_cigar;
    {
        std::atomic<size_t> next_seg{0};
        auto work = [&]() {
            for (size_t g; (g = next_seg.fetch_add(1)) < nseg;) {
                Seg& c = sg[g];
                const size_t guess = (seg_off[g + 1] - seg_off[g]) / 200 + 16;
                c.tid.reserve(guess);
                c.pos.reserve(guess);
                c.span.reserve(guess);
                for (size_t q = seg_off[g]; q < seg_off[g + 1];) {
                    const int32_t block_size = rdi32(d + q);
                    const uint8_t* r = d + q + 4;
                    const uint8_t* rend = r + block_size;
                    q += 4 + (size_t)block_size;
                    const int32_t tid = rdi32(r);
                    const uint16_t flag = rd16(r + 14);
                    ++c.records;
                    if (tid >= 0 && !(flag & 4)) ++c.mapped;
                    else ++c.unmapped;
                    if (tid < 0 || (flag & flag_filter)) continue;
                    if (tid >= n_ref) {
                        c.err = 1;
                        c.err_at = q;
                        break;
                    }
                    const uint8_t* cig;
                    uint32_t n_cigar;
                    if (!cigar_of(r, rend, &cig, &n_cigar)) {
                        c.err = 2;
                        c.err_at = q;
                        break;
                    }
                    int64_t rlen = cigar_rlen(cig, n_cigar);
                    if (rlen <= 0 && (flag_filter & MC_LEGACY_ENDPOS)) rlen = 1;
                    if (rlen > INT32_MAX) {
                        c.err = 3;
                        c.err_at = q;
                        break;
                    }
                    c.tid.push_back(tid);
                    c.pos.push_back(rdi32(r + 4));
                    c.span.push_back((int32_t)rlen);
                    if (keep_cigar) {
                        c.cigar.insert(c.cigar.end(), reinterpret_cast<const uint32_t*>(cig),
                                       reinterpret_cast<const uint32_t*>(cig) + n_cigar);
                        c.nw.push_back(n_cigar);
                    }
                }
            }
        };
        std::vector<std::thread> pool;
        for (int i = 1; i < std::min<int>(nt, (int)nseg); ++i) pool.emplace_back(work);
        work();
        for (auto& t : pool) t.join();
    }
    lap("parse");
    std::vector<int64_t> kept_off(nseg + 1, 0), word_off(nseg + 1, 0);
    kept_off[0] = (int64_t)bam->tid.size();
    word_off[0] = keep_cigar ? (int64_t)bam->cigar.size() : 0;
    if (keep_cigar && bam->cig_off.empty()) bam->cig_off.push_back(0);
    for (size_t g = 0; g < nseg; ++g) {
        if (sg[g].err) {
            return fail(sg[g].err == 1 ? "record tid beyond the reference list"
                        : sg[g].err == 2 ? "CIGAR overruns record" : "reference span exceeds int32",
                        sg[g].err_at);
        }
        kept_off[g + 1] = kept_off[g] + (int64_t)sg[g].tid.size();
        word_off[g + 1] = word_off[g] + (int64_t)sg[g].cigar.size();
        bam->n_mapped += sg[g].mapped;
        bam->n_records += sg[g].records;
        bam->n_unmapped += sg[g].unmapped;
    }
    bam->tid.resize(kept_off[nseg]);
    bam->pos.resize(kept_off[nseg]);
    bam->span.resize(kept_off[nseg]);
    if (keep_cigar) {
        bam->cigar.resize(word_off[nseg]);
        bam->cig_off.resize(kept_off[nseg] + 1, 0);
    }
    {
        std::atomic<size_t> next_seg{0};
        auto copy = [&]() {
            for (size_t g; (g = next_seg.fetch_add(1)) < nseg;) {
                const Seg& c = sg[g];
                const size_t k = c.tid.size();
                if (k) {
                    std::memcpy(bam->tid.data() + kept_off[g], c.tid.data(), k * 4);
                    std::memcpy(bam->pos.data() + kept_off[g], c.pos.data(), k * 4);
                    std::memcpy(bam->span.data() + kept_off[g], c.span.data(), k * 4);
                }
                if (keep_cigar) {
                    if (!c.cigar.empty())
                        std::memcpy(bam->cigar.data() + word_off[g], c.cigar.data(), c.cigar.size() * 4);
                    int64_t w = word_off[g];
                    for (size_t i = 0; i < k; ++i) {
                        w += c.nw[i];
                        bam->cig_off[kept_off[g] + i + 1] = w;
                    }
                }
            }
        };
        std::vector<std::thread> pool;
        for (int i = 1; i < std::min<int>(nt, (int)nseg); ++i) pool.emplace_back(copy);
        copy();
        for (auto& t : pool) t.join();
    }
    return MC_OK;
}

}  // namespace

extern "C" int mc_bam_close(mc_bam* bam) {
    delete bam;
    return MC_OK;
}

extern "C" int mc_bam_n_targets(const mc_bam* bam, int32_t* n) {
    MC_REQUIRE(bam && n, MC_E_INVALID, "null argument");
    *n = (int32_t)bam->names.size();
    return MC_OK;
}

extern "C" int mc_bam_target(const mc_bam* bam, int32_t i, const char** name, int64_t* length) {
    MC_REQUIRE(bam && name && length, MC_E_INVALID, "null argument");
    MC_REQUIRE(i >= 0 && i < (int32_t)bam->names.size(), MC_E_INVALID, "target %d out of range", i);
    *name = bam->names[i].c_str();
    *length = bam->lens[i];
    return MC_OK;
}

extern "C" int mc_bam_counts(const mc_bam* bam, int64_t* n_records, int64_t* n_kept,
                             int64_t* n_mapped, int64_t* n_unmapped) {
    MC_REQUIRE(bam, MC_E_INVALID, "null bam");
    if (n_records) *n_records = bam->n_records;
    if (n_kept) *n_kept = (int64_t)bam->tid.size();
    if (n_mapped) *n_mapped = bam->n_mapped;
    if (n_unmapped) *n_unmapped = bam->n_unmapped;
    return MC_OK;
}

extern "C" int mc_bam_intervals(const mc_bam* bam, int32_t* tid, int32_t* pos, int32_t* span) {
    MC_REQUIRE(bam && tid && pos && span, MC_E_INVALID, "null argument");
    const size_t n = bam->tid.size();
    if (n) {
        std::memcpy(tid, bam->tid.data(), n * 4);
        std::memcpy(pos, bam->pos.data(), n * 4);
        std::memcpy(span, bam->span.data(), n * 4);
    }
    return MC_OK;
}

extern "C" int mc_bam_n_cigar_words(const mc_bam* bam, int64_t* n) {
    MC_REQUIRE(bam && n, MC_E_INVALID, "null argument");
    MC_REQUIRE(bam->keep_cigar, MC_E_STATE, "opened without keep_cigar");
    *n = (int64_t)bam->cigar.size();
    return MC_OK;
}

extern "C" int mc_bam_cigars(const mc_bam* bam, int64_t* cig_off, uint32_t* cigar) {
    MC_REQUIRE(bam && cig_off, MC_E_INVALID, "null argument");
    MC_REQUIRE(bam->keep_cigar, MC_E_STATE, "opened without keep_cigar");
    std::memcpy(cig_off, bam->cig_off.data(), bam->cig_off.size() * 8);
    if (!bam->cigar.empty()) {
        MC_REQUIRE(cigar, MC_E_INVALID, "null cigar");
        std::memcpy(cigar, bam->cigar.data(), bam->cigar.size() * 4);
    }
    return MC_OK;
}

// ---- streaming decode ------------------------------------------------------
//
// Bounded memory: BGZF blocks are inflated a window at a time (on all
// threads), the window's complete records are parsed (the parallel parse
// above, in partial mode) and a record cut by the window end is carried into
// the next window.  Intervals are handed out in caller-sized batches.
struct mc_bam_stream {
    MappedFile mf;
    std::string path;
    int nt = 1;
    uint32_t flag_filter = 0;
    size_t window = 0;                // inflated bytes per window
    size_t next_off = 0;              // file offset of the next BGZF block
    std::unique_ptr<uint8_t[]> buf;   // carried bytes + the current window (uninitialised)
    size_t cap = 0;
    size_t carry = 0;
    int32_t n_ref = 0;
    mc_bam out;                       // header, counters, parsed intervals not yet handed out
    size_t out_pos = 0;
    bool eof = false;
    double t_scan = 0, t_inflate = 0, t_parse = 0;   // MC_DECODE_TIMING
    ~mc_bam_stream() {
        if (std::getenv("MC_DECODE_TIMING"))
            std::fprintf(stderr, "[bam stream] scan %.3f s  inflate %.3f s  parse %.3f s\n", t_scan,
                         t_inflate, t_parse);
    }
};

namespace {
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

namespace {

// Inflates the next window of blocks after the carried bytes; returns the
// number of new bytes (0 at the end of the file).
int stream_fill(mc_bam_stream* s, size_t* added) {
    const double t0 = now_s();
    std::vector<Block> blocks;
    size_t total = 0;
    while (s->next_off < s->mf.size && total < s->window) {
        const size_t first = blocks.size();
        if (int rc = scan_blocks(s->mf.data, s->mf.size, s->next_off, s->next_off, blocks, total))
            return rc;
        const Block& b = blocks[first];
        s->next_off = b.cdata + b.clen + 8;
    }
    const size_t need = s->carry + total + 8;
    if (need > s->cap) {              // grow without zero-filling; keep the carried bytes
        const size_t ncap = std::max(need, s->cap + s->cap / 4);
        std::unique_ptr<uint8_t[]> nb(new (std::nothrow) uint8_t[ncap]);
        MC_REQUIRE(nb, MC_E_IO, "cannot allocate %zu bytes for %s", ncap, s->path.c_str());
        if (s->carry) std::memcpy(nb.get(), s->buf.get(), s->carry);
        s->buf = std::move(nb);
        s->cap = ncap;
    }
    const double t1 = now_s();
    MC_REQUIRE(blocks.empty() || inflate_blocks(s->mf.data, blocks, s->buf.get() + s->carry, s->nt),
               MC_E_IO, "BGZF inflate failed in %s", s->path.c_str());
    s->t_scan += t1 - t0;
    s->t_inflate += now_s() - t1;
    *added = total;
    return MC_OK;
}

// Parses buf[from, carry + added) (partial unless the file is done) and
// keeps the unparsed tail as the next carry.
int stream_parse(mc_bam_stream* s, size_t from, size_t added) {
    const size_t n = s->carry + added;
    const bool last = s->next_off >= s->mf.size;
    if (s->out_pos) {                 // drop what was already handed out
        s->out.tid.erase(s->out.tid.begin(), s->out.tid.begin() + s->out_pos);
        s->out.pos.erase(s->out.pos.begin(), s->out.pos.begin() + s->out_pos);
        s->out.span.erase(s->out.span.begin(), s->out.span.begin() + s->out_pos);
        s->out_pos = 0;
    }
    size_t consumed = from;
    const double t0 = now_s();
    const std::function<void(const char*)> nolap = [](const char*) {};
    if (int rc = parse_records(s->buf.get(), from, n, !last, s->n_ref, s->flag_filter, s->nt,
                               &s->out, &consumed, s->path.c_str(), nolap))
        return rc;
    s->carry = n - consumed;
    if (s->carry) std::memmove(s->buf.get(), s->buf.get() + consumed, s->carry);
    s->t_parse += now_s() - t0;
    if (last) {
        MC_REQUIRE(s->carry == 0, MC_E_IO, "%s: truncated record at the end of the file",
                   s->path.c_str());
        s->eof = true;
    }
    return MC_OK;
}

}  // namespace

namespace {

int stream_open(const char* path, int n_threads, uint32_t flag_filter, int64_t window_bytes,
                bool keep_cigar, std::unique_ptr<mc_bam_stream>& s) {
    s.reset(new mc_bam_stream());
    if (int rc = s->mf.open(path)) return rc;
    s->path = path;
    s->nt = n_threads_or_all(n_threads);
    s->flag_filter = flag_filter;
    s->window = (size_t)std::max<int64_t>(window_bytes > 0 ? window_bytes : (256ll << 20), 1 << 16);
    s->out.keep_cigar = keep_cigar;
    // header: windows until the reference list parses, then the first records
    size_t o = 0;
    for (;;) {
        size_t added = 0;
        if (int rc = stream_fill(s.get(), &added)) return rc;
        s->carry += added;
        std::vector<std::string> names;
        std::vector<int64_t> lens;
        if (parse_header(s->buf.get(), s->carry, path, names, lens, &o) == MC_OK) {
            s->out.names = std::move(names);
            s->out.lens = std::move(lens);
            break;
        }
        MC_REQUIRE(s->next_off < s->mf.size, MC_E_IO, "%s: no valid BAM header", path);
    }
    s->n_ref = (int32_t)s->out.names.size();
    const size_t have = s->carry;
    s->carry = 0;
    return stream_parse(s.get(), o, have);
}

}  // namespace

extern "C" int mc_bam_stream_open(const char* path, int n_threads, uint32_t flag_filter,
                                  int64_t window_bytes, mc_bam_stream** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<mc_bam_stream> s;
    if (int rc = stream_open(path, n_threads, flag_filter, window_bytes, false, s)) return rc;
    *out = s.release();
    return MC_OK;
}

// The whole file: the same windows (the buffer stays warm instead of faulting
// in the entire inflated file), every kept interval accumulated.
extern "C" int mc_bam_open(const char* path, int n_threads, uint32_t flag_filter, int keep_cigar,
                           mc_bam** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<mc_bam_stream> s;
    if (int rc = stream_open(path, n_threads, flag_filter, 0, keep_cigar != 0, s)) return rc;
    while (!s->eof) {
        size_t added = 0;
        if (int rc = stream_fill(s.get(), &added)) return rc;
        if (int rc = stream_parse(s.get(), 0, added)) return rc;
    }
    *out = new mc_bam(std::move(s->out));
    return MC_OK;
}

extern "C" int mc_bam_stream_next(mc_bam_stream* s, int64_t cap, int32_t* tid, int32_t* pos,
                                  int32_t* span, int64_t* n_out) {
    MC_REQUIRE(s && n_out && cap >= 0 && (cap == 0 || (tid && pos && span)), MC_E_INVALID,
               "bad argument");
    while ((int64_t)(s->out.tid.size() - s->out_pos) < cap && !s->eof) {
        size_t added = 0;
        if (int rc = stream_fill(s, &added)) return rc;
        if (int rc = stream_parse(s, 0, added)) return rc;
    }
    const int64_t k = std::min<int64_t>(cap, (int64_t)(s->out.tid.size() - s->out_pos));
    if (k) {
        std::memcpy(tid, s->out.tid.data() + s->out_pos, k * 4);
        std::memcpy(pos, s->out.pos.data() + s->out_pos, k * 4);
        std::memcpy(span, s->out.span.data() + s->out_pos, k * 4);
        s->out_pos += (size_t)k;
    }
    *n_out = k;
    return MC_OK;
}

extern "C" int mc_bam_stream_header(const mc_bam_stream* s, const mc_bam** header) {
    MC_REQUIRE(s && header, MC_E_INVALID, "null argument");
    *header = &s->out;      // names, lengths and (so far) counts via the mc_bam accessors
    return MC_OK;
}

extern "C" int mc_bam_stream_close(mc_bam_stream* s) {
    delete s;
    return MC_OK;
}
