// Read-side reductions of the reference's experimental estimator
// (pileup.experimental, metacov/pileup.py:38-173), host C++.
//
// mc_reads_open decodes every placed record (tid >= 0) of a coordinate-sorted
// BAM into a compact table: the fields experimental() reads from pysam's
// AlignedSegment (is_secondary / is_proper_pair / is_reverse / is_read1 =
// flag bits 0x100 / 0x2 / 0x10 / 0x40, query_name, reference_start,
// reference_length, the first K bases of query_alignment_sequence) plus the
// record's end for the fetch overlap test.  Third-party semantics restated
// (pysam / htslib, unpinned by the reference, requirements.txt:2):
//   fetch(ref, start, end)          records of ref with pos < end and
//                                   bam_endpos > start, in file order
//   bam_endpos                      pos + bam_cigar2rlen, or pos + 1 when the
//                                   read is unmapped or the length is 0
//   reference_length                None when unmapped or without CIGAR,
//                                   else bam_endpos - pos
//   query_alignment_sequence        None when l_seq == 0, else
//                                   seq[leading S .. l_seq - trailing S]
//                                   (getQueryStart / getQueryEnd: H skipped,
//                                   the backwards walk stops at op 1)
//
// mc_experimental_reads then runs the per-read loop of pileup.py:101-151 for
// R regions on a thread pool (regions are independent) and returns exact
// aggregates; the Python layer (metacov_amd/experimental.py) turns them into
// the 13 result fields with the reference's expression types.  The per-
// position arrays of the reference are never materialised:
//   cov   sum over reads of |[max(0,rstart), min(L,rend))|         (exact)
//   covc  per-position 1/rcor sums in read order, np.mean's pairwise sum
//         (the array is built only when some 1/rcor != 1)          (exact)
//   starts / cor   the distinct rstart in [0, L) and the 1/rcor of the last
//         read starting there; np.mean(cor) is re-summed exactly the way
//         numpy 2.x's add.reduce does (8192-element chunks, pairwise within)
//         and the builtin sum(cor) sequentially (pileup.py:166)      (exact)
//   cov2  sum of the numpy slice lengths of cov2[s-1:e+1]           (exact)
//   wnf   the pair terms in pairing order                          (exact)
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string_view>
#include <thread>
#include <unordered_map>

#include "bgzf.h"
#include "common.h"
#include "exp_gpu.h"

using namespace mc::bgzf;

namespace {

constexpr uint32_t kNoKmer = 0xFFFFFFFFu;
constexpr uint8_t kNoSeq = 1, kNoRefLen = 2;

enum Status : int64_t {
    kOk = 0,
    kNoSeqError = 1,      // query_alignment_sequence is None (TypeError in the reference)
    kNoRefLenError = 2,   // reference_length is None (TypeError)
    kNoKcorError = 3,     // k_cor is None and a pair was found (TypeError)
};

}  // namespace

struct mc_reads {
    int k = 0;
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    int64_t n_records = 0, n_unplaced = 0;
    // placed records, file order
    std::vector<int32_t> pos;
    std::vector<int64_t> end;       // bam_endpos
    std::vector<uint16_t> flag;
    std::vector<uint8_t> bits;      // kNoSeq | kNoRefLen
    std::vector<uint32_t> kmer;     // 2-bit code of the first K aligned bases, or kNoKmer
    std::vector<uint64_t> name_off;
    std::vector<uint8_t> name_len;
    std::string arena;
    std::vector<int64_t> first;     // per contig [first[t], first[t+1])
    std::vector<int64_t> max_span;  // per contig max(end - pos)
    std::vector<std::vector<uint64_t>> events;   // per region of the last call: (readno << 32) | kmer
    // a GPU decode's table stays in HBM (mc_reads_open_gpu*): the read pass
    // runs on the device (csrc/exp_gpu.hip); the host vectors above are
    // filled only when mc_reads_fields asks for them
    mc_bam_gpu* g = nullptr;
    ExpDevTable dev;
    bool host_ready = true;
    double pass_ms = 0;             // the last mc_experimental_reads call
    ExpScratch* scratch = nullptr;  // the device pass's buffers, kept between calls
    ~mc_reads() {
        if (scratch) exp_gpu_scratch_free(scratch);
        if (g) mc_bam_gpu_close(g);
    }
};

namespace {

// 2-bit code of nt16 base b (A=1 C=2 G=4 T=8), or 4 for any other symbol.
inline uint32_t nt16_2bit(uint32_t b) {
    switch (b) {
        case 1: return 0;
        case 2: return 1;
        case 4: return 2;
        case 8: return 3;
        default: return 4;
    }
}

// The first k bases of query_alignment_sequence as a 2-bit code, kNoKmer when
// shorter than k or not all of A/C/G/T (such a prefix matches no K-mer key).
uint32_t kmer_prefix(const uint8_t* cig, uint32_t n_cigar, const uint8_t* seq, int32_t l_seq,
                     int k) {
    int64_t qs = 0, qe = l_seq;
    for (uint32_t i = 0; i < n_cigar; ++i) {          // getQueryStart
        const uint32_t op = rd32(cig + 4 * i) & 0xF;
        if (op == 5) continue;
        if (op == 4) { qs += rd32(cig + 4 * i) >> 4; continue; }
        break;
    }
    for (uint32_t i = n_cigar; i-- > 1;) {            // getQueryEnd (stops at op 1)
        const uint32_t op = rd32(cig + 4 * i) & 0xF;
        if (op == 5) continue;
        if (op == 4) { qe -= rd32(cig + 4 * i) >> 4; continue; }
        break;
    }
    if (qe - qs < k) return kNoKmer;
    uint32_t code = 0;
    for (int m = 0; m < k; ++m) {
        const int64_t q = qs + m;
        const uint32_t b = nt16_2bit((seq[q >> 1] >> ((~q & 1) << 2)) & 0xF);
        if (b > 3) return kNoKmer;
        code = (code << 2) | b;
    }
    return code;
}

// The complete records of d[o, n): a serial pass over the record sizes and
// the order / range checks (a few ns per record), then the placed records'
// fields on nt threads, each into its own slice of the tables and its own
// name arena (one serial walk was ~0.3 s of the 0.42 s read pass on 3.2 M
// records, profiles/r05/r05f_experimental.json).
int walk_records(mc_reads* r, const uint8_t* d, size_t o, size_t n, size_t* consumed, int32_t* last_tid,
                 int32_t* last_pos, const char* path, int nt) {
    const int32_t n_ref = (int32_t)r->names.size();
    std::vector<size_t> placed;   // offsets of the placed records (tid >= 0)
    std::vector<int32_t> ptid;    // and their contigs
    while (o + 4 <= n) {
        const int32_t bs = rdi32(d + o);
        MC_REQUIRE(bs >= 32, MC_E_IO, "%s: bad record size at inflated byte %zu", path, o);
        if (o + 4 + (size_t)bs > n) break;
        __builtin_prefetch(d + std::min(n - 1, o + 4096));   // (the size chain is a serial walk)
        const uint8_t* b = d + o + 4;
        const int32_t tid = rdi32(b), pos = rdi32(b + 4);
        const uint8_t l_read_name = b[8];
        const int32_t l_seq = rdi32(b + 16);
        MC_REQUIRE(tid >= -1 && tid < n_ref && l_read_name > 0 && l_seq >= 0, MC_E_IO,
                   "%s: corrupt record at inflated byte %zu", path, o);
        ++r->n_records;
        if (tid < 0) {
            ++r->n_unplaced;
        } else {
            MC_REQUIRE(tid > *last_tid || (tid == *last_tid && pos >= *last_pos), MC_E_INVALID,
                       "%s is not coordinate-sorted (record %lld); experimental() fetches "
                       "regions of a sorted, indexed BAM", path, (long long)r->n_records - 1);
            *last_tid = tid;
            *last_pos = pos;
            placed.push_back(o);
            ptid.push_back(tid);
        }
        o += 4 + (size_t)bs;
    }
    *consumed = o;
    const size_t m = placed.size();
    if (m == 0) return MC_OK;
    const size_t base = r->pos.size();
    r->pos.resize(base + m);
    r->end.resize(base + m);
    r->flag.resize(base + m);
    r->bits.resize(base + m);
    r->kmer.resize(base + m);
    r->name_off.resize(base + m);
    r->name_len.resize(base + m);
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(nt, 1), m / 4096 + 1));
    std::vector<std::string> arenas(T);
    std::vector<size_t> bad(T, SIZE_MAX);   // first record a thread found truncated
    auto work = [&](int t) {
        const size_t i0 = m * t / T, i1 = m * (t + 1) / T;
        std::string& ar = arenas[t];
        for (size_t i = i0; i < i1; ++i) {
            const uint8_t* b = d + placed[i] + 4;
            const uint8_t* bend = b + rdi32(d + placed[i]);
            const int32_t pos = rdi32(b + 4);
            const uint8_t l_read_name = b[8];
            const uint16_t flag = rd16(b + 14);
            const int32_t l_seq = rdi32(b + 16);
            const uint8_t* cig;
            uint32_t n_cigar;
            const uint8_t* seq = b + 32 + l_read_name + 4 * (size_t)rd16(b + 12);
            if (!cigar_of(b, bend, &cig, &n_cigar) || seq + ((size_t)l_seq + 1) / 2 > bend) {
                bad[t] = i;
                return;
            }
            const bool unmapped = flag & 4;
            int64_t rlen = unmapped ? 0 : cigar_rlen(cig, n_cigar);
            if (rlen == 0) rlen = 1;
            const size_t k = base + i;
            r->pos[k] = pos;
            r->end[k] = pos + rlen;
            r->flag[k] = flag;
            r->bits[k] = (uint8_t)((l_seq == 0 ? kNoSeq : 0) | ((unmapped || n_cigar == 0) ? kNoRefLen : 0));
            r->kmer[k] = l_seq ? kmer_prefix(cig, n_cigar, seq, l_seq, r->k) : kNoKmer;
            const size_t nl = strnlen((const char*)b + 32, l_read_name);
            r->name_off[k] = ar.size();   // (thread-relative until the arenas are joined)
            r->name_len[k] = (uint8_t)nl;
            ar.append((const char*)b + 32, nl);
        }
    };
    if (T == 1) {
        work(0);
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < T; ++t) pool.emplace_back(work, t);
        for (auto& th : pool) th.join();
    }
    for (int t = 0; t < T; ++t) {
        MC_REQUIRE(bad[t] == SIZE_MAX, MC_E_IO, "%s: truncated CIGAR or SEQ at inflated byte %zu", path,
                   placed[bad[t]]);
    }
    size_t names = r->arena.size();   // join the arenas
    for (int t = 0; t < T; ++t) names += arenas[t].size();
    if (names > r->arena.capacity()) r->arena.reserve(std::max(names, r->arena.capacity() + r->arena.capacity() / 2));
    for (int t = 0; t < T; ++t) {
        const size_t i0 = m * t / T, i1 = m * (t + 1) / T, shift = r->arena.size();
        for (size_t i = i0; i < i1; ++i) r->name_off[base + i] += shift;
        r->arena += arenas[t];
    }
    for (size_t i = 0; i < m; ++i) {   // per contig first record and maximum span
        const int32_t tid = ptid[i];
        const size_t k = base + i;
        if (r->first.size() <= (size_t)tid) r->first.resize(tid + 1, (int64_t)k);
        int64_t& ms = r->max_span[tid];
        ms = std::max<int64_t>(ms, r->end[k] - r->pos[k]);
    }
    return MC_OK;
}

// One window of the file: its BGZF blocks inflated after kCarryRoom bytes of
// room, where the previous window's unfinished record is copied in front.
struct Window {
    std::unique_ptr<uint8_t[]> buf;
    size_t cap = 0, total = 0;
    bool last = false;
};
constexpr size_t kCarryRoom = 1 << 20;

// Finds the blocks of up to `window` inflated bytes from *next_off and
// inflates them into w (after kCarryRoom).  Runs on a background thread for
// the next window while the current one is walked: the walk's serial parts
// (the record-size chain, the joins) overlap the inflate.
int produce_window(const MappedFile& mf, size_t* next_off, size_t window, int nt, const char* path, Window& w,
                   std::string* err) {
    std::vector<Block> blocks;
    size_t total = 0;
    while (*next_off < mf.size && total < window) {
        const size_t b0 = blocks.size();
        if (int rc = scan_blocks(mf.data, mf.size, *next_off, *next_off, blocks, total)) {
            *err = mc::last_error();
            return rc;
        }
        *next_off = blocks[b0].cdata + blocks[b0].clen + 8;
    }
    w.last = *next_off >= mf.size;
    w.total = total;
    if (kCarryRoom + total + 8 > w.cap) {
        w.cap = kCarryRoom + total + 8;
        w.buf.reset(new (std::nothrow) uint8_t[w.cap]);
        if (!w.buf) {
            *err = "cannot allocate the read window for " + std::string(path);
            w.cap = 0;
            return MC_E_IO;
        }
    }
    if (!blocks.empty() && !inflate_blocks(mf.data, blocks, w.buf.get() + kCarryRoom, nt)) {
        *err = "BGZF inflate failed in " + std::string(path);
        return MC_E_IO;
    }
    return MC_OK;
}

int reads_open(const char* path, int n_threads, int k, mc_reads* r) {
    MappedFile mf;
    if (int rc = mf.open(path)) return rc;
    const int nt = n_threads_or_all(n_threads);
    size_t window = 256ull << 20;
    if (const char* e = std::getenv("MC_READS_WINDOW")) window = std::max<size_t>(1, std::strtoull(e, nullptr, 10));
    const char* pe = std::getenv("MC_READS_PIPELINE");
    const bool pipeline = !(pe && pe[0] == '0');
    size_t next_off = 0;
    bool have_header = false;
    int32_t last_tid = -1, last_pos = -1;
    std::vector<uint8_t> carry;   // the previous window's unfinished bytes
    Window cur, nxt;
    std::string perr;
    if (int rc = produce_window(mf, &next_off, window, nt, path, cur, &perr)) {
        mc::set_error("%s", perr.c_str());
        return rc;
    }
    for (;;) {
        int prc = MC_OK;
        std::thread producer;
        if (!cur.last) {
            if (pipeline)
                producer = std::thread([&] { prc = produce_window(mf, &next_off, window, nt, path, nxt, &perr); });
            else
                prc = produce_window(mf, &next_off, window, nt, path, nxt, &perr);
        }
        auto join = [&] {
            if (producer.joinable()) producer.join();
        };
        // the window's bytes with the carry in front
        uint8_t* d;
        std::unique_ptr<uint8_t[]> big;   // (a carry larger than the room)
        if (carry.size() <= kCarryRoom) {
            d = cur.buf.get() + kCarryRoom - carry.size();
            if (!carry.empty()) std::memcpy(d, carry.data(), carry.size());
        } else {
            big.reset(new (std::nothrow) uint8_t[carry.size() + cur.total + 8]);
            if (!big) {
                join();
                MC_REQUIRE(false, MC_E_IO, "cannot allocate %zu bytes for %s", carry.size() + cur.total, path);
            }
            std::memcpy(big.get(), carry.data(), carry.size());
            std::memcpy(big.get() + carry.size(), cur.buf.get() + kCarryRoom, cur.total);
            d = big.get();
        }
        const size_t n = carry.size() + cur.total;
        size_t o = 0;
        if (!have_header) {
            std::vector<std::string> names;
            std::vector<int64_t> lens;
            if (parse_header(d, n, path, names, lens, &o) != MC_OK) {
                join();
                MC_REQUIRE(!cur.last, MC_E_IO, "%s: no valid BAM header", path);
                MC_REQUIRE(prc == MC_OK, prc, "%s", perr.c_str());
                carry.assign(d, d + n);
                std::swap(cur, nxt);
                continue;
            }
            have_header = true;
            r->names = std::move(names);
            r->lens = std::move(lens);
            r->max_span.assign(r->names.size(), 0);
        }
        size_t consumed = o;
        const int wrc = walk_records(r, d, o, n, &consumed, &last_tid, &last_pos, path, nt);
        join();
        if (wrc) return wrc;
        carry.assign(d + consumed, d + n);
        if (cur.last) {
            MC_REQUIRE(carry.empty(), MC_E_IO, "%s: truncated record at the end of the file", path);
            break;
        }
        MC_REQUIRE(prc == MC_OK, prc, "%s", perr.c_str());
        std::swap(cur, nxt);
    }
    r->first.resize(r->names.size() + 1, (int64_t)r->pos.size());
    return MC_OK;
}

struct Tables {
    const double* val[2];
    const uint8_t* has[2];
    bool none;   // k_cor is None
    bool lookup(int which, uint32_t code, double* v) const {
        if (none || code == kNoKmer || !has[which][code]) return false;
        *v = val[which][code];
        return true;
    }
};

// Python slice index normalisation (step 1) for an array of length L.
inline int64_t slice_index(int64_t i, int64_t L) {
    if (i < 0) {
        i += L;
        return i < 0 ? 0 : i;
    }
    return i > L ? L : i;
}

// numpy 2.x pairwise sum of a block of n float64 (n <= 8192) whose only
// non-zero entries are v[0..m) at sorted offsets off[0..m) (relative to the
// block start).  Zeros are exact no-ops, so only the entries are replayed.
double pairwise_block(const int64_t* off, const double* v, size_t m, int64_t base, int64_t n) {
    if (n < 8) {   // numpy starts from -0.0; with a zero element present that is +0.0
        double res = 0.0;
        for (size_t i = 0; i < m; ++i) res += v[i];
        return res;
    }
    if (n <= 128) {
        double r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int64_t body = n - (n % 8);
        size_t i = 0;
        for (; i < m && off[i] - base < body; ++i) r[(off[i] - base) & 7] += v[i];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < m; ++i) res += v[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    const size_t split = (size_t)(std::lower_bound(off, off + m, base + n2) - off);
    return pairwise_block(off, v, split, base, n2) +
           pairwise_block(off + split, v + split, m - split, base + n2, n - n2);
}

// numpy 2.x pairwise sum of a dense block of n float64 (n <= 8192)
double pairwise_dense(const double* a, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_dense(a, n2) + pairwise_dense(a + n2, n - n2);
}

// np.add.reduce over a dense float64 array: 8192-element chunks, pairwise within
// np.add.reduce of the per-position sums of covers [a, b) += inv (added per
// position in cover order) over [0, L), chunk by chunk: the covers touching
// each 8192-position chunk are listed in cover order (CSR), their sums built
// in one chunk buffer, which is summed as numpy_sum_dense sums that chunk.
template <class Cover>
double numpy_sum_covers(const Cover* cv, size_t m, int64_t L) {
    constexpr int64_t kChunk = 8192;
    const int64_t nb = (L + kChunk - 1) / kChunk;
    std::vector<int64_t> first((size_t)nb + 1, 0);
    for (size_t j = 0; j < m; ++j)
        for (int64_t k = cv[j].a / kChunk; k <= (cv[j].b - 1) / kChunk; ++k) ++first[(size_t)k + 1];
    for (int64_t k = 0; k < nb; ++k) first[(size_t)k + 1] += first[(size_t)k];
    std::vector<uint32_t> list((size_t)first[(size_t)nb]);
    std::vector<int64_t> fill(first.begin(), first.end() - 1);
    for (size_t j = 0; j < m; ++j)
        for (int64_t k = cv[j].a / kChunk; k <= (cv[j].b - 1) / kChunk; ++k) list[(size_t)fill[(size_t)k]++] = (uint32_t)j;
    std::vector<double> buf((size_t)kChunk);
    double total = 0;
    for (int64_t k = 0; k < nb; ++k) {
        const int64_t c0 = k * kChunk, n = std::min(kChunk, L - c0);
        std::fill(buf.begin(), buf.begin() + n, 0.0);
        for (int64_t q = first[(size_t)k]; q < first[(size_t)k + 1]; ++q) {
            const Cover& c = cv[list[(size_t)q]];
            const int64_t a = std::max(c.a, c0), b = std::min(c.b, c0 + n);
            for (int64_t p = a; p < b; ++p) buf[(size_t)(p - c0)] += c.inv;
        }
        const double s = pairwise_dense(buf.data(), n);
        total = k == 0 ? s : total + s;
    }
    return total;
}

double numpy_sum_dense(const std::vector<double>& v) {
    constexpr int64_t kChunk = 8192;
    const int64_t L = (int64_t)v.size();
    double total = 0;
    for (int64_t c = 0; c < L; c += kChunk) {
        const double s = pairwise_dense(v.data() + c, std::min(kChunk, L - c));
        total = c == 0 ? s : total + s;
    }
    return total;
}

// np.add.reduce over a float64 array of length L with the given sparse
// entries: 8192-element chunks, pairwise within, chunk sums added in order.
double numpy_sum_sparse(const std::vector<int64_t>& off, const std::vector<double>& v, int64_t L) {
    constexpr int64_t kChunk = 8192;
    double total = 0;
    size_t i = 0;
    for (int64_t c = 0; c < L; c += kChunk) {
        const int64_t n = std::min(kChunk, L - c);
        size_t j = i;
        while (j < off.size() && off[j] < c + n) ++j;
        const double s = j > i ? pairwise_block(off.data() + i, v.data() + i, j - i, c, n) : 0.0;
        total = c == 0 ? s : total + s;
        i = j;
    }
    return total;
}

struct RegionOut {
    int64_t* counts;   // [8]
    double* sums;      // [4]
};

// pileup.py:101-151 for one region; see the file comment for the outputs.
void one_region(const mc_reads& r, const Tables& tab, int32_t tid, int64_t start, int64_t end,
                RegionOut out, std::vector<uint64_t>& events) {
    const int64_t L = end - start;
    int64_t secondary = 0, improper = 0, nreads = 0, cov_sum = 0, cov2_sum = 0;
    double wnf = 0;
    // cov_cor (pileup.py:141): per position, the reads' 1/rcor added in read
    // order, then np.mean's sum: numpy's add.reduce over 8192-element chunks,
    // pairwise within each.  The reads' covers are kept in read order and the
    // per-position sums are built one 8192-position chunk at a time at the
    // end (memory O(reads + one chunk), not O(region length)); with every
    // 1/rcor == 1 the float sums are exact integers and equal cov's.
    struct Cover {
        int64_t a, b;
        double inv;
    };
    std::vector<Cover> covers;
    bool any_inv = false;
    int64_t status = kOk;
    struct Start {
        int64_t at;
        int64_t order;
        double inv;
    };
    std::vector<Start> starts;
    std::unordered_map<std::string_view, int64_t> mates;
    const int64_t c0 = r.first[tid], c1 = r.first[tid + 1];
    const int64_t lo_pos = start - r.max_span[tid];
    int64_t i = std::lower_bound(r.pos.begin() + c0, r.pos.begin() + c1,
                                 lo_pos < INT32_MIN ? INT32_MIN : lo_pos) - r.pos.begin();
    auto name = [&](int64_t j) {
        return std::string_view(r.arena.data() + r.name_off[j], r.name_len[j]);
    };
    for (; i < c1 && r.pos[i] < end && status == kOk; ++i) {
        if (r.end[i] <= start) continue;
        const uint16_t f = r.flag[i];
        if (f & 0x100) { ++secondary; continue; }
        if (!(f & 0x2)) { ++improper; continue; }
        auto it = mates.find(name(i));
        if (it != mates.end()) {
            const int64_t j = it->second;
            const int64_t s = std::min<int64_t>(r.pos[i], r.pos[j]) - start;
            const int64_t e = std::max<int64_t>(r.pos[i], r.pos[j]) - start;
            cov2_sum += std::max<int64_t>(0, slice_index(e + 1, L) - slice_index(s - 1, L));
            // wnf term (pileup.py:115-125): operands evaluated left to right
            if (tab.none) { status = kNoKcorError; break; }
            if (r.bits[i] & kNoSeq) { status = kNoSeqError; break; }
            double a, b;
            if (!tab.lookup((f & 0x10) ? 1 : 0, r.kmer[i], &a)) {
                wnf += 1;
            } else if (r.bits[j] & kNoSeq) {
                status = kNoSeqError;
                break;
            } else if (!tab.lookup((r.flag[j] & 0x10) ? 1 : 0, r.kmer[j], &b)) {
                wnf += 1;
            } else {
                const double p = a * b;
                wnf += p == 0 ? 1.0 : 1.0 / p;
            }
            mates.erase(it);
        } else {
            mates.emplace(name(i), i);
        }
        if (r.bits[i] & kNoSeq) { status = kNoSeqError; break; }
        const int readno = (f & 0x40) ? 0 : 1;
        double rcor;
        if (!tab.lookup(readno, r.kmer[i], &rcor)) rcor = 1;
        if (rcor == 0) {
            events.push_back(((uint64_t)readno << 32) | r.kmer[i]);
            rcor = 1;
        }
        const double inv = 1.0 / rcor;
        if (r.bits[i] & kNoRefLen) { status = kNoRefLenError; break; }
        const int64_t rl = r.end[i] - r.pos[i];
        int64_t rs, re;
        if (f & 0x10) {
            re = r.pos[i] - start;
            rs = re - rl;
        } else {
            rs = r.pos[i] - start;
            re = rs + rl;
        }
        const int64_t a0 = std::max<int64_t>(0, rs), b0 = std::min(L, re);
        if (b0 > a0) {
            cov_sum += b0 - a0;
            covers.push_back({a0, b0, inv});
            any_inv |= inv != 1.0;
        }
        if (rs >= 0 && rs < L) {
            starts.push_back({rs, i, inv});
            ++nreads;
        }
    }
    // last write per start position
    std::sort(starts.begin(), starts.end(), [](const Start& x, const Start& y) {
        return x.at != y.at ? x.at < y.at : x.order < y.order;
    });
    std::vector<int64_t> off;
    std::vector<double> val;
    off.reserve(starts.size());
    val.reserve(starts.size());
    for (size_t k = 0; k < starts.size(); ++k)
        if (k + 1 == starts.size() || starts[k + 1].at != starts[k].at) {
            off.push_back(starts[k].at);
            val.push_back(starts[k].inv);
        }
    double seq_sum = 0;
    for (double v : val) seq_sum += v;
    out.counts[0] = status;
    out.counts[1] = secondary;
    out.counts[2] = improper;
    out.counts[3] = nreads;
    out.counts[4] = cov_sum;
    out.counts[5] = (int64_t)off.size();
    out.counts[6] = cov2_sum;
    out.counts[7] = (int64_t)events.size();
    out.sums[0] = any_inv ? numpy_sum_covers(covers.data(), covers.size(), L) : (double)cov_sum;
    out.sums[1] = seq_sum;
    out.sums[2] = numpy_sum_sparse(off, val, L);
    out.sums[3] = wnf;
}

}  // namespace

extern "C" int mc_reads_open(const char* path, int n_threads, int k_len, mc_reads** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    MC_REQUIRE(k_len >= 1 && k_len <= 13, MC_E_RANGE, "k-mer length %d outside 1..13", k_len);
    *out = nullptr;
    std::unique_ptr<mc_reads> r(new mc_reads());
    r->k = k_len;
    if (int rc = reads_open(path, n_threads, k_len, r.get())) return rc;
    *out = r.release();
    return MC_OK;
}

namespace {

// mc_reads_open_gpu's table: the reads-mode GPU decode stays open and its
// fields in HBM; the order check and the per contig first record / maximum
// span run on the device (exp_gpu_index).
int reads_keep_gpu(mc_bam_gpu* g, const char* path, int device, int k, mc_reads* r) {
    const mc_bam* h = nullptr;
    if (int rc = mc_bam_gpu_header(g, &h)) return rc;
    int64_t m = 0, nb = 0;
    const int32_t *dt, *dp, *df;
    const int64_t *de, *dno;
    const uint8_t *db, *dnl, *dn;
    const uint32_t* dk;
    if (int rc = mc_bam_gpu_reads_device(g, &m, &dt, &dp, &de, &df, &db, &dk, &dnl, &dno, &dn, &nb)) return rc;
    r->names = h->names;
    r->lens = h->lens;
    r->n_records = h->n_records;
    r->n_unplaced = h->n_records - m;
    r->dev = ExpDevTable{device, k, m, dt, dp, de, df, db, dk, dnl, dno, dn};
    const int32_t n_ref = (int32_t)r->names.size();
    r->first.assign((size_t)n_ref + 1, m);
    r->max_span.assign((size_t)n_ref, 0);
    int64_t bad = -1;
    if (int rc = exp_gpu_index(r->dev, n_ref, r->first.data(), r->max_span.data(), &bad)) return rc;
    MC_REQUIRE(bad < 0, MC_E_INVALID,
               "%s is not coordinate-sorted (placed record %lld); experimental() fetches "
               "regions of a sorted, indexed BAM", path, (long long)bad);
    r->g = g;
    r->host_ready = false;
    (void)nb;
    return MC_OK;
}

// the device table's fields copied back (mc_reads_fields on a GPU table)
int reads_to_host(mc_reads* r) {
    if (r->host_ready) return MC_OK;
    const int64_t m = r->dev.n;
    int64_t nb = 0;
    {
        int64_t m2 = 0;
        const int32_t *dt, *dp, *df;
        const int64_t *de, *dno;
        const uint8_t *db, *dnl, *dn;
        const uint32_t* dk;
        if (int rc = mc_bam_gpu_reads_device(r->g, &m2, &dt, &dp, &de, &df, &db, &dk, &dnl, &dno, &dn, &nb))
            return rc;
    }
    std::vector<int32_t> tid((size_t)m), flag((size_t)m);
    std::vector<int64_t> name_off((size_t)m);
    r->pos.resize((size_t)m);
    r->end.resize((size_t)m);
    r->flag.resize((size_t)m);
    r->bits.resize((size_t)m);
    r->kmer.resize((size_t)m);
    r->name_off.resize((size_t)m);
    r->name_len.resize((size_t)m);
    r->arena.resize((size_t)nb);
    if (int rc = mc_bam_gpu_reads_copy(r->g, tid.data(), r->pos.data(), r->end.data(), flag.data(), r->bits.data(),
                                       r->kmer.data(), r->name_len.data(), name_off.data(),
                                       (uint8_t*)r->arena.data()))
        return rc;
    for (int64_t i = 0; i < m; ++i) {
        r->flag[(size_t)i] = (uint16_t)flag[(size_t)i];
        r->name_off[(size_t)i] = (uint64_t)name_off[(size_t)i];
    }
    r->host_ready = true;
    return MC_OK;
}

}  // namespace

extern "C" int mc_reads_open_gpu_extents(const char* path, int device, int n_threads, int k_len, int32_t n_ref,
                                         const mc_contig_extent* ext, int64_t n_no_coor, int32_t n_sel,
                                         const int32_t* sel, mc_reads** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    MC_REQUIRE(k_len >= 1 && k_len <= 13, MC_E_RANGE, "k-mer length %d outside 1..13", k_len);
    *out = nullptr;
    std::unique_ptr<mc_reads> r(new mc_reads());
    r->k = k_len;
    mc_bam_gpu* g = nullptr;
    if (int rc = mc_bam_gpu_open_reads_extents(path, device, n_threads, k_len, n_ref, ext, n_no_coor, n_sel, sel, &g))
        return rc;
    if (int rc = reads_keep_gpu(g, path, device, k_len, r.get())) {
        if (!r->g) mc_bam_gpu_close(g);
        return rc;
    }
    *out = r.release();
    return MC_OK;
}

extern "C" int mc_reads_open_gpu(const char* path, int device, int n_threads, int k_len, mc_reads** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    MC_REQUIRE(k_len >= 1 && k_len <= 13, MC_E_RANGE, "k-mer length %d outside 1..13", k_len);
    *out = nullptr;
    std::unique_ptr<mc_reads> r(new mc_reads());
    r->k = k_len;
    mc_bam_gpu* g = nullptr;
    int64_t window = 0;   // (tests: MC_READS_GPU_WINDOW forces the windowed decode)
    if (const char* e = std::getenv("MC_READS_GPU_WINDOW")) window = std::strtoll(e, nullptr, 10);
    if (int rc = mc_bam_gpu_open_reads(path, device, n_threads, k_len, window, &g)) return rc;
    if (int rc = reads_keep_gpu(g, path, device, k_len, r.get())) {
        if (!r->g) mc_bam_gpu_close(g);
        return rc;
    }
    *out = r.release();
    return MC_OK;
}

extern "C" int mc_reads_close(mc_reads* r) {
    delete r;
    return MC_OK;
}

extern "C" int mc_reads_header(const mc_reads* r, int32_t* n_ref, int64_t* n_records,
                               int64_t* n_placed) {
    MC_REQUIRE(r, MC_E_INVALID, "null handle");
    if (n_ref) *n_ref = (int32_t)r->names.size();
    if (n_records) *n_records = r->n_records;
    if (n_placed) *n_placed = r->g ? r->dev.n : (int64_t)r->pos.size();
    return MC_OK;
}

extern "C" int mc_reads_fields(const mc_reads* r, const int32_t** pos, const int64_t** end, const uint16_t** flag,
                               const uint8_t** bits, const uint32_t** kmer, const uint64_t** name_off,
                               const uint8_t** name_len, const char** names, int64_t* name_bytes,
                               const int64_t** first, const int64_t** max_span) {
    MC_REQUIRE(r && pos && end && flag && bits && kmer && name_off && name_len && names && name_bytes && first &&
                   max_span,
               MC_E_INVALID, "null argument");
    if (int rc = reads_to_host(const_cast<mc_reads*>(r))) return rc;
    *pos = r->pos.data();
    *end = r->end.data();
    *flag = r->flag.data();
    *bits = r->bits.data();
    *kmer = r->kmer.data();
    *name_off = r->name_off.data();
    *name_len = r->name_len.data();
    *names = r->arena.data();
    *name_bytes = (int64_t)r->arena.size();
    *first = r->first.data();
    *max_span = r->max_span.data();
    return MC_OK;
}

extern "C" int mc_reads_target(const mc_reads* r, int32_t i, const char** name, int64_t* length) {
    MC_REQUIRE(r && i >= 0 && (size_t)i < r->names.size(), MC_E_INVALID, "bad target %d", i);
    if (name) *name = r->names[i].c_str();
    if (length) *length = r->lens[i];
    return MC_OK;
}

extern "C" int mc_experimental_reads(mc_reads* r, int k_len, const double* val1, const uint8_t* has1,
                                     const double* val2, const uint8_t* has2, int64_t R,
                                     const int32_t* tid, const int64_t* start, const int64_t* end,
                                     int n_threads, int64_t* counts, double* sums) {
    MC_REQUIRE(r && tid && start && end && counts && sums, MC_E_INVALID, "null argument");
    MC_REQUIRE(k_len == r->k, MC_E_INVALID, "k-mer length %d differs from the table's %d", k_len,
               r->k);
    const bool none = !val1 || !has1 || !val2 || !has2;
    for (int64_t q = 0; q < R; ++q) {
        MC_REQUIRE(tid[q] >= 0 && (size_t)tid[q] < r->names.size(), MC_E_INVALID,
                   "region %lld: bad contig id %d", (long long)q, tid[q]);
        MC_REQUIRE(end[q] > start[q], MC_E_INVALID, "region %lld: length must be > 0", (long long)q);
    }
    if (r->g && !(std::getenv("MC_EXP_READS") && std::strcmp(std::getenv("MC_EXP_READS"), "host") == 0))
        return exp_gpu_reads(r->dev, r->first.data(), r->max_span.data(), none ? nullptr : val1, none ? nullptr : has1,
                             none ? nullptr : val2, none ? nullptr : has2, R, tid, start, end, counts, sums, r->events,
                             &r->pass_ms, &r->scratch);
    if (int rc = reads_to_host(r)) return rc;   // (MC_EXP_READS=host on a GPU table: the host pass)
    Tables tab{{val1, val2}, {has1, has2}, none};
    r->events.assign((size_t)R, {});
    const int nt = std::max(1, std::min<int>(n_threads_or_all(n_threads), (int)std::max<int64_t>(R, 1)));
    std::atomic<int64_t> next{0};
    std::atomic<int64_t> failed{-1};      // a region whose pass threw (e.g. std::bad_alloc)
    auto worker = [&]() {
        for (;;) {
            const int64_t q = next.fetch_add(1);
            if (q >= R) break;
            try {
                one_region(*r, tab, tid[q], start[q], end[q], {counts + 8 * q, sums + 4 * q},
                           r->events[q]);
            } catch (const std::exception&) {
                int64_t none = -1;
                failed.compare_exchange_strong(none, q);
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    MC_REQUIRE(failed.load() < 0, MC_E_RANGE, "region %lld: the reads pass ran out of host memory",
               (long long)failed.load());
    return MC_OK;
}

extern "C" int mc_experimental_events(const mc_reads* r, int64_t region, int64_t cap,
                                      uint64_t* events, int64_t* n) {
    MC_REQUIRE(r && n && region >= 0 && (size_t)region < r->events.size(), MC_E_INVALID,
               "bad region %lld", (long long)region);
    const auto& ev = r->events[region];
    *n = (int64_t)ev.size();
    if (events) std::copy(ev.begin(), ev.begin() + std::min<int64_t>(cap, *n), events);
    return MC_OK;
}
