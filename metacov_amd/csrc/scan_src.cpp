// Host read sources of `metacov scan` (reference metacov/cli.py:162-285,
// metacov/scan.pyx:188-340, metacov/pyfq.pyx:60-270): every record of a BAM
// or of one / two FASTQ files, cut into SoA batches for the GPU histogram
// kernel (scan.hip).  Per record the batch holds exactly what the
// reference's ReadIterator hands its ReadProcessors:
//
//   rlen    get_len    BAM l_qseq (scan.pyx:261-262); FASTQ the length of
//                      the sequence line INCLUDING its '\n' (getline,
//                      pyfq.pyx:166-175, get_len :185-187)
//   flag    get_flags  BAM flag (:264-265); FASTQ 0, or PAIRED|READ1 /
//                      PAIRED|READ2 for a pair (pyfq.pyx:213-215)
//   gpos    get_pos    BAM pos, or pos + l_qseq on the reverse strand
//                      (:273-277); FASTQ -1 (:325-326)
//   gisize  get_isize  BAM tlen when PROPER_PAIR (0x2) is set, else 0
//                      (:267-271, is_paired :291-292); FASTQ -1 (:322-323)
//   tid     get_tid    BAM refID (:282-283); FASTQ -1
//   seq     get_seq    the BAM nt16 nibbles as stored (2 per byte, high
//                      nibble first; each read's bytes start on a 4-byte
//                      boundary, zero padded); FASTQ bytes mapped to the same code
//                      (A/C/G/T either case -> 1/2/4/8, anything else -> 15,
//                      which the kernel's nt16 -> nt4 makes 4 exactly like
//                      iupac_to_nt4, pyfq.pyx:26-49).  The kernel undoes the
//                      mapper's reverse complement itself (:240-259).
//
// Record order is the reference's: IteratorRowAll = file order, placed and
// unplaced alike (scan.pyx:204); a FASTQ pair alternates starting with the
// SECOND file (FastQFilePair.cnext flips `cur` to 1 first, pyfq.pyx:264-269)
// and ends when the file whose turn it is runs out; a FASTQ record is read
// as 4 lines and a file ending inside a record ends the stream there
// (FastQFile.cnext, pyfq.pyx:166-175).
#include <zlib.h>

#include <cctype>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <string>
#include <unordered_map>
#include <thread>

#include "bgzf.h"
#include "common.h"

using namespace mc::bgzf;

namespace {

// FASTQ byte -> nt16 code (iupac_to_nt4 then nt4 -> nt16 with N = 15)
struct Ascii16 {
    uint8_t t[256];
    Ascii16() {
        std::memset(t, 15, sizeof t);
        t['A'] = t['a'] = 1;
        t['C'] = t['c'] = 2;
        t['G'] = t['g'] = 4;
        t['T'] = t['t'] = 8;
    }
};
const Ascii16 kAscii16;

// SAM SEQ byte -> nt16 code as htslib's seq_nt16_table stores it in a BAM
// record ("=ACMGRSVTWYHKDBN", either case; anything else N = 15)
struct SamNt16 {
    uint8_t t[256];
    SamNt16() {
        std::memset(t, 15, sizeof t);
        const char* code = "=ACMGRSVTWYHKDBN";
        for (int i = 0; i < 16; ++i) {
            t[(uint8_t)code[i]] = (uint8_t)i;
            t[(uint8_t)std::tolower(code[i])] = (uint8_t)i;
        }
    }
};
const SamNt16 kSamNt16;

// Buffered getline over a zlib stream (gzread reads plain files as-is).
struct LineReader {
    gzFile f = nullptr;
    std::vector<char> buf;
    size_t lo = 0, hi = 0;
    bool eof = false;
    int open(const char* path) {
        f = gzopen(path, "rb");
        MC_REQUIRE(f, MC_E_IO, "cannot open %s", path);
        gzbuffer(f, 1 << 20);
        buf.resize(4 << 20);
        return MC_OK;
    }
    ~LineReader() {
        if (f) gzclose(f);
    }
    // Next line (with its '\n' when present) appended to `out`; false at the
    // end of the file (getline returning -1).
    int getline(std::string& out, bool* got) {
        out.clear();
        for (;;) {
            if (lo == hi) {
                if (eof) {
                    *got = !out.empty();
                    return MC_OK;
                }
                const int n = gzread(f, buf.data(), (unsigned)buf.size());
                if (n < 0) {
                    int ez = 0;
                    const char* m = gzerror(f, &ez);
                    mc::set_error("FASTQ read error: %s", m ? m : "?");
                    return MC_E_IO;
                }
                if (n == 0) eof = true;
                lo = 0;
                hi = (size_t)n;
                continue;
            }
            const char* s = buf.data() + lo;
            const void* nl = std::memchr(s, '\n', hi - lo);
            if (nl) {
                const size_t k = (size_t)((const char*)nl - s) + 1;
                out.append(s, k);
                lo += k;
                *got = true;
                return MC_OK;
            }
            out.append(s, hi - lo);
            lo = hi;
        }
    }
};

}  // namespace

struct mc_scan_src {
    int kind = 0;   // 0 = BAM, 1 = FASTQ, 2 = SAM text
    std::string path;
    int64_t n_records = 0;
    // BAM
    MappedFile mf;
    int nt = 1;
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    std::unordered_map<std::string, int32_t> name_tid;   // SAM: RNAME -> tid (the first @SQ of a name)
    std::string last_rname;                               // SAM: the previous record's RNAME and tid
    int32_t last_tid = -1;
    std::unique_ptr<uint8_t[]> buf;
    size_t cap = 0, n = 0, o = 0, next_off = 0;
    bool have_header = false, last = false, done = false;
    // FASTQ (SAM: fq[0], the pending first record in line[0])
    LineReader fq[2];
    int n_fq = 0, cur = 0;
    std::string line[4];
    bool sam_pending = false;
    int64_t sam_line = 0;
    // the next window, inflated on a background thread while the current
    // one is walked (bam_fill)
    std::unique_ptr<uint8_t[]> nbuf;
    size_t window = 256ull << 20;   // inflated bytes per window (MC_SCAN_WINDOW for tests)
    size_t ncap = 0, ntotal = 0;
    bool nlast = false;
    std::thread prod;
    int prc = 0;
    std::string perr;
    ~mc_scan_src() {
        if (prod.joinable()) prod.join();
    }
    // the batch handed out by mc_scan_src_next
    std::vector<int32_t> rlen, flag, gpos, gisize, tid;
    std::vector<int64_t> seq_off;
    std::vector<uint8_t> seq;
    void clear_batch() {
        rlen.clear();
        flag.clear();
        gpos.clear();
        gisize.clear();
        tid.clear();
        seq_off.assign(1, 0);
        seq.clear();
    }
};

namespace {

constexpr size_t kCarryRoom = 1 << 20;   // room before a window for the previous one's unfinished record

// Inflates the window of BGZF blocks after s->next_off into s->nbuf (after
// kCarryRoom).  Runs on s->prod while the current window is walked.
int bam_produce(mc_scan_src* s) {
    std::vector<Block> blocks;
    size_t total = 0;
    while (s->next_off < s->mf.size && total < s->window) {
        const size_t b0 = blocks.size();
        if (int rc = scan_blocks(s->mf.data, s->mf.size, s->next_off, s->next_off, blocks, total)) {
            s->perr = mc::last_error();
            return rc;
        }
        s->next_off = blocks[b0].cdata + blocks[b0].clen + 8;
    }
    s->nlast = s->next_off >= s->mf.size;
    s->ntotal = total;
    if (kCarryRoom + total + 8 > s->ncap) {
        s->nbuf.reset(new (std::nothrow) uint8_t[kCarryRoom + total + 8]);
        if (!s->nbuf) {
            s->ncap = 0;
            s->perr = "cannot allocate the read window for " + s->path;
            return MC_E_IO;
        }
        s->ncap = kCarryRoom + total + 8;
    }
    if (!blocks.empty() && !inflate_blocks(s->mf.data, blocks, s->nbuf.get() + kCarryRoom, s->nt)) {
        s->perr = "BGZF inflate failed in " + s->path;
        return MC_E_IO;
    }
    return MC_OK;
}

// Moves to the next window: the unparsed tail of the current one goes in
// front of it, and the window after it starts inflating in the background.
int bam_fill(mc_scan_src* s) {
    if (s->prod.joinable()) {
        s->prod.join();
    } else {
        s->prc = bam_produce(s);
    }
    MC_REQUIRE(s->prc == MC_OK, s->prc, "%s", s->perr.c_str());
    const size_t carry = s->n - s->o;
    if (carry <= kCarryRoom) {
        if (carry) std::memcpy(s->nbuf.get() + kCarryRoom - carry, s->buf.get() + s->o, carry);
        std::swap(s->buf, s->nbuf);
        std::swap(s->cap, s->ncap);
        s->o = kCarryRoom - carry;
        s->n = kCarryRoom + s->ntotal;
    } else {   // (a carry longer than the room: one buffer with both)
        const size_t need = carry + s->ntotal + 8;
        std::unique_ptr<uint8_t[]> nb(new (std::nothrow) uint8_t[need]);
        MC_REQUIRE(nb, MC_E_IO, "cannot allocate %zu bytes for %s", need, s->path.c_str());
        std::memcpy(nb.get(), s->buf.get() + s->o, carry);
        std::memcpy(nb.get() + carry, s->nbuf.get() + kCarryRoom, s->ntotal);
        s->buf = std::move(nb);
        s->cap = need;
        s->o = 0;
        s->n = carry + s->ntotal;
    }
    s->last = s->nlast;
    if (!s->last) s->prod = std::thread([s] { s->prc = bam_produce(s); });
    if (!s->have_header) {
        size_t o = 0;
        if (parse_header(s->buf.get() + s->o, s->n - s->o, s->path.c_str(), s->names, s->lens, &o) == MC_OK) {
            s->have_header = true;
            s->o += o;
        } else {
            MC_REQUIRE(!s->last, MC_E_IO, "%s: no valid BAM header", s->path.c_str());
        }
    }
    return MC_OK;
}

int bam_next(mc_scan_src* s, int64_t max_reads, int64_t max_bytes) {
    const int32_t n_ref = (int32_t)s->names.size();
    while ((int64_t)s->rlen.size() < max_reads && (int64_t)s->seq.size() < max_bytes) {
        const uint8_t* d = s->buf.get();
        if (!s->have_header || s->o + 4 > s->n || s->o + 4 + (size_t)rdi32(d + s->o) > s->n) {
            if (s->last) {
                MC_REQUIRE(s->have_header && s->o == s->n, MC_E_IO,
                           "%s: truncated record at the end of the file", s->path.c_str());
                s->done = true;
                return MC_OK;
            }
            if (int rc = bam_fill(s)) return rc;
            continue;
        }
        const int32_t bs = rdi32(d + s->o);
        MC_REQUIRE(bs >= 32, MC_E_IO, "%s: bad record size at byte %zu of the inflated stream",
                   s->path.c_str(), s->o);
        const uint8_t* r = d + s->o + 4;
        const int32_t tid = rdi32(r), pos = rdi32(r + 4);
        const uint32_t l_name = r[8], n_cigar = rd16(r + 12), flag = rd16(r + 14);
        const int32_t l_seq = rdi32(r + 16), tlen = rdi32(r + 28);
        const uint64_t seq_at = 32ull + l_name + 4ull * n_cigar;
        const uint64_t nbytes = ((uint64_t)std::max(l_seq, 0) + 1) / 2;
        MC_REQUIRE(l_seq >= 0 && seq_at + nbytes <= (uint64_t)bs && tid >= -1 && tid < n_ref,
                   MC_E_IO, "%s: malformed record at byte %zu of the inflated stream",
                   s->path.c_str(), s->o);
        s->rlen.push_back(l_seq);
        s->flag.push_back((int32_t)flag);
        s->gpos.push_back((flag & 0x10) ? pos + l_seq : pos);
        s->gisize.push_back((flag & 0x2) ? tlen : 0);
        s->tid.push_back(tid);
        s->seq.insert(s->seq.end(), r + seq_at, r + seq_at + nbytes);
        s->seq.resize((s->seq.size() + 3) & ~size_t(3), 0);   // 4-byte aligned starts
        s->seq_off.push_back((int64_t)s->seq.size());
        s->o += 4 + (size_t)bs;
        ++s->n_records;
    }
    return MC_OK;
}

// One FASTQ record of file f appended to the batch; *got false at the end.
int fq_record(mc_scan_src* s, int f, int32_t flag, bool* got) {
    *got = false;
    for (int i = 0; i < 4; ++i) {
        bool ok = false;
        if (int rc = s->fq[f].getline(s->line[i], &ok)) return rc;
        if (!ok) return MC_OK;
    }
    const std::string& q = s->line[1];
    const size_t L = q.size();
    MC_REQUIRE(L <= (size_t)INT32_MAX, MC_E_RANGE, "FASTQ sequence line too long");
    const size_t at = s->seq.size();
    s->seq.resize(at + (((L + 1) / 2 + 3) & ~size_t(3)), 0);   // 4-byte aligned starts
    uint8_t* o = s->seq.data() + at;
    const uint8_t* c = reinterpret_cast<const uint8_t*>(q.data());
    for (size_t i = 0; i + 1 < L; i += 2) o[i >> 1] = (uint8_t)(kAscii16.t[c[i]] << 4 | kAscii16.t[c[i + 1]]);
    if (L & 1) o[L >> 1] = (uint8_t)(kAscii16.t[c[L - 1]] << 4);
    s->rlen.push_back((int32_t)L);
    s->flag.push_back(flag);
    s->gpos.push_back(-1);
    s->gisize.push_back(-1);
    s->tid.push_back(-1);
    s->seq_off.push_back((int64_t)s->seq.size());
    ++s->n_records;
    *got = true;
    return MC_OK;
}

int fq_next(mc_scan_src* s, int64_t max_reads, int64_t max_bytes) {
    while (!s->done && (int64_t)s->rlen.size() < max_reads && (int64_t)s->seq.size() < max_bytes) {
        bool got = false;
        if (s->n_fq == 1) {
            if (int rc = fq_record(s, 0, 0, &got)) return rc;
        } else {
            s->cur ^= 1;   // the second file's read comes first
            if (int rc = fq_record(s, s->cur ? 1 : 0, s->cur ? 0x81 : 0x41, &got)) return rc;
        }
        if (!got) s->done = true;
    }
    return MC_OK;
}

// SAM text (plain, gzip or BGZF): the record fields scan reads, as htslib's
// sam_parse1 stores them in a bam1_t (pysam AlignmentFile over a .sam, what
// the reference opens for `scan x.sam`: metacov/cli.py:171-173,
// scan.pyx:188-216): FLAG, RNAME -> tid (the @SQ order; "*" = -1), POS - 1,
// TLEN, SEQ as nt16 ("*" = no bases).
int sam_fields(mc_scan_src* s, const std::string& ln, const char* f[11], size_t fl[11]) {
    size_t a = 0;
    int k = 0;
    for (; k < 11; ++k) {
        const size_t b = ln.find('\t', a);
        const size_t e = b == std::string::npos ? ln.size() : b;
        f[k] = ln.data() + a;
        fl[k] = e - a;
        if (b == std::string::npos) {
            ++k;
            break;
        }
        a = b + 1;
    }
    MC_REQUIRE(k >= 11, MC_E_IO, "%s: line %lld: a SAM record needs 11 fields, found %d", s->path.c_str(),
               (long long)s->sam_line, k);
    return MC_OK;
}

int sam_int(mc_scan_src* s, const char* p, size_t n, int base, int64_t* out) {
    std::string t(p, n);
    char* end = nullptr;
    errno = 0;
    const long long v = std::strtoll(t.c_str(), &end, base);
    MC_REQUIRE(n && end == t.c_str() + n && errno == 0, MC_E_IO, "%s: line %lld: bad number '%s'",
               s->path.c_str(), (long long)s->sam_line, t.c_str());
    *out = v;
    return MC_OK;
}

// Next non-empty line without its line end into line[0]; *got false at the end.
int sam_getline(mc_scan_src* s, bool* got) {
    for (;;) {
        if (int rc = s->fq[0].getline(s->line[0], got)) return rc;
        if (!*got) return MC_OK;
        ++s->sam_line;
        std::string& l = s->line[0];
        while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
        if (!l.empty()) return MC_OK;
    }
}

int sam_header(mc_scan_src* s) {
    for (;;) {
        bool got = false;
        if (int rc = sam_getline(s, &got)) return rc;
        if (!got) return MC_OK;
        const std::string& l = s->line[0];
        if (l[0] != '@') {
            s->sam_pending = true;
            return MC_OK;
        }
        if (l.compare(0, 4, "@SQ\t") != 0) continue;
        std::string name;
        int64_t len = -1;
        for (size_t a = 4; a < l.size();) {
            size_t b = l.find('\t', a);
            if (b == std::string::npos) b = l.size();
            const std::string tag = l.substr(a, b - a);
            if (tag.compare(0, 3, "SN:") == 0) name = tag.substr(3);
            if (tag.compare(0, 3, "LN:") == 0 && sam_int(s, tag.data() + 3, tag.size() - 3, 10, &len)) return MC_E_IO;
            a = b + 1;
        }
        MC_REQUIRE(!name.empty() && len >= 0, MC_E_IO, "%s: line %lld: @SQ needs SN and LN", s->path.c_str(),
                   (long long)s->sam_line);
        s->name_tid.emplace(name, (int32_t)s->names.size());
        s->names.push_back(name);
        s->lens.push_back(len);
    }
}

int sam_next(mc_scan_src* s, int64_t max_reads, int64_t max_bytes) {
    const char* f[11];
    size_t fl[11];
    while ((int64_t)s->rlen.size() < max_reads && (int64_t)s->seq.size() < max_bytes) {
        if (!s->sam_pending) {
            bool got = false;
            if (int rc = sam_getline(s, &got)) return rc;
            if (!got) {
                s->done = true;
                return MC_OK;
            }
        }
        s->sam_pending = false;
        const std::string& ln = s->line[0];
        MC_REQUIRE(ln[0] != '@', MC_E_IO, "%s: line %lld: header line after the records", s->path.c_str(),
                   (long long)s->sam_line);
        if (int rc = sam_fields(s, ln, f, fl)) return rc;
        int64_t flag = 0, pos = 0, tlen = 0;
        if (int rc = sam_int(s, f[1], fl[1], 0, &flag)) return rc;
        if (int rc = sam_int(s, f[3], fl[3], 10, &pos)) return rc;
        if (int rc = sam_int(s, f[8], fl[8], 10, &tlen)) return rc;
        MC_REQUIRE(flag >= 0 && flag <= 0xffff && pos >= 0 && pos <= (int64_t)INT32_MAX + 1 &&
                       tlen >= INT32_MIN && tlen <= INT32_MAX,
                   MC_E_IO, "%s: line %lld: FLAG, POS or TLEN out of range", s->path.c_str(), (long long)s->sam_line);
        int32_t tid = -1;
        if (!(fl[2] == 1 && f[2][0] == '*')) {
            if (s->last_tid >= 0 && s->last_rname.size() == fl[2] &&
                std::memcmp(s->last_rname.data(), f[2], fl[2]) == 0) {
                tid = s->last_tid;   // sorted SAM: runs of one RNAME
            } else {
                const std::string rn(f[2], fl[2]);
                auto it = s->name_tid.find(rn);
                MC_REQUIRE(it != s->name_tid.end(), MC_E_IO, "%s: line %lld: reference '%s' is not in the header",
                           s->path.c_str(), (long long)s->sam_line, rn.c_str());
                tid = it->second;
                s->last_rname = rn;
                s->last_tid = tid;
            }
        }
        const bool no_seq = fl[9] == 1 && f[9][0] == '*';
        const size_t L = no_seq ? 0 : fl[9];
        MC_REQUIRE(L <= (size_t)INT32_MAX, MC_E_RANGE, "SAM sequence too long");
        const int32_t l_seq = (int32_t)L, p0 = (int32_t)(pos - 1);
        s->rlen.push_back(l_seq);
        s->flag.push_back((int32_t)flag);
        s->gpos.push_back((flag & 0x10) ? p0 + l_seq : p0);
        s->gisize.push_back((flag & 0x2) ? (int32_t)tlen : 0);
        s->tid.push_back(tid);
        const size_t at = s->seq.size();
        s->seq.resize(at + (((L + 1) / 2 + 3) & ~size_t(3)), 0);   // 4-byte aligned starts
        uint8_t* o = s->seq.data() + at;
        const uint8_t* c = reinterpret_cast<const uint8_t*>(f[9]);
        for (size_t i = 0; i + 1 < L; i += 2) o[i >> 1] = (uint8_t)(kSamNt16.t[c[i]] << 4 | kSamNt16.t[c[i + 1]]);
        if (L & 1) o[L >> 1] = (uint8_t)(kSamNt16.t[c[L - 1]] << 4);
        s->seq_off.push_back((int64_t)s->seq.size());
        ++s->n_records;
    }
    return MC_OK;
}

}  // namespace

extern "C" int mc_scan_src_open_sam(const char* path, mc_scan_src** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<mc_scan_src> s(new mc_scan_src());
    s->kind = 2;
    s->path = path;
    if (int rc = s->fq[0].open(path)) return rc;
    if (int rc = sam_header(s.get())) return rc;
    s->clear_batch();
    *out = s.release();
    return MC_OK;
}

extern "C" int mc_scan_src_open_bam(const char* path, int n_threads, mc_scan_src** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<mc_scan_src> s(new mc_scan_src());
    s->kind = 0;
    s->path = path;
    s->nt = n_threads_or_all(n_threads);
    if (const char* e = std::getenv("MC_SCAN_WINDOW")) s->window = std::max<size_t>(1, std::strtoull(e, nullptr, 10));
    if (int rc = s->mf.open(path)) return rc;
    while (!s->have_header) {
        if (int rc = bam_fill(s.get())) return rc;
    }
    s->clear_batch();
    *out = s.release();
    return MC_OK;
}

extern "C" int mc_scan_src_open_fastq(const char* path1, const char* path2, mc_scan_src** out) {
    MC_REQUIRE(path1 && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<mc_scan_src> s(new mc_scan_src());
    s->kind = 1;
    s->path = path1;
    s->n_fq = path2 ? 2 : 1;
    if (int rc = s->fq[0].open(path1)) return rc;
    if (path2) {
        if (int rc = s->fq[1].open(path2)) return rc;
    }
    s->clear_batch();
    *out = s.release();
    return MC_OK;
}

extern "C" int mc_scan_src_close(mc_scan_src* s) {
    delete s;
    return MC_OK;
}

extern "C" int mc_scan_src_n_targets(const mc_scan_src* s, int32_t* n) {
    MC_REQUIRE(s && n, MC_E_INVALID, "null argument");
    *n = (int32_t)s->names.size();
    return MC_OK;
}

extern "C" int mc_scan_src_target(const mc_scan_src* s, int32_t i, const char** name,
                                  int64_t* length) {
    MC_REQUIRE(s && i >= 0 && (size_t)i < s->names.size(), MC_E_INVALID, "bad target %d", i);
    if (name) *name = s->names[i].c_str();
    if (length) *length = s->lens[i];
    return MC_OK;
}

extern "C" int mc_scan_src_next(mc_scan_src* s, int64_t max_reads, int64_t max_seq_bytes,
                                int64_t* n_out) {
    MC_REQUIRE(s && n_out && max_reads > 0 && max_seq_bytes > 0, MC_E_INVALID, "bad argument");
    s->clear_batch();
    if (!s->done) {
        if (int rc = s->kind == 0   ? bam_next(s, max_reads, max_seq_bytes)
                     : s->kind == 2 ? sam_next(s, max_reads, max_seq_bytes)
                                    : fq_next(s, max_reads, max_seq_bytes))
            return rc;
    }
    *n_out = (int64_t)s->rlen.size();
    return MC_OK;
}

extern "C" int mc_scan_src_batch(const mc_scan_src* s, const int32_t** rlen, const int32_t** flag,
                                 const int32_t** gpos, const int32_t** gisize,
                                 const int32_t** tid, const int64_t** seq_off,
                                 const uint8_t** seq, int64_t* seq_bytes) {
    MC_REQUIRE(s, MC_E_INVALID, "null handle");
    if (rlen) *rlen = s->rlen.data();
    if (flag) *flag = s->flag.data();
    if (gpos) *gpos = s->gpos.data();
    if (gisize) *gisize = s->gisize.data();
    if (tid) *tid = s->tid.data();
    if (seq_off) *seq_off = s->seq_off.data();
    if (seq) *seq = s->seq.data();
    if (seq_bytes) *seq_bytes = (int64_t)s->seq.size();
    return MC_OK;
}

extern "C" int mc_scan_src_records(const mc_scan_src* s, int64_t* n_records) {
    MC_REQUIRE(s && n_records, MC_E_INVALID, "null argument");
    *n_records = s->n_records;
    return MC_OK;
}
