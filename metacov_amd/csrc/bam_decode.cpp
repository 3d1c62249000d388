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
//   span = bam_cigar2rlen (ops M/D/N/=/X, op-type mask 0x18D), or 1 when the
//          read has no reference-consuming op (bam_endpos: pos + 1)
// Records with more than 65535 CIGAR ops carry the real CIGAR in a CG:B,I
// tag behind a `<l_seq>S<rlen>N` placeholder (SAMv1 §4.2.2), as htslib's
// bam_read1 resolves it.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/metacov_amd.h"
#include "common.h"

struct mc_bam {
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    int64_t n_records = 0, n_mapped = 0, n_unmapped = 0;
    std::vector<int32_t> tid, pos, span;
    bool keep_cigar = false;
    std::vector<int64_t> cig_off;
    std::vector<uint32_t> cigar;
};

namespace {

struct Block {
    size_t off;       // compressed block offset in the file
    size_t cdata;     // offset of the deflate payload
    size_t clen;      // deflate payload length
    size_t isize;     // inflated size
    size_t out;       // offset in the inflated stream
};

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline int32_t rdi32(const uint8_t* p) { return (int32_t)rd32(p); }

struct MappedFile {
    int fd = -1;
    const uint8_t* data = nullptr;
    size_t size = 0;
    ~MappedFile() {
        if (data && size) munmap((void*)data, size);
        if (fd >= 0) close(fd);
    }
};

int scan_blocks(const uint8_t* d, size_t n, std::vector<Block>& blocks, size_t& total) {
    size_t o = 0;
    total = 0;
    while (o < n) {
        MC_REQUIRE(o + 18 <= n, MC_E_IO, "truncated BGZF header at offset %zu", o);
        MC_REQUIRE(d[o] == 31 && d[o + 1] == 139 && d[o + 2] == 8 && (d[o + 3] & 4), MC_E_IO,
                   "not a BGZF block at offset %zu (is the file bgzip-compressed BAM?)", o);
        const uint16_t xlen = rd16(d + o + 10);
        size_t bsize = 0;
        for (size_t x = o + 12; x + 4 <= o + 12 + xlen;) {
            const uint16_t slen = rd16(d + x + 2);
            if (d[x] == 66 && d[x + 1] == 67 && slen == 2) bsize = (size_t)rd16(d + x + 4) + 1;
            x += 4 + slen;
        }
        MC_REQUIRE(bsize >= (size_t)xlen + 20 && o + bsize <= n, MC_E_IO,
                   "bad BGZF block size at offset %zu", o);
        Block b;
        b.off = o;
        b.cdata = o + 12 + xlen;
        b.clen = bsize - xlen - 20;
        b.isize = rd32(d + o + bsize - 4);
        b.out = total;
        total += b.isize;
        blocks.push_back(b);
        o += bsize;
    }
    return MC_OK;
}

bool inflate_block(const uint8_t* src, size_t clen, uint8_t* dst, size_t isize) {
    if (isize == 0) return true;
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return false;
    zs.next_in = const_cast<Bytef*>(src);
    zs.avail_in = (uInt)clen;
    zs.next_out = dst;
    zs.avail_out = (uInt)isize;
    const int rc = inflate(&zs, Z_FINISH);
    const bool ok = rc == Z_STREAM_END && zs.total_out == isize;
    inflateEnd(&zs);
    return ok;
}

int find_cg(const uint8_t* p, const uint8_t* end, const uint8_t** words, uint32_t* count) {
    while (p + 3 <= end) {
        const char t0 = (char)p[0], t1 = (char)p[1], ty = (char)p[2];
        p += 3;
        switch (ty) {
            case 'A': case 'c': case 'C': p += 1; break;
            case 's': case 'S': p += 2; break;
            case 'i': case 'I': case 'f': p += 4; break;
            case 'Z': case 'H':
                while (p < end && *p) ++p;
                ++p;
                break;
            case 'B': {
                if (p + 5 > end) return MC_E_IO;
                const char sub = (char)p[0];
                const uint32_t cnt = rd32(p + 1);
                p += 5;
                size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
                if (t0 == 'C' && t1 == 'G' && sub == 'I') {
                    if (p + (size_t)cnt * 4 > end) return MC_E_IO;
                    *words = p;
                    *count = cnt;
                    return MC_OK;
                }
                p += es * cnt;
                break;
            }
            default:
                return MC_E_IO;
        }
    }
    return MC_OK;
}

}  // namespace

extern "C" int mc_bam_open(const char* path, int n_threads, uint32_t flag_filter, int keep_cigar,
                           mc_bam** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    MappedFile mf;
    mf.fd = open(path, O_RDONLY);
    MC_REQUIRE(mf.fd >= 0, MC_E_IO, "cannot open %s: %s", path, strerror(errno));
    struct stat st;
    MC_REQUIRE(fstat(mf.fd, &st) == 0, MC_E_IO, "cannot stat %s", path);
    mf.size = (size_t)st.st_size;
    MC_REQUIRE(mf.size > 0, MC_E_IO, "%s is empty", path);
    void* m = mmap(nullptr, mf.size, PROT_READ, MAP_PRIVATE, mf.fd, 0);
    MC_REQUIRE(m != MAP_FAILED, MC_E_IO, "mmap %s failed", path);
    mf.data = (const uint8_t*)m;

    std::vector<Block> blocks;
    size_t total = 0;
    if (int rc = scan_blocks(mf.data, mf.size, blocks, total)) return rc;
    std::vector<uint8_t> buf(total + 8);
    int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = std::max(1, std::min<int>(nt, (int)blocks.size()));
    std::atomic<size_t> next{0};
    std::atomic<bool> failed{false};
    auto worker = [&]() {
        for (;;) {
            const size_t k = next.fetch_add(16);
            if (k >= blocks.size()) break;
            const size_t ke = std::min(blocks.size(), k + 16);
            for (size_t j = k; j < ke; ++j) {
                const Block& b = blocks[j];
                if (!inflate_block(mf.data + b.cdata, b.clen, buf.data() + b.out, b.isize))
                    failed = true;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < nt; ++i) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    MC_REQUIRE(!failed, MC_E_IO, "BGZF inflate failed in %s", path);

    const uint8_t* d = buf.data();
    const size_t n = total;
    MC_REQUIRE(n >= 12 && std::memcmp(d, "BAM\1", 4) == 0, MC_E_IO, "%s: missing BAM magic", path);
    size_t o = 4;
    const int32_t l_text = rdi32(d + o);
    MC_REQUIRE(l_text >= 0 && o + 8 + (size_t)l_text <= n, MC_E_IO, "bad header text length");
    o += 4 + (size_t)l_text;
    const int32_t n_ref = rdi32(d + o);
    MC_REQUIRE(n_ref >= 0, MC_E_IO, "bad n_ref");
    o += 4;
    mc_bam* bam = new mc_bam();
    bam->keep_cigar = keep_cigar != 0;
    auto fail = [&](const char* msg, size_t at) {
        delete bam;
        mc::set_error("%s: %s at byte %zu of the inflated stream", path, msg, at);
        return MC_E_IO;
    };
    for (int32_t i = 0; i < n_ref; ++i) {
        if (o + 4 > n) return fail("truncated reference list", o);
        const int32_t l_name = rdi32(d + o);
        o += 4;
        if (l_name <= 0 || o + (size_t)l_name + 4 > n) return fail("bad reference name", o);
        bam->names.emplace_back((const char*)d + o, strnlen((const char*)d + o, (size_t)l_name));
        o += (size_t)l_name;
        bam->lens.push_back(rdi32(d + o));
        o += 4;
    }
    if (bam->keep_cigar) bam->cig_off.push_back(0);
    while (o < n) {
        if (o + 4 > n) return fail("truncated record", o);
        const int32_t block_size = rdi32(d + o);
        if (block_size < 32 || o + 4 + (size_t)block_size > n) return fail("bad record size", o);
        const uint8_t* r = d + o + 4;
        const uint8_t* rend = r + block_size;
        const int32_t tid = rdi32(r);
        const int32_t pos = rdi32(r + 4);
        const uint8_t l_read_name = r[8];
        uint32_t n_cigar = rd16(r + 12);
        const uint16_t flag = rd16(r + 14);
        const int32_t l_seq = rdi32(r + 16);
        ++bam->n_records;
        if (tid >= 0 && !(flag & 4)) ++bam->n_mapped;
        else ++bam->n_unmapped;
        o += 4 + (size_t)block_size;
        if (tid < 0 || (flag & flag_filter)) continue;
        if (tid >= n_ref) return fail("record tid beyond the reference list", o);
        const uint8_t* cig = r + 32 + l_read_name;
        if (cig + (size_t)n_cigar * 4 > rend) return fail("CIGAR overruns record", o);
        if (n_cigar == 2 && rd32(cig) == (((uint32_t)l_seq << 4) | 4u) && (rd32(cig + 4) & 0xF) == 3) {
            const uint8_t* aux = cig + 8 + ((size_t)l_seq + 1) / 2 + (size_t)l_seq;
            const uint8_t* words = nullptr;
            uint32_t cnt = 0;
            if (aux <= rend && find_cg(aux, rend, &words, &cnt) == MC_OK && words) {
                cig = words;
                n_cigar = cnt;
            }
        }
        int64_t rlen = 0;
        for (uint32_t k = 0; k < n_cigar; ++k) {
            const uint32_t c = rd32(cig + 4 * k);
            if ((0x18Du >> (c & 0xF)) & 1u) rlen += c >> 4;
        }
        if (rlen <= 0) rlen = 1;
        if (rlen > INT32_MAX) return fail("reference span exceeds int32", o);
        bam->tid.push_back(tid);
        bam->pos.push_back(pos);
        bam->span.push_back((int32_t)rlen);
        if (bam->keep_cigar) {
            for (uint32_t k = 0; k < n_cigar; ++k) bam->cigar.push_back(rd32(cig + 4 * k));
            bam->cig_off.push_back((int64_t)bam->cigar.size());
        }
    }
    *out = bam;
    return MC_OK;
}

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
