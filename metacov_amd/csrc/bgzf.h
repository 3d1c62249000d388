// BGZF / BAM building blocks shared by the decoder (bam_decode.cpp) and the
// index builder / indexed range reader (bam_index.cpp).  Host code only.
#pragma once

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/metacov_amd.h"
#include "common.h"

// The decoded file (mc_bam_open / mc_bam_open_contigs): header, kept
// records as pileup intervals, optionally their CIGARs.
struct mc_bam {
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    int64_t n_records = 0, n_mapped = 0, n_unmapped = 0;
    std::vector<int32_t> tid, pos, span;
    bool keep_cigar = false;
    std::vector<int64_t> cig_off;
    std::vector<uint32_t> cigar;
};

namespace mc {
namespace bgzf {

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
inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

struct MappedFile {
    int fd = -1;
    const uint8_t* data = nullptr;
    size_t size = 0;
    MappedFile() = default;
    MappedFile(const MappedFile&) = delete;
    MappedFile& operator=(const MappedFile&) = delete;
    ~MappedFile() {
        if (data && size) munmap((void*)data, size);
        if (fd >= 0) close(fd);
    }
    // map = false: the descriptor and size only (the GPU decode reads through
    // pread: unmapping a multi-GB mapping whose header pages the scan had
    // faulted in cost ~60 ms at the end of its open)
    int open(const char* path, bool map = true) {
        fd = ::open(path, O_RDONLY);
        MC_REQUIRE(fd >= 0, MC_E_IO, "cannot open %s: %s", path, strerror(errno));
        struct stat st;
        MC_REQUIRE(fstat(fd, &st) == 0, MC_E_IO, "cannot stat %s", path);
        size = (size_t)st.st_size;
        MC_REQUIRE(size > 0, MC_E_IO, "%s is empty", path);
        if (!map) return MC_OK;
        void* m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        MC_REQUIRE(m != MAP_FAILED, MC_E_IO, "mmap %s failed", path);
        data = (const uint8_t*)m;
        (void)madvise(m, size, MADV_SEQUENTIAL);   // read ahead: blocks are visited in order
        return MC_OK;
    }
};

// Block headers from file offset `from` while the block offset is <= `last`
// (SIZE_MAX: to the end of the file).  `out` offsets continue from *total.
inline int scan_blocks(const uint8_t* d, size_t n, size_t from, size_t last,
                       std::vector<Block>& blocks, size_t& total) {
    size_t o = from;
    while (o < n && o <= last) {
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

// libdeflate (the image's libdeflate.so.0, Debian libdeflate0 1.10) inflates a
// BGZF block 2-3x faster than zlib.  It has no header in the image, so its
// stable C entry points are bound with dlopen / dlsym; without the library
// (or with MC_NO_LIBDEFLATE set) zlib does the work.
struct Libdeflate {
    void* (*alloc)() = nullptr;
    int (*decompress)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
    void (*free_d)(void*) = nullptr;
    bool ok = false;
    Libdeflate() {
        if (std::getenv("MC_NO_LIBDEFLATE")) return;
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = reinterpret_cast<void* (*)()>(dlsym(h, "libdeflate_alloc_decompressor"));
        decompress = reinterpret_cast<int (*)(void*, const void*, size_t, void*, size_t, size_t*)>(
            dlsym(h, "libdeflate_deflate_decompress"));
        free_d = reinterpret_cast<void (*)(void*)>(dlsym(h, "libdeflate_free_decompressor"));
        ok = alloc && decompress && free_d;
    }
};

inline const Libdeflate& libdeflate() {
    static const Libdeflate ld;
    return ld;
}

struct LibdeflateState {   // one decompressor per thread
    void* d = nullptr;
    ~LibdeflateState() {
        if (d) libdeflate().free_d(d);
    }
};

inline bool inflate_block(const uint8_t* src, size_t clen, uint8_t* dst, size_t isize) {
    if (isize == 0) return true;
    const Libdeflate& ld = libdeflate();
    if (ld.ok) {
        thread_local LibdeflateState st;
        if (!st.d) st.d = ld.alloc();
        if (st.d) {
            size_t got = 0;
            return ld.decompress(st.d, src, clen, dst, isize, &got) == 0 && got == isize;
        }
    }
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

// Inflate every block into buf + block.out on nt threads (16-block grains).
inline bool inflate_blocks(const uint8_t* file, const std::vector<Block>& blocks, uint8_t* buf,
                           int nt) {
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
                if (!inflate_block(file + b.cdata, b.clen, buf + b.out, b.isize)) failed = true;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < nt; ++i) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    return !failed;
}

inline int n_threads_or_all(int n_threads) {
    return n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
}

// BAM header in the inflated stream d[0, n): magic, text, reference list.
// On success *o is the offset of the first record.
inline int parse_header(const uint8_t* d, size_t n, const char* path,
                        std::vector<std::string>& names, std::vector<int64_t>& lens, size_t* o_out) {
    MC_REQUIRE(n >= 12 && std::memcmp(d, "BAM\1", 4) == 0, MC_E_IO, "%s: missing BAM magic", path);
    size_t o = 4;
    const int32_t l_text = rdi32(d + o);
    MC_REQUIRE(l_text >= 0 && o + 8 + (size_t)l_text <= n, MC_E_IO, "%s: bad header text length", path);
    o += 4 + (size_t)l_text;
    const int32_t n_ref = rdi32(d + o);
    MC_REQUIRE(n_ref >= 0, MC_E_IO, "%s: bad n_ref", path);
    o += 4;
    for (int32_t i = 0; i < n_ref; ++i) {
        MC_REQUIRE(o + 4 <= n, MC_E_IO, "%s: truncated reference list", path);
        const int32_t l_name = rdi32(d + o);
        o += 4;
        MC_REQUIRE(l_name > 0 && o + (size_t)l_name + 4 <= n, MC_E_IO, "%s: bad reference name", path);
        names.emplace_back((const char*)d + o, strnlen((const char*)d + o, (size_t)l_name));
        o += (size_t)l_name;
        lens.push_back(rdi32(d + o));
        o += 4;
    }
    *o_out = o;
    return MC_OK;
}

// CG:B,I tag (SAMv1 §4.2.2) in the aux data [p, end): the real CIGAR of a
// record with more than 65535 ops.
inline int find_cg(const uint8_t* p, const uint8_t* end, const uint8_t** words, uint32_t* count) {
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

// The CIGAR of the record body r[0, rend - r) (after block_size), with the
// CG:B,I placeholder `<l_seq>S<rlen>N` resolved as htslib's bam_read1 does.
inline bool cigar_of(const uint8_t* r, const uint8_t* rend, const uint8_t** cig_out,
                     uint32_t* n_out) {
    const uint8_t l_read_name = r[8];
    uint32_t n_cigar = rd16(r + 12);
    const int32_t l_seq = rdi32(r + 16);
    const uint8_t* cig = r + 32 + l_read_name;
    if (cig + (size_t)n_cigar * 4 > rend) return false;
    if (n_cigar == 2 && rd32(cig) == (((uint32_t)l_seq << 4) | 4u) && (rd32(cig + 4) & 0xF) == 3) {
        const uint8_t* aux = cig + 8 + ((size_t)l_seq + 1) / 2 + (size_t)l_seq;
        const uint8_t* words = nullptr;
        uint32_t cnt = 0;
        if (aux <= rend && find_cg(aux, rend, &words, &cnt) == MC_OK && words) {
            cig = words;
            n_cigar = cnt;
        }
    }
    *cig_out = cig;
    *n_out = n_cigar;
    return true;
}

// bam_cigar2rlen: lengths of the reference-consuming ops (M, D, N, =, X).
inline int64_t cigar_rlen(const uint8_t* cig, uint32_t n_cigar) {
    int64_t rlen = 0;
    for (uint32_t k = 0; k < n_cigar; ++k) {
        const uint32_t cw = rd32(cig + 4 * k);
        if ((0x18Du >> (cw & 0xF)) & 1u) rlen += cw >> 4;
    }
    return rlen;
}

}  // namespace bgzf
}  // namespace mc
