// BAM writer for synthetic workloads (the role `metacov simulate` plays in
// the reference, metacov/cli.py:288-414, without ART): records from SoA
// arrays, BGZF blocks deflated in parallel (each block is independent).
// Bases and qualities are pseudo-random per record (uniform ACGT, Phred 2-40)
// so the files compress like real BAMs (~3x), names are "r<index>".  Blocks
// are deflated with libdeflate when the image has it (dlopen), else zlib.
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/metacov_amd.h"
#include "common.h"

namespace {

inline void put32(std::vector<uint8_t>& b, uint32_t v) {
    b.push_back(v & 0xff);
    b.push_back((v >> 8) & 0xff);
    b.push_back((v >> 16) & 0xff);
    b.push_back((v >> 24) & 0xff);
}
inline void put16(std::vector<uint8_t>& b, uint16_t v) {
    b.push_back(v & 0xff);
    b.push_back((v >> 8) & 0xff);
}

int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

struct LibdeflateC {
    void* (*alloc)(int) = nullptr;
    size_t (*compress)(void*, const void*, size_t, void*, size_t) = nullptr;
    void (*free_c)(void*) = nullptr;
    bool ok = false;
    LibdeflateC() {
        if (std::getenv("MC_NO_LIBDEFLATE")) return;
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = reinterpret_cast<void* (*)(int)>(dlsym(h, "libdeflate_alloc_compressor"));
        compress = reinterpret_cast<size_t (*)(void*, const void*, size_t, void*, size_t)>(
            dlsym(h, "libdeflate_deflate_compress"));
        free_c = reinterpret_cast<void (*)(void*)>(dlsym(h, "libdeflate_free_compressor"));
        ok = alloc && compress && free_c;
    }
};

const LibdeflateC& libdeflate_c() {
    static const LibdeflateC ld;
    return ld;
}

// raw deflate of src[0, n) into dst (capacity cap); returns the size, 0 on failure
size_t deflate_raw(const uint8_t* src, size_t n, int level, uint8_t* dst, size_t cap) {
    const LibdeflateC& ld = libdeflate_c();
    if (ld.ok) {
        struct State {
            void* c = nullptr;
            int level = -1;
            ~State() {
                if (c) libdeflate_c().free_c(c);
            }
        };
        thread_local State st;
        if (st.level != level) {
            if (st.c) ld.free_c(st.c);
            st.c = ld.alloc(level);
            st.level = level;
        }
        if (st.c) return ld.compress(st.c, src, n, dst, cap);
    }
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return 0;
    zs.next_in = const_cast<Bytef*>(src);
    zs.avail_in = (uInt)n;
    zs.next_out = dst;
    zs.avail_out = (uInt)cap;
    const int rc = deflate(&zs, Z_FINISH);
    const size_t clen = zs.total_out;
    deflateEnd(&zs);
    return rc == Z_STREAM_END ? clen : 0;
}

// one BGZF block (header + raw deflate + crc + isize) for <= 65280 bytes
bool bgzf_block(const uint8_t* src, size_t n, int level, std::vector<uint8_t>& out) {
    out.resize(18 + compressBound((uLong)n) + 8 + 64);
    const size_t clen = deflate_raw(src, n, level, out.data() + 18, out.size() - 26);
    if (clen == 0 && n > 0) return false;
    const size_t bsize = clen + 26;
    const uint8_t hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0,
                             (uint8_t)((bsize - 1) & 0xff), (uint8_t)((bsize - 1) >> 8)};
    std::memcpy(out.data(), hdr, 18);
    const uint32_t crc = (uint32_t)crc32(0L, src, (uInt)n);
    uint8_t* t = out.data() + 18 + clen;
    for (int i = 0; i < 4; ++i) t[i] = (crc >> (8 * i)) & 0xff;
    for (int i = 0; i < 4; ++i) t[4 + i] = ((uint32_t)n >> (8 * i)) & 0xff;
    out.resize(bsize);
    return true;
}

}  // namespace

extern "C" int mc_bam_write(const char* path, int32_t n_ref, const char* const* names,
                            const int64_t* lengths, int64_t n, const int32_t* tid,
                            const int32_t* pos, const uint16_t* flag, const int64_t* cig_off,
                            const uint32_t* cigar, int32_t l_seq, int level, int n_threads) {
    MC_REQUIRE(path && (n_ref == 0 || (names && lengths)), MC_E_INVALID, "null argument");
    MC_REQUIRE(n == 0 || (tid && pos && flag && cig_off), MC_E_INVALID, "null record array");
    MC_REQUIRE(l_seq >= 0 && l_seq < (1 << 20), MC_E_INVALID, "bad l_seq");
    // ---- serialise header + records (uncompressed stream)
    std::vector<uint8_t> raw;
    std::string text = "@HD\tVN:1.6\tSO:coordinate\n";
    for (int32_t i = 0; i < n_ref; ++i)
        text += std::string("@SQ\tSN:") + names[i] + "\tLN:" + std::to_string(lengths[i]) + "\n";
    raw.insert(raw.end(), {'B', 'A', 'M', 1});
    put32(raw, (uint32_t)text.size());
    raw.insert(raw.end(), text.begin(), text.end());
    put32(raw, (uint32_t)n_ref);
    for (int32_t i = 0; i < n_ref; ++i) {
        const size_t ln = std::strlen(names[i]) + 1;
        put32(raw, (uint32_t)ln);
        raw.insert(raw.end(), names[i], names[i] + ln);
        put32(raw, (uint32_t)lengths[i]);
    }
    const size_t seq_bytes = ((size_t)l_seq + 1) / 2;
    char name[32];
    for (int64_t i = 0; i < n; ++i) {
        const int64_t c0 = cig_off[i], c1 = cig_off[i + 1];
        MC_REQUIRE(c1 >= c0 && c1 - c0 < 65536, MC_E_INVALID, "record %lld: bad CIGAR range",
                   (long long)i);
        const int ln = std::snprintf(name, sizeof name, "r%lld", (long long)i) + 1;
        int64_t rlen = 0;
        for (int64_t k = c0; k < c1; ++k)
            if ((0x18Du >> (cigar[k] & 0xF)) & 1u) rlen += cigar[k] >> 4;
        const int64_t end = pos[i] + std::max<int64_t>(rlen, 1);
        const uint32_t bin = tid[i] >= 0 ? (uint32_t)reg2bin(std::max(pos[i], 0), std::max<int64_t>(end, 1))
                                         : 4680u;
        const uint32_t block = 32 + ln + 4 * (uint32_t)(c1 - c0) + (uint32_t)seq_bytes + (uint32_t)l_seq;
        put32(raw, block);
        put32(raw, (uint32_t)tid[i]);
        put32(raw, (uint32_t)pos[i]);
        raw.push_back((uint8_t)ln);
        raw.push_back(60);
        put16(raw, (uint16_t)bin);
        put16(raw, (uint16_t)(c1 - c0));
        put16(raw, flag[i]);
        put32(raw, (uint32_t)l_seq);
        put32(raw, (uint32_t)tid[i]);
        put32(raw, (uint32_t)pos[i]);
        put32(raw, 0);
        raw.insert(raw.end(), name, name + ln);
        for (int64_t k = c0; k < c1; ++k) put32(raw, cigar[k]);
        uint64_t h = (uint64_t)i + 0x632BE59BD9B4E019ull;   // per-record stream start:
        h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;          // hashed, so records do not
        h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;          // share shifted streams
        h ^= h >> 31;
        auto rnd = [&h]() {       // splitmix64 step
            uint64_t z = (h += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            return z ^ (z >> 31);
        };
        static const uint8_t kNt16[4] = {1, 2, 4, 8};      // A C G T
        uint64_t bits = 0;
        for (size_t k = 0; k < seq_bytes; ++k) {
            if ((k & 15) == 0) bits = rnd();
            const uint8_t b = (uint8_t)((kNt16[bits & 3] << 4) | kNt16[(bits >> 2) & 3]);
            bits >>= 4;
            raw.push_back(b);
        }
        for (int32_t k = 0; k < l_seq; ++k) {
            if ((k & 7) == 0) bits = rnd();
            raw.push_back((uint8_t)(2 + (bits & 0xff) % 39));
            bits >>= 8;
        }
    }
    // ---- deflate 65280-byte blocks in parallel, write in order
    const size_t kBlk = 0xff00;
    const size_t nblk = (raw.size() + kBlk - 1) / kBlk;
    std::vector<std::vector<uint8_t>> out(nblk);
    std::atomic<size_t> next{0};
    std::atomic<bool> failed{false};
    int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = std::max(1, std::min<int>(nt, (int)std::max<size_t>(nblk, 1)));
    auto worker = [&]() {
        for (size_t b; (b = next.fetch_add(1)) < nblk;) {
            const size_t o = b * kBlk;
            if (!bgzf_block(raw.data() + o, std::min(kBlk, raw.size() - o), level, out[b]))
                failed = true;
        }
    };
    std::vector<std::thread> pool;
    for (int i = 1; i < nt; ++i) pool.emplace_back(worker);
    worker();
    for (auto& t : pool) t.join();
    MC_REQUIRE(!failed, MC_E_IO, "deflate failed");
    FILE* f = std::fopen(path, "wb");
    MC_REQUIRE(f, MC_E_IO, "cannot create %s", path);
    bool ok = true;
    for (auto& b : out) ok &= std::fwrite(b.data(), 1, b.size(), f) == b.size();
    static const uint8_t kEof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67,
                                     2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    ok &= std::fwrite(kEof, 1, 28, f) == 28;
    ok &= std::fclose(f) == 0;
    MC_REQUIRE(ok, MC_E_IO, "write to %s failed", path);
    return MC_OK;
}
