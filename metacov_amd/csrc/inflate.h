// DEFLATE (RFC 1951) decoding of one BGZF block by one GPU lane, and the BAM
// record arithmetic of the GPU decode (bam_gpu.hip).
//
// The host decoder (bgzf.h) inflates BGZF blocks with libdeflate on host
// threads; at 16 threads it is the end-to-end bound of `metacov pileup`
// (profiles/r03pp_e2e.json: 1.56 s of 1.78 s for a 5.2 GB BAM).  Here every
// BGZF block (<= 64 KiB out, an independent deflate stream) is one lane's
// work: a 64-bit bit buffer fed from a per-lane LDS ring of input words,
// canonical Huffman codes decoded by a primary lookup table (MC_GZ_LIT_BITS =
// 7 bits literal/length, MC_GZ_DIST_BITS = 5 bits distance; longer codes by
// branch-free compares against the left-aligned length bounds, held in
// registers, into byte symbol lists), up to MC_GZ_LIT_EXTRA more literals per
// step, LZ77 copies from the lane's own output queued per lane.  The kernel
// keeps each lane's tables, symbol lists, ring and queue in LDS (bam_gpu.hip);
// the build's counts and code lengths in a per-lane global scratch slot
// (kScratchWords u16).
//
// Every function is __host__ __device__: mc_gz_inflate_host runs the same
// code on the CPU for the unit tests (tests/test_gpu_decode.py compares it
// with zlib), the kernels run it per lane.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mc {
namespace gz {

#define MC_HD __host__ __device__ __forceinline__

#ifndef MC_GZ_QUEUE
#define MC_GZ_QUEUE 16          // matches a lane defers (>= 1)
#endif
#ifndef MC_GZ_COPY_BATCH
#define MC_GZ_COPY_BATCH 2      // lz_copy: 2 = 16-byte chunks (dist >= 16), 1 = byte groups, 0 = byte loop
#endif

// Tuning knobs (scripts/gz_ab.py): primary table bits, tables in LDS.
#ifndef MC_GZ_LIT_BITS
#define MC_GZ_LIT_BITS 7        // primary table index bits (7 / 5-bit tables, 6 waves per CU)
#endif
#ifndef MC_GZ_DIST_BITS
#define MC_GZ_DIST_BITS 5
#endif
constexpr int kLitBits = MC_GZ_LIT_BITS;    // primary table index bits, literal/length alphabet
constexpr int kDistBits = MC_GZ_DIST_BITS;  // distance alphabet
static_assert(kLitBits >= 7, "the code length code (<= 7 bits) uses the literal table");
constexpr int kPrimaryWords = (1 << kLitBits) + (1 << kDistBits);   // both primary tables (u16)
// per-lane scratch (u16 words): counts, lengths (the primary tables and the
// symbol lists are separate: LDS in the kernel)
constexpr int kLitCnt = 0;                        // [16] codes per length
constexpr int kDistCnt = kLitCnt + 16;            // [16]
constexpr int kLens = kDistCnt + 16;              // [320] code lengths being read
constexpr int kOffs = kLens + 320;                // [16] build temporary
constexpr int kLitHi = kOffs + 16;                // [16] per length: canonical index of its first symbol >= 256
constexpr int kScratchWords = kLitHi + 16;
// symbol lists in canonical order, one byte per symbol: within one code
// length the symbols are in increasing order, so the literal/length symbols
// >= 256 of a length follow its literals, from the index kLitHi records
constexpr int kLitSyms = 288;
constexpr int kDistSyms = 32;
constexpr int kSymWords = (kLitSyms + kDistSyms) / 2;   // u16 words of both lists

enum : int {
    kOk = 0,
    kErrBlockType = 1,     // BTYPE 3
    kErrStored = 2,        // stored block LEN / NLEN mismatch
    kErrCodes = 3,         // bad code lengths (over-subscribed, counts out of range, no end code)
    kErrSymbol = 4,        // a bit pattern that is no code, or a length/distance symbol out of range
    kErrDistance = 5,      // distance before the block's output start
    kErrOutput = 6,        // more output than ISIZE
    kErrInput = 7,         // read past the compressed payload
    kErrSize = 8,          // the stream ended before ISIZE bytes
};

MC_HD bool wave_any(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __any(p);
#else
    return p;
#endif
}

// Bit reader over src[0, clen) through a per-lane ring of kRingWords u32 in
// LDS (the kernel; a plain array on the host).  The ring is topped up only at
// wave-uniform points (bits_topup: a vote, then every lane fills its ring
// with 16-byte groups and one wait covers the whole wave).
// Loading 16 bytes ahead in registers instead (round 3), every lane's refill
// copied the in-flight group into the loop-carried registers at once: the
// wave waited a full memory latency, draining every output store in flight
// too (vmcnt counts stores), at almost every symbol step of some lane.  The
// buffer src points into must be readable up to 16 bytes past clen rounded up
// to 16 (callers pad it).
#ifndef MC_GZ_RING
#define MC_GZ_RING 16
#endif
constexpr int kRingWords = MC_GZ_RING;            // power of two, >= 8 (A/B: 8 words 39.4 vs 36.0 ms)
constexpr int kRingLow = 4;                       // a lane below this many words calls the top-up
static_assert((kRingWords & (kRingWords - 1)) == 0 && kRingWords >= 8, "ring: power of two >= 8 words");

// the ring's and the match queue's pointer types for a table pointer type
// (LDS-qualified or plain)
template <class TP> struct RingOf;
template <> struct RingOf<uint16_t*> {
    using type = uint32_t*;
    using queue = uint64_t*;
    using sym = uint8_t*;
};
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
template <> struct RingOf<__attribute__((address_space(3))) uint16_t*> {
    using type = __attribute__((address_space(3))) uint32_t*;
    using queue = __attribute__((address_space(3))) uint64_t*;
    using sym = __attribute__((address_space(3))) uint8_t*;
};
#endif

template <class RP>
struct Bits {
    const uint4* p;         // next 16-byte group to load
    const uint4* pend;      // groups at or past it read the last one again (past the payload)
    RP ring;                // kRingWords words: [rpos, rfill) not yet in buf
    uint32_t rpos, rfill;   // absolute word counters (slot = counter % kRingWords)
    uint64_t buf;
    int cnt;                // valid bits in buf
    int64_t end_bits;       // bits from src[0] to the end of the words moved into buf
};

// The address is clamped, not the value.  Groups past the payload are never
// consumed by a valid stream (bits_pos checks).
MC_HD uint4 ld_group(const uint4* p, const uint4* pend) { return *(p < pend ? p : pend - 1); }

template <int kWords, class RP>
MC_HD void ring_load(Bits<RP>& b) {   // every load issued before the first ring write
    uint4 v[kWords / 4];
#pragma unroll
    for (int g = 0; g < kWords / 4; ++g) v[g] = ld_group(b.p + g, b.pend);
    b.p += kWords / 4;
#pragma unroll
    for (int g = 0; g < kWords / 4; ++g) {
        const uint32_t s = (b.rfill + 4 * g) & (kRingWords - 1);   // 4-aligned: no wrap inside a group
        b.ring[s] = v[g].x;
        b.ring[s + 1] = v[g].y;
        b.ring[s + 2] = v[g].z;
        b.ring[s + 3] = v[g].w;
    }
    b.rfill += kWords;
}

// Every lane that may consume input calls it at a point where the whole wave
// (or the active part of it) does: when some lane is low, every lane fills its
// ring (as many 16-byte groups as fit), and the wave waits once.  Filling only
// the lanes at or below half (round 3) left lanes just above it to trigger
// the next wait a few steps later (A/B: 37.5 vs 36.0 ms); full rings space
// the waits by at least kRingWords - 3 - kRingLow words of the fastest lane.
template <class RP>
MC_HD void bits_topup(Bits<RP>& b) {
    if (wave_any((int)(b.rfill - b.rpos) < kRingLow)) {
        const int ng = (kRingWords - (int)(b.rfill - b.rpos)) >> 2;   // free groups
        uint4 v[kRingWords / 4];
#pragma unroll
        for (int g = 0; g < kRingWords / 4; ++g)
            if (g < ng) v[g] = ld_group(b.p + g, b.pend);
#pragma unroll
        for (int g = 0; g < kRingWords / 4; ++g)
            if (g < ng) {
                const uint32_t s = (b.rfill + 4 * g) & (kRingWords - 1);
                b.ring[s] = v[g].x;
                b.ring[s + 1] = v[g].y;
                b.ring[s + 2] = v[g].z;
                b.ring[s + 3] = v[g].w;
            }
        b.p += ng;
        b.rfill += 4 * ng;
    }
}

// (pointer arithmetic only, no integer round trip: the compiler keeps the
// global address space and issues global loads, not flat ones)
template <class RP>
MC_HD void bits_init(Bits<RP>& b, const uint8_t* src, int64_t byte_off, int64_t clen) {
    const uint8_t* a = src + byte_off;
    const int mis = (int)((uintptr_t)a & 15);
    const uint8_t* e = src + clen;
    b.p = reinterpret_cast<const uint4*>(a - mis);
    b.pend = reinterpret_cast<const uint4*>(e + ((16 - (int)((uintptr_t)e & 15)) & 15)) + 1;
    b.rpos = b.rfill = 0;
    ring_load<kRingWords>(b);
    const int wi = mis >> 2, bi = mis & 3;
    b.rpos = wi + 1;
    b.buf = (uint64_t)b.ring[wi] >> (8 * bi);
    b.cnt = 32 - 8 * bi;
    b.end_bits = (byte_off + 4 - bi) * 8;
}

template <class RP>
MC_HD void bits_refill(Bits<RP>& b) {   // afterwards cnt > 32 (rpos < rfill: bits_topup's job)
    if (b.cnt <= 32) {
        b.buf |= (uint64_t)b.ring[b.rpos & (kRingWords - 1)] << b.cnt;
        ++b.rpos;
        b.cnt += 32;
        b.end_bits += 32;
    }
}

template <class RP>
MC_HD uint32_t bits_take(Bits<RP>& b, int n) {   // n <= cnt, n < 32
    const uint32_t v = (uint32_t)b.buf & ((1u << n) - 1u);
    b.buf >>= n;
    b.cnt -= n;
    return v;
}

template <class RP>
MC_HD int64_t bits_pos(const Bits<RP>& b) { return b.end_bits - b.cnt; }   // next unread bit

MC_HD uint32_t bitrev(uint32_t code, int len) {
    uint32_t r = 0;
    for (int i = 0; i < len; ++i) {
        r = (r << 1) | (code & 1u);
        code >>= 1;
    }
    return r;
}

// Canonical Huffman code from lens[0, n): counts, symbols in code order and
// the primary table of `tb` index bits.  Over-subscribed lengths are an
// error; incomplete codes are accepted (their missing patterns fail in
// decode_slow).
template <class TP, class SP>
MC_HD int build_code(uint16_t* S, TP T, int tb, int cnt_off, SP sym, const uint16_t* lens, int n) {
    uint16_t* cnt = S + cnt_off;
    uint16_t* offs = S + kOffs;
    for (int l = 0; l < 16; ++l) cnt[l] = 0;
    for (int s = 0; s < n; ++s) cnt[lens[s] & 15]++;
    int left = 1;
    for (int l = 1; l < 16; ++l) {
        left = (left << 1) - cnt[l];
        if (left < 0) return kErrCodes;
    }
    offs[1] = 0;
    for (int l = 1; l < 15; ++l) offs[l + 1] = (uint16_t)(offs[l] + cnt[l]);
    const bool lit = n > 256;   // the literal/length alphabet (symbols >= 256 in a byte list: kLitHi)
    for (int s = 0; s < n; ++s) {
        if (s == 256)
            for (int l = 0; l < 16; ++l) S[kLitHi + l] = offs[l];
        const int l = lens[s] & 15;
        if (l) sym[offs[l]++] = (uint8_t)s;
    }
    const int size = 1 << tb;
    for (int i = 0; i < size; ++i) T[i] = 0;
    uint32_t code = 0;
    int k = 0;
    for (int l = 1; l <= tb; ++l) {
        for (int c = 0; c < cnt[l]; ++c, ++k, ++code) {
            const int v = (int)sym[k] | (lit && k >= (int)S[kLitHi + l] ? 256 : 0);
            const uint16_t e = (uint16_t)((v << 4) | l);
            for (uint32_t r = bitrev(code, l); r < (uint32_t)size; r += 1u << l) T[r] = e;
        }
        code <<= 1;
    }
    return kOk;
}

// Codes longer than the primary table's TB bits.  Canonical codes of length
// l, left-aligned to 15 bits, fill the interval [lim[l-1], lim[l]) of the
// 15-bit code space, one length after the other; so for the next 15 bits c
// (first bit most significant) the length is TB + 1 + the number of l in
// [TB + 1, 14] with c >= lim[l], the symbol's canonical index is off[len] +
// (c >> (15 - len)), and c >= lim[15] is no code (an incomplete code).  The
// bounds and offsets are registers (built once per table); the search is
// branch-free compares, since the whole wave runs it whenever one lane meets
// a long code (round 3's 15-step RFC 1951 §3.2.2 count walk was 52 / 65
// instructions for the literal / distance alphabets, this one about half).
// HI: the literal/length alphabet, whose symbols >= 256 are told apart in the
// byte list by hi[k], the canonical index of the first of them at length
// TB + 1 + k (kLitHi).
template <int TB, bool HI>
struct CodeRegs {
    int lim[16 - TB];                  // lim[k]: bound of length TB + 1 + k (k = 0 .. 14 - TB)
    int off[16 - TB];                  // off[k]: canonical index - (code >> shift) base of that length
    int hi[HI ? 16 - TB : 1];
};

template <int TB, bool HI>
MC_HD void load_code(const uint16_t* S, int cnt_off, CodeRegs<TB, HI>& R) {
    int first = 0, index = 0;          // canonical first code / codes before, at length l
#pragma unroll
    for (int l = 1; l <= 15; ++l) {
        const int c = S[cnt_off + l];
        if (l > TB) {
            R.lim[l - TB - 1] = (first + c) << (15 - l);
            R.off[l - TB - 1] = index - first;
            if (HI) R.hi[l - TB - 1] = S[kLitHi + l];
        }
        index += c;
        first = (first + c) << 1;
    }
}

MC_HD uint32_t bitrev32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse32(x);
#else
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    x = ((x >> 8) & 0x00FF00FFu) | ((x & 0x00FF00FFu) << 8);
    return (x >> 16) | (x << 16);
#endif
}

// Keeps v a register value the compiler cannot fold into an address: a chain
// of selects over a register array otherwise becomes a select of the array
// index and one load, and the array moves to scratch (a private-memory round
// trip whose vmcnt wait drains the lane's output stores too).
MC_HD int opaque(int v) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(v));
#endif
    return v;
}

template <int TB, bool HI, class SP>
MC_HD int decode_slow(uint64_t bits, const CodeRegs<TB, HI>& R, SP sym, int* used) {
    const int c = (int)(bitrev32((uint32_t)bits) >> 17);   // the next 15 bits, first bit on top
    int k = 0, off = R.off[0], hi = R.hi[0];
#pragma unroll
    for (int j = 0; j < 14 - TB; ++j) {
        const bool past = c >= R.lim[j];
        k += past ? 1 : 0;
        off = opaque(past ? R.off[j + 1] : off);
        if (HI) hi = opaque(past ? R.hi[j + 1] : hi);
    }
    if (c >= R.lim[14 - TB]) return -1;
    const int len = TB + 1 + k;
    *used = len;
    const int idx = off + (c >> (15 - len));
    return (int)sym[idx] | (HI && idx >= hi ? 256 : 0);
}

template <int TB, bool HI, class TP, class SP, class RP>
MC_HD int decode_sym(Bits<RP>& b, TP T, const CodeRegs<TB, HI>& R, SP sym) {
    const uint16_t e = T[(uint32_t)b.buf & ((1u << TB) - 1u)];
    int used, s;
    if (e) {
        used = e & 15;
        s = e >> 4;
    } else {
        s = decode_slow<TB, HI>(b.buf, R, sym, &used);
        if (s < 0) return -1;
    }
    b.buf >>= used;
    b.cnt -= used;
    return s;
}

// Dynamic block header: code length code, then the literal/length and
// distance code lengths (RFC 1951 §3.2.7), then both tables.
template <class TP, class RP>
MC_HD int read_dynamic(Bits<RP>& b, uint16_t* S, TP TL, TP TD, typename RingOf<TP>::sym SL,
                       typename RingOf<TP>::sym SD) {
    bits_topup(b);
    bits_refill(b);
    const int nlen = (int)bits_take(b, 5) + 257;
    const int ndist = (int)bits_take(b, 5) + 1;
    const int ncode = (int)bits_take(b, 4) + 4;
    if (nlen > 286 || ndist > 30) return kErrCodes;
    uint16_t* lens = S + kLens;
    const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    for (int i = 0; i < 19; ++i) lens[i] = 0;
    for (int i = 0; i < ncode; ++i) {
        if ((i & 7) == 0) bits_topup(b);   // (8 x 3 bits per top-up at most)
        bits_refill(b);
        lens[order[i]] = (uint16_t)bits_take(b, 3);
    }
    // the code length code (<= 7 bits) goes through the literal table's slots
    int rc = build_code(S, TL, 7, kLitCnt, SL, lens, 19);
    if (rc) return rc;
    CodeRegs<7, false> ccode;
    load_code<7, false>(S, kLitCnt, ccode);
    int idx = 0;
    while (idx < nlen + ndist) {
        bits_topup(b);
        bits_refill(b);
        const int sym = decode_sym<7, false>(b, TL, ccode, SL);
        if (sym < 0) return kErrCodes;
        if (sym < 16) {
            lens[idx++] = (uint16_t)sym;
            continue;
        }
        int len = 0, rep;
        if (sym == 16) {
            if (idx == 0) return kErrCodes;
            len = lens[idx - 1];
            rep = 3 + (int)bits_take(b, 2);
        } else if (sym == 17) {
            rep = 3 + (int)bits_take(b, 3);
        } else {
            rep = 11 + (int)bits_take(b, 7);
        }
        if (idx + rep > nlen + ndist) return kErrCodes;
        while (rep--) lens[idx++] = (uint16_t)len;
    }
    if (lens[256] == 0) return kErrCodes;
    // the distance lengths follow the literal ones in lens[]; the literal
    // table is built last because its build overwrites nothing of them
    rc = build_code(S, TD, kDistBits, kDistCnt, SD, lens + nlen, ndist);
    if (rc) return rc;
    return build_code(S, TL, kLitBits, kLitCnt, SL, lens, nlen);
}

template <class TP>
MC_HD int read_fixed(uint16_t* S, TP TL, TP TD, typename RingOf<TP>::sym SL, typename RingOf<TP>::sym SD) {
    uint16_t* lens = S + kLens;
    for (int s = 0; s < 288; ++s) lens[s] = (uint16_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
    int rc = build_code(S, TL, kLitBits, kLitCnt, SL, lens, 288);
    if (rc) return rc;
    for (int s = 0; s < 30; ++s) lens[s] = 5;
    return build_code(S, TD, kDistBits, kDistCnt, SD, lens, 30);
}

// LZ77 copy of len bytes from dist back: every source byte precedes the
// copy's first output byte, so a group's loads are all issued before its
// stores (one memory round trip per 16 bytes, not per byte); the source
// index runs modulo dist for overlapping copies.
MC_HD void lz_copy_bytes(uint8_t* q, int len, int dist) {
#if MC_GZ_COPY_BATCH
    const uint8_t* s = q - dist;
    int si = 0;
    for (int k = 0; k < len; k += 16) {
        uint8_t v[16];
        int sj = si;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            v[j] = k + j < len ? s[sj] : 0;
            sj = sj + 1 == dist ? 0 : sj + 1;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (k + j < len) q[k + j] = v[j];
        si = sj;
    }
#else
    for (int k = 0; k < len; ++k) q[k] = q[k - dist];
#endif
}

// 16 bytes at p, any alignment (gfx950 runs in unaligned access mode: one
// global_load / store_dwordx4; memcpy tells the compiler the alignment is 1)
MC_HD uint4 ld16(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
MC_HD void st16(uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }

// A copy whose source ends at least 16 bytes before its destination starts
// (dist >= 16): whole 16-byte chunks; the last partial one as 8 / 4 / 2 / 1
// byte stores, since the bytes past the copy may hold literals already
// written (copies are deferred, literals are not).  Each chunk's source lies
// before the chunk itself, so a chunk read after earlier chunks' stores sees
// them (one lane, in order).
// v0: the copy's first 16 source bytes, already loaded.
MC_HD void lz_copy_wide(uint8_t* q, int len, int dist, uint4 v0) {
    const uint8_t* s = q - dist;
    int k = 0;
    uint4 v = v0;
    if (len >= 16) {
        st16(q, v0);
        for (k = 16; k + 16 <= len; k += 16) st16(q + k, ld16(s + k));
        if (k == len) return;
        v = ld16(s + k);
    }
    const int r = len - k;
    uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
    const uint64_t hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
    uint8_t* d = q + k;
    if (r & 8) {
        __builtin_memcpy(d, &lo, 8);
        d += 8;
        lo = hi;
    }
    if (r & 4) {
        const uint32_t w = (uint32_t)lo;
        __builtin_memcpy(d, &w, 4);
        d += 4;
        lo >>= 32;
    }
    if (r & 2) {
        const uint16_t h = (uint16_t)lo;
        __builtin_memcpy(d, &h, 2);
        d += 2;
        lo >>= 16;
    }
    if (r & 1) *d = (uint8_t)lo;
}

MC_HD void lz_copy(uint8_t* q, int len, int dist) {
#if MC_GZ_COPY_BATCH == 2
    if (dist >= 16) {
        lz_copy_wide(q, len, dist, ld16(q - dist));
        return;
    }
#endif
    lz_copy_bytes(q, len, dist);
}

// A lane's deferred LZ77 copies.  With one lane per BGZF block, a copy
// waits on its source bytes (global memory); done as decoded, some lane of
// the wave has one at almost every symbol step (6 % of symbols are matches,
// 1 - 0.94^64 = 98 %), so every step waited a memory round trip.  Queued, the
// copies of all lanes run together when some lane's queue is full (a wave
// vote), then at the block end.  The queue is the lane's kQueue u64 slots in
// LDS (a push is one ds_write; in registers, an entry selected by unrolled
// compares cost 3 x kQueue VALU per push, which every step with some lane
// matching paid), and the flush loops over the entries at run time.
constexpr int kQueue = MC_GZ_QUEUE;

// Literals decoded after a literal in the same symbol step (inflate_block),
// each while at least kLitBits bits are buffered (after bits_refill more than
// 32 are; a first symbol takes at most 15, an extra literal at most kLitBits).
#ifndef MC_GZ_LIT_EXTRA
#define MC_GZ_LIT_EXTRA 4
#endif
constexpr int kLitExtra = MC_GZ_LIT_EXTRA;
static_assert(kLitExtra >= 0, "extra literals");
static_assert(kQueue >= 1, "match queue: >= 1 entry");

template <class QP>
struct MatchQueue {
    QP e;                              // [kQueue] offset << 32 | dist << 9 | len
    int n;
};

template <class QP>
MC_HD void mq_flush(MatchQueue<QP>& q, uint8_t* dst) {
    for (int j = 0; j < q.n; ++j) {
        const uint64_t e = q.e[j];
        lz_copy(dst + (uint32_t)(e >> 32), (int)(e & 511u), (int)((uint32_t)e >> 9));
    }
    q.n = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    // vmcnt(0) here, once per flush: otherwise the compiler's wait for the
    // flush's loads lands at the join after it, on the symbol loop's common
    // path, and every symbol step waited for the output stores in flight
    // (A/B: 32 vs 33.3 ms).  Loading a batch of four entries' first chunks
    // together before their stores was slower (38.4 vs 36.0 ms).
    __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
}

// One raw deflate stream src[0, clen) into dst[0, isize): kOk iff it ends
// (BFINAL) with exactly isize bytes and without reading past clen.  S: the
// lane's scratch; TL / TD: its primary tables (1 << kLitBits, 1 << kDistBits);
// SL / SD: its symbol lists (kLitSyms, kDistSyms); ring: its input ring
// (kRingWords u32, see Bits).  TP: the pointer type
// (uint16_t* on the host, an LDS-qualified pointer in the kernel, so every
// lookup of the symbol loop is a ds_read waited on by lgkmcnt alone: with the
// symbol lists in the global scratch, a code longer than the primary table,
// which some lane of the wave meets at almost every step, cost a global round
// trip whose vmcnt wait also drained the lane's output stores).
template <class TP>
MC_HD int inflate_block(const uint8_t* src, int64_t clen, uint8_t* dst, int64_t isize, uint16_t* S, TP TL, TP TD,
                        typename RingOf<TP>::sym SL, typename RingOf<TP>::sym SD, typename RingOf<TP>::type ring,
                        typename RingOf<TP>::queue queue) {
    if (isize == 0) return kOk;
    MatchQueue<typename RingOf<TP>::queue> mq;
    mq.e = queue;
    mq.n = 0;
    Bits<typename RingOf<TP>::type> b;
    b.ring = ring;
    bits_init(b, src, 0, clen);
    const int64_t limit_bits = clen * 8;
    int64_t o = 0;
    for (;;) {
        bits_topup(b);
        bits_refill(b);
        const int final = (int)bits_take(b, 1);
        const int type = (int)bits_take(b, 2);
        if (type == 0) {
            // stored: skip to the byte boundary, LEN, NLEN, then LEN raw bytes
            const int64_t p = (bits_pos(b) + 7) >> 3;
            if (p + 4 > clen) return kErrInput;
            const uint32_t len = (uint32_t)src[p] | ((uint32_t)src[p + 1] << 8);
            const uint32_t nlen = (uint32_t)src[p + 2] | ((uint32_t)src[p + 3] << 8);
            if ((len ^ 0xffffu) != nlen) return kErrStored;
            if (p + 4 + (int64_t)len > clen) return kErrInput;
            if (o + (int64_t)len > isize) return kErrOutput;
            for (uint32_t k = 0; k < len; ++k) dst[o + k] = src[p + 4 + k];
            o += len;
            bits_init(b, src, p + 4 + len, clen);
        } else if (type == 3) {
            return kErrBlockType;
        } else {
            const int rc = type == 1 ? read_fixed(S, TL, TD, SL, SD) : read_dynamic(b, S, TL, TD, SL, SD);
            if (rc) return rc;
            CodeRegs<kLitBits, true> lcode;
            CodeRegs<kDistBits, false> dcode;
            load_code<kLitBits, true>(S, kLitCnt, lcode);
            load_code<kDistBits, false>(S, kDistCnt, dcode);
            for (;;) {
                // all lanes still in a symbol loop vote: one full queue
                // flushes every lane's (at most one push per iteration)
                if (wave_any(mq.n == kQueue)) mq_flush(mq, dst);
                // (no per-step input bound: loads past the payload are clamped
                // to its last group, every step but the end of block adds
                // output, bounded by isize, and the block end checks bits_pos)
                bits_topup(b);   // (a symbol with its distance takes <= 2 words)
                bits_refill(b);
                int s = decode_sym<kLitBits, true>(b, TL, lcode, SL);
                if (s < 0) return kErrSymbol;
                if (s < 256) {
                    if (o >= isize) return kErrOutput;
                    dst[o++] = (uint8_t)s;
                    // up to kLitExtra more literals of primary-table codes
                    // from the bits already buffered (anything else waits for
                    // the next iteration): a wave step's fixed cost - votes,
                    // checks, refill, the other paths some lane takes - is
                    // paid per iteration, and 72 % of BAM symbols are literals
#pragma unroll
                    for (int x = 0; x < kLitExtra; ++x) {
                        const uint32_t e2 = TL[(uint32_t)b.buf & ((1u << kLitBits) - 1u)];
                        if (e2 == 0 || e2 >= (256u << 4) || o >= isize ||
                            (33 - 15 - x * kLitBits < kLitBits && b.cnt < kLitBits))
                            break;
                        const int u = (int)(e2 & 15u);
                        b.buf >>= u;
                        b.cnt -= u;
                        dst[o++] = (uint8_t)(e2 >> 4);
                    }
                    continue;
                }
                if (s == 256) break;
                s -= 257;
                if (s >= 29) return kErrSymbol;
                int len;
                if (s < 8) {
                    len = s + 3;
                } else if (s == 28) {
                    len = 258;
                } else {
                    const int e = (s - 4) >> 2;
                    len = ((4 + (s & 3)) << e) + 3 + (int)bits_take(b, e);
                }
                bits_refill(b);
                const int d = decode_sym<kDistBits, false>(b, TD, dcode, SD);
                if (d < 0 || d >= 30) return kErrSymbol;
                int dist;
                if (d < 4) {
                    dist = d + 1;
                } else {
                    const int e = (d - 2) >> 1;
                    dist = ((2 + (d & 1)) << e) + 1 + (int)bits_take(b, e);
                }
                if ((int64_t)dist > o) return kErrDistance;
                if (o + len > isize) return kErrOutput;
                mq.e[mq.n++] = ((uint64_t)o << 32) | ((uint32_t)dist << 9) | (uint32_t)len;
                o += len;
            }
        }
        if (bits_pos(b) > limit_bits) return kErrInput;
        if (final) break;
    }
    mq_flush(mq, dst);
    return o == isize ? kOk : kErrSize;
}

// ---------------------------------------------------------------- BAM records
// (the host decoder's rules, bam_decode.cpp:32-205 / bgzf.h:222-289)

MC_HD uint32_t ld_u16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
MC_HD uint32_t ld_u32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
MC_HD int32_t ld_i32(const uint8_t* p) { return (int32_t)ld_u32(p); }

// hts_reg2bin(beg, end, 14, 5): the bin field of a record spanning [beg, end)
MC_HD uint32_t reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (uint32_t)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (uint32_t)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (uint32_t)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (uint32_t)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (uint32_t)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

// A structurally valid record starts at q of d[0, n): sizes that fit, ids
// in range, a NUL-terminated name and, for a mapped record, the bin field
// equal to reg2bin over its bam_endpos span (SAMv1 §4.2.1; the CG:B,I
// placeholder `<l_seq>S<rlen>N` has the real reference length).  Unmapped
// records' bins are not checked (writers differ on them).  *key (optional):
// the record's sort key (tid as unsigned, so tid -1 sorts last; pos + 1).
MC_HD bool rec_plausible(const uint8_t* d, int64_t q, int64_t n, int32_t n_ref, uint64_t* key = nullptr) {
    if (q + 36 > n) return false;
    const int32_t bs = ld_i32(d + q);
    if (bs < 32 || q + 4 + (int64_t)bs > n) return false;
    const int32_t tid = ld_i32(d + q + 4), pos = ld_i32(d + q + 8);
    const uint32_t lrn = d[q + 12];
    const uint32_t ncig = ld_u16(d + q + 16);
    const int32_t lseq = ld_i32(d + q + 20), ntid = ld_i32(d + q + 24);
    if (tid < -1 || tid >= n_ref || ntid < -1 || ntid >= n_ref || pos < -1 || lrn == 0 || lseq < 0)
        return false;
    const uint64_t need = 32 + (uint64_t)lrn + 4ull * ncig + ((uint64_t)lseq + 1) / 2 + (uint64_t)lseq;
    if (need > (uint64_t)bs) return false;
    if (d[q + 36 + lrn - 1] != 0) return false;
    // QNAME: 1-254 printable characters (SAMv1 §1.4: "*" when absent; some
    // aligners, BBMap among them, write spaces too)
    if (lrn < 2) return false;
    for (uint32_t k = 0; k + 1 < lrn; ++k)
        if ((uint32_t)(d[q + 36 + k] - 0x20) > 0x7e - 0x20) return false;
    const uint32_t flag = ld_u16(d + q + 18);
    if (flag >> 12) return false;   // no flag bits beyond 0x800 are defined
    if (tid >= 0 && pos >= 0 && !(flag & 4u)) {
        // ops 0-8 only; the query length of the CIGAR is l_seq (or no
        // sequence stored); the bin field is reg2bin of the span
        const uint8_t* cig = d + q + 36 + lrn;
        int64_t rlen = 0, qlen = 0;
        for (uint32_t k = 0; k < ncig; ++k) {
            const uint32_t cw = ld_u32(cig + 4ull * k), op = cw & 0xFu;
            if (op > 8) return false;
            if ((0x18Du >> op) & 1u) rlen += cw >> 4;
            if ((0x193u >> op) & 1u) qlen += cw >> 4;
        }
        if (ncig && lseq && qlen != lseq) return false;
        if (ld_u16(d + q + 14) != reg2bin(pos, pos + (rlen > 0 ? rlen : 1))) return false;
    }
    if (key) *key = ((uint64_t)(uint32_t)tid << 32) | (uint32_t)(pos + 1);
    return true;
}

// q starts a chain of `chain` plausible records in sort order, or a shorter
// chain ending exactly at n (the host decoder's sync rule, with the bin and
// order checks: a false start inside a record's bytes rarely chains).
MC_HD bool rec_chain(const uint8_t* d, int64_t q, int64_t n, int32_t n_ref, int chain) {
    uint64_t prev = 0, key = 0;
    int64_t z = q;
    int k = 0;
    for (; k < chain && z < n; ++k) {
        if (!rec_plausible(d, z, n, n_ref, &key) || key < prev) return false;
        prev = key;
        z += 4 + (int64_t)ld_i32(d + z);
    }
    return k == chain || z == n;
}

// CG:B,I in the aux data [p, end) (SAMv1 §4.2.2)
MC_HD bool find_cg(const uint8_t* p, const uint8_t* end, const uint8_t** words, uint32_t* count) {
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
                if (p + 5 > end) return false;
                const char sub = (char)p[0];
                const uint32_t cnt = ld_u32(p + 1);
                p += 5;
                const uint64_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
                if (t0 == 'C' && t1 == 'G' && sub == 'I') {
                    if (p + (uint64_t)cnt * 4 > end) return false;
                    *words = p;
                    *count = cnt;
                    return true;
                }
                p += es * cnt;
                break;
            }
            default:
                return false;
        }
    }
    return true;
}

// Record body r[0, rend - r) after block_size: 0 = dropped, 1 = kept with
// (tid, pos, span), or an error: 2 tid beyond the reference list, 3 CIGAR
// overruns record, 4 reference span exceeds int32.
struct RecOut {
    int32_t tid, pos, span;
    bool mapped;
};

MC_HD int rec_parse(const uint8_t* r, const uint8_t* rend, int32_t n_ref, uint32_t flag_filter, RecOut& out) {
    const int32_t tid = ld_i32(r);
    const uint32_t flag = ld_u16(r + 14);
    out.mapped = tid >= 0 && !(flag & 4u);
    if (tid < 0 || (flag & flag_filter)) return 0;
    if (tid >= n_ref) return 2;
    const uint32_t l_read_name = r[8];
    uint32_t n_cigar = ld_u16(r + 12);
    const int32_t l_seq = ld_i32(r + 16);
    const uint8_t* cig = r + 32 + l_read_name;
    if (cig + (uint64_t)n_cigar * 4 > rend) return 3;
    if (n_cigar == 2 && ld_u32(cig) == (((uint32_t)l_seq << 4) | 4u) && (ld_u32(cig + 4) & 0xFu) == 3u) {
        const uint8_t* aux = cig + 8 + ((uint64_t)l_seq + 1) / 2 + (uint64_t)l_seq;
        const uint8_t* words = nullptr;
        uint32_t cnt = 0;
        if (aux <= rend && find_cg(aux, rend, &words, &cnt) && words) {
            cig = words;
            n_cigar = cnt;
        }
    }
    int64_t rlen = 0;
    for (uint32_t k = 0; k < n_cigar; ++k) {
        const uint32_t cw = ld_u32(cig + 4ull * k);
        if ((0x18Du >> (cw & 0xFu)) & 1u) rlen += cw >> 4;
    }
    if (rlen <= 0 && (flag_filter & MC_LEGACY_ENDPOS)) rlen = 1;   // else raw rlen (bam_plp_push)
    if (rlen > 0x7fffffffll) return 4;
    out.tid = tid;
    out.pos = ld_i32(r + 4);
    out.span = (int32_t)rlen;
    return 1;
}

#undef MC_HD

}  // namespace gz
}  // namespace mc
