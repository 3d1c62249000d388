// `metacov scan` read histograms on gfx950 (reference metacov/scan.pyx:380-672,
// SURVEY.md §8 f rank 3): BaseHist, KmerHist, MirrorHist and IsizeHist under
// ByFlag, accumulated over batches of reads from scan_src.cpp in one kernel.
//
// Per read (restated from the reference's process_read methods):
//   group g   ByFlag: g = sum over the -g flags in order of bit(flag & mask),
//             the first flag most significant (scan.pyx:406-419)
//   read[x]   get_seq: nt4 of the x-th base; on the reverse strand
//             comp(nt4(seq[rlen-1-x])) (:240-259); nt4 maps nt16 1/2/4/8 to
//             0..3 and every other code to 4; comp(n) = 3-n, comp(4) = 4
//   ref[i]    get_ref: nt4 of the FASTA sequence of the read's reference,
//             Cython memoryview indexing: i < 0 wraps once (i += L)
//   BaseHist  (:422-470) pos = gpos; skip when pos < start_pos.  Mismatches
//             over x < rlen of read[x] against ref[pos + x] (forward) or
//             comp(ref[pos - x - 1]) (reverse); skip when mismatch*32 > rlen.
//             Then count[x][ref[pos + x - start_pos]] (forward) or
//             count[x][comp(ref[pos - x - 1 + start_pos])] (reverse) for
//             x < start_pos, and count[x + start_pos][read[x]] for x < rlen.
//   KmerHist  (:480-501) when rlen >= OFFSET + STEP*NK: for i < NK the code
//             of read[OFFSET + i*STEP + j], j < K, base j at bits 2j; any base
//             > 3 makes it the N bucket 4^K.  count[code][i] += 1.
//   MirrorHist (:525-543) p = gpos + OFFSET; skip when p < N - OFFSET;
//             plain / comp = #i<N with ref[p+i+1] != ref[p-i-1] /
//             != comp(ref[p-i-1]).  count[plain][0], count[comp][1] += 1.
//   IsizeHist (:561-579) count[|gisize|] += 1; max_isize = max(...).
//
// Where the reference reads memory it does not own the result is undefined
// there; this build fixes it (parity unpinned):
//   * reference positions outside [0, L) after the one wrap, and every
//     reference position when there is no FASTA sequence for the read, read
//     as N (4);
//   * k-mer bases outside [0, rlen) (negative OFFSET, K > STEP) read as N
//     (the reference reads stale bytes of earlier reads).
//
// Layout: one lane per read.  Waves take slices of kScanSlice reads from a
// queue and walk them in batches of up to 64 consecutive reads whose bases
// (and, when they share a reference sequence, the reference window they
// touch) are staged in LDS; every per-read access after that is LDS.
// BaseHist, MirrorHist and IsizeHist are privatised per workgroup in LDS
// when they fit (every read hits the same few hundred bins) and flushed once
// per workgroup; BaseHist's per-position counts are taken position-parallel
// (count_bases_pairs).  KmerHist codes go to HBM and kmer_count_kernel counts
// them in LDS tables (global atomics for K >= 8).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/metacov_amd.h"
#include "common.h"

#define HIP_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            mc::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                          __FILE__, __LINE__);                                 \
            return MC_E_HIP;                                                   \
        }                                                                      \
    } while (0)

namespace {

// Build knobs (A/B of the round-5 changes, profiles/r05/r05s-r05z):
//   MC_SCAN_CUT    a batch ends where its reference window outgrows the stage
//   MC_SCAN_PAIRS  BaseHist by strand/length sets, two positions per lane
//                  (0: count_bases, one position per lane)
//   MC_SCAN_DYN    slices from a queue (0: one static slice per wave)
//   MC_SCAN_PREFETCH  the next batch's accessor columns load during this one
//   MC_SCAN_SLICE  reads per queued slice
#ifndef MC_SCAN_CUT
#define MC_SCAN_CUT 1
#endif
#ifndef MC_SCAN_PAIRS
#define MC_SCAN_PAIRS 1
#endif
#ifndef MC_SCAN_DYN
#define MC_SCAN_DYN 1
#endif
#ifndef MC_SCAN_PREFETCH
#define MC_SCAN_PREFETCH 1
#endif
#ifndef MC_SCAN_SLICE
#define MC_SCAN_SLICE 256
#endif
constexpr int64_t kScanSlice = MC_SCAN_SLICE;   // reads per queued slice (MC_SCAN_DYN)
//   MC_SCAN_STAGE16  a batch's bases and reference window staged with 16-byte
//                  loads all issued before the first wait (0: dword loop,
//                  one round trip per 4 dwords per lane)
#ifndef MC_SCAN_STAGE16
#define MC_SCAN_STAGE16 1
#endif
//   MC_SCAN_REGCOLS  the per-read columns (rlen, flag, gpos, gisize) taken
//                  from the prefetched registers (0: reloaded from global
//                  memory where they are used, an L2 round trip each)
#ifndef MC_SCAN_REGCOLS
#define MC_SCAN_REGCOLS 1
#endif
//   MC_SCAN_NEED   stage / cut a batch only for what its tables read
#ifndef MC_SCAN_NEED
#define MC_SCAN_NEED 1
#endif
//   MC_SCAN_PF2    a second batch of accessor columns in flight (see scan_kernel)
#ifndef MC_SCAN_PF2
#define MC_SCAN_PF2 1
#endif
//   MC_SCAN_KMER8  KmerHist codes (K <= 8) from one 8-base window each (kmer8;
//                  0: base by base)
#ifndef MC_SCAN_KMER8
#define MC_SCAN_KMER8 1
#endif
//   MC_SCAN_MISM8  BaseHist's mismatch test 8 bases at a time (mism8; 0: per
//                  base, the compiler's unrolled byte compares).  Slower: all
//                  four 14.09 -> 14.19 ms, BaseHist alone 10.65 -> 10.77
//                  (profiles/r06/r06x_scan_mism8_ab.txt)
#ifndef MC_SCAN_MISM8
#define MC_SCAN_MISM8 0
#endif
//   MC_SCAN_QUEUES slice queues (take_slice).  100 M reads, ms for IsizeHist
//                  alone / KmerHist alone / all four: 1 queue 4.53 / 5.29 /
//                  14.22, 2: 2.37 / 3.58 / 14.11, 4: 1.32 / 3.54 / 14.05,
//                  8 (one per XCD): 1.02 / 3.52 / 14.30
//                  (profiles/r06/r06s_scan_queues_ab.txt)
#ifndef MC_SCAN_QUEUES
#define MC_SCAN_QUEUES 4
#endif
#ifndef MC_SCAN_QPEEK
#define MC_SCAN_QPEEK 0             // take_slice reads a queue's counter before its atomic
#endif
#ifndef MC_SCAN_STAGE_REGS
#define MC_SCAN_STAGE_REGS 3      // 16-byte units per lane in flight (VGPRs: 4 each)
#endif

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kLdsWords = 8192;     // histogram arena: 32 KiB
// scan_kernel residency: 4 workgroups per CU (launch bounds: VGPRs <= 128)
// with 5 KB of read stage and 1.5 KB of reference window per wave (whole
// 64-read batches of 150 bp, a window of ~0.8 kbp at C3 density): C3 scan
// 20.5 -> 17.9 ms against 3 per CU with 6 + 2 KB; 5 per CU with 3 + 1.5 KB
// 24.4 ms (short batches) (profiles/r05/r05zh_scan_occupancy.txt)
#ifndef MC_SCAN_OCC
#define MC_SCAN_OCC 4
#endif
#ifndef MC_SCAN_SEQ
#define MC_SCAN_SEQ (MC_SCAN_OCC >= 4 ? 5120 : 6144)
#endif
#ifndef MC_SCAN_REF
#define MC_SCAN_REF (MC_SCAN_OCC >= 4 ? 1536 : 2048)
#endif
constexpr int kSeqStage = MC_SCAN_SEQ;   // per wave: packed bases of the batch
constexpr int kRefStage = MC_SCAN_REF;   // per wave: reference window of the batch
constexpr int kStagePad = 16;
constexpr int kStageBytes = kSeqStage + kRefStage + 2 * kStagePad;
constexpr int kMaxFlags = 16;
constexpr int kRefPad = 64;         // zero bytes before and after the device reference

struct ScanArgs {
    const int32_t* rlen;
    const int32_t* flag;
    const int32_t* gpos;
    const int32_t* gisize;
    const int32_t* ref_id;
    const int64_t* seq_off;
    const uint8_t* seq;
    int64_t n;
    int64_t per_wave;         // reads per slice (a multiple of 64)
    unsigned* work;           // the slice queues (0 at launch, kQueueStride apart), or null: one static slice per wave
    int32_t nq;               // queues: queue q hands out slices [q * per_q, (q + 1) * per_q) of n_slices
    uint32_t per_q, n_slices;
    const uint8_t* ref;       // nt4 codes, all sequences back to back (padded both ends)
    const int64_t* ref_off;
    const int64_t* ref_len;
    int32_t n_ref;
    int32_t n_flags;
    uint32_t fmask[kMaxFlags];
    int32_t G;
    // BaseHist: [row][G][5]
    int32_t base_on, base_start, base_rows, base_lds;
    uint32_t* base;
    // KmerHist: [G][NK][4^K + 1] (slot-major on the device).  kcodes != null:
    // the codes go to kcodes[slot][read] (u16, 0xFFFF = no k-mer) and
    // kmer_count_kernel counts them; else global atomics here.
    int32_t kmer_on, K, NK, STEP, OFF;
    uint32_t* kmer;
    uint16_t* kcodes;
    uint16_t* kgroup;         // per read group (G > 1 with kcodes)
    int64_t kstride;          // kcodes row stride: n rounded up to 8 (16-byte rows)
    // MirrorHist: [G][N + 1][2]
    int32_t mir_on, MOFF, MN, mir_lds;
    uint32_t* mir;
    // IsizeHist: [a][G] and max per group
    int32_t isz_on, isz_cap, isz_lds;
    uint32_t* isz;
    int32_t* isz_max;
    // LDS arena (words) and the staging area after it
    int32_t lds_base, lds_mir, lds_isz, lds_isz_max, lds_words, stage_off;
    int32_t* error;           // set when a read's bases are not 4-byte aligned
};

// LDS pointers carry their address space explicitly: generic pointers into
// LDS compile to flat instructions (vector-memory path, several times
// slower than ds_* for the atomics and byte reads this kernel lives on).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
typedef __attribute__((address_space(3))) const uint8_t lds_cu8;

// nt16 code -> nt4 (scan.pyx:26-29): 1/2/4/8 -> 0..3, anything else -> 4
constexpr uint64_t kNt4 = 0x4444444344424104ull;   // nibble v holds nt4(v)

__device__ __forceinline__ int nt4_of(uint32_t v) { return (int)((kNt4 >> (4 * v)) & 15); }

__device__ __forceinline__ int comp4(int n) { return n < 4 ? 3 - n : 4; }

// base j (0 = high nibble of byte 0) of a dword holding 8 packed bases
__device__ __forceinline__ uint32_t nib8(uint32_t w, int j) {
    return (w >> (8 * (j >> 1) + 4 * (1 - (j & 1)))) & 15u;
}

// The read's reference sequence: a staged LDS window [wlo, whi) of it (the
// batch's span) and the global copy for everything else.  Cython indexing:
// one negative wrap; outside [0, L) reads N.
struct RefWin {
    const uint8_t* g;     // global nt4, sequence start (nullptr: no sequence)
    int64_t L;
    lds_cu8* w;           // LDS: position wlo
    int64_t wlo, whi;
    __device__ __forceinline__ int at(int64_t i) const {
        if (!g) return 4;
        if (i < 0) i += L;
        if (i < 0 || i >= L) return 4;
        return (i >= wlo && i < whi) ? (int)w[i - wlo] : (int)g[i];
    }
    // 8 consecutive positions p..p+7, all inside [wlo, whi + 8) (window
    // padding covers the overhang): nt4 bytes little-endian in two dwords
    __device__ __forceinline__ void at8(int64_t p, uint32_t& lo, uint32_t& hi) const {
        const uint32_t a = (uint32_t)(uintptr_t)(w + (p - wlo));   // LDS byte address
        lds_cu32* q = (lds_cu32*)(uintptr_t)(a & ~3u);
        const uint32_t sh = a & 3u;
        const uint32_t d0 = q[0], d1 = q[1], d2 = q[2];
        lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
        hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
    }
};

// BaseHist's mismatches of 8 packed bases (w, BAM order) against the
// reference's nt4 bytes lo (positions 0-3) / hi (4-7), the first n8 only:
// nt4 of every nibble at once (the kmer8 arithmetic; a nibble that is not
// A/C/G/T becomes 4, the reference's N code), spread to bytes, compared by
// XOR, the non-zero bytes counted.
__device__ __forceinline__ int mism8(uint32_t w, uint32_t lo, uint32_t hi, int n8) {
    constexpr uint32_t M1 = 0x11111111u, B1 = 0x01010101u;
    w = ((w >> 4) & 0x0F0F0F0Fu) | ((w & 0x0F0F0F0Fu) << 4);   // base j at nibble j
    const uint32_t t0 = w & M1, t1 = (w >> 1) & M1, t2 = (w >> 2) & M1, t3 = (w >> 3) & M1;
    const uint32_t f = (t0 + t1 + t2 + t3) ^ M1;                // non-zero: not one bit set
    const uint32_t fb = (f | (f >> 1) | (f >> 2)) & M1;
    const uint32_t n = (((t1 | t3) | ((t2 | t3) << 1)) & ~(fb * 3u)) | (fb << 2);
    auto spread = [](uint32_t x) {   // nibbles 0-3 -> bytes 0-3
        x &= 0xFFFFu;
        x = (x | (x << 8)) & 0x00FF00FFu;
        return (x | (x << 4)) & 0x0F0F0F0Fu;
    };
    const uint32_t dl = spread(n) ^ lo, dh = spread(n >> 16) ^ hi;
    const uint32_t ml = n8 >= 4 ? B1 : ((1u << (8 * n8)) - 1u) & B1;
    const uint32_t mh = n8 >= 8 ? B1 : n8 <= 4 ? 0u : ((1u << (8 * (n8 - 4))) - 1u) & B1;
    return __builtin_popcount((dl | (dl >> 1) | (dl >> 2)) & ml) + __builtin_popcount((dh | (dh >> 1) | (dh >> 2)) & mh);
}

// KmerHist's code of the K <= 8 bases b .. b+K-1 of a read (forward), or of
// comp(b+K-1) .. comp(b) (reverse strand: base j of the k-mer is the read's
// base b+K-1-j, complemented), from one 8-base window: two dwords of packed
// bases (the pair is clamped to the read's last dwords, ndw = dwords of its
// bases, so nothing past it is read), the nibbles of each byte swapped into
// base order, then per nibble n (nt16): nt4 = (bit1 | bit3) | (bit2 | bit3) << 1
// for n in {1, 2, 4, 8}; any other n (one bit set is the test) puts the k-mer
// in the N bucket 4^K.  Base j of the code at bits 2j (scan.pyx:480-501).
template <typename P32>
__device__ __forceinline__ uint32_t kmer8(P32 s32, int b, int ndw, int K, bool rev) {
    const int byte = b >> 1;
    const int q = min(byte >> 2, ndw - 2);
    uint64_t w = (uint64_t)s32[q] | ((uint64_t)s32[q + 1] << 32);
    w >>= 8 * (byte - 4 * q);   // (0..7 bytes: the window ends inside the pair)
    w = ((w >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((w & 0x0F0F0F0F0F0F0F0Full) << 4);
    const uint32_t n = (uint32_t)(w >> (4 * (b & 1)));   // base b + j at nibble j
    constexpr uint32_t M1 = 0x11111111u;
    const uint32_t t0 = n & M1, t1 = (n >> 1) & M1, t2 = (n >> 2) & M1, t3 = (n >> 3) & M1;
    const uint32_t nib = K == 8 ? 0xFFFFFFFFu : (1u << (4 * K)) - 1u;
    if (((t0 + t1 + t2 + t3) ^ M1) & nib) return 1u << (2 * K);   // a base other than A/C/G/T
    uint32_t c = (t1 | t3) | ((t2 | t3) << 1);   // nt4 in the low 2 bits of each nibble
    c = (c | (c >> 2)) & 0x0F0F0F0Fu;
    c = (c | (c >> 4)) & 0x00FF00FFu;
    c = (c | (c >> 8)) & 0x0000FFFFu;            // base b + j at bits 2j
    const uint32_t km = (1u << (2 * K)) - 1u;
    if (!rev) return c & km;
    c = ((c & 0x3333u) << 2) | ((c >> 2) & 0x3333u);   // the eight 2-bit fields reversed
    c = ((c & 0x0F0Fu) << 4) | ((c >> 4) & 0x0F0Fu);
    c = ((c & 0x00FFu) << 8) | ((c >> 8) & 0x00FFu);
    return (c >> (2 * (8 - K))) ^ km;                  // comp(n) = 3 - n
}

__device__ __forceinline__ void inc(lds_u32* lds_base, uint32_t* g, int64_t i, bool in_lds) {
    if (in_lds)
        __hip_atomic_fetch_add(lds_base + i, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else
        atomicAdd(g + i, 1u);
}

// Per-read rules (see the header): s = the read's packed bases (LDS or
// global, 4-byte aligned), rw = its reference.
// Returns true when the read passed BaseHist's match test and `defer` left
// the counting of its bases to the caller.
template <typename P8, typename P32>
__device__ __forceinline__ bool process_read(const ScanArgs& a, int64_t r, P8 s, P32 s32,
                                             const RefWin& rw, lds_u32* lds, bool defer,
                                             bool isize_done, int32_t rlen, int32_t flag, int32_t gpos,
                                             int32_t isz) {
    const bool rev = (flag & 0x10) != 0;
    int g = 0;
    for (int f = 0; f < a.n_flags; ++f) g = (g << 1) | ((flag & a.fmask[f]) ? 1 : 0);

    if (a.isz_on && !isize_done) {
        int32_t v = isz;
        v = v < 0 ? -v : v;
        inc(lds + a.lds_isz, a.isz, (int64_t)v * a.G + g, a.isz_lds);
        if (a.isz_lds)
            __hip_atomic_fetch_max((__attribute__((address_space(3))) int32_t*)(lds + a.lds_isz_max) + g,
                                   v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
            atomicMax(a.isz_max + g, v);
    }

    if (a.kmer_on) {
        const uint32_t nbucket = 1u << (2 * a.K);
        const bool ok = rlen >= a.OFF + a.STEP * a.NK;
        if (a.kcodes && a.G > 1) a.kgroup[r] = (uint16_t)g;
        // every k-mer's bases inside the read (and K <= 8, two dwords of
        // bases): each code from one 8-base window (kmer8), not base by base
        const bool fast = MC_SCAN_KMER8 && ok && a.K <= 8 && a.OFF >= 0 && rlen >= 9 &&
                          a.OFF + (a.NK - 1) * a.STEP + a.K <= rlen;
        for (int i = 0; i < a.NK; ++i) {
            uint32_t k = 0xFFFFu;
            if (fast) {
                const int x0 = a.OFF + i * a.STEP;
                k = kmer8(s32, rev ? rlen - a.K - x0 : x0, (rlen + 7) >> 3, a.K, rev);
            } else if (ok) {
                k = 0;
                for (int j = 0; j < a.K; ++j) {
                    const int x = a.OFF + i * a.STEP + j;
                    int c = 4;
                    if (x >= 0 && x < rlen) {
                        const int b = rev ? rlen - 1 - x : x;
                        const uint32_t byte = s[b >> 1];
                        c = nt4_of((b & 1) ? (byte & 15u) : (byte >> 4));
                        if (rev) c = comp4(c);
                    }
                    if (c > 3) {
                        k = nbucket;
                        break;
                    }
                    k |= (uint32_t)c << (2 * j);
                }
            }
            if (a.kcodes)
                a.kcodes[(int64_t)i * a.kstride + r] = (uint16_t)k;
            else if (ok)
                atomicAdd(a.kmer + ((int64_t)g * a.NK + i) * (nbucket + 1) + k, 1u);
        }
    }

    if (a.mir_on) {
        const int64_t p = (int64_t)gpos + a.MOFF;
        if (p >= (int64_t)a.MN - a.MOFF) {
            int plain = 0, cmp = 0;
            for (int i = 0; i < a.MN; ++i) {
                const int x = rw.at(p + i + 1), y = rw.at(p - i - 1);
                plain += x != y;
                cmp += x != comp4(y);
            }
            const int64_t b = ((int64_t)g * (a.MN + 1)) * 2;
            inc(lds + a.lds_mir, a.mir, b + plain * 2, a.mir_lds);
            inc(lds + a.lds_mir, a.mir, b + cmp * 2 + 1, a.mir_lds);
        }
    }

    if (a.base_on && gpos >= a.base_start) {
        // mismatches in BAM orientation: base j against position b0 + j
        // (the reverse strand's comparison mapped back; comp is a bijection)
        const int64_t b0 = rev ? (int64_t)gpos - rlen : (int64_t)gpos;
        const int nw = (rlen + 7) >> 3;
        const bool fast = rw.g && b0 >= rw.wlo && b0 + rlen <= rw.whi;
        // The mismatch count only grows, so testing it once at the end
        // rejects exactly the reads the reference's early exit does; without
        // the exit the staged-window loop has no loop-carried branch and its
        // LDS reads of several words are in flight together.
        int mism = 0;
        if (fast) {
#pragma unroll 4
            for (int k = 0; k < nw; ++k) {
                const uint32_t w = s32[k];
                const int n8 = min(8, rlen - 8 * k);
                uint32_t lo, hi;
                rw.at8(b0 + 8 * k, lo, hi);
                if (MC_SCAN_MISM8) {
                    mism += mism8(w, lo, hi, n8);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int rv = (int)(((j < 4 ? lo : hi) >> (8 * (j & 3))) & 255u);
                        mism += (j < n8) & (nt4_of(nib8(w, j)) != rv);
                    }
                }
            }
        } else {
            for (int k = 0; k < nw && mism * 32 <= rlen; ++k) {
                const uint32_t w = s32[k];
                const int n8 = min(8, rlen - 8 * k);
                for (int j = 0; j < n8; ++j) mism += nt4_of(nib8(w, j)) != rw.at(b0 + 8 * k + j);
            }
        }
        const bool reject = mism * 32 > rlen;
        if (!reject) {
            const int64_t rowstride = (int64_t)a.G * 5;
            for (int x = 0; x < a.base_start; ++x) {
                const int v = rev ? comp4(rw.at((int64_t)gpos - x - 1 + a.base_start))
                                  : rw.at((int64_t)gpos + x - a.base_start);
                inc(lds + a.lds_base, a.base, x * rowstride + g * 5 + v, a.base_lds);
            }
            if (defer) return true;   // the wave counts the read's bases (count_bases)
            for (int j = 0; j < rlen; ++j) {
                const uint32_t byte = s[j >> 1];
                int v = nt4_of((j & 1) ? (byte & 15u) : (byte >> 4));
                int x = j;
                if (rev) {
                    v = comp4(v);
                    x = rlen - 1 - j;
                }
                inc(lds + a.lds_base, a.base, (int64_t)(x + a.base_start) * rowstride + g * 5 + v,
                    a.base_lds);
            }
        }
    }
    return false;
}

// BaseHist counts of the batch's passing reads, position-parallel: lane L
// owns read positions L, L+64, L+128, L+192 and keeps 5 packed 12-bit
// counters per position in a 64-bit register while the wave walks the
// reads one by one (broadcast LDS reads of each read's bytes); one LDS add
// per non-zero counter at the end.  Positions from 256 on, and batches
// whose passing reads are in several groups, are counted per lane.
#ifndef MC_SCAN_INC_TAB
#define MC_SCAN_INC_TAB 1
#endif
typedef __attribute__((address_space(3))) const uint64_t lds_cu64;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
constexpr int kIncTabWords = 64;   // 32 u64: nibble -> packed-counter increment, forward then reverse

// A batch whose passing reads are in several groups (or with BaseHist in
// global memory): each lane counts its own read.
__device__ __forceinline__ void count_bases_lanes(const ScanArgs& a, bool pending, int rlen, int fl, int g,
                                                  int soff, lds_u32* sseq, lds_u32* lds) {
    if (!pending) return;
    const int rowstride = a.G * 5;
    lds_cu8* s = (lds_cu8*)(sseq + soff);
    const bool rev = (fl & 0x10) != 0;
    for (int j = 0; j < rlen; ++j) {
        const uint32_t byte = s[j >> 1];
        int v = nt4_of((j & 1) ? (byte & 15u) : (byte >> 4));
        int x = j;
        if (rev) {
            v = comp4(v);
            x = rlen - 1 - j;
        }
        inc(lds + a.lds_base, a.base, (int64_t)(x + a.base_start) * rowstride + g * 5 + v, a.base_lds);
    }
}

__device__ __forceinline__ void count_bases(lds_cu64* inc_tab, const ScanArgs& a, int64_t r, bool pending, bool act,
                                            int soff, lds_u32* sseq, lds_u32* lds, int lane, int32_t rlen_r,
                                            int32_t flag_r) {
    uint64_t pend = __ballot(pending);
    if (!pend) return;
    const int32_t rlen = act ? rlen_r : 0;
    const int32_t fl = act ? flag_r : 0;
    int g = 0;
    for (int f = 0; f < a.n_flags; ++f) g = (g << 1) | ((fl & a.fmask[f]) ? 1 : 0);
    const int first = __builtin_ctzll(pend);
    const int g0 = __builtin_amdgcn_readlane(g, first);
    const int rowstride = a.G * 5;
    if (!a.base_lds || __ballot(pending && g != g0)) {
        count_bases_lanes(a, pending, rlen, fl, g, soff, sseq, lds);
        return;
    }
    uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    // two reads per step, branch-free (a position past the read end reads
    // the read's first byte and adds 0), so both reads' LDS loads are in
    // flight together instead of one read's latency at a time
    while (pend) {
        const int l = __builtin_ctzll(pend);
        pend &= pend - 1;
        const bool two = pend != 0;
        const int l2 = two ? __builtin_ctzll(pend) : l;
        if (two) pend &= pend - 1;
        const int rl = __builtin_amdgcn_readlane(rlen, l);
        const int rv = __builtin_amdgcn_readlane(fl, l) & 0x10;
        const int so = __builtin_amdgcn_readlane(soff, l);
        const int rl2 = two ? __builtin_amdgcn_readlane(rlen, l2) : 0;
        const int rv2 = __builtin_amdgcn_readlane(fl, l2) & 0x10;
        const int so2 = __builtin_amdgcn_readlane(soff, l2);
        lds_cu8* s = (lds_cu8*)(sseq + so);
        lds_cu8* s2 = (lds_cu8*)(sseq + so2);
        auto count_pos = [inc_tab](lds_cu8* sp, int len, int rev, int x, uint64_t& c) {
            const bool ok = x < len;
            const int j = ok ? (rev ? len - 1 - x : x) : 0;
            const uint32_t byte = sp[j >> 1];
            const uint32_t nib = (j & 1) ? (byte & 15u) : (byte >> 4);
#if MC_SCAN_INC_TAB
            c += ok ? inc_tab[(rev ? 16 : 0) + nib] : 0ull;   // the packed counter's increment
#else
            int v = nt4_of(nib);
            if (rev) v = comp4(v);
            c += ok ? (1ull << (12 * v)) : 0ull;
#endif
        };
        count_pos(s, rl, rv, lane, c0);
        count_pos(s2, rl2, rv2, lane, c0);
        count_pos(s, rl, rv, lane + 64, c1);
        count_pos(s2, rl2, rv2, lane + 64, c1);
        if (max(rl, rl2) > 128) {
            count_pos(s, rl, rv, lane + 128, c2);
            count_pos(s2, rl2, rv2, lane + 128, c2);
        }
        if (max(rl, rl2) > 192) {
            count_pos(s, rl, rv, lane + 192, c3);
            count_pos(s2, rl2, rv2, lane + 192, c3);
        }
        for (int k = 0; k < 2; ++k) {
            const int len = k ? rl2 : rl, rev = k ? rv2 : rv;
            lds_cu8* sp = k ? s2 : s;
            for (int x = 256 + lane; x < len; x += 64) {
                const int j = rev ? len - 1 - x : x;
                const uint32_t byte = sp[j >> 1];
                int v = nt4_of((j & 1) ? (byte & 15u) : (byte >> 4));
                if (rev) v = comp4(v);
                __hip_atomic_fetch_add(lds + a.lds_base + (x + a.base_start) * rowstride + g0 * 5 + v,
                                       1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    const uint64_t cs[4] = {c0, c1, c2, c3};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (!cs[q]) continue;
        lds_u32* row = lds + a.lds_base + (lane + 64 * q + a.base_start) * rowstride + g0 * 5;
#pragma unroll
        for (int v = 0; v < 5; ++v) {
            const uint32_t c = (uint32_t)(cs[q] >> (12 * v)) & 0xFFFu;
            if (c) __hip_atomic_fetch_add(row + v, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// BaseHist counts, two positions per lane (MC_SCAN_PAIRS).  Lane L owns the
// read-position pairs P = L and P = 64 + L: one LDS byte holds a pair's two
// bases, and one 8-byte table entry (pair_tab) both positions' increments as
// 8-bit A/C/G/T counters in a dword each; N is the position's coverage less
// the four.  The reads are counted in BAM orientation: a read set of one
// group is walked forward strand first (position x = base j), then per
// length L the reverse-strand reads of that length, whose counts land at x =
// L-1-j, complemented, when the set's counters are flushed.  So every read
// costs a byte load, a table load and a 64-bit add per 128 positions, with no
// per-read strand arithmetic (the one-position-per-lane walk, count_bases,
// spent ~100 instructions per read).  A batch has at most 64 reads: no 8-bit
// counter overflows before its flush.
constexpr int kPairTabWords = 256 * 2;   // 256 u64

__device__ __forceinline__ uint32_t inc8(int v) { return v < 4 ? 1u << (8 * v) : 0u; }

__device__ __forceinline__ void pair_tab_init(lds_u64* tab) {
    for (int i = threadIdx.x; i < 256; i += kThreads) {
        // the high nibble is the even base
        tab[i] = (uint64_t)inc8(nt4_of((uint32_t)i >> 4)) | ((uint64_t)inc8(nt4_of((uint32_t)i & 15u)) << 32);
    }
}

// Counts of the reads in `set` (lane mask; each read's length in rlen, its
// first staged dword in soff) at base pairs P = lane (acc0) and 64 + lane
// (acc1), two reads per step so their loads are in flight together.
__device__ __forceinline__ void count_set(lds_cu64* tab, uint64_t set, int rlen, int soff, lds_u32* sseq, int lane,
                                          uint64_t& acc0, uint32_t& cov0, uint64_t& acc1, uint32_t& cov1) {
    auto one = [&](int len, lds_cu8* sp, int P, uint64_t& acc, uint32_t& cov) {
        const bool ok0 = 2 * P < len, ok1 = 2 * P + 1 < len;
        const uint64_t v = tab[sp[ok0 ? P : 0]];
        acc += v & (ok0 ? (ok1 ? ~0ull : 0xffffffffull) : 0ull);
        cov += (ok0 ? 1u : 0u) + (ok1 ? 0x10000u : 0u);
    };
    while (set) {
        const int l = __builtin_ctzll(set);
        set &= set - 1;
        const bool two = set != 0;
        const int l2 = two ? __builtin_ctzll(set) : l;
        if (two) set &= set - 1;
        const int len = __builtin_amdgcn_readlane(rlen, l);
        const int len2 = two ? __builtin_amdgcn_readlane(rlen, l2) : 0;
        lds_cu8* s = (lds_cu8*)(sseq + __builtin_amdgcn_readlane(soff, l));
        lds_cu8* s2 = (lds_cu8*)(sseq + __builtin_amdgcn_readlane(soff, l2));
        one(len, s, lane, acc0, cov0);
        one(len2, s2, lane, acc0, cov0);
        if (max(len, len2) > 128) {
            one(len, s, 64 + lane, acc1, cov1);
            one(len2, s2, 64 + lane, acc1, cov1);
        }
    }
}

// Adds base pair P's counts (c, cov) to the rows of group g0: forward
// (rlen_rev < 0) at positions 2P, 2P+1; reverse at rlen_rev-1-2P and
// rlen_rev-2-2P, complemented.  Zeroes (c, cov).
__device__ __forceinline__ void flush_pair(const ScanArgs& a, lds_u32* lds, int g0, int P, int rlen_rev,
                                           uint64_t& c, uint32_t& cov) {
    if (cov) {
        const int rowstride = a.G * 5;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t n = (cov >> (16 * h)) & 0xFFFFu;
            if (!n) continue;
            const uint32_t w = (uint32_t)(c >> (32 * h));
            const int j = 2 * P + h;
            const int x = rlen_rev < 0 ? j : rlen_rev - 1 - j;
            lds_u32* row = lds + a.lds_base + (x + a.base_start) * rowstride + g0 * 5;
            uint32_t sum = 0;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint32_t k = (w >> (8 * v)) & 0xFFu;
                sum += k;
                if (k) __hip_atomic_fetch_add(row + (rlen_rev < 0 ? v : 3 - v), k, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (n > sum) __hip_atomic_fetch_add(row + 4, n - sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    c = 0;
    cov = 0;
}

__device__ __forceinline__ void count_bases_pairs(lds_cu64* tab, const ScanArgs& a, int64_t r, bool pending,
                                                  bool act, int soff, lds_u32* sseq, lds_u32* lds, int lane,
                                                  int32_t rlen_r, int32_t flag_r) {
    uint64_t pend = __ballot(pending);
    if (!pend) return;
    const int32_t rlen = act ? rlen_r : 0;
    const int32_t fl = act ? flag_r : 0;
    int g = 0;
    for (int f = 0; f < a.n_flags; ++f) g = (g << 1) | ((fl & a.fmask[f]) ? 1 : 0);
    if (!a.base_lds || __ballot(pending && rlen > 256)) {   // BaseHist in global memory, or long reads
        count_bases_lanes(a, pending, rlen, fl, g, soff, sseq, lds);
        return;
    }
    const uint64_t rev = __ballot((fl & 0x10) != 0);
    uint64_t c0 = 0, c1 = 0;
    uint32_t v0 = 0, v1 = 0;
    while (pend) {   // per group of the batch's passing reads (one, normally)
        const int g0 = __builtin_amdgcn_readlane(g, __builtin_ctzll(pend));
        const uint64_t set = pend & __ballot(g == g0);
        pend &= ~set;
        count_set(tab, set & ~rev, rlen, soff, sseq, lane, c0, v0, c1, v1);
        flush_pair(a, lds, g0, lane, -1, c0, v0);
        flush_pair(a, lds, g0, 64 + lane, -1, c1, v1);
        uint64_t rs = set & rev;
        while (rs) {   // reverse strand, per read length (one, normally)
            const int L = __builtin_amdgcn_readlane(rlen, __builtin_ctzll(rs));
            const uint64_t same = rs & __ballot(rlen == L);
            rs &= ~same;
            count_set(tab, same, rlen, soff, sseq, lane, c0, v0, c1, v1);
            flush_pair(a, lds, g0, lane, L, c0, v0);
            flush_pair(a, lds, g0, 64 + lane, L, c1, v1);
        }
    }
}

// Reference positions a read's BaseHist / MirrorHist may read: [lo, hi).
__device__ __forceinline__ void ref_span(const ScanArgs& a, int32_t rlen, int32_t gpos, int32_t flag, int64_t& lo,
                                         int64_t& hi) {
    const bool rev = (flag & 0x10) != 0;
    lo = INT64_MAX;
    hi = INT64_MIN;
    if (a.base_on && gpos >= a.base_start) {
        const int64_t b0 = rev ? (int64_t)gpos - rlen : (int64_t)gpos;
        lo = min(lo, b0);
        hi = max(hi, b0 + rlen);
        if (a.base_start) {
            lo = min(lo, rev ? (int64_t)gpos : (int64_t)gpos - a.base_start);
            hi = max(hi, rev ? (int64_t)gpos + a.base_start : (int64_t)gpos);
        }
    }
    if (a.mir_on) {
        const int64_t p = (int64_t)gpos + a.MOFF;
        if (p >= (int64_t)a.MN - a.MOFF) {
            lo = min(lo, p - a.MN);
            hi = max(hi, p + a.MN + 1);
        }
    }
}

// A batch's accessor columns at read r (the first read of the batch plus
// the lane): loaded for the next batch while the current one is processed
// (MC_SCAN_PREFETCH), so a batch starts without a global round trip.
struct Cols {
    int64_t so = 0, se = 0;
    int32_t rid = -1, rlen = 0, gpos = 0, flag = 0, isz = 0;
};
__device__ __forceinline__ Cols load_cols(const ScanArgs& a, int64_t r, bool valid) {
    Cols c;
    if (valid) {
        c.so = a.seq_off[r];
        c.se = a.seq_off[r + 1];
        c.rid = a.ref_id[r];
        c.rlen = a.rlen[r];
        c.gpos = a.gpos[r];
        c.flag = a.flag[r];
        if (a.isz_on) c.isz = a.gisize[r];
    }
    return c;
}

__device__ __forceinline__ int64_t wave_max(int64_t v) {
    for (int d = 32; d > 0; d >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, d, 64));
    return v;
}

// Copies the 16-byte units [0, nq) of src (16-byte aligned) to dst (LDS,
// 16-byte aligned): every lane's loads issued before the first wait, one
// round trip per batch.  An aligned 16-byte unit never crosses a page, so the
// bytes around a buffer's first and last valid ones are safe to read.
template <int kMaxUnits>
__device__ __forceinline__ void stage16(lds_u32* dst, const u32x4* __restrict__ src, int nq, int lane) {
    constexpr int kPer = (kMaxUnits + 63) / 64;
    constexpr int kRound = kPer < MC_SCAN_STAGE_REGS ? kPer : MC_SCAN_STAGE_REGS;   // units per lane in flight
#pragma unroll 1
    for (int k0 = 0; k0 < kPer && 64 * k0 < nq; k0 += kRound) {
        u32x4 v[kRound];
#pragma unroll
        for (int k = 0; k < kRound; ++k) {
            const int i = lane + 64 * (k0 + k);
            if (i < nq) v[k] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int k = 0; k < kRound; ++k) {
            const int i = lane + 64 * (k0 + k);
            if (i < nq) *((lds_u32x4*)dst + i) = v[k];
        }
    }
}

// One wave walks its slice of reads in batches of up to 64 consecutive
// reads (one lane each) whose packed bases fit the wave's staging buffer:
// the batch's bases (contiguous in HBM) and, when the batch shares one
// reference sequence, the reference window it touches are copied to LDS
// with coalesced dword loads; every per-read access after that is LDS.
// A read too long to stage is processed from global memory.
// The next slice for a wave of workgroup queue `home` (blockIdx % nq; with
// nq dividing the 8 XCDs, the workgroups of one XCD share a queue over a
// contiguous stretch of the reads), else the first queue after it with slices
// left; n_slices when none is.  One queue for all waves made its counter the
// launch's serialisation point: ~11 ns per grab, 4.5 ms of a 100 M-read launch
// with IsizeHist alone (profiles/r06/r06s_scan_queues_ab.txt).  Reading a
// counter before its atomic (MC_SCAN_QPEEK) cost a round trip per grab.
constexpr int kQueueStride = 32;   // counters 128 bytes apart
__device__ __forceinline__ unsigned take_slice(const ScanArgs& a, int home) {
    for (int k = 0; k < a.nq; ++k) {
        const int q = home + k < a.nq ? home + k : home + k - a.nq;
        const unsigned lo = (unsigned)q * a.per_q;
        if (lo >= a.n_slices) continue;
        const unsigned cnt = min(a.per_q, a.n_slices - lo);
        unsigned* ctr = a.work + q * kQueueStride;
        if (MC_SCAN_QPEEK && __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= cnt) continue;
        const unsigned t = atomicAdd(ctr, 1u);
        if (t < cnt) return lo + t;
    }
    return a.n_slices;
}

__global__ __launch_bounds__(kThreads, MC_SCAN_OCC) void scan_kernel(ScanArgs a) {
    extern __shared__ uint32_t lds_[];
    lds_u32* lds = (lds_u32*)lds_;
    for (int i = threadIdx.x; i < a.lds_words; i += kThreads) lds[i] = 0;
    // BaseHist's per-base increment of the packed counters (1 << 12 * nt4,
    // complemented on the reverse strand), after the staging buffers
    lds_u64* inc_tab = (lds_u64*)(lds + a.stage_off + kWaves * (kStageBytes / 4));
    if (threadIdx.x < 32) {
        const int v = nt4_of(threadIdx.x & 15u);
        inc_tab[threadIdx.x] = 1ull << (12 * (threadIdx.x < 16 ? v : comp4(v)));
    }
    lds_u64* pair_tab = inc_tab + kIncTabWords / 2;
    if (MC_SCAN_PAIRS) pair_tab_init(pair_tab);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    lds_u32* sseq = lds + a.stage_off + wave * (kStageBytes / 4);
    lds_u32* sref = sseq + (kSeqStage + kStagePad) / 4;
    const int64_t gw = (int64_t)blockIdx.x * kWaves + wave;
    // which tables read the bases / the reference: a batch stages (and is cut
    // for) only what they read (kmer-only and isize-only runs skip the window)
    const bool need_seq = MC_SCAN_NEED ? (a.base_on || a.kmer_on) : true;
    const bool need_ref = MC_SCAN_NEED ? (a.base_on || a.mir_on) : true;
    // work != null: each wave takes slices of per_wave reads from a queue
    // (a static slice per wave left the kernel waiting on the waves whose
    // slices cover sparse stretches: many short batches); else slice gw
    for (int64_t c = gw;;) {
        if (a.work) {
            unsigned t = 0;
            if (lane == 0) t = take_slice(a, (int)(blockIdx.x % (unsigned)a.nq));
            c = __shfl((int)t, 0, 64);
        }
        int64_t r0 = c * a.per_wave;
        if (r0 >= a.n) break;
        const int64_t rend = min(a.n, r0 + a.per_wave);
        Cols nx = load_cols(a, r0 + lane, r0 + lane < rend);
        // MC_SCAN_PF2: the columns of the 64 reads after the next batch, loaded
        // one batch early; used when the next batch is a whole 64 reads (most
        // batches), so two batches' loads are in flight
        Cols nx2;
        int64_t spec = -1;   // first read of nx2 (-1: none)
        if (MC_SCAN_PF2) {
            nx2 = load_cols(a, r0 + 64 + lane, r0 + 64 + lane < rend);
            spec = r0 + 64;
        }
        while (r0 < rend) {
            const int64_t r = r0 + lane;
            const bool valid = r < rend;
            const Cols cc = nx;
            const int64_t so = cc.so, se = cc.se;
            if (valid && (so & 3)) atomicOr(a.error, 1);
            const int64_t base = __shfl((long long)so, 0, 64);
            const uint64_t fit = __ballot(valid && (!need_seq || se - base <= kSeqStage));
            const int m_seq = fit == ~0ull ? 64 : __builtin_ctzll(~fit);
            // the batch also ends where its reads leave lane 0's sequence or the
            // reference window they touch outgrows kRefStage (inclusive prefix
            // min / max of the reads' spans): a batch over a sparse stretch of a
            // contig used to leave the window unstaged and every base of its
            // reads to global loads (scan C3: 1/3 of the launch)
            const int32_t ridv = cc.rid;
            const int32_t rid0 = __shfl(ridv, 0, 64);
            const bool rid0_ok = rid0 >= 0 && rid0 < a.n_ref;
            int64_t plo = INT64_MAX, phi = INT64_MIN;
            int m_ref = 64;
            if (need_ref) {
                if (valid && rid0_ok) ref_span(a, cc.rlen, cc.gpos, cc.flag, plo, phi);
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int64_t ol = __shfl_up((long long)plo, d, 64), oh = __shfl_up((long long)phi, d, 64);
                    if (lane >= d) {
                        plo = min(plo, ol);
                        phi = max(phi, oh);
                    }
                }
                const int64_t L0 = rid0_ok ? a.ref_len[rid0] : 0;
                const int64_t cwlo = max<int64_t>(plo, 0), cwhi = min<int64_t>(phi, L0);
                const bool wfit = rid0_ok ? ridv == rid0 && (cwhi <= cwlo || cwhi - cwlo <= kRefStage)
                                          : (ridv < 0 || ridv >= a.n_ref);
                const uint64_t wf = __ballot(valid && wfit);
                m_ref = wf == ~0ull ? 64 : __builtin_ctzll(~wf);
            }
            const int m = m_seq == 0 ? 0 : MC_SCAN_CUT ? min(m_seq, max(m_ref, 1)) : m_seq;
            {   // the next batch's columns, in flight while this one is processed
                const int64_t s1 = r0 + max(m, 1), rn = s1 + lane;
                if (MC_SCAN_PF2) {
                    if (spec == s1) nx = nx2;
                    else nx = load_cols(a, rn, rn < rend);
                    nx2 = load_cols(a, rn + 64, rn + 64 < rend);
                    spec = s1 + 64;
                } else if (MC_SCAN_PREFETCH) {
                    nx = load_cols(a, rn, rn < rend);
                } else {
                    nx = load_cols(a, rn, false);
                }
            }
            if (m == 0) {   // the first read alone exceeds the stage: global path
                if (lane == 0) {
                    const int32_t rid = a.ref_id[r];
                    RefWin rw{nullptr, 0, nullptr, 0, 0};
                    if (rid >= 0 && rid < a.n_ref) rw = RefWin{a.ref + a.ref_off[rid], a.ref_len[rid], nullptr, 0, 0};
                    process_read(a, r, a.seq + so, reinterpret_cast<const uint32_t*>(a.seq + so), rw,
                                 lds, false, false, a.rlen[r], a.flag[r], a.gpos[r], a.isz_on ? a.gisize[r] : 0);
                }
                r0 += 1;
                if (!MC_SCAN_PREFETCH) nx = load_cols(a, r0 + lane, r0 + lane < rend);
                continue;
            }
            const bool act = lane < m;
            const int64_t end = __shfl((long long)se, m - 1, 64);
            // stage the batch's bases (sdl: dwords between the staged origin
            // and the batch's first base)
            int sdl = 0;
            if (!need_seq) {
                // (no table reads the bases: nothing staged)
            } else if (MC_SCAN_STAGE16) {
                const uintptr_t g0 = reinterpret_cast<uintptr_t>(a.seq + base), g16 = g0 & ~uintptr_t(15);
                const int nq = (int)((reinterpret_cast<uintptr_t>(a.seq + end) - g16 + 15) >> 4);
                stage16<(kSeqStage + kStagePad) / 16>(sseq, reinterpret_cast<const u32x4*>(g16), nq, lane);
                sdl = (int)(g0 - g16) >> 2;
            } else {
                const uint32_t* g32 = reinterpret_cast<const uint32_t*>(a.seq + (base & ~int64_t(3)));
                const int nwd = (int)((end - (base & ~int64_t(3)) + 3) >> 2);
                for (int i = lane; i < nwd; i += 64) sseq[i] = g32[i];
            }
            // the reference window, when the batch shares one sequence (the
            // prefix span at its last read)
            const int32_t rid = act ? ridv : -1;
            const bool one_ref = __ballot(act && rid != rid0) == 0 && rid0_ok;
            RefWin rw{nullptr, 0, nullptr, 0, 0};
            if (rid >= 0 && rid < a.n_ref) rw = RefWin{a.ref + a.ref_off[rid], a.ref_len[rid], nullptr, 0, 0};
            if (one_ref && need_ref) {
                const int64_t L = a.ref_len[rid0];
                const int64_t wlo = max<int64_t>(__shfl((long long)plo, m - 1, 64), 0);
                const int64_t whi = min<int64_t>(__shfl((long long)phi, m - 1, 64), L);
                if (whi > wlo && whi - wlo <= kRefStage) {
                    const uint8_t* gref = a.ref + a.ref_off[rid0];
                    const uintptr_t ga = reinterpret_cast<uintptr_t>(gref + wlo);
                    if (MC_SCAN_STAGE16) {
                        const uintptr_t g16 = ga & ~uintptr_t(15);
                        const int nq = (int)((whi - wlo + (int64_t)(ga - g16) + 15) >> 4);
                        stage16<(kRefStage + kStagePad) / 16>(sref, reinterpret_cast<const u32x4*>(g16), nq, lane);
                        rw.w = (lds_cu8*)sref + (ga - g16);
                    } else {
                        const uint32_t* q = reinterpret_cast<const uint32_t*>(ga & ~uintptr_t(3));
                        const int nrw = (int)((whi - wlo + (int64_t)(ga & 3) + 3) >> 2);
                        for (int i = lane; i < nrw; i += 64) sref[i] = q[i];
                        rw.w = (lds_cu8*)sref + (ga & 3);
                    }
                    rw.wlo = wlo;
                    rw.whi = whi;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // IsizeHist max, aggregated when the batch is one group
            bool isize_done = false;
            if (a.isz_on && a.isz_lds) {
                int g = 0;
                const int32_t fl = act ? (MC_SCAN_REGCOLS ? cc.flag : a.flag[r]) : 0;
                for (int f = 0; f < a.n_flags; ++f) g = (g << 1) | ((fl & a.fmask[f]) ? 1 : 0);
                const int g0 = __shfl(g, 0, 64);
                if (__ballot(act && g != g0) == 0) {
                    int32_t v = act ? (MC_SCAN_REGCOLS ? cc.isz : a.gisize[r]) : 0;
                    v = v < 0 ? -v : v;
                    if (act)
                        __hip_atomic_fetch_add(lds + a.lds_isz + (int64_t)v * a.G + g, 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                    const int64_t mx = wave_max(act ? (int64_t)v : 0);
                    if (lane == 0)
                        __hip_atomic_fetch_max((__attribute__((address_space(3))) int32_t*)(lds + a.lds_isz_max) + g0,
                                               (int32_t)mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    isize_done = true;
                }
            }
            const int soff = (int)((so - (base & ~int64_t(3))) >> 2) + sdl;   // the read's first dword
            bool pending = false;
            if (act) {
                lds_cu32* rs32 = sseq + soff;
                pending = process_read(a, r, (lds_cu8*)rs32, rs32, rw, lds, true, isize_done,
                                       MC_SCAN_REGCOLS ? cc.rlen : a.rlen[r], MC_SCAN_REGCOLS ? cc.flag : a.flag[r],
                                       MC_SCAN_REGCOLS ? cc.gpos : a.gpos[r],
                                       a.isz_on ? (MC_SCAN_REGCOLS ? cc.isz : a.gisize[r]) : 0);
            }
            if (a.base_on) {
                const int32_t rl = MC_SCAN_REGCOLS ? cc.rlen : act ? a.rlen[r] : 0;
                const int32_t fl = MC_SCAN_REGCOLS ? cc.flag : act ? a.flag[r] : 0;
                if (MC_SCAN_PAIRS) count_bases_pairs(pair_tab, a, r, pending, act, soff, sseq, lds, lane, rl, fl);
                else count_bases(inc_tab, a, r, pending, act, soff, sseq, lds, lane, rl, fl);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            r0 += m;
            if (!MC_SCAN_PREFETCH) nx = load_cols(a, r0 + lane, r0 + lane < rend);
        }
        if (!a.work) break;
    }
    __syncthreads();
    // flush the workgroup's private bins
    for (int i = threadIdx.x; i < a.lds_words; i += kThreads) {
        const uint32_t v = lds[i];
        if (!v) continue;
        if (a.isz_lds && i >= a.lds_isz_max && i < a.lds_isz_max + a.G) {
            atomicMax(a.isz_max + (i - a.lds_isz_max), (int32_t)v);
        } else if (a.base_lds && i >= a.lds_base && i < a.lds_base + a.base_rows * a.G * 5) {
            atomicAdd(a.base + (i - a.lds_base), v);
        } else if (a.mir_lds && i >= a.lds_mir && i < a.lds_mir + a.G * (a.MN + 1) * 2) {
            atomicAdd(a.mir + (i - a.lds_mir), v);
        } else if (a.isz_lds && i >= a.lds_isz && i < a.lds_isz + a.isz_cap * a.G) {
            atomicAdd(a.isz + (i - a.lds_isz), v);
        }
    }
}

// KmerHist counts from the per-read codes scan_kernel wrote (u16,
// kcodes[slot][read], 0xFFFF = read too short).  The table of 4^K+1 bins
// for `spp` slots of one group sits in LDS (u32; K = 7: two slots, 128 KiB),
// so the random-key increments are LDS atomics; blockIdx.y picks the slots,
// blockIdx.z the group.  Each workgroup adds its table into the device's
// slot-major [G][NK][4^K+1] table once: consecutive bins, coalesced.
constexpr int kKmerThreads = 512;
constexpr int kKmerLdsBytes = 160 * 1024;

__global__ __launch_bounds__(kKmerThreads) void kmer_count_kernel(
    const uint16_t* __restrict__ kcodes, const uint16_t* __restrict__ kgroup, int64_t n, int64_t kstride, int NK,
    int nbins, int spp, int G, uint32_t* __restrict__ kmer) {
    extern __shared__ uint32_t t_[];
    lds_u32* t = (lds_u32*)t_;
    const int s0 = blockIdx.y * spp, ns = min(spp, NK - s0), g = blockIdx.z;
    const int words = ns * nbins;
    for (int i = threadIdx.x; i < words; i += kKmerThreads) t[i] = 0;
    __syncthreads();
    // 8 reads' codes per 16-byte load (rows are kstride = n rounded up to 8
    // apart); two steps' loads in flight (one u16 per thread and step was
    // latency-bound: ~3 ms of 100 M reads x 8 slots)
    const int64_t stride = (int64_t)gridDim.x * kKmerThreads * 8;
    auto count8 = [&](lds_u32* tq, int64_t r8, uint4 v, uint4 gr) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        const uint32_t gw[4] = {gr.x, gr.y, gr.z, gr.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const uint32_t c = (w[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
            const uint32_t gg = (gw[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
            if (r8 + e < n && c != 0xFFFFu && (G == 1 || (int)gg == g))
                __hip_atomic_fetch_add(tq + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    for (int q = 0; q < ns; ++q) {
        const uint16_t* row = kcodes + (int64_t)(s0 + q) * kstride;
        lds_u32* tq = t + q * nbins;
        for (int64_t r8 = ((int64_t)blockIdx.x * kKmerThreads + threadIdx.x) * 8; r8 < n; r8 += 2 * stride) {
            const int64_t r8b = r8 + stride;
            const uint4 va = *reinterpret_cast<const uint4*>(row + r8);
            const uint4 vb = r8b < n ? *reinterpret_cast<const uint4*>(row + r8b) : uint4{};
            uint4 ga{}, gb{};
            if (G > 1) {
                ga = *reinterpret_cast<const uint4*>(kgroup + r8);
                if (r8b < n) gb = *reinterpret_cast<const uint4*>(kgroup + r8b);
            }
            count8(tq, r8, va, ga);
            if (r8b < n) count8(tq, r8b, vb, gb);
        }
    }
    __syncthreads();
    uint32_t* out = kmer + ((int64_t)g * NK + s0) * nbins;
    for (int i = threadIdx.x; i < words; i += kKmerThreads) {
        const uint32_t v = t[i];
        if (v) atomicAdd(out + i, v);
    }
}

// mc_scan_run_gpu: idx[i] = i when read i's tid maps to a loaded sequence,
// else -1 (then an inclusive max-scan gives each read the latest such read at
// or before it), and the batch's longest read / largest |insert size|.
__global__ void ref_idx_kernel(const int32_t* __restrict__ tid, int64_t n, const int32_t* __restrict__ map,
                               int32_t n_map, int64_t* __restrict__ idx, const int32_t* __restrict__ rlen,
                               const int32_t* __restrict__ gisize, int* __restrict__ maxes) {
    int mr = 0, mi = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t t = tid[i];
        idx[i] = (t >= 0 && t < n_map && map[t] >= 0) ? i : -1;
        mr = max(mr, rlen[i]);
        const int32_t v = gisize[i];
        mi = max(mi, v < 0 ? -v : v);   // (|INT_MIN| overflows: such a read is out of range anyway)
    }
    for (int d = 32; d > 0; d >>= 1) {
        mr = max(mr, __shfl_xor(mr, d, 64));
        mi = max(mi, __shfl_xor(mi, d, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(maxes, mr);
        atomicMax(maxes + 1, mi);
    }
}

// carry: the reference id in force before this chunk of reads (-1: none)
__global__ void ref_fill_kernel(const int64_t* __restrict__ last, const int32_t* __restrict__ tid, int64_t n,
                                const int32_t* __restrict__ map, int32_t carry, int32_t* __restrict__ ref_id) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = last[i];
        ref_id[i] = j >= 0 ? map[tid[j]] : carry;
    }
}

// nt4 of FASTA bytes (iupac_to_nt4, scan.pyx:37-60)
__global__ void ascii_nt4_kernel(uint8_t* p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    switch (p[i]) {
        case 'A': case 'a': p[i] = 0; break;
        case 'C': case 'c': p[i] = 1; break;
        case 'G': case 'g': p[i] = 2; break;
        case 'T': case 't': p[i] = 3; break;
        default: p[i] = 4;
    }
}

template <typename T>
struct Dev {
    T* p = nullptr;
    size_t cap = 0;
    ~Dev() {
        if (p) (void)hipFree(p);
    }
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) cap = n;
        return e;
    }
};

struct Pinned {
    void* p = nullptr;
    size_t cap = 0;
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
        if (e == hipSuccess) cap = n;
        return e;
    }
};

struct Slot {   // one in-flight batch: pinned staging + device copy
    Pinned host;
    Dev<uint8_t> dev;
    hipEvent_t done = nullptr;
    bool busy = false;
};

}  // namespace

struct mc_scan {
    int device = 0;
    hipStream_t stream = nullptr;
    mc_scan_config cfg{};
    int G = 1;
    int64_t base_rows = 0, isz_cap = 0, kmer_bins = 0;
    int32_t max_rlen = 50;
    int64_t n_reads = 0;
    Dev<uint32_t> base, kmer, mir, isz;
    Dev<int32_t> isz_max;
    Dev<uint8_t> ref;
    Dev<int64_t> ref_off, ref_len;
    Dev<int32_t> error;
    Dev<uint32_t> work;         // scan_kernel's slice queue
    Dev<int64_t> ridx;          // mc_scan_run_gpu: the forward-fill scan
    Dev<int32_t> rid, rmap, rmax;
    Dev<uint8_t> rtemp;
    Dev<uint16_t> kcodes, kgroup;
    int cus = 1;
    int32_t n_ref = 0;
    Slot slot[2];
    int next_slot = 0;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    float kernel_ms = 0;
    int64_t launches = 0;
    int grid = 0;
    ~mc_scan() {
        if (stream) (void)hipStreamSynchronize(stream);
        for (auto& s : slot)
            if (s.done) (void)hipEventDestroy(s.done);
        if (t0) (void)hipEventDestroy(t0);
        if (t1) (void)hipEventDestroy(t1);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

// Grows a [rows][G*w] table to new_rows, keeping its contents.
int grow_rows(mc_scan* s, Dev<uint32_t>& buf, int64_t old_rows, int64_t new_rows, int64_t w) {
    if (new_rows <= old_rows && buf.p) return MC_OK;
    Dev<uint32_t> nb;
    HIP_TRY(nb.reserve((size_t)(new_rows * w)));
    HIP_TRY(hipMemsetAsync(nb.p, 0, (size_t)(new_rows * w) * 4, s->stream));
    if (buf.p && old_rows > 0)
        HIP_TRY(hipMemcpyAsync(nb.p, buf.p, (size_t)(old_rows * w) * 4, hipMemcpyDeviceToDevice,
                               s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    std::swap(buf.p, nb.p);
    std::swap(buf.cap, nb.cap);
    return MC_OK;
}

int ensure_shape(mc_scan* s, int32_t batch_max_rlen, int64_t batch_max_isize) {
    if (s->cfg.base_on && batch_max_rlen > s->max_rlen) {
        const int64_t rows = (int64_t)batch_max_rlen + s->cfg.base_start;
        if (int rc = grow_rows(s, s->base, s->base_rows, rows, (int64_t)s->G * 5)) return rc;
        s->base_rows = rows;
    }
    s->max_rlen = std::max(s->max_rlen, batch_max_rlen);
    if (s->cfg.isize_on && batch_max_isize + 1 > s->isz_cap) {
        int64_t cap = std::max<int64_t>(s->isz_cap, 128);
        while (cap <= batch_max_isize) cap *= 2;
        if (int rc = grow_rows(s, s->isz, s->isz_cap, cap, s->G)) return rc;
        s->isz_cap = cap;
    }
    return MC_OK;
}

// Launch over device-resident batch arrays.
int launch(mc_scan* s, int64_t n, const int32_t* rlen, const int32_t* flag, const int32_t* gpos,
           const int32_t* gisize, const int32_t* ref_id, const int64_t* seq_off,
           const uint8_t* seq) {
    if (n == 0) return MC_OK;
    const mc_scan_config& c = s->cfg;
    ScanArgs a;
    std::memset(&a, 0, sizeof a);
    a.rlen = rlen;
    a.flag = flag;
    a.gpos = gpos;
    a.gisize = gisize;
    a.ref_id = ref_id;
    a.seq_off = seq_off;
    a.seq = seq;
    a.n = n;
    a.ref = s->ref.p ? s->ref.p + kRefPad : nullptr;
    a.ref_off = s->ref_off.p;
    a.ref_len = s->ref_len.p;
    a.n_ref = s->n_ref;
    a.n_flags = c.n_flags;
    for (int i = 0; i < c.n_flags; ++i) a.fmask[i] = c.flags[i];
    a.G = s->G;
    int32_t words = 0;
    auto place = [&](int64_t need, int32_t* off) -> int32_t {
        if (need <= 0 || words + need > kLdsWords) return 0;
        *off = words;
        words += (int32_t)need;
        return 1;
    };
    a.mir_on = c.mirror_on;
    a.MOFF = c.mirror_offset;
    a.MN = c.mirror_n;
    a.mir = s->mir.p;
    if (c.mirror_on) a.mir_lds = place((int64_t)s->G * (c.mirror_n + 1) * 2, &a.lds_mir);
    a.isz_on = c.isize_on;
    a.isz_cap = (int32_t)s->isz_cap;
    a.isz = s->isz.p;
    a.isz_max = s->isz_max.p;
    if (c.isize_on) {
        int32_t off0 = 0, off1 = 0;
        const int32_t w0 = words;
        if (place(s->isz_cap * s->G, &off0) && place(s->G, &off1)) {
            a.isz_lds = 1;
            a.lds_isz = off0;
            a.lds_isz_max = off1;
        } else {
            words = w0;
        }
    }
    a.base_on = c.base_on;
    a.base_start = c.base_start;
    a.base_rows = (int32_t)s->base_rows;
    a.base = s->base.p;
    if (c.base_on) a.base_lds = place(s->base_rows * s->G * 5, &a.lds_base);
    a.kmer_on = c.kmer_on;
    a.K = c.kmer_k;
    a.NK = c.kmer_nk;
    a.STEP = c.kmer_step;
    a.OFF = c.kmer_offset;
    a.kmer = s->kmer.p;
    const int nbins = (1 << (2 * c.kmer_k)) + 1;
    const int spp = c.kmer_on ? std::min(c.kmer_nk, kKmerLdsBytes / (nbins * 4)) : 0;
    if (c.kmer_on && spp >= 1) {       // K <= 7: codes + LDS counting kernel
        a.kstride = (n + 7) & ~int64_t(7);
        HIP_TRY(s->kcodes.reserve((size_t)(a.kstride * c.kmer_nk)));
        a.kcodes = s->kcodes.p;
        if (s->G > 1) {
            HIP_TRY(s->kgroup.reserve((size_t)a.kstride));
            a.kgroup = s->kgroup.p;
        }
    }
    a.lds_words = words;
    if (!a.isz_lds) a.lds_isz_max = kLdsWords;   // outside the arena: never matched by the flush
    a.stage_off = (words + 3) & ~3;
    a.error = s->error.p;
    // one slice of whole 64-read batches per wave
    const int64_t batches = (n + 63) / 64;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((batches + kWaves - 1) / kWaves,
                                                                  s->grid));
    const int64_t waves = (int64_t)grid * kWaves;
    a.per_wave = (batches + waves - 1) / waves * 64;
    if (MC_SCAN_DYN && a.per_wave > 64) {
        a.per_wave = std::min<int64_t>(a.per_wave, kScanSlice);
        const int64_t slices = (n + a.per_wave - 1) / a.per_wave;
        a.nq = (int32_t)std::max<int64_t>(1, std::min<int64_t>(MC_SCAN_QUEUES, slices));
        a.n_slices = (uint32_t)slices;
        a.per_q = (uint32_t)((slices + a.nq - 1) / a.nq);
        HIP_TRY(s->work.reserve((size_t)a.nq * kQueueStride));
        HIP_TRY(hipMemsetAsync(s->work.p, 0, (size_t)a.nq * kQueueStride * 4, s->stream));
        a.work = s->work.p;
    }
    const size_t lds_bytes = (size_t)a.stage_off * 4 + (size_t)kWaves * kStageBytes + kIncTabWords * 4 +
                             (MC_SCAN_PAIRS ? kPairTabWords * 4 : 0);
    hipLaunchKernelGGL(scan_kernel, dim3(grid), dim3(kThreads), lds_bytes, s->stream, a);
    HIP_TRY(hipGetLastError());
    if (a.kcodes) {
        const int passes = (c.kmer_nk + spp - 1) / spp;
        const int64_t wantb = (n + 8 * kKmerThreads - 1) / (8 * kKmerThreads);
        const int gx = (int)std::max<int64_t>(1, std::min<int64_t>(wantb, s->cus));
        hipLaunchKernelGGL(kmer_count_kernel, dim3(gx, passes, s->G), dim3(kKmerThreads),
                           (size_t)spp * nbins * 4, s->stream, a.kcodes, a.kgroup, n, a.kstride, c.kmer_nk,
                           nbins, spp, s->G, s->kmer.p);
        HIP_TRY(hipGetLastError());
    }
    ++s->launches;
    return MC_OK;
}

}  // namespace

extern "C" int mc_scan_create(int device, const mc_scan_config* cfg, mc_scan** out) {
    MC_REQUIRE(cfg && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    MC_REQUIRE(cfg->n_flags >= 0 && cfg->n_flags <= 11, MC_E_RANGE,
               "%d group-by flags (at most the 11 BAM flags)", cfg->n_flags);
    MC_REQUIRE(!cfg->base_on || (cfg->base_start >= 0 && cfg->base_start <= 200), MC_E_RANGE,
               "base offset %d outside 0..200", cfg->base_start);
    MC_REQUIRE(!cfg->kmer_on || (cfg->kmer_k >= 1 && cfg->kmer_k <= 12 && cfg->kmer_nk >= 1 &&
                                 cfg->kmer_nk <= 100 && cfg->kmer_step >= 1 &&
                                 cfg->kmer_step <= 100 && cfg->kmer_offset >= -100 &&
                                 cfg->kmer_offset <= 100),
               MC_E_RANGE, "k-mer histogram parameters out of range");
    MC_REQUIRE(!cfg->mirror_on || (cfg->mirror_n >= 1 && cfg->mirror_n <= 50 &&
                                   cfg->mirror_offset >= -100 && cfg->mirror_offset <= 100),
               MC_E_RANGE, "mirror histogram parameters out of range");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    MC_REQUIRE(device >= 0 && device < ndev, MC_E_HIP, "no HIP device %d (%d present)", device, ndev);
    HIP_TRY(hipSetDevice(device));
    std::unique_ptr<mc_scan> s(new mc_scan());
    s->device = device;
    s->cfg = *cfg;
    s->G = 1 << cfg->n_flags;
    HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&s->t0));
    HIP_TRY(hipEventCreate(&s->t1));
    for (auto& sl : s->slot) HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    s->cus = std::max(1, cus);
    s->grid = s->cus * MC_SCAN_OCC;
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(kmer_count_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kKmerLdsBytes));
    HIP_TRY(s->error.reserve(1));
    HIP_TRY(hipMemsetAsync(s->error.p, 0, 4, s->stream));
    if (cfg->base_on) {
        s->base_rows = (int64_t)s->max_rlen + cfg->base_start;   // set_max_readlen(50)
        HIP_TRY(s->base.reserve((size_t)(s->base_rows * s->G * 5)));
        HIP_TRY(hipMemsetAsync(s->base.p, 0, (size_t)(s->base_rows * s->G * 5) * 4, s->stream));
    }
    if (cfg->kmer_on) {
        s->kmer_bins = ((int64_t(1) << (2 * cfg->kmer_k)) + 1) * cfg->kmer_nk * s->G;
        HIP_TRY(s->kmer.reserve((size_t)s->kmer_bins));
        HIP_TRY(hipMemsetAsync(s->kmer.p, 0, (size_t)s->kmer_bins * 4, s->stream));
    }
    if (cfg->mirror_on) {
        const size_t w = (size_t)s->G * (cfg->mirror_n + 1) * 2;
        HIP_TRY(s->mir.reserve(w));
        HIP_TRY(hipMemsetAsync(s->mir.p, 0, w * 4, s->stream));
    }
    if (cfg->isize_on) {
        s->isz_cap = 128;
        HIP_TRY(s->isz.reserve((size_t)(s->isz_cap * s->G)));
        HIP_TRY(hipMemsetAsync(s->isz.p, 0, (size_t)(s->isz_cap * s->G) * 4, s->stream));
        HIP_TRY(s->isz_max.reserve((size_t)s->G));
        HIP_TRY(hipMemsetAsync(s->isz_max.p, 0, (size_t)s->G * 4, s->stream));
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    *out = s.release();
    return MC_OK;
}

extern "C" int mc_scan_destroy(mc_scan* s) {
    if (s) {
        (void)hipSetDevice(s->device);
        delete s;
    }
    return MC_OK;
}

extern "C" int mc_scan_set_reference(mc_scan* s, int32_t n_seq, const int64_t* off,
                                     const int64_t* len, int64_t n_bytes, const uint8_t* ascii) {
    MC_REQUIRE(s && n_seq >= 0 && (n_seq == 0 || (off && len)) && n_bytes >= 0 &&
                   (n_bytes == 0 || ascii),
               MC_E_INVALID, "bad argument");
    for (int32_t i = 0; i < n_seq; ++i)
        MC_REQUIRE(off[i] >= 0 && len[i] >= 0 && off[i] + len[i] <= n_bytes, MC_E_RANGE,
                   "sequence %d [%lld, +%lld) outside the %lld bytes given", i, (long long)off[i],
                   (long long)len[i], (long long)n_bytes);
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    HIP_TRY(s->ref.reserve((size_t)n_bytes + 2 * kRefPad));
    HIP_TRY(s->ref_off.reserve((size_t)std::max(n_seq, 1)));
    HIP_TRY(s->ref_len.reserve((size_t)std::max(n_seq, 1)));
    HIP_TRY(hipMemset(s->ref.p, 4, (size_t)n_bytes + 2 * kRefPad));
    if (n_bytes) {
        HIP_TRY(hipMemcpy(s->ref.p + kRefPad, ascii, (size_t)n_bytes, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(ascii_nt4_kernel, dim3((unsigned)((n_bytes + 255) / 256)), dim3(256), 0,
                           s->stream, s->ref.p + kRefPad, n_bytes);
        HIP_TRY(hipGetLastError());
    }
    if (n_seq) {
        HIP_TRY(hipMemcpy(s->ref_off.p, off, (size_t)n_seq * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(s->ref_len.p, len, (size_t)n_seq * 8, hipMemcpyHostToDevice));
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->n_ref = n_seq;
    return MC_OK;
}

// Host batch: staged through a pinned slot (two in flight), then one launch.
extern "C" int mc_scan_add_batch(mc_scan* s, int64_t n, const int32_t* rlen, const int32_t* flag,
                                 const int32_t* gpos, const int32_t* gisize, const int32_t* ref_id,
                                 const int64_t* seq_off, const uint8_t* seq) {
    MC_REQUIRE(s && n >= 0, MC_E_INVALID, "bad argument");
    if (n == 0) return MC_OK;
    MC_REQUIRE(rlen && flag && gpos && gisize && ref_id && seq_off && seq, MC_E_INVALID,
               "null array");
    HIP_TRY(hipSetDevice(s->device));
    int32_t mr = 0;
    int64_t mi = 0;
    for (int64_t i = 0; i < n; ++i) {
        MC_REQUIRE(rlen[i] >= 0 && seq_off[i + 1] - seq_off[i] >= ((int64_t)rlen[i] + 1) / 2 &&
                       seq_off[i] >= 0,
                   MC_E_RANGE, "read %lld: %d bases in %lld bytes", (long long)i, rlen[i],
                   (long long)(seq_off[i + 1] - seq_off[i]));
        mr = std::max(mr, rlen[i]);
        const int64_t v = gisize[i] < 0 ? -(int64_t)gisize[i] : gisize[i];
        mi = std::max(mi, v);
    }
    MC_REQUIRE(mi < (int64_t(1) << 28), MC_E_RANGE,
               "insert size %lld too large for a dense histogram", (long long)mi);
    if (int rc = ensure_shape(s, mr, s->cfg.isize_on ? mi : 0)) return rc;
    // the kernel stages bases in dwords: every read's bases start on a
    // 4-byte boundary (the sources emit that; anything else is repacked)
    bool aligned = true;
    int64_t packed = 0;
    for (int64_t i = 0; i < n; ++i) {
        aligned &= (seq_off[i] - seq_off[0]) % 4 == 0;
        packed += (seq_off[i + 1] - seq_off[i] + 3) & ~int64_t(3);
    }
    const int64_t nbytes = aligned ? seq_off[n] - seq_off[0] : packed;
    const size_t cols = (size_t)n * 4, offb = (size_t)(n + 1) * 8;
    const size_t total = 5 * cols + offb + (size_t)nbytes + 16;
    Slot& sl = s->slot[s->next_slot];
    s->next_slot ^= 1;
    if (sl.busy) {
        HIP_TRY(hipEventSynchronize(sl.done));
        sl.busy = false;
    }
    HIP_TRY(sl.host.reserve(total));
    HIP_TRY(sl.dev.reserve(total));
    // staging layout: seq_off (n+1 int64, rebased), 5 int32 columns, bases
    uint8_t* h = static_cast<uint8_t*>(sl.host.p);
    int64_t* ho = reinterpret_cast<int64_t*>(h);
    uint8_t* hc = h + offb;
    std::memcpy(hc, rlen, cols);
    std::memcpy(hc + cols, flag, cols);
    std::memcpy(hc + 2 * cols, gpos, cols);
    std::memcpy(hc + 3 * cols, gisize, cols);
    std::memcpy(hc + 4 * cols, ref_id, cols);
    uint8_t* hs = hc + 5 * cols;
    if (aligned) {
        for (int64_t i = 0; i <= n; ++i) ho[i] = seq_off[i] - seq_off[0];
        std::memcpy(hs, seq + seq_off[0], (size_t)nbytes);
    } else {
        int64_t o = 0;
        for (int64_t i = 0; i < n; ++i) {
            ho[i] = o;
            const int64_t k = seq_off[i + 1] - seq_off[i];
            std::memcpy(hs + o, seq + seq_off[i], (size_t)k);
            std::memset(hs + o + k, 0, (size_t)(((k + 3) & ~int64_t(3)) - k));
            o += (k + 3) & ~int64_t(3);
        }
        ho[n] = o;
    }
    std::memset(hs + nbytes, 0, 16);
    HIP_TRY(hipMemcpyAsync(sl.dev.p, h, total, hipMemcpyHostToDevice, s->stream));
    const uint8_t* d = sl.dev.p + offb;
    HIP_TRY(hipEventRecord(s->t0, s->stream));
    if (int rc = launch(s, n, (const int32_t*)d, (const int32_t*)(d + cols),
                        (const int32_t*)(d + 2 * cols), (const int32_t*)(d + 3 * cols),
                        (const int32_t*)(d + 4 * cols), (const int64_t*)sl.dev.p, d + 5 * cols))
        return rc;
    HIP_TRY(hipEventRecord(s->t1, s->stream));
    HIP_TRY(hipEventRecord(sl.done, s->stream));
    sl.busy = true;
    s->n_reads += n;
    return MC_OK;
}

// Device-resident batch (bench): the caller states the batch's longest read
// and largest |insert size| (the histogram shapes depend on them).
extern "C" int mc_scan_add_batch_device(mc_scan* s, int64_t n, const int32_t* rlen,
                                        const int32_t* flag, const int32_t* gpos,
                                        const int32_t* gisize, const int32_t* ref_id,
                                        const int64_t* seq_off, const uint8_t* seq,
                                        int32_t max_rlen, int64_t max_abs_isize,
                                        float* kernel_ms) {
    MC_REQUIRE(s && n >= 0 && max_rlen >= 0 && max_abs_isize >= 0, MC_E_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(s->device));
    MC_REQUIRE(max_abs_isize < (int64_t(1) << 28), MC_E_RANGE, "insert size too large");
    if (int rc = ensure_shape(s, max_rlen, s->cfg.isize_on ? max_abs_isize : 0)) return rc;
    HIP_TRY(hipEventRecord(s->t0, s->stream));
    if (int rc = launch(s, n, rlen, flag, gpos, gisize, ref_id, seq_off, seq)) return rc;
    HIP_TRY(hipEventRecord(s->t1, s->stream));
    s->n_reads += n;
    if (kernel_ms) {
        HIP_TRY(hipEventSynchronize(s->t1));
        HIP_TRY(hipEventElapsedTime(kernel_ms, s->t0, s->t1));
    }
    return MC_OK;
}

// The source -> GPU loop: batches of `batch_reads` decoded on the host while
// the previous batch's copy and kernel run.  tid_to_ref maps the source's
// reference ids to mc_scan_set_reference sequences (-1: not in the FASTA);
// a record's sequence is that of the latest record at or before it whose
// tid has one (AlignmentFileIterator reloads only on a tid change and keeps
// the old sequence when the new name has none, scan.pyx:213-232).
extern "C" int mc_scan_run(mc_scan* s, mc_scan_src* src, int32_t n_map, const int32_t* tid_to_ref,
                           int64_t max_reads, int64_t batch_reads, int64_t* n_done) {
    MC_REQUIRE(s && src && n_done && n_map >= 0 && (n_map == 0 || tid_to_ref), MC_E_INVALID,
               "bad argument");
    if (batch_reads <= 0) batch_reads = 1 << 21;
    *n_done = 0;
    int32_t last_ref = -1;
    std::vector<int32_t> rid;
    for (;;) {
        int64_t want = batch_reads;
        if (max_reads > 0) want = std::min(want, max_reads - *n_done);
        if (want <= 0) break;
        int64_t n = 0;
        if (int rc = mc_scan_src_next(src, want, int64_t(1) << 30, &n)) return rc;
        if (n == 0) break;
        const int32_t *rlen, *flag, *gpos, *gisize, *tid;
        const int64_t* seq_off;
        const uint8_t* seq;
        if (int rc = mc_scan_src_batch(src, &rlen, &flag, &gpos, &gisize, &tid, &seq_off, &seq,
                                       nullptr))
            return rc;
        rid.resize((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            const int32_t t = tid[i];
            if (t >= 0 && t < n_map && tid_to_ref[t] >= 0) last_ref = tid_to_ref[t];
            rid[i] = last_ref;
        }
        if (int rc = mc_scan_add_batch(s, n, rlen, flag, gpos, gisize, rid.data(), seq_off, seq))
            return rc;
        *n_done += n;
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MC_OK;
}

// The same run over a BAM decoded on the GPU (mc_bam_gpu_open_scan): the
// whole file is one device-resident batch; the reference ids are forward-
// filled on the device (an inclusive max-scan of "latest read whose tid has
// a sequence"), as mc_scan_run does on the host.
extern "C" int mc_scan_run_gpu(mc_scan* s, const mc_bam_gpu* g, int32_t n_map, const int32_t* tid_to_ref,
                               int64_t max_reads, int64_t* n_done) {
    MC_REQUIRE(s && g && n_done && n_map >= 0 && (n_map == 0 || tid_to_ref), MC_E_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(s->device));
    *n_done = 0;
    int64_t n = 0, nbytes = 0;
    const int32_t *rlen, *flag, *gpos, *gisize, *tid;
    const int64_t* seq_off;
    const uint8_t* seq;
    if (int rc = mc_bam_gpu_scan_device(g, &n, &rlen, &flag, &gpos, &gisize, &tid, &seq_off, &seq, &nbytes))
        return rc;
    if (max_reads > 0) n = std::min(n, max_reads);
    hipStream_t st = s->stream;
    // in chunks of up to 2^30 reads (the scan's counts are int32); the
    // forward fill carries the reference id in force across chunks
    int64_t kChunk = int64_t(1) << 30;
    if (const char* e = std::getenv("MC_SCAN_RUN_CHUNK")) kChunk = std::max<int64_t>(1, std::atoll(e));   // (tests)
    const int64_t cmax = std::min(n, kChunk);
    if (n > 0) {
        HIP_TRY(s->ridx.reserve((size_t)cmax));
        HIP_TRY(s->rid.reserve((size_t)cmax));
        HIP_TRY(s->rmap.reserve((size_t)std::max(n_map, 1)));
        HIP_TRY(s->rmax.reserve(2));
        if (n_map) HIP_TRY(hipMemcpyAsync(s->rmap.p, tid_to_ref, (size_t)n_map * 4, hipMemcpyHostToDevice, st));
    }
    int32_t carry = -1;
    for (int64_t c0 = 0; c0 < n; c0 += kChunk) {
        const int64_t m = std::min(kChunk, n - c0);
        HIP_TRY(hipMemsetAsync(s->rmax.p, 0, 8, st));
        const int grid = (int)std::min<int64_t>((m + 255) / 256, (int64_t)s->cus * 8);
        hipLaunchKernelGGL(ref_idx_kernel, dim3(grid), dim3(256), 0, st, tid + c0, m, s->rmap.p, n_map, s->ridx.p,
                           rlen + c0, gisize + c0, s->rmax.p);
        HIP_TRY(hipGetLastError());
        size_t temp = 0;
        HIP_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, temp, s->ridx.p, s->ridx.p, hipcub::Max(), (int)m, st));
        HIP_TRY(s->rtemp.reserve(temp + 16));
        HIP_TRY(hipcub::DeviceScan::InclusiveScan(s->rtemp.p, temp, s->ridx.p, s->ridx.p, hipcub::Max(), (int)m, st));
        hipLaunchKernelGGL(ref_fill_kernel, dim3(grid), dim3(256), 0, st, s->ridx.p, tid + c0, m, s->rmap.p, carry,
                           s->rid.p);
        HIP_TRY(hipGetLastError());
        int mx[2] = {0, 0};
        HIP_TRY(hipMemcpyAsync(mx, s->rmax.p, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&carry, s->rid.p + (m - 1), 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (int rc = mc_scan_add_batch_device(s, m, rlen + c0, flag + c0, gpos + c0, gisize + c0, s->rid.p,
                                              seq_off + c0, seq, mx[0], mx[1], nullptr))
            return rc;
        HIP_TRY(hipStreamSynchronize(st));   // (ridx / rid are reused by the next chunk)
        *n_done += m;
    }
    return MC_OK;
}

extern "C" int mc_scan_dims(mc_scan* s, int32_t* groups, int64_t* base_rows, int64_t* isize_cap,
                            int32_t* max_rlen, int64_t* n_reads) {
    MC_REQUIRE(s, MC_E_INVALID, "null handle");
    if (groups) *groups = s->G;
    if (base_rows) *base_rows = s->base_rows;
    if (isize_cap) *isize_cap = s->isz_cap;
    if (max_rlen) *max_rlen = s->max_rlen;
    if (n_reads) *n_reads = s->n_reads;
    return MC_OK;
}

// Results in the reference's per-processor layouts, group-major:
// base [G][rows][5], kmer [G][4^K+1][NK], mirror [G][N+1][2],
// isize [G][cap] and isize_max [G].  NULL skips a table.
extern "C" int mc_scan_results(mc_scan* s, uint32_t* base, uint32_t* kmer, uint32_t* mirror,
                               uint32_t* isize, int32_t* isize_max) {
    MC_REQUIRE(s, MC_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    int32_t err = 0;
    HIP_TRY(hipMemcpy(&err, s->error.p, 4, hipMemcpyDeviceToHost));
    MC_REQUIRE(err == 0, MC_E_INVALID,
               "a device batch had read bases that do not start on a 4-byte boundary");
    const int G = s->G;
    if (base && s->cfg.base_on) {
        std::vector<uint32_t> t((size_t)(s->base_rows * G * 5));
        HIP_TRY(hipMemcpy(t.data(), s->base.p, t.size() * 4, hipMemcpyDeviceToHost));
        for (int64_t r = 0; r < s->base_rows; ++r)
            for (int g = 0; g < G; ++g)
                std::memcpy(base + ((int64_t)g * s->base_rows + r) * 5, &t[(r * G + g) * 5], 20);
    }
    if (kmer && s->cfg.kmer_on) {   // device [G][NK][bins] -> [G][bins][NK]
        const int64_t nb = (int64_t(1) << (2 * s->cfg.kmer_k)) + 1, NK = s->cfg.kmer_nk;
        std::vector<uint32_t> t((size_t)s->kmer_bins);
        HIP_TRY(hipMemcpy(t.data(), s->kmer.p, t.size() * 4, hipMemcpyDeviceToHost));
        for (int64_t g = 0; g < G; ++g)
            for (int64_t i = 0; i < NK; ++i)
                for (int64_t k = 0; k < nb; ++k)
                    kmer[(g * nb + k) * NK + i] = t[(size_t)((g * NK + i) * nb + k)];
    }
    if (mirror && s->cfg.mirror_on)
        HIP_TRY(hipMemcpy(mirror, s->mir.p, (size_t)G * (s->cfg.mirror_n + 1) * 2 * 4,
                          hipMemcpyDeviceToHost));
    if (s->cfg.isize_on) {
        if (isize) {
            std::vector<uint32_t> t((size_t)(s->isz_cap * G));
            HIP_TRY(hipMemcpy(t.data(), s->isz.p, t.size() * 4, hipMemcpyDeviceToHost));
            for (int64_t a = 0; a < s->isz_cap; ++a)
                for (int g = 0; g < G; ++g) isize[(int64_t)g * s->isz_cap + a] = t[a * G + g];
        }
        if (isize_max)
            HIP_TRY(hipMemcpy(isize_max, s->isz_max.p, (size_t)G * 4, hipMemcpyDeviceToHost));
    }
    return MC_OK;
}

extern "C" int mc_scan_timing(mc_scan* s, float* last_kernel_ms, int64_t* launches) {
    MC_REQUIRE(s, MC_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (last_kernel_ms) HIP_TRY(hipEventElapsedTime(last_kernel_ms, s->t0, s->t1));
    if (launches) *launches = s->launches;
    return MC_OK;
}
