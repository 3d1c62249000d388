// gfx950 kernels of the coverage engine.  Integer work only, HBM-bound:
// no MFMA anywhere (SURVEY.md §8 d: "integer scatter, scan and reduction").
//
//   ingest_kernel        validation + extents + aligned-base count (prepare)
//                        + the BAI-style chunk index (first read of each chunk)
//   cigar_span_kernel    K1: packed BAM CIGAR words -> pileup span
//   depth_kernel         K2: LDS-ring difference array + wave prefix scan
//   region_seg_kernel    K3a: per-segment min/max/sum/sumsq + value histogram
//   region_final_kernel  K3b: exact order statistics from the histogram
//   region_final_wave_kernel  K3b of the fused path: one wave per region
//
// Reference semantics being reproduced: htslib PileupColumn.n under pysam's
// default "all" stepper (called at metacov/pileup.py:13) and the region
// statistics of metacov/pileup.py:18-26.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mc {

// Tuning knobs (compile-time; scripts/ab_inproc.py A/Bs builds of them).
#ifndef MC_TILE_W
#define MC_TILE_W 4096                 // positions per tile (multiple of 1024)
#endif
#ifndef MC_RING
#define MC_RING (2 * MC_TILE_W)        // LDS ring ints (multiple of 256; power of two is cheapest)
#endif
#ifndef MC_TILES_PER_CHUNK
#define MC_TILES_PER_CHUNK 8
#endif
#ifndef MC_PREFETCH
#define MC_PREFETCH 1                  // load read batch k+1 while applying batch k
#endif
#ifndef MC_PREFETCH_STATS
#define MC_PREFETCH_STATS 1            // the same for the fused-statistics K2
#endif
#ifndef MC_APPLY_SHORT
#define MC_APPLY_SHORT 1               // K2 without long reads: one branch per read in the apply loop
                                       // (A/B, profiles/r05/r05ab1: direct C3 1.019 -> 1.002 ms, C2 0.0653 ->
                                       // 0.0611; 2 = no branch, zero adds: 1.004 vs 0.990 ms, r05ab2)
#endif
#ifndef MC_FAR_HALO
#define MC_FAR_HALO 1                  // direct K2: the chunk halo's far part by spans only (far_halo)
#endif
#ifndef MC_FAR_HALO_MIN
#define MC_FAR_HALO_MIN 4096
#endif
#ifndef MC_DIRECT_ONE_CONTIG
#define MC_DIRECT_ONE_CONTIG 1         // direct K2: a batch on the cached contig skips the contig lookup loop
                                       // (C3 1.019 -> 1.007 ms, C2 0.0653 -> 0.0615; both: 0.988 / 0.0558)
#endif
#ifndef MC_K2_WAVE_ADVANCE
#define MC_K2_WAVE_ADVANCE 0           // K2's read batches advance per wave (no block vote in the apply loop)
#endif
#ifndef MC_FILL_WAVE_COUNTS
#define MC_FILL_WAVE_COUNTS 0          // long_fill_words_kernel: one count atomic per distinct tile of a wave
#endif
#ifndef MC_FILL_SORTED
#define MC_FILL_SORTED 0               // long_fill_words_kernel: a round's events grouped by tile in LDS before the stores
                                       // (measured at C5: 0.114 -> 0.128 ms, prepare 0.410 -> 0.421 ms; the 32 KB
                                       // buffer halves the resident workgroups: profiles/r06/r06h_*)
#endif
#ifndef MC_DEFER_LONG
#define MC_DEFER_LONG 1                // the fused long-read K2 defers its tile stores too (in-process A/B,
                                       // C5 K2 median 1.087 -> 1.070 and 1.081 -> 1.072 ms: profiles/r06/r06j_*, r06k_*;
                                       // the fused short-read K2 has no long-read registers to trade and loses 1.6 %)
#endif
#ifndef MC_DEFER_DIRECT
#define MC_DEFER_DIRECT 0              // the fused direct K2 defers its tile stores too (in-process A/B: C3 K2
                                       // 0.990 -> 1.009 ms, C2 0.0527 -> 0.0534: profiles/r06/r06l_*)
#endif
#ifndef MC_NT_STORE
#define MC_NT_STORE 1                  // non-temporal depth stores (written once, not re-read soon)
#endif
#ifndef MC_WAVES_PLAIN
#define MC_WAVES_PLAIN 0               // __launch_bounds__ waves/SIMD, plain K2 (0 = none)
#endif
#ifndef MC_WAVES_STATS
#define MC_WAVES_STATS 4               // __launch_bounds__ waves/SIMD, fused K2 (<= 128 VGPRs)
#endif
// K2 reads each read of a prepared batch as ONE 4-byte word, written by
// ingest_kernel: the low kGposBits bits of its global start (chunk-relative
// starts are exact as the sign-extended difference, since every read K2
// applies starts at most one tile before its chunk or inside it) and its span
// capped at kGspanCap (> short_max, so the cap still marks a long read; K2
// needs a long read's span only to tell that it is one).  In-process A/B
// against (start, span) words (profiles/r02zz_pack_ab_c*.txt): plain K2 C3
// 0.811 -> 0.762 ms, C5 0.848 -> 0.806; against (tid, pos, span) 0.904 ->
// 0.762.  The direct path (probe_kernel) reads the raw tuples instead.
constexpr int kGposBits = 18;
constexpr unsigned kGposMask = (1u << kGposBits) - 1u;
constexpr int kGspanCap = (1 << (32 - kGposBits)) - 1;   // 16383

constexpr int kBlock = 256;            // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr int kTileW = MC_TILE_W;
constexpr int kRing = MC_RING;
static_assert(kRing % 256 == 0 && kRing > kTileW, "ring must hold a tile plus a halo");

// ring slot of a chunk-relative position (the ring is re-zeroed per chunk)
__device__ __forceinline__ int ring_slot(int rel) { return rel % kRing; }
constexpr int kTilesPerChunk = MC_TILES_PER_CHUNK;
// Chunks of a contig set with long reads (C5): twice as long.  Their
// per-chunk costs (the first event and read batches, the histogram flush, the
// carry) weigh more there: C5 K2 1.081 -> 1.057 ms, while C3 loses 2-4 % on
// them (profiles/r03u_chunk16_ab.txt).
#ifndef MC_TILES_PER_CHUNK_LONG
#define MC_TILES_PER_CHUNK_LONG 16
#endif
constexpr int kTilesPerChunkLong = MC_TILES_PER_CHUNK_LONG;
constexpr int kReadsPerThread = 4;     // int4 loads of tid/pos/span
constexpr int kBatch = kBlock * kReadsPerThread;
// K2's workgroup (depth_kernel alone): MC_K2_WAVES waves.  The K2-shape
// micro (profiles/r05/r05g_micro_k2_shape.txt) moves K2's byte mix in 0.79-0.80
// ms with 2 x 512-thread workgroups per CU against 0.92 ms with 4 x 256 at
// the same 16 waves per CU: half as many concurrent chunk streams, each with
// twice the bytes in flight.
#ifndef MC_K2_WAVES
#define MC_K2_WAVES 4
#endif
constexpr int kK2Waves = MC_K2_WAVES;
constexpr int kK2Block = 64 * kK2Waves;
constexpr int kK2Batch = kK2Block * kReadsPerThread;   // reads per K2 batch
constexpr int kPadBatch = kK2Batch > kBatch ? kK2Batch : kBatch;   // read arrays' padding past n
static_assert(kK2Waves == 4 || kK2Waves == 8, "K2 workgroups of 4 or 8 waves");
// K2's LDS header (ints): [0] chunk id, [4, 4 + W) wave totals, [4 + W, 4 +
// 2W) wave maxima, then block_all2's two 8-byte vote words
constexpr int kLdsHeader = (4 + 2 * kK2Waves + 4 + 3) / 4 * 4 > 20 ? (4 + 2 * kK2Waves + 4 + 3) / 4 * 4 : 20;
constexpr int kSeg = 65536;            // K3 segment length (positions)
constexpr int kLdsBins = 16384;        // K3 LDS histogram bins (64 KiB)

typedef int i32x4 __attribute__((ext_vector_type(4)));

struct RegionAcc {                     // K3 per-region accumulator
    unsigned long long sum;
    unsigned long long sumsq;
    int min;
    int max;
};

// ----------------------------------------------------------------- helpers

// Inclusive wave scan on DPP (VALU lane moves, no LDS round trips):
// row_shr 1/2/4/8 scans each row of 16 lanes, row_bcast:15 / :31 carry the
// row totals into the following rows (gfx9 DPP; lanes without a source add
// the `old` operand, 0).
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
    (void)lane;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}

// Sum over the wave, uniform result (DPP scan, then lane 63).
__device__ __forceinline__ int wave_sum_i32(int v) {
    return __builtin_amdgcn_readlane(wave_incl_scan(v, 0), 63);
}

__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// 64-bit lane moves on DPP (two 32-bit halves, same control), for the
// 64-bit scans and sums of the statistics kernels
template <int kCtrl, int kRowMask>
__device__ __forceinline__ long long dpp64(long long v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(v & 0xffffffff), kCtrl, kRowMask, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), kCtrl, kRowMask, 0xf, false);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ long long wave_incl_scan64(long long v) {
    v += dpp64<0x111, 0xf>(v);   // row_shr:1
    v += dpp64<0x112, 0xf>(v);   // row_shr:2
    v += dpp64<0x114, 0xf>(v);   // row_shr:4
    v += dpp64<0x118, 0xf>(v);   // row_shr:8
    v += dpp64<0x142, 0xa>(v);   // row_bcast:15
    v += dpp64<0x143, 0xc>(v);   // row_bcast:31
    return v;
}

__device__ __forceinline__ long long readlane64(long long v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return v;
}

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = min(v, __shfl_xor(v, d, 64));
    return v;
}

// Load at a wave-uniform index through the scalar cache (s_load, counted by
// lgkmcnt).  A per-lane vector load of the same value would need a
// vmcnt wait, which on gfx9 also waits for every store still in flight (K2's
// depth stores).  Only for data no kernel of the launch writes.
template <class T>
__device__ __forceinline__ T uload(const T* p, int64_t i) {
    return ((const __attribute__((address_space(4))) T*)(p))[i];
}

// An LDS value every lane reads alike, made wave-uniform (SGPR) for the compiler.
__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
    const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xffffffff));
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// ----------------------------------------------------------------- ingest

// One streaming pass over the reads (prepare) computes everything K2 needs
// from them besides the long-read buckets:
//   out[0] = invalid records, out[1] = order violations, out[2] = aligned
//   bases, out[3] = max span; maxend[t] = furthest read end of contig t (the
//   host takes max(len, maxend) as the extent); cbases[t] = aligned bases of
//   contig t;
//   the chunk index, for base chunks of width w = 2^lw in the layout coff:
//     index[2k]   = first short read (span <= short_max) crossing k*w, i.e.
//                   starting before it and ending after it (UINT64_MAX: none)
//     index[2k+1] = first read starting at or after (k+1)*w
//   so base chunk k's reads start at min(index[2k], index[2k-1]) (0 for
//   k = 0) and end at index[2k+1].  The fused K2's chunk c is base chunks
//   [c*s, c*s + s).  Reads longer than short_max are the long-read path's.
// The layout is the one prepare expects (extents = contig lengths); when a
// read runs past its contig (maxend > len), the extents grow and prepare runs
// the pass again with the final layout.
//
// Each wave owns a contiguous range of int4 read groups (the arrays are
// padded past n) and walks it kIngestU groups per lane at a time (lane L,
// slot u: group gb + 64u + L, so every load instruction is 1 KiB
// contiguous), the next step's 3 x kIngestU loads in flight while the
// current one is checked.  Nothing is loaded that depends on a load: a
// read's predecessor comes from the neighbouring lane (or the previous slot /
// step), the contig offset of the step's contig(s) by a scalar load, and
// per-contig sums and ends accumulate in registers while the wave stays on
// one contig, one atomic each when it moves on.  Index entries are stores at
// the reads where a chunk boundary falls between two starts (every entry has
// exactly one writer), and one atomicMin per boundary and slot for the first
// crossing read.  (The first ingest gathered len[tid] per read and re-loaded
// each group's predecessor: 0.57 ms per 100 M reads; the index then took two
// more kernels of binary searches and halo scans: 0.24 ms.)
#ifndef MC_INGEST_U
#define MC_INGEST_U 1                  // C3 prepare: 1 0.406, 2 0.426, 4 0.82 ms (VGPR-bound occupancy)
#endif
constexpr int kIngestU = MC_INGEST_U;
#ifndef MC_INGEST_NT_LOAD
// ingest's read loads non-temporal (streamed once): C3 prepare -4.5 %.  The
// same for K2's read batches (plain +3 %), the long-read kernels (+2 %) and
// K1's CIGAR words (+13 %) measured worse.
#define MC_INGEST_NT_LOAD 1
#endif
__device__ __forceinline__ i32x4 ingest_load(const int32_t* p) {
    if (MC_INGEST_NT_LOAD) return __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(p));
    return *reinterpret_cast<const i32x4*>(p);
}

struct IngestAcc {                     // running record of contig cur (wave-uniform)
    int cur = -1;
    long long bases = 0, end = 0;      // per lane, reduced at the flush
};

// every lane calls it (cur is uniform)
__device__ __forceinline__ void ingest_flush(IngestAcc& a, unsigned long long* cbases,
                                             long long* maxend, int lane) {
    if (a.cur >= 0) {
        const long long b = wave_sum64(a.bases);
        long long e = a.end;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) e = max(e, (long long)__shfl_xor(e, d, 64));
        if (lane == 0) {
            if (b) atomicAdd(&cbases[a.cur], (unsigned long long)b);
            atomicMax(&maxend[a.cur], e);
        }
    }
    a.bases = a.end = 0;
}

struct IngestIndex {
    const int64_t* coff;               // [n_contigs + 1] layout of the pass
    int lw;                            // base chunk width 2^lw
    int short_max;
    int64_t n_base;                    // base chunks
    int64_t* index;                    // [2 * n_base]
    // long_count_kernel's counts, folded into this pass when the batch is
    // expected to hold long reads (the previous one did); null: not counted
    unsigned* tile_cnt;                // [n_tiles + 1] end events per tile
    int* chunk_diff;                   // [n_chunks + 1] long reads covering a chunk start (difference form)
    int64_t alloc_len;                 // the depth vector's length
    int lcw;                           // (full) chunk width 2^lcw
    // with the counts: each read's end event as long_fill_words_kernel takes
    // it (its global end, ~0u for a read with no event: short, invalid, past
    // the allocation or ending on a chunk start); null: not written
    uint32_t* end_words;
};

// Per-wave LDS windows of the folded long-read counts: end tiles within 64
// tiles (256 Ki positions) and chunk boundaries within 16 chunks of the
// step's first long read start; farther ones take a global atomic.
constexpr int kIngestTileWin = 64;
constexpr int kIngestChunkWin = 16;

__device__ __forceinline__ int64_t shfl_up_i64(int64_t v) {
    const int lo = __shfl_up((int)(v & 0xffffffff), 1, 64), hi = __shfl_up((int)(v >> 32), 1, 64);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ int64_t readlane_i64(int64_t v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// The wave's long-read count windows into the global counts (every lane of
// the wave calls it; win_tb < 0: nothing placed yet).
__device__ __forceinline__ void ingest_window_flush(const IngestIndex& X, int* wtile, int* wchunk, int64_t win_tb,
                                                    int64_t win_cb, int lane) {
    if (win_tb < 0) return;
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the wave's LDS atomics are done
    const int v = wtile[lane];
    if (v) {
        atomicAdd(&X.tile_cnt[win_tb + lane], (unsigned)v);
        wtile[lane] = 0;
    }
    if (lane < kIngestChunkWin) {
        const int c = wchunk[lane];
        if (c) {
            atomicAdd(&X.chunk_diff[win_cb + lane], c);
            wchunk[lane] = 0;
        }
    }
}

// kCount: the long-read counting compiled in (its registers cost the plain
// pass an occupancy step: 90 -> 111 VGPRs)
template <bool kCount>
__global__ void __launch_bounds__(kBlock)
ingest_kernel(const int32_t* __restrict__ tid, const int32_t* __restrict__ pos,
              const int32_t* __restrict__ span, int64_t n, int32_t n_contigs,
              unsigned long long* __restrict__ out, long long* __restrict__ maxend,
              unsigned long long* __restrict__ cbases, IngestIndex X, uint32_t* __restrict__ gpos) {
    constexpr int U = kIngestU;
    static_assert(kIngestTileWin == 64 && kIngestChunkWin <= 64, "one window entry per lane");
    const int lane = threadIdx.x & 63;
    __shared__ int lw_tiles[kWaves][kIngestTileWin];
    __shared__ int lw_chunks[kWaves][kIngestChunkWin];
    int* wtile = lw_tiles[threadIdx.x >> 6];
    int* wchunk = lw_chunks[threadIdx.x >> 6];
    int64_t win_tb = -1, win_cb = 0;   // the windows' first tile / chunk (-1: not placed)
    if (kCount) {   // (this wave's windows only: no barrier)
        wtile[lane] = 0;
        if (lane < kIngestChunkWin) wchunk[lane] = 0;
    }
    const int64_t n4 = (n + 3) / 4;
    const int64_t n_waves = (int64_t)gridDim.x * kWaves;
    const int64_t gw = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    constexpr int64_t kStep = 64 * U;
    const int64_t per = ((n4 + n_waves - 1) / n_waves + kStep - 1) / kStep * kStep;
    const int64_t g0 = gw * per, g1 = min(n4, g0 + per);
    long long bases = 0;
    unsigned nbad = 0, nuns = 0;
    int mspan = 0;
    IngestAcc acc;
    // the read before the wave's range (every wave checks its first read too);
    // carry_c = -1: none (the first read of all: boundaries from 1 on)
    int carry_t = -1, carry_p = 0, carry_c = -1;   // carry_c: its base chunk
    if (g0 < g1 && g0 > 0) {
        carry_t = uload(tid, g0 * 4 - 1);
        carry_p = uload(pos, g0 * 4 - 1);
        const int carry_s = uload(span, g0 * 4 - 1);
        if (carry_t >= 0 && carry_t < n_contigs && (carry_p | carry_s) >= 0)
            carry_c = (int)((uload(X.coff, carry_t) + carry_p) >> X.lw);
    }
    i32x4 ct[U], cp[U], cs[U], nt[U], np[U], ns[U];
#define MC_INGEST_LOAD(T, P, S, GB)                                                  \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                                  \
        const int64_t q_ = (GB) + 64 * u + lane;                                     \
        const bool in_ = q_ < g1;                                                    \
        const int64_t o_ = in_ ? q_ * 4 : 0;                                         \
        T[u] = ingest_load(tid + o_);                                                \
        P[u] = ingest_load(pos + o_);                                                \
        S[u] = ingest_load(span + o_);                                               \
    }
    if (g0 < g1) { MC_INGEST_LOAD(ct, cp, cs, g0) }
    for (int64_t gb = g0; gb < g1; gb += kStep) {
        if (gb + kStep < g1) { MC_INGEST_LOAD(nt, np, ns, gb + kStep) }
        int tt[4 * U], ps[4 * U], ss[4 * U], tprev[U], pprev[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            tt[4 * u] = ct[u].x; tt[4 * u + 1] = ct[u].y; tt[4 * u + 2] = ct[u].z; tt[4 * u + 3] = ct[u].w;
            ps[4 * u] = cp[u].x; ps[4 * u + 1] = cp[u].y; ps[4 * u + 2] = cp[u].z; ps[4 * u + 3] = cp[u].w;
            ss[4 * u] = cs[u].x; ss[4 * u + 1] = cs[u].y; ss[4 * u + 2] = cs[u].z; ss[4 * u + 3] = cs[u].w;
            // predecessor of this group's first read: lane L-1's last read; lane 0
            // takes the previous slot's lane 63 (or the previous step's)
            const int up_t = __shfl_up(ct[u].w, 1, 64), up_p = __shfl_up(cp[u].w, 1, 64);
            const int l0_t = u ? __builtin_amdgcn_readlane(ct[u - 1].w, 63) : carry_t;
            const int l0_p = u ? __builtin_amdgcn_readlane(cp[u - 1].w, 63) : carry_p;
            tprev[u] = lane ? up_t : l0_t;
            pprev[u] = lane ? up_p : l0_p;
        }
        carry_t = __builtin_amdgcn_readlane(ct[U - 1].w, 63);
        carry_p = __builtin_amdgcn_readlane(cp[U - 1].w, 63);
        // validity and order, branch-free (32-bit per-lane counters)
        unsigned todo = 0;   // bit 4u+k: valid live read
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = gb + 64 * u + lane;
            int tp = tprev[u], pp = pprev[u];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 4 * u + k;
                // past the end: every later slot of the lane is past it too
                const bool live = (q < g1) & (q * 4 + k < n);
                const int t = tt[j], p = ps[j], sp = ss[j];
                const bool ok = ((unsigned)t < (unsigned)n_contigs) & ((p | sp) >= 0);
                const bool uns = (tp > t) | ((tp == t) & (pp > p));
                nbad += (live & !ok) ? 1u : 0u;
                nuns += (live & ok & uns) ? 1u : 0u;
                todo |= (live & ok) ? 1u << j : 0u;
                tp = t;
                pp = p;
            }
        }
        const unsigned valid = todo;
        // per contig of this step (one, unless the wave crosses a boundary):
        // base chunk ids and offsets in 32 bits (contig offset c0 = hi * w +
        // lo, lo < w: the chunk of c0 + p is hi + ((lo + p) >> lw)), bases /
        // max end / max span into the running record
        int cid[4 * U], off[4 * U];
#pragma unroll
        for (int j = 0; j < 4 * U; ++j) cid[j] = off[j] = -1;
        const unsigned wmask = (1u << X.lw) - 1u;
        for (;;) {
            int cand = -1;
#pragma unroll
            for (int j = 4 * U - 1; j >= 0; --j)
                if ((todo >> j) & 1u) cand = tt[j];
            const unsigned long long act = __ballot(cand >= 0);
            if (!act) break;
            const int t0 = __builtin_amdgcn_readlane(cand, __ffsll((long long)act) - 1);
            const int64_t c0 = uload(X.coff, t0);
            const int c0hi = (int)(c0 >> X.lw);
            const unsigned c0lo = (unsigned)c0 & wmask;
            unsigned long long b = 0;
            unsigned e = 0;
            int m = 0;
#pragma unroll
            for (int j = 0; j < 4 * U; ++j) {
                const bool in = ((todo >> j) & 1u) & (tt[j] == t0);
                const unsigned rel = c0lo + (unsigned)ps[j];
                b += in ? (unsigned)ss[j] : 0u;
                e = max(e, in ? (unsigned)ps[j] + (unsigned)ss[j] : 0u);
                m = max(m, in ? ss[j] : 0);
                cid[j] = in ? c0hi + (int)(rel >> X.lw) : cid[j];
                off[j] = in ? (int)(rel & wmask) : off[j];
                todo &= in ? ~(1u << j) : ~0u;
            }
            mspan = max(mspan, m);
            bases += b;
            if (t0 != acc.cur) {
                ingest_flush(acc, cbases, maxend, lane);
                acc.cur = t0;
            }
            acc.bases += b;
            acc.end = max(acc.end, (long long)e);
        }
        if (kCount) {
            // long reads (span > short_max): end event per tile and chunk carry
            // differences, as long_count_kernel counts them (the same rules),
            // into the wave's LDS windows; a window is flushed only when the
            // wave's long reads have moved half its width past its base (a
            // flush per step cost C5's ingest 0.08 ms)
            uint32_t ew[4 * U];
#pragma unroll
            for (int j = 0; j < 4 * U; ++j) ew[j] = ~0u;
            unsigned lng = 0;
#pragma unroll
            for (int j = 0; j < 4 * U; ++j)
                lng |= (((valid >> j) & 1u) && ss[j] > X.short_max) ? 1u << j : 0u;
            const unsigned long long la = __ballot(lng != 0);
            if (la) {
                // the step's first long read (its smallest start when sorted;
                // on unsorted input, which prepare rejects, windows just miss)
                const int jf = lng ? __ffs(lng) - 1 : 0;
                int64_t gl = 0;
#pragma unroll
                for (int j = 0; j < 4 * U; ++j)
                    if (j == jf) gl = ((int64_t)cid[j] << X.lw) + off[j];
                const int64_t gf = readlane_i64(gl, __ffsll((long long)la) - 1);
                const int64_t tb = gf / kTileW;
                if (win_tb < 0 || tb < win_tb || tb - win_tb >= kIngestTileWin / 2) {
                    ingest_window_flush(X, wtile, wchunk, win_tb, win_cb, lane);
                    win_tb = tb;
                    win_cb = gf >> X.lcw;
                }
                const int64_t cmask = ((int64_t)1 << X.lcw) - 1;
#pragma unroll
                for (int j = 0; j < 4 * U; ++j) {
                    if (!((lng >> j) & 1u)) continue;
                    const int64_t g = ((int64_t)cid[j] << X.lw) + off[j];
                    const int64_t ge = g + ss[j];
                    if (ge < X.alloc_len && (ge & cmask)) {   // (an end on a chunk start: no event)
                        const int64_t te = ge / kTileW;
                        if ((uint64_t)(te - win_tb) < (uint64_t)kIngestTileWin) atomicAdd(&wtile[te - win_tb], 1);
                        else atomicAdd(&X.tile_cnt[te], 1u);
                        ew[j] = (uint32_t)ge;
                    }
                    const int64_t c0 = (g >> X.lcw) + 1, c1 = ((ge - 1) >> X.lcw) + 1;
                    if (c1 > c0) {
                        if ((uint64_t)(c0 - win_cb) < (uint64_t)kIngestChunkWin) atomicAdd(&wchunk[c0 - win_cb], 1);
                        else atomicAdd(&X.chunk_diff[c0], 1);
                        if ((uint64_t)(c1 - win_cb) < (uint64_t)kIngestChunkWin) atomicAdd(&wchunk[c1 - win_cb], -1);
                        else atomicAdd(&X.chunk_diff[c1], -1);
                    }
                }
            }
            if (X.end_words) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int64_t q = gb + 64 * u + lane;
                    if (q < g1)
                        *reinterpret_cast<i32x4*>(X.end_words + q * 4) =
                            i32x4{(int)ew[4 * u], (int)ew[4 * u + 1], (int)ew[4 * u + 2], (int)ew[4 * u + 3]};
                }
            }
        }
        if (gpos) {   // K2's read words: start bits (coff[tid] + pos = chunk * w + offset) and span
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t q = gb + 64 * u + lane;
                unsigned g[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    g[k] = ((unsigned)cid[4 * u + k] << X.lw) + (unsigned)off[4 * u + k];
                    g[k] = (g[k] & kGposMask) | ((unsigned)min(ss[4 * u + k], kGspanCap) << kGposBits);
                }
                if (q < g1) {
                    const i32x4 w = i32x4{(int)g[0], (int)g[1], (int)g[2], (int)g[3]};
                    // (non-temporal stores: C3 prepare 0.353 -> 0.368 ms, r02zz_nt_prep.txt)
                    *reinterpret_cast<i32x4*>(gpos + q * 4) = w;
                }
            }
        }
        // chunk index: boundaries m*w with prev < m*w <= g get "first read at
        // or after" = i (usually none between two neighbouring starts); the
        // last read of all also closes every boundary after it with n
        int cprev[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int up = __shfl_up(cid[4 * u + 3], 1, 64);
            const int l0 = u ? __builtin_amdgcn_readlane(cid[4 * u - 1], 63) : carry_c;
            cprev[u] = lane ? up : l0;
        }
        carry_c = __builtin_amdgcn_readlane(cid[4 * U - 1], 63);
        // bit j of bnd: a base chunk boundary lies in (prev start, start]
        // (rare: one read in ~1,600 at C3); bit j of cross: a short read
        // crossing the boundary after its start
        unsigned bnd = 0, cross = 0;
        const int w = 1 << X.lw;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int cp_id = cprev[u];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int j = 4 * u + k;
                const int sp = ss[j];
                const bool ok = (valid >> j) & 1u;   // cid[j] = -1 otherwise
                bnd |= (ok & (cid[j] > cp_id)) ? 1u << j : 0u;
                cross |= (ok & (sp > 0) & (sp <= X.short_max) & (cid[j] + 1 < X.n_base) &
                          (off[j] + sp > w)) ? 1u << j : 0u;
                cp_id = cid[j];
            }
        }
        if (__builtin_expect(__any(bnd != 0), 0)) {
            // boundaries m with prev < m*w <= start get "first read at or after" = i
            while (bnd) {
                const int j = __ffs(bnd) - 1;
                bnd &= bnd - 1;
                const int u = j >> 2, k = j & 3;
                const int64_t i = (gb + 64 * u + lane) * 4 + k;
                int cp = -1, ch = 0;
#pragma unroll
                for (int jj = 0; jj < 4 * U; ++jj)
                    if (jj == j) {
                        cp = (k == 0) ? cprev[u] : cid[jj - 1];
                        ch = cid[jj];
                    }
                const int64_t m_lo = (cp < 0 ? 0 : cp) + 1;
                const int64_t m_hi = ch < X.n_base ? ch : X.n_base;
                for (int64_t mm = m_lo; mm <= m_hi; ++mm) X.index[2 * mm - 1] = i;
            }
        }
        // the last read of all closes every boundary after its start with n
        if (__builtin_expect((gb + kStep) * 4 >= n && gb * 4 < n, 0)) {
#pragma unroll
            for (int j = 0; j < 4 * U; ++j) {
                const int64_t i = (gb + 64 * (j >> 2) + lane) * 4 + (j & 3);
                if (i == n - 1 && ((valid >> j) & 1u))
                    for (int64_t mm = (int64_t)cid[j] + 1; mm <= X.n_base; ++mm) X.index[2 * mm - 1] = n;
            }
        }
        // first crossing read per boundary: per slot, the wave's earliest
        // pending crossing read takes an atomicMin, every later read of the
        // same boundary in the slot is dropped
#pragma unroll
        for (int u = 0; u < U; ++u) {
            unsigned pend = (cross >> (4 * u)) & 0xfu;
            for (;;) {
                int cm = -1, ck = 0;
#pragma unroll
                for (int k = 3; k >= 0; --k)
                    if ((pend >> k) & 1u) {
                        cm = cid[4 * u + k] + 1;
                        ck = k;
                    }
                const unsigned long long act = __ballot(cm >= 0);
                if (!act) break;
                const int leader = __ffsll((long long)act) - 1;
                const int m0 = __builtin_amdgcn_readlane(cm, leader);
                if (lane == leader)
                    atomicMin(reinterpret_cast<unsigned long long*>(&X.index[2 * (int64_t)m0]),
                              (unsigned long long)((gb + 64 * u + lane) * 4 + ck));
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (((pend >> k) & 1u) && cid[4 * u + k] + 1 == m0) pend &= ~(1u << k);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ct[u] = nt[u];
            cp[u] = np[u];
            cs[u] = ns[u];
        }
    }
#undef MC_INGEST_LOAD
    if (kCount) ingest_window_flush(X, wtile, wchunk, win_tb, win_cb, lane);
    ingest_flush(acc, cbases, maxend, lane);
    // one atomic per workgroup and counter: same-address atomics from every
    // wave of the grid serialise at the end of the launch
    __shared__ long long red[4][kWaves];
    const int wave = threadIdx.x >> 6;
    const long long bad = wave_sum64(nbad);
    const long long unsorted = wave_sum64(nuns);
    bases = wave_sum64(bases);
    mspan = wave_max(mspan);
    if (lane == 0) {
        red[0][wave] = bad;
        red[1][wave] = unsorted;
        red[2][wave] = bases;
        red[3][wave] = mspan;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        long long v = red[threadIdx.x][0];
#pragma unroll
        for (int w = 1; w < kWaves; ++w)
            v = threadIdx.x == 3 ? max(v, red[3][w]) : v + red[threadIdx.x][w];
        if (threadIdx.x == 3) atomicMax(&out[3], (unsigned long long)v);
        else if (v) atomicAdd(&out[threadIdx.x], (unsigned long long)v);
    }
}

// ------------------------------------------------------ direct prepare
//
// The per-batch path without the ingest pass.  ingest_kernel streams all
// 12 B/read once before K2 (0.35 ms at C3) only to find each chunk's reads,
// the extents and the per-contig bases.  The direct path gets the chunk
// ranges from a sparse sample instead and lets K2, which reads every read
// anyway, do the validation:
//
//   probe_kernel   one thread per sample (every kProbeStride-th read): its
//                  global start key_j = coff[tid] + pos in the layout the
//                  contig lengths give.  For each chunk-grid target P, J(P) =
//                  the number of samples with key < P is j + 1 exactly when
//                  key_j < P <= key_{j+1}, so thread j writes J for the
//                  targets in that interval (usually none or one): no search.
//                  lb(P), the first read with key >= P, then lies in
//                  ((J-1)*S, J*S].  The same sweep gives each contig's first
//                  sample and the sampled spans' sum (for the histogram
//                  windows: direct_window_base) and flags unsorted or
//                  invalid samples and long spans.
//   depth_kernel<.., kDirect = true>  chunk c loads the reads in
//                  [lower(J(C0 - halo)), upper(J(C0 + W))) as raw
//                  (tid, pos, span), applies those that overlap it, and
//                  validates the reads in [lower(J(C0)), lower(J(C0 + W))):
//                  these ranges partition [0, n) whenever the samples are
//                  sorted (J is monotone), so every read is checked exactly
//                  once (range, order against its predecessor, overhang past
//                  its contig, span <= short_max).
// Anything the direct path cannot represent (unsorted or invalid reads, a
// read past its contig's end, a long read) is reported in DirectRes; the host
// then re-runs the batch through the full prepare, which raises the exact
// errors or builds the extents and long-read buckets.
constexpr int kProbeShift = 8;                 // sample stride S = 256 reads
// Reads starting more than kNearHalo positions before a chunk reach into it
// only with a span above kNearHalo: K2 takes that far part of the chunk's
// halo by spans alone (far_halo), the rest as whole tuples.
constexpr int kNearHalo = 256;
constexpr int kFarHaloMin = MC_FAR_HALO_MIN;   // reads
constexpr int kProbeStride = 1 << kProbeShift;

// dres[]: probe flags (the call's generation stamp, so they need no reset)
// and K2's verdict (zeroed by the probe, or-ed / added by K2's workgroups)
enum : int {
    kDresBadSample = 0,      // gen: an unsorted or invalid sample
    kDresLongSample = 1,     // gen: a sampled span > short_max
    kDresFlags = 2,          // K2: kDirectInvalid | kDirectUnfit
    kDresBases = 3,          // span_sum_kernel: aligned bases (on request)
    kDresMaxSpan = 4,        // K2: the batch's maximum span (atomicMax per workgroup)
    kDresSpanSum = 5,        // probe: sampled spans' sum / count, [5, 6] for even generations, [7, 8] for
    kDresSpanCnt = 6,        //   odd ones (each probe zeroes the other pair for the next batch)
    kDresWords = 9
};
constexpr unsigned kDirectInvalid = 1;   // an invalid or unsorted read: mc_prepare's error
constexpr unsigned kDirectUnfit = 2;     // a read past its contig's end (long reads: kDresMaxSpan)

struct ProbeArgs {
    const int32_t* tid;
    const int32_t* pos;
    const int32_t* span;
    int64_t n;
    int32_t nc;
    const int64_t* coff;               // [nc + 1] layout from the contig lengths
    int lw;                            // grid step w = 2^lw (the plain K2's chunks)
    int short_max;
    int halo;                          // <= short_max: the batch's spans are taken to be <= halo
    int64_t n_base;                    // grid targets k = 0 .. n_base
    int32_t* j0;                       // [n_base + 1] J(k * w)
    int32_t* jh;                       // [n_base + 1] J(k * w - halo)
    int32_t* jn;                       // [n_base + 1] J(k * w - kNearHalo) (MC_FAR_HALO)
    int32_t* fsamp;                    // [nc + 1] first sample of contig t
    unsigned long long* dres;
    unsigned long long gen;
};

// The histogram window of a region on the direct path, from the probe's
// samples: its contig's reads ~ (samples of the contig) x S, the mean span of
// the sampled spans, its depth over the contig less one mean span (the same
// estimate the full prepare makes from exact per-contig bases), kWinBelow
// bins of the window below it.  K2 and K3b both evaluate it, bit for bit
// alike (a window_kernel launch between the probe and K2 was 0.012 ms of a
// C3 step with its gap).
struct DirectWindow {
    const int32_t* fsamp;              // [nc + 1] first sample of each contig (probe)
    const int64_t* len;                // [nc]
    const unsigned long long* dres;    // the span sums of this generation at [kDresSpanSum + 2 * parity]
    int parity;
    int win_below;
};

// (parity: this call's; W.parity is unused by K2, which takes it by value)
template <class WT>
__device__ __forceinline__ int direct_window_base(const WT& W, int parity, int t) {
    const long long ns = (long long)uload(W.fsamp, t + 1) - uload(W.fsamp, t);
    const unsigned long long ssum = uload(W.dres, kDresSpanSum + 2 * parity);
    const unsigned long long scnt = uload(W.dres, kDresSpanCnt + 2 * parity);
    if (ns <= 0 || scnt == 0) return 0;
    const double mean = (double)ssum / (double)scnt;
    const double bases = (double)ns * (double)kProbeStride * mean;
    const double ext = (double)uload(W.len, t);
    const double body = ext > 2.0 * mean ? ext - mean : ext;
    const double est = ext > 0 ? bases / body : 0.0;
    const long long b0 = llrint(est) - W.win_below;
    return b0 > 0 ? (int)b0 : 0;
}

__device__ __forceinline__ int64_t probe_key(const ProbeArgs& A, int t, int p) {
    const int ct = t < 0 ? 0 : t >= A.nc ? A.nc - 1 : t;
    const int64_t k = A.coff[ct] + (int64_t)(p < 0 ? 0 : p);
    return k;
}

// J(P) = j + 1 for the targets k of one grid with key_j < P(k) <= key_next,
// P(k) = k * w - off: k in [(key_j + off) >> lw + 1, (key_next + off) >> lw]
__device__ __forceinline__ void probe_fill(int32_t* J, int64_t n_base, int lw, int64_t off, int64_t key,
                                           int64_t key_next, bool first, bool last, int32_t val) {
    int64_t k0 = first ? 0 : ((key + off) >> lw) + 1;
    int64_t k1 = last ? n_base : ((key_next + off) >> lw);
    if (k1 > n_base) k1 = n_base;
    if (first) {   // targets at or below the first sample: J = 0
        int64_t kz = (key + off) >> lw;
        if (kz > n_base) kz = n_base;
        for (int64_t k = 0; k <= kz; ++k) J[k] = 0;
        k0 = kz + 1;
    }
    for (int64_t k = k0; k <= k1; ++k) J[k] = val;
}

// probe_kernel samples every read's (tid, pos) at stride S, its span at
// stride 4 S (only the long-read flag reads it: a long read the sparser
// sample misses is still caught by K2's check)
constexpr int kProbeSpanEvery = 4;
constexpr unsigned kProbeMeanBlocks = 64;

__global__ void __launch_bounds__(kBlock)
probe_kernel(ProbeArgs A) {
    const int64_t M = (A.n + kProbeStride - 1) >> kProbeShift;
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int par = (int)(A.gen & 1);
    // K2's counters (K2 runs after this launch) and the next generation's span sums
    if (blockIdx.x == 0 && threadIdx.x >= kDresFlags && threadIdx.x <= kDresMaxSpan) A.dres[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x < 2) A.dres[kDresSpanSum + 2 * (par ^ 1) + threadIdx.x] = 0;
    const bool sampled = j < M && (j % kProbeSpanEvery) == 0;
    const int s0 = sampled ? A.span[j << kProbeShift] : 0;
    // the mean span for the windows: the sampled spans of kProbeMeanBlocks
    // workgroups spread over the batch, one atomic pair per workgroup (one
    // pair per wave of all workgroups, on one address, serialised: +0.1 ms)
    const unsigned every = max(1u, gridDim.x / kProbeMeanBlocks);
    if (blockIdx.x % every == 0) {
        __shared__ long long red[2 * kWaves];
        const bool s_ok = sampled && s0 >= 0;
        const long long wsum = wave_sum64(s_ok ? (long long)s0 : 0);
        const long long wcnt = wave_sum64(s_ok ? 1 : 0);
        if ((threadIdx.x & 63) == 0) {
            red[threadIdx.x >> 6] = wsum;
            red[kWaves + (threadIdx.x >> 6)] = wcnt;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            long long ts = 0, tc = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) {
                ts += red[w];
                tc += red[kWaves + w];
            }
            if (tc) {
                atomicAdd(&A.dres[kDresSpanSum + 2 * par], (unsigned long long)ts);
                atomicAdd(&A.dres[kDresSpanCnt + 2 * par], (unsigned long long)tc);
            }
        }
    }
    if (j >= M) return;
    const bool last = j == M - 1;
    // this sample and the next one, all loads issued together (the next
    // sample's from the neighbouring lane would leave lane 63 a second round trip)
    const int64_t i = j << kProbeShift, i1 = last ? i : i + kProbeStride;
    const int t = A.tid[i], p = A.pos[i];
    const int t_next = A.tid[i1], p_next = A.pos[i1];
    const int s = s0;
    const int64_t key = probe_key(A, t, p);
    const int64_t key_next = probe_key(A, t_next, p_next);
    const bool bad = ((unsigned)t >= (unsigned)A.nc) | (p < 0) | (s < 0);
    const bool uns = !last && ((t > t_next) | ((t == t_next) & (p > p_next)) | (key > key_next));
    if (bad | uns) atomicMax(&A.dres[kDresBadSample], A.gen);
    if (s > A.short_max) atomicMax(&A.dres[kDresLongSample], A.gen);
    const bool first = j == 0;
    probe_fill(A.j0, A.n_base, A.lw, 0, key, key_next, first, last, (int32_t)(j + 1));
    probe_fill(A.jh, A.n_base, A.lw, A.halo, key, key_next, first, last, (int32_t)(j + 1));
    if (MC_FAR_HALO) probe_fill(A.jn, A.n_base, A.lw, kNearHalo, key, key_next, first, last, (int32_t)(j + 1));
    // contigs (tid_j, tid_next] start after sample j
    const int ct = t < 0 ? 0 : t >= A.nc ? A.nc - 1 : t;
    const int cn = last ? A.nc : (t_next < 0 ? 0 : t_next >= A.nc ? A.nc - 1 : t_next);
    if (first)
        for (int k = 0; k <= ct; ++k) A.fsamp[k] = 0;
    for (int k = ct + 1; k <= cn; ++k) A.fsamp[k] = (int32_t)(j + 1);
}

// The full prepare's window bases on the device (a repeated call over the
// same layout with a new batch): the estimate the host makes at staging time
// (depth over the contig less one mean read span, kWinBelow bins of the
// window below it) from ingest's per-contig bases, with the contig length
// for the extent.  One thread per region row.
__global__ void __launch_bounds__(kBlock)
window_bases_kernel(const unsigned long long* __restrict__ ingest_out, const unsigned long long* __restrict__ cbases,
                    int64_t n, const int64_t* __restrict__ len, const int32_t* __restrict__ rtid,
                    const int32_t* __restrict__ rfused, int64_t R, int win_below, int32_t* __restrict__ brow,
                    int32_t* __restrict__ fbase) {
    const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (r >= R) return;
    const int t = rtid[r];
    const double mean = n > 0 ? (double)ingest_out[2] / (double)n : 0.0;
    const double ext = (double)len[t];
    const double body = ext > 2.0 * mean ? ext - mean : ext;
    const double est = ext > 0 ? (double)cbases[t] / body : 0.0;
    const long long b0 = llrint(est) - win_below;
    const int32_t base = (int32_t)(b0 > 0 ? b0 : 0);
    brow[r] = base;
    const int32_t k = rfused[r];
    if (k >= 0) fbase[k] = base;
}

// Prepare's buffer setup in one launch (three fills were three commands in
// the stream ahead of ingest_kernel): the tid padding K2's whole-batch loads
// read past n (zeros: a valid contig), the ingest counters / ends / bases
// (zeros) and the chunk index (all ones: no crossing read yet; zeros when
// there are no reads).
__global__ void __launch_bounds__(kBlock)
prep_clear_kernel(int32_t* __restrict__ tid_pad, int64_t n_pad, unsigned long long* __restrict__ scratch,
                  int64_t n_scratch, unsigned long long* __restrict__ index, int64_t n_index,
                  unsigned long long index_fill, int32_t* __restrict__ zero32, int64_t n_zero32,
                  int32_t* __restrict__ zero32b, int64_t n_zero32b) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int64_t e1 = n_pad + n_scratch, e2 = e1 + n_index, e3 = e2 + n_zero32, e4 = e3 + n_zero32b;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < e4; i += stride) {
        if (i < n_pad) tid_pad[i] = 0;
        else if (i < e1) scratch[i - n_pad] = 0;
        else if (i < e2) index[i - e1] = index_fill;
        else if (i < e3) zero32[i - e2] = 0;          // (the folded long-read counts)
        else zero32b[i - e3] = 0;
    }
}

// ------------------------------------------------------ long reads (prepare)
//
// Reads longer than `short_max` (= ring - kTileW) cannot keep their -1 end
// event in the LDS ring.  For them:
//   * +1 is applied by K2 in-stream at the read start (its own chunk only);
//   * -1 goes to an end-event bucket of the tile holding the end (CSR over
//     tiles: long_count_kernel counts, long_scan_kernel turns the counts into
//     offsets, long_fill_kernel fills; K2 streams a chunk's events in tile
//     order);
//   * chunk_diff builds the count of long reads covering each chunk's first
//     position that started in an earlier chunk (K2's initial carry).
//
// Each workgroup walks a contiguous range of reads in sub-ranges of
// kLongSub reads (16 per thread, int4 loads).  Reads are sorted by start, so
// a sub-range's end events fall in a short run of tiles from the tile of its
// first start: they are counted in an LDS window of kLongTileWin tiles (and
// kLongChunkWin chunks for the carries), then flushed with one global atomic
// per non-empty bin; an event past the window goes straight to global memory.
// The fill pass reserves each bin's slots with one atomic per bin and ranks
// the sub-range's events inside it with LDS atomics.  (Per-wave ballot
// grouping with a returning global atomic per 64 reads was latency-bound:
// 0.35 + 0.39 ms for C5's 47 M long reads, plus a host round trip for the
// offsets.)
#ifndef MC_LONG_PER
#define MC_LONG_PER 4                  // C5 prepare: 4 0.606, 8 0.612, 16 0.674 ms (profiles/r02za_long_per.txt)
#endif
constexpr int kLongPer = MC_LONG_PER;             // reads per thread and sub-range
constexpr int kLongSub = kBlock * kLongPer;
constexpr int kLongTileWin = 256;                 // 1 Mi positions past the sub-range's first start
constexpr int kLongChunkWin = 64;

struct LongGeo {
    const int32_t* tid;
    const int32_t* pos;
    const int32_t* span;
    int64_t n;
    const int64_t* coff;
    int short_max;
    int64_t alloc_len;
    int lcw;                                      // chunk width 2^lcw
    int64_t per;                                  // reads per workgroup (multiple of kLongSub)
};

struct LongRaw {                                  // a thread's reads of one sub-range, as loaded
    i32x4 t[kLongPer / 4], p[kLongPer / 4], s[kLongPer / 4];
};

// this thread's reads of the sub-range at `sub`: read sub + (v * kBlock +
// threadIdx.x) * 4 + k (the read arrays are padded by a batch past n)
__device__ __forceinline__ void long_issue(const LongGeo& G, int64_t sub, int64_t r1, LongRaw& r) {
#pragma unroll
    for (int v = 0; v < kLongPer / 4; ++v) {
        const int64_t i0 = sub + ((int64_t)v * kBlock + threadIdx.x) * 4;
        const int64_t o = i0 < r1 ? i0 : 0;
        r.t[v] = *reinterpret_cast<const i32x4*>(G.tid + o);
        r.p[v] = *reinterpret_cast<const i32x4*>(G.pos + o);
        r.s[v] = *reinterpret_cast<const i32x4*>(G.span + o);
    }
}

// Global starts and spans of the loaded reads; live = bit mask of the long
// reads below r1.  Contig offsets by scalar loads per distinct contig of the
// wave (one or two per sub-range).
__device__ __forceinline__ void long_finish(const LongGeo& G, int64_t sub, int64_t r1, const LongRaw& r,
                                            int64_t (&g)[kLongPer], int (&sp)[kLongPer], unsigned& live) {
    int tt[kLongPer], pp[kLongPer];
    live = 0;
#pragma unroll
    for (int v = 0; v < kLongPer / 4; ++v) {
        const int64_t i0 = sub + ((int64_t)v * kBlock + threadIdx.x) * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            tt[4 * v + k] = r.t[v][k];
            pp[4 * v + k] = r.p[v][k];
            sp[4 * v + k] = r.s[v][k];
            if (i0 + k < r1 && r.s[v][k] > G.short_max) live |= 1u << (4 * v + k);
        }
    }
    unsigned todo = live;
    for (;;) {
        int cand = -1;
#pragma unroll
        for (int j = kLongPer - 1; j >= 0; --j)
            if ((todo >> j) & 1u) cand = tt[j];
        const unsigned long long act = __ballot(cand >= 0);
        if (!act) break;
        const int t0 = __builtin_amdgcn_readlane(cand, __ffsll((long long)act) - 1);
        const int64_t c = uload(G.coff, t0);
#pragma unroll
        for (int j = 0; j < kLongPer; ++j)
            if (((todo >> j) & 1u) && tt[j] == t0) {
                g[j] = c + pp[j];
                todo &= ~(1u << j);
            }
    }
}

// global start of read i (wave-uniform i): the sub-range's window base
__device__ __forceinline__ int64_t long_first_start(const LongGeo& G, int64_t i) {
    return uload(G.coff, uload(G.tid, i)) + uload(G.pos, i);
}

// the tile of read j's end event, or -1 (past the allocation, or exactly on
// a chunk start, where the next chunk's carry already excludes it)
__device__ __forceinline__ int64_t long_end_tile(const LongGeo& G, int64_t ge) {
    return (ge < G.alloc_len && (ge & (((int64_t)1 << G.lcw) - 1))) ? ge / kTileW : -1;
}

// Sub-range loop shared by the count and fill passes: the next sub-range's
// loads are in flight while the current one is counted / filled.
template <class F>
__device__ __forceinline__ void long_walk(const LongGeo& G, F&& body) {
    const int64_t r0 = blockIdx.x * G.per, r1 = min(G.n, r0 + G.per);
    LongRaw cur, nxt;
    if (r0 < r1) long_issue(G, r0, r1, cur);
    for (int64_t sub = r0; sub < r1; sub += kLongSub) {
        if (sub + kLongSub < r1) long_issue(G, sub + kLongSub, r1, nxt);
        int64_t g[kLongPer];
        int sp[kLongPer];
        unsigned live;
        long_finish(G, sub, r1, cur, g, sp, live);
        body(sub, g, sp, live);
        cur = nxt;
    }
}

__global__ void __launch_bounds__(kBlock)
long_count_kernel(LongGeo G, unsigned* __restrict__ tile_cnt, int* __restrict__ chunk_diff) {
    __shared__ int wt[kLongTileWin];
    __shared__ int wc[kLongChunkWin];
    for (int k = threadIdx.x; k < kLongTileWin; k += kBlock) wt[k] = 0;
    for (int k = threadIdx.x; k < kLongChunkWin; k += kBlock) wc[k] = 0;
    __syncthreads();
    long_walk(G, [&](int64_t sub, const int64_t (&g)[kLongPer], const int (&sp)[kLongPer], unsigned live) {
        const int64_t gf = long_first_start(G, sub);
        const int64_t TB = gf / kTileW, CB = gf >> G.lcw;
#pragma unroll
        for (int j = 0; j < kLongPer; ++j) {
            if (!((live >> j) & 1u)) continue;
            const int64_t ge = g[j] + sp[j];
            const int64_t te = long_end_tile(G, ge);
            if (te >= 0) {
                if (te - TB < kLongTileWin) atomicAdd(&wt[te - TB], 1);
                else atomicAdd(&tile_cnt[te], 1u);
            }
            const int64_t c0 = (g[j] >> G.lcw) + 1, c1 = ((ge - 1) >> G.lcw) + 1;
            if (c1 > c0) {
                if (c0 - CB < kLongChunkWin) atomicAdd(&wc[c0 - CB], 1);
                else atomicAdd(&chunk_diff[c0], 1);
                if (c1 - CB < kLongChunkWin) atomicAdd(&wc[c1 - CB], -1);
                else atomicAdd(&chunk_diff[c1], -1);
            }
        }
        __syncthreads();
        for (int k = threadIdx.x; k < kLongTileWin; k += kBlock) {
            const int v = wt[k];
            if (v) {
                atomicAdd(&tile_cnt[TB + k], (unsigned)v);
                wt[k] = 0;
            }
        }
        for (int k = threadIdx.x; k < kLongChunkWin; k += kBlock) {
            const int v = wc[k];
            if (v) {
                atomicAdd(&chunk_diff[CB + k], v);
                wc[k] = 0;
            }
        }
        __syncthreads();
    });
}

// tile_off = exclusive prefix of tile_cnt (n_tiles + 1 entries), tile_cnt
// zeroed (the fill pass's cursors), chunk_diff turned into the per-chunk
// carry (inclusive prefix, in place): a reduce-then-scan over segments of
// kScanSeg entries, the first bt blocks on the tiles, the next on the chunks.
constexpr int kScanPer = 16;
constexpr int kScanSeg = kBlock * kScanPer;

struct ScanArgs {
    unsigned* tile_cnt;
    int64_t n_tiles;
    int64_t* tile_off;
    int* chunk;
    int64_t n_chunks;
    long long* partial;                            // [bt + bc]
    int bt;
};

__device__ __forceinline__ long long block_sum_ll(long long v, long long* red) {
    v = wave_sum64(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    long long t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += red[w];
    __syncthreads();
    return t;
}

__global__ void __launch_bounds__(kBlock)
long_scan_partial_kernel(ScanArgs A) {
    __shared__ long long red[kWaves];
    const bool tiles = (int)blockIdx.x < A.bt;
    const int64_t b = tiles ? blockIdx.x : blockIdx.x - A.bt;
    const int64_t N = tiles ? A.n_tiles : A.n_chunks;
    long long v = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = b * kScanSeg + (int64_t)k * kBlock + threadIdx.x;
        if (i < N) v += tiles ? (long long)A.tile_cnt[i] : (long long)A.chunk[i];
    }
    v = block_sum_ll(v, red);
    if (threadIdx.x == 0) A.partial[blockIdx.x] = v;
}

__global__ void __launch_bounds__(kBlock)
long_scan_final_kernel(ScanArgs A) {
    __shared__ long long red[kWaves];
    const bool tiles = (int)blockIdx.x < A.bt;
    const int64_t b = tiles ? blockIdx.x : blockIdx.x - A.bt;
    const int64_t N = tiles ? A.n_tiles : A.n_chunks;
    const int p0 = tiles ? 0 : A.bt;
    long long pre = 0;                             // the segments before this one
    for (int q = p0 + threadIdx.x; q < (int)blockIdx.x; q += kBlock) pre += A.partial[q];
    pre = block_sum_ll(pre, red);
    // this thread's kScanPer consecutive entries
    const int64_t i0 = b * kScanSeg + (int64_t)threadIdx.x * kScanPer;
    long long x[kScanPer], tot = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = i0 + k;
        x[k] = i < N ? (tiles ? (long long)A.tile_cnt[i] : (long long)A.chunk[i]) : 0;
        tot += x[k];
    }
    // exclusive block scan of the thread totals (64-bit wave scans + wave carries)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    long long incl = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const long long y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) red[wave] = incl;
    __syncthreads();
    long long run = pre + incl - tot;
    for (int w = 0; w < wave; ++w) run += red[w];
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = i0 + k;
        if (i >= N) break;
        if (tiles) {
            A.tile_off[i] = run;
            A.tile_cnt[i] = 0;
            run += x[k];
        } else {
            run += x[k];
            A.chunk[i] = (int)run;                // inclusive
        }
    }
    if (tiles && i0 < N && i0 + kScanPer >= N) A.tile_off[N] = run;   // the thread holding the last tile
}

__global__ void __launch_bounds__(kBlock)
long_fill_kernel(LongGeo G, const int64_t* __restrict__ tile_off, unsigned* __restrict__ cursor,
                 int32_t* __restrict__ ev) {
    __shared__ int wt[kLongTileWin];      // counts, then ranks
    __shared__ int wb[kLongTileWin];      // first slot of the sub-range's events per tile
    const int64_t cmask = ((int64_t)1 << G.lcw) - 1;
    for (int k = threadIdx.x; k < kLongTileWin; k += kBlock) wt[k] = 0;
    __syncthreads();
    long_walk(G, [&](int64_t sub, const int64_t (&g)[kLongPer], const int (&sp)[kLongPer], unsigned live) {
        const int64_t TB = long_first_start(G, sub) / kTileW;
        int te[kLongPer];                  // window bin, or -1
#pragma unroll
        for (int j = 0; j < kLongPer; ++j) {
            te[j] = -1;
            if (!((live >> j) & 1u)) continue;
            const int64_t t = long_end_tile(G, g[j] + sp[j]);
            if (t < 0) {
                live &= ~(1u << j);
            } else if (t - TB < kLongTileWin) {
                te[j] = (int)(t - TB);
                atomicAdd(&wt[te[j]], 1);
            }
        }
        __syncthreads();
        for (int k = threadIdx.x; k < kLongTileWin; k += kBlock) {
            const int v = wt[k];
            if (v) {
                wb[k] = (int)(tile_off[TB + k] + atomicAdd(&cursor[TB + k], (unsigned)v));
                wt[k] = 0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kLongPer; ++j) {
            if (!((live >> j) & 1u)) continue;
            const int64_t ge = g[j] + sp[j];
            int64_t slot;
            if (te[j] >= 0) {
                slot = wb[te[j]] + atomicAdd(&wt[te[j]], 1);
            } else {
                const int64_t t = ge / kTileW;
                slot = tile_off[t] + atomicAdd(&cursor[t], 1u);
            }
            ev[slot] = (int32_t)(ge & cmask);   // chunk-relative end
        }
        __syncthreads();
        for (int k = threadIdx.x; k < kLongTileWin; k += kBlock) wt[k] = 0;
        __syncthreads();
    });
}

// The fill pass on the end words ingest_kernel<true> wrote (4 B per read
// instead of the 12 B tuples long_fill_kernel re-reads: 0.2 instead of 0.6
// GB at C5).  Same buckets and slots.  A round takes kFillSubs sub-ranges
// (kFillSubs int4 of end words per thread) and its window starts at the tile
// of its smallest end (ends are not sorted, starts are).  The count atomics
// return each event's rank in its tile (round 3 took the ranks in a second
// atomic pass; SQ: LDS bank-conflict cycles 2.5x the LDS-active cycles, waves
// waiting on LDS 36 % of their cycles): C5 call 1.670 -> 1.634 ms.  Measured
// and dropped: one or eight sub-ranges per round (no change), counters striped
// over 8 / 16 lanes (1.680 / 1.686 ms; profiles/r04/r04o_long_fill_ab.txt).
constexpr int kFillSubs = 4;

__global__ void __launch_bounds__(kBlock)
long_fill_words_kernel(const uint32_t* __restrict__ ew, int64_t n, int64_t per, int lcw,
                       const int64_t* __restrict__ tile_off, unsigned* __restrict__ cursor,
                       int32_t* __restrict__ ev) {
    static_assert(kLongPer == 4, "one int4 of end words per thread and sub-range");
    constexpr int kE = 4 * kFillSubs;     // end words per thread and round
    __shared__ int wt[kLongTileWin];      // per window tile: count (ranks come back from the atomics)
    __shared__ int wb[kLongTileWin];      // per window tile: first slot
    __shared__ unsigned red[kWaves];
    // MC_FILL_SORTED: per window tile its first position in the round's LDS
    // event buffer; the buffer (values and their global slots)
    __shared__ int wc[MC_FILL_SORTED ? kLongTileWin : 1];
    __shared__ int32_t sbuf[MC_FILL_SORTED ? kBlock * 4 * kFillSubs : 1];
    __shared__ int32_t sslot[MC_FILL_SORTED ? kBlock * 4 * kFillSubs : 1];
    const int64_t cmask = ((int64_t)1 << lcw) - 1;
    for (int k = threadIdx.x; k < kLongTileWin; k += kBlock) wt[k] = 0;
    const int64_t r0 = blockIdx.x * per, r1 = min(n, r0 + per);
    for (int64_t sub = r0; sub < r1; sub += (int64_t)kLongSub * kFillSubs) {
        uint32_t e[kE];
#pragma unroll
        for (int q = 0; q < kFillSubs; ++q) {
            const int64_t i0 = sub + (int64_t)q * kLongSub + (int64_t)threadIdx.x * 4;   // padded past n
            const i32x4 v = i0 < r1 ? *reinterpret_cast<const i32x4*>(ew + i0) : i32x4{-1, -1, -1, -1};
            e[4 * q] = (uint32_t)v.x;
            e[4 * q + 1] = (uint32_t)v.y;
            e[4 * q + 2] = (uint32_t)v.z;
            e[4 * q + 3] = (uint32_t)v.w;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (i0 + k >= r1) e[4 * q + k] = ~0u;
        }
        // the window base: the smallest end of the round
        unsigned m = ~0u;
#pragma unroll
        for (int k = 0; k < kE; ++k) m = min(m, e[k]);
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) m = min(m, (unsigned)__shfl_xor((int)m, d, 64));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        m = min(min(red[0], red[1]), min(red[2], red[3]));
        const int64_t TB = m == ~0u ? 0 : (int64_t)(m / kTileW);
        int te[kE];     // window tile, or -1
        int rk[kE];     // rank in its tile
        const int lane = threadIdx.x & 63;
        const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
        for (int k = 0; k < kE; ++k) {
            te[k] = -1;
            rk[k] = 0;
            if (e[k] != ~0u) {
                const int64_t t = (int64_t)(e[k] / kTileW);
                if (t - TB < kLongTileWin) te[k] = (int)(t - TB);
            }
            if (MC_FILL_WAVE_COUNTS) {
                // one LDS atomic per distinct tile of the wave (the lanes of
                // a tile take consecutive ranks after the leader's add)
                unsigned long long todo = __ballot(te[k] >= 0);
                while (todo) {
                    const int leader = __ffsll((long long)todo) - 1;
                    const int tt = __builtin_amdgcn_readlane(te[k], leader);
                    const unsigned long long m = __ballot(te[k] == tt);
                    int base = 0;
                    if (lane == leader) base = atomicAdd(&wt[tt], (int)__popcll(m));
                    base = __builtin_amdgcn_readlane(base, leader);
                    if (te[k] == tt) rk[k] = base + (int)__popcll(m & below);
                    todo &= ~m;
                }
            } else if (te[k] >= 0) {
                rk[k] = atomicAdd(&wt[te[k]], 1);
            }
        }
        __syncthreads();
        for (int t = threadIdx.x; t < kLongTileWin; t += kBlock) {
            const int v = wt[t];
            if (v) {
                wb[t] = (int)(tile_off[TB + t] + atomicAdd(&cursor[TB + t], (unsigned)v));
                wt[t] = 0;
            }
            if (MC_FILL_SORTED) wc[t] = v;
        }
        if (MC_FILL_SORTED) {
            // the round's window events grouped by tile in LDS, then written
            // out in that order: consecutive lanes store consecutive slots of a
            // tile's run (one scattered 4-byte store per event left each wave
            // store instruction spread over ~a dozen tiles' runs)
            __syncthreads();
            // exclusive prefix of the window's counts: one tile per thread,
            // wave scans by shuffles, then the waves' totals
            static_assert(kBlock == kLongTileWin, "one window tile per thread");
            const int own = wc[threadIdx.x];
            int inc = own;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(inc, d, 64);
                if (lane >= d) inc += y;
            }
            if (lane == 63) red[threadIdx.x >> 6] = (unsigned)inc;
            __syncthreads();
            int add = 0;
            for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) add += (int)red[w];
            wc[threadIdx.x] = add + inc - own;
            const int total = (int)(red[0] + red[1] + red[2] + red[3]);
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kE; ++k) {
                if (e[k] == ~0u) continue;
                const int32_t val = (int32_t)((int64_t)e[k] & cmask);   // chunk-relative end
                if (te[k] >= 0) {
                    const int at = wc[te[k]] + rk[k];
                    sbuf[at] = val;
                    sslot[at] = wb[te[k]] + rk[k];
                } else {
                    const int64_t t = (int64_t)(e[k] / kTileW);
                    ev[tile_off[t] + atomicAdd(&cursor[t], 1u)] = val;
                }
            }
            __syncthreads();
            for (int j = threadIdx.x; j < total; j += kBlock) ev[sslot[j]] = sbuf[j];
            __syncthreads();   // sbuf / wb / wc are rewritten by the next round
            continue;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kE; ++k) {
            if (e[k] == ~0u) continue;
            int64_t slot;
            if (te[k] >= 0) {
                slot = wb[te[k]] + rk[k];
            } else {
                const int64_t t = (int64_t)(e[k] / kTileW);
                slot = tile_off[t] + atomicAdd(&cursor[t], 1u);
            }
            ev[slot] = (int32_t)((int64_t)e[k] & cmask);   // chunk-relative end
        }
        __syncthreads();   // wb is read before the next round's phase 2 rewrites it
    }
}

// ----------------------------------------------------------------- K1

// One workgroup per 256 reads: the block streams the contiguous CIGAR words
// of its reads as int4 (kU loads in flight per thread) and sums the
// reference-consuming lengths per read (op-type mask 0x18D = M, D, N, =, X;
// htslib bam_cigar2rlen).  A mapped read without such an op gets span
// min_span: 0 as current htslib's bam_plp_push (raw rlen), 1 for the legacy
// bam_endpos rule (mc_set_legacy_endpos).  Each lane splits its 4 words into runs by read (one
// LDS binary search per int4, then forward steps); a wave whose runs touch few
// reads (long CIGARs) reduces them with shuffles before one LDS atomic per
// read, otherwise (short CIGARs, low contention) each run adds directly.
#ifndef MC_K1_LOADS
#define MC_K1_LOADS 2                  // K1: int4 loads per lane per step (sweep: 1/2/4/8)
#endif
constexpr int kCigarLoads = MC_K1_LOADS;
constexpr int kOwnerBuckets = 2048;       // K1 word -> read lookup buckets (bytes of LDS)

__device__ __forceinline__ int cigar_ref_len(uint32_t c) {
    return ((0x18Du >> (c & 0xFu)) & 1u) ? (int)(c >> 4) : 0;
}

__global__ void __launch_bounds__(kBlock)
cigar_span_kernel(const int64_t* __restrict__ cig_off, const uint32_t* __restrict__ cigar,
                  int64_t n, int min_span, int32_t* __restrict__ span) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    long long* off = reinterpret_cast<long long*>(smem_raw);                 // kBlock + 1
    int* acc = reinterpret_cast<int*>(smem_raw + (kBlock + 1) * 8 + 8);      // kBlock
    unsigned char* owner = smem_raw + (kBlock + 1) * 8 + 8 + kBlock * 4;     // kOwnerBuckets
    const int64_t r0 = blockIdx.x * (int64_t)kBlock;
    const int nr = (int)min<int64_t>(kBlock, n - r0);
    for (int k = threadIdx.x; k <= nr; k += kBlock) off[k] = cig_off[r0 + k];
    acc[threadIdx.x] = 0;
    __syncthreads();
    const long long w0 = off[0], w1 = off[nr];
    // owner[k]: the read holding word w0 + (k << sh) (2^sh words per bucket,
    // kOwnerBuckets buckets cover the block's words): a lookup plus a step or
    // two replaces a binary search per int4
    int sh = 0;
    while (((long long)kOwnerBuckets << sh) < w1 - w0) ++sh;
    if ((int)threadIdx.x < nr) {                       // each read claims its buckets
        const long long lo = off[threadIdx.x] - w0, hi = off[threadIdx.x + 1] - w0;
        for (long long k = (lo + (1ll << sh) - 1) >> sh; (k << sh) < hi; ++k)
            owner[k] = (unsigned char)threadIdx.x;
    }
    __syncthreads();
    // each lane sums kLaneWords consecutive words per step (4 int4 loads,
    // the next step's in flight), so a long CIGAR's words stay in one lane's
    // registers and a lane adds at most a few per-read partial sums to LDS
    constexpr int kLaneWords = 4 * kCigarLoads;
    constexpr long long kStep = (long long)kLaneWords * kBlock;
    const long long a4 = w0 & ~3ll;
    auto load = [&](uint32_t (&wd)[kLaneWords], long long base) {
        const long long p0 = base + (long long)kLaneWords * threadIdx.x;
#pragma unroll
        for (int u = 0; u < kCigarLoads; ++u) {
            const long long p = p0 + 4 * u;
            if (p + 3 < w1 && p >= w0) {
                const uint4 x = *reinterpret_cast<const uint4*>(cigar + p);
                wd[4 * u] = x.x;
                wd[4 * u + 1] = x.y;
                wd[4 * u + 2] = x.z;
                wd[4 * u + 3] = x.w;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    wd[4 * u + k] = (p + k >= w0 && p + k < w1) ? cigar[p + k] : 0u;
            }
        }
    };
    uint32_t cur[kLaneWords], nxt[kLaneWords];
    if (a4 < w1) load(cur, a4);
    for (long long base = a4; base < w1; base += kStep) {
        if (base + kStep < w1) load(nxt, base + kStep);   // next step in flight meanwhile
        const long long p = base + (long long)kLaneWords * threadIdx.x;
        const long long first = p > w0 ? p : w0;
        if (first < w1 && first < p + kLaneWords) {
            int r = owner[(first - w0) >> sh];
            long long next = off[r + 1];                   // first word of read r + 1
            int run = 0, s = 0;
#pragma unroll
            for (int k = 0; k < kLaneWords; ++k) {
                const long long w = p + k;
                if (w < first || w >= w1) continue;
                if (next <= w) {                           // a new read: flush the run
                    if (s) atomicAdd(&acc[run], s);
                    do {
                        ++r;
                        next = off[r + 1];
                    } while (next <= w);
                    s = 0;
                }
                run = r;
                s += cigar_ref_len(cur[k]);
            }
            if (s) atomicAdd(&acc[run], s);
        }
#pragma unroll
        for (int k = 0; k < kLaneWords; ++k) cur[k] = nxt[k];
    }
    __syncthreads();
    if (threadIdx.x < nr) {
        const int s = acc[threadIdx.x];
        span[r0 + threadIdx.x] = s > min_span ? s : min_span;
    }
}

// ----------------------------------------------------------------- K2

struct ReadBatch {                     // 4 reads in chunk-relative coordinates
    int rs[kReadsPerThread];           // start - chunk start, clamped to +-2^30
    int sp[kReadsPerThread];           // span
    unsigned pending;                  // bit k: read k still to apply
};

// One batch of reads as loaded (int4 per array): the packed read words of a
// prepared batch (ingest_kernel), or the raw tuples (direct path).
template <bool kDirect> struct RawBatch;
template <> struct RawBatch<false> {
    i32x4 g;                           // packed start bits and capped span
};
template <> struct RawBatch<true> {
    i32x4 t, p, s;
    int pt, pp;                        // lane 0: the read before the lane's first (order check)
};

// The read arrays K2 loads: the packed words, or tid / pos / span
struct ReadArrays {
    const uint32_t* __restrict__ gpos;
    const int32_t* __restrict__ tid;
    const int32_t* __restrict__ pos;
    const int32_t* __restrict__ span;
};

// Issue the 16-byte loads of this thread's 4 reads.  The arrays are padded
// by one batch past n, so no bounds check.  Lanes whose 4 reads all lie at or
// past `cend` (the chunk's last batch runs past the chunk) load nothing:
// those are the next chunk's reads, which another workgroup, usually on
// another XCD, fetches again (PMC: the overshoot was most of K2's 21-39 %
// fetch excess over its algorithmic bytes).
template <bool kDirect, class AT>
__device__ __forceinline__ void issue_raw(RawBatch<kDirect>& r, int64_t base, const AT& A,
                                          int64_t cend) {
    const int64_t i0 = base + (int64_t)threadIdx.x * kReadsPerThread;
    if constexpr (kDirect) {
        if (i0 < cend) {
            r.t = *reinterpret_cast<const i32x4*>(A.tid + i0);
            r.p = *reinterpret_cast<const i32x4*>(A.pos + i0);
            r.s = *reinterpret_cast<const i32x4*>(A.span + i0);
        } else {
            r.t = r.p = r.s = i32x4{0, 0, 0, 0};
        }
        // lane 0's predecessor (the previous wave's last read) comes with the
        // batch: a scalar load of it at the batch advance stalled every batch
        // on an L2 round trip (0.12 ms of a C3 launch)
        r.pt = 0;
        r.pp = 0;
        if ((threadIdx.x & 63) == 0 && i0 > 0 && i0 < cend) {
            r.pt = A.tid[i0 - 1];
            r.pp = A.pos[i0 - 1];
        }
    } else {
        r.g = i0 < cend ? *reinterpret_cast<const i32x4*>(A.gpos + i0) : i32x4{0, 0, 0, 0};
    }
}

// Packed read words: chunk-relative start and span of the 4 reads; reads at
// or past n (the chunk's read end) are masked.  lo: the chunk's first read
// (reads before it in the first batch's aligned group are masked: their start
// may lie any distance before the chunk, outside the wrap-around range).
__device__ __forceinline__ void finish_batch(ReadBatch& b, const RawBatch<false>& r, int64_t base,
                                             int64_t n, int64_t C0, int64_t lo) {
    const int64_t i0 = base + (int64_t)threadIdx.x * kReadsPerThread;
    static_assert((int64_t)(kTilesPerChunkLong > kTilesPerChunk ? kTilesPerChunkLong : kTilesPerChunk) * kTileW +
                          kRing < (1 << (kGposBits - 1)),
                  "packed starts: a chunk and its halo must fit the signed wrap-around range");
    static_assert(kGspanCap > kRing - kTileW, "the span cap must exceed short_max");
    const unsigned c0 = (unsigned)C0 & kGposMask;
    const unsigned gg[4] = {(unsigned)r.g.x, (unsigned)r.g.y, (unsigned)r.g.z, (unsigned)r.g.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // sign-extend the kGposBits-bit difference
        const int d = (int)(((gg[k] - c0) & kGposMask) << (32 - kGposBits)) >> (32 - kGposBits);
        b.rs[k] = d;
        b.sp[k] = (int)(gg[k] >> kGposBits);
    }
    const int64_t left = n - i0;
    b.pending = left >= 4 ? 0xfu : left <= 0 ? 0u : ((1u << left) - 1u);
    const int64_t skip = lo - i0;   // > 0 only in thread 0 of the chunk's first batch
    if (skip > 0) b.pending &= skip >= 4 ? 0u : ~((1u << skip) - 1u);
}

// Direct path (see probe_kernel): K2's own view of the batch and what it checks.
struct DirectArgs {
    const int32_t* j0;                 // [n_base + 1] J(k * w)       (probe_kernel)
    const int32_t* jh;                 // [n_base + 1] J(k * w - halo)
    const int32_t* jn;                 // [n_base + 1] J(k * w - kNearHalo)
    const int64_t* len;                // [nc] contig lengths (= extents on this path)
    int32_t nc;
    unsigned long long* dres;
    DirectWindow win;                  // the fused regions' window bases (direct_window_base; its
                                       // parity is K2's win_parity argument)
};

struct DirectChunk {                   // wave-uniform per chunk
    int64_t lo, hi;                    // reads loaded (and applied where they overlap)
    int64_t vlo, vhi;                  // reads this chunk validates
};

struct DirectAcc {                     // per-lane verdict
    unsigned flags = 0;                // kDirectInvalid | kDirectUnfit
    int max_span = 0;                  // over the valid reads loaded for [lo, hi)
    // the last contig looked up (wave-uniform: its offset and length by
    // scalar loads; sorted reads meet a new contig rarely, and the loads'
    // round trip was paid per batch)
    int ct = -1;
    int64_t c_off = 0, c_len = 0;
};

// Raw tuples: chunk-relative starts (contig offsets and lengths by scalar
// loads per distinct contig of the wave: a per-lane vector load would need a
// vmcnt(0), which on gfx9 also waits for every depth store in flight), the
// apply mask (valid reads of [lo, hi) starting before the chunk end), and the
// checks of the reads in [vlo, vhi): range, order against the predecessor
// (the neighbouring lane's last read; lane 0 loads its own by scalar loads),
// overhang, span.
template <class DT>
__device__ __forceinline__ void finish_batch_direct(ReadBatch& b, const RawBatch<true>& r, int64_t base,
                                                    int64_t C0, int64_t chunk_w, const DirectChunk& dc,
                                                    const int64_t* __restrict__ coff,
                                                    const DT& D, int short_max, DirectAcc& acc) {
    const int lane4 = (int)threadIdx.x * kReadsPerThread;   // this lane's first read, relative to base
    const int tt[4] = {r.t.x, r.t.y, r.t.z, r.t.w};
    const int pp[4] = {r.p.x, r.p.y, r.p.z, r.p.w};
    int sp[4];
    asm volatile("v_mov_b32 %0, %1" : "=v"(sp[0]) : "v"(r.s.x));
    asm volatile("v_mov_b32 %0, %1" : "=v"(sp[1]) : "v"(r.s.y));
    asm volatile("v_mov_b32 %0, %1" : "=v"(sp[2]) : "v"(r.s.z));
    asm volatile("v_mov_b32 %0, %1" : "=v"(sp[3]) : "v"(r.s.w));
    unsigned valid = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        valid |= (((unsigned)tt[k] < (unsigned)D.nc) & ((pp[k] | sp[k]) >= 0)) ? 1u << k : 0u;
    constexpr int64_t kClamp = int64_t(1) << 30;
    int rs[4] = {0, 0, 0, 0};
    unsigned L[4] = {0, 0, 0, 0};          // contig length (positions fit 32 bits)
    unsigned todo = valid;
    // 4-bit masks of this lane's reads: in [lo, hi) (applied) and in [vlo,
    // vhi) (checked here); the bounds relative to the batch are scalar
    auto range4 = [&](int64_t lo, int64_t hi) -> unsigned {
        const int la = (int)(lo - base < -8 ? -8 : lo - base > kK2Batch + 8 ? kK2Batch + 8 : lo - base);
        const int ha = (int)(hi - base < -8 ? -8 : hi - base > kK2Batch + 8 ? kK2Batch + 8 : hi - base);
        const int ka = min(max(la - lane4, 0), 4), kz = min(max(ha - lane4, 0), 4);
        return ((1u << kz) - 1u) & ~((1u << ka) - 1u);
    };
    const unsigned inr = range4(dc.lo, dc.hi);
    const unsigned own = range4(dc.vlo, dc.vhi);
    bool fast = false;   // wave-uniform
    if (MC_DIRECT_ONE_CONTIG && acc.ct >= 0) {
        // every read this batch applies or checks is on the contig of the
        // previous batch (sorted reads: almost every batch): one vote instead
        // of the lookup loop's two and its per-read selects
        const unsigned use = (inr | own) & valid;
        bool other = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) other |= ((use >> k) & 1u) && tt[k] != acc.ct;
        if (!__ballot(other)) {
            const int64_t c = acc.c_off - C0, ln = acc.c_len;
            const unsigned l32 = ln > 0xffffffffll ? 0xffffffffu : (unsigned)ln;
            int c32, p_lo, p_hi;
            if (c > kClamp) {
                c32 = (int)kClamp;
                p_lo = p_hi = 0;
            } else if (c < -kClamp - (int64_t)INT32_MAX) {
                c32 = -(int)kClamp;
                p_lo = p_hi = 0;
            } else {
                c32 = (int)(uint32_t)(uint64_t)c;
                p_lo = (int)(c < -kClamp ? -kClamp - c : 0);
                p_hi = (int)(kClamp - c > (int64_t)INT32_MAX ? (int64_t)INT32_MAX : kClamp - c);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                rs[k] = (int)((unsigned)c32 + (unsigned)min(max(pp[k], p_lo), p_hi));
                L[k] = l32;
            }
            fast = true;   // (reads outside use: their rs / L are never used)
        }
    }
    for (; !fast;) {
        const int cand = (todo & 1u) ? tt[0] : (todo & 2u) ? tt[1] : (todo & 4u) ? tt[2]
                       : (todo & 8u) ? tt[3] : -1;
        const unsigned long long act = __ballot(cand >= 0);
        if (!act) break;
        const int t0 = __builtin_amdgcn_readlane(cand, __ffsll((long long)act) - 1);
        if (t0 != acc.ct) {
            acc.ct = t0;
            acc.c_off = uload(coff, t0);
            acc.c_len = uload(D.len, t0);
        }
        const int64_t c = acc.c_off - C0, ln = acc.c_len;
        const unsigned l32 = ln > 0xffffffffll ? 0xffffffffu : (unsigned)ln;
        // rs = clamp(c + pos, -2^30, 2^30) in 32 bits: pos (>= 0 when valid)
        // clamped to [p_lo, p_hi] per contig (scalar), then c + pos wraps
        // into an int32 that is exact (one med3 and one add per read instead
        // of a 64-bit add, two 64-bit compares and selects)
        int c32, p_lo, p_hi;
        if (c > kClamp) {
            c32 = (int)kClamp;
            p_lo = p_hi = 0;
        } else if (c < -kClamp - (int64_t)INT32_MAX) {
            c32 = -(int)kClamp;
            p_lo = p_hi = 0;
        } else {
            c32 = (int)(uint32_t)(uint64_t)c;
            p_lo = (int)(c < -kClamp ? -kClamp - c : 0);
            p_hi = (int)(kClamp - c > (int64_t)INT32_MAX ? (int64_t)INT32_MAX : kClamp - c);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool m = ((todo >> k) & 1u) && tt[k] == t0;
            rs[k] = m ? (int)((unsigned)c32 + (unsigned)min(max(pp[k], p_lo), p_hi)) : rs[k];
            L[k] = m ? l32 : L[k];
            todo &= m ? ~(1u << k) : ~0u;
        }
    }
    // predecessor of read 0: lane - 1's read 3 (DPP wave_shr:1, no LDS
    // permute); lane 0 keeps its own, which came with the batch
    const int pt = __builtin_amdgcn_update_dpp(r.pt, tt[3], 0x138, 0xf, 0xf, false);
    const int ppv = __builtin_amdgcn_update_dpp(r.pp, pp[3], 0x138, 0xf, 0xf, false);
    unsigned pend = 0, bad = 0, unfit = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b.rs[k] = rs[k];
        b.sp[k] = sp[k];
        const bool ok = (valid >> k) & 1u;
        pend |= (ok & (rs[k] < chunk_w) & (sp[k] <= short_max)) ? 1u << k : 0u;
        const int qt = k ? tt[k - 1] : pt, qp = k ? pp[k - 1] : ppv;
        // (tid, pos) as one unsigned 64-bit key: one compare (3 compares and 2
        // mask operations as a lexicographic pair: C3 K2 -0.02 ms).  Reads
        // with a negative field are invalid whatever the order says; the first
        // read of all has the predecessor (0, 0).
        const bool uns = (((uint64_t)(unsigned)tt[k] << 32) | (unsigned)pp[k]) <
                         (((uint64_t)(unsigned)qt << 32) | (unsigned)qp);
        bad |= (!ok | uns) ? 1u << k : 0u;
        unfit |= ((unsigned)pp[k] + (unsigned)sp[k] > L[k]) ? 1u << k : 0u;
    }
    b.pending = pend & inr;
    // the batch's maximum span (every read is loaded by the chunk it belongs
    // to, so the maximum over the workgroups is exact): the host takes long
    // reads (> short_max) to the full prepare and sizes the next batch's halo
    const unsigned mm = valid & inr;
    acc.max_span = max(acc.max_span, max(max((mm & 1u) ? sp[0] : 0, (mm & 2u) ? sp[1] : 0),
                                         max((mm & 4u) ? sp[2] : 0, (mm & 8u) ? sp[3] : 0)));
    acc.flags |= (bad & own) ? kDirectInvalid : (unfit & own) ? kDirectUnfit : 0u;
}

// The far part of a direct chunk's halo, reads [lo, hi) that start more
// than kNearHalo positions before the chunk (C0): only those with a span
// above kNearHalo can reach it, so their spans are read (4 B per read, int4
// per lane) and only such reads' (tid, pos) (rare: the span mix's spliced
// reads).  A read reaching past C0 adds +1 at the chunk's first slot and -1
// at its end, as the batch loop applies a halo read.  The reads are checked
// by their own chunk.  At C2 depth this is ~45 % of the reads a chunk loads.
template <class DT>
__device__ __forceinline__ void far_halo(const ReadArrays& A, const DT& D, const int64_t* __restrict__ coff,
                                         int64_t lo, int64_t hi, int64_t C0, int short_max, int* ring) {
    // (one int4 of spans per thread and step: keeping 8 in flight raised the
    // kernel's VGPRs and cost C3 +10 %, r05/r05ab13_*)
    // the lane offset is opaque to the optimiser: hoisted out of the chunk
    // loop, the three per-lane array addresses were the fused direct K2's
    // VGPR spills (6), reloaded from scratch with a vmcnt(0) each per chunk
    int lane_off = (int)threadIdx.x * 4;
    asm volatile("" : "+v"(lane_off));
    for (int64_t i0 = (lo & ~(int64_t)3) + lane_off; i0 < hi; i0 += (int64_t)kK2Block * 4) {
        const i32x4 s4 = *reinterpret_cast<const i32x4*>(A.span + i0);
        const int sp[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = i0 + k;
            if (i < lo || i >= hi || sp[k] <= kNearHalo || sp[k] > short_max) continue;
            const int t = A.tid[i], p = A.pos[i];
            if ((unsigned)t >= (unsigned)D.nc || p < 0) continue;
            const int64_t e = coff[t] + p + sp[k] - C0;
            if (e > 0 && e <= short_max) {   // (sorted input: e <= short_max - kNearHalo)
                atomicAdd(&ring[ring_slot(0)], 1);
                atomicAdd(&ring[ring_slot((int)e)], -1);
            }
        }
    }
}

// K2 direct: the per-workgroup verdict into dres (one atomic, only when a
// read failed a check).  The aligned bases are not counted here: summing
// the spans cost 0.03 ms of a C3 launch for a figure few callers ask for
// (span_sum_kernel computes it on request).
template <class DT>
__device__ __forceinline__ void direct_flush(const DirectAcc& a, const DT& D, int* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned f = a.flags;
    int m = a.max_span;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        f |= __shfl_xor(f, d, 64);
        m = max(m, __shfl_xor(m, d, 64));
    }
    __syncthreads();
    if (lane == 0) {
        red[wave] = (int)f;
        red[kK2Waves + wave] = m;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned ff = 0;
        int mm = 0;
#pragma unroll
        for (int w = 0; w < kK2Waves; ++w) {
            ff |= (unsigned)red[w];
            mm = max(mm, red[kK2Waves + w]);
        }
        if (ff) atomicOr(&D.dres[kDresFlags], (unsigned long long)ff);
        if (mm > 0) atomicMax(&D.dres[kDresMaxSpan], (unsigned long long)mm);
    }
}

// The aligned bases of a direct batch K2 accepted (every span >= 0): the sum
// of span[0, n), on request (mc_aligned_bases).  Each thread keeps 4 int4
// loads in flight; each workgroup writes one partial (span_sum_final_kernel
// adds them): one same-address atomic per wave, 8192 of them, serialised
// into most of the launch at C2 (0.105 ms for 40 MB, round 4).
__global__ void __launch_bounds__(kBlock)
span_sum_kernel(const int32_t* __restrict__ span, int64_t n, unsigned long long* __restrict__ part) {
    long long s = 0;
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        i32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(span) + i + u * stride);
#pragma unroll
        for (int u = 0; u < 4; ++u) s += (long long)v[u].x + v[u].y + v[u].z + v[u].w;
    }
    for (; i < n4; i += stride) {
        const i32x4 v = reinterpret_cast<const i32x4*>(span)[i];
        s += (long long)v.x + v.y + v.z + v.w;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) s += span[(n4 << 2) + threadIdx.x];
    s = wave_sum64(s);
    __shared__ long long ws[kWaves];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) t += ws[w];
        part[blockIdx.x] = (unsigned long long)t;
    }
}

// One workgroup: out = the sum of span_sum_kernel's m partials.
__global__ void __launch_bounds__(kBlock)
span_sum_final_kernel(const unsigned long long* __restrict__ part, int m, unsigned long long* __restrict__ out) {
    long long s = 0;
    for (int i = threadIdx.x; i < m; i += kBlock) s += (long long)part[i];
    s = wave_sum64(s);
    __shared__ long long ws[kWaves];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) t += ws[w];
        *out = (unsigned long long)t;
    }
}

// Fused region statistics of K2 (optional): non-overlapping regions sorted by
// global start.  Each tile folds the positions it owns into the region(s)
// covering them: min/max/sum/sum of squares per thread, value histogram of
// the current region in LDS (kHistBins bins; larger values go to an LDS
// overflow accumulator, and regions whose ranks reach them are recomputed by
// the host with region_seg_kernel).
//
// The LDS histogram is kept in kHistCopies lane-striped copies (lane L adds
// into copy L % kHistCopies).  Neighbouring lanes hold neighbouring positions,
// which mostly have the same depth: with one copy, the 32 lanes of an LDS
// atomic group pile onto a handful of bins (same-address lanes serialise; the
// fused K2 showed 8x the plain kernel's SQ_LDS_BANK_CONFLICT cycles).  Copies
// start 32 / kHistCopies banks apart, and the flush sums them.  Budget: ring +
// copies + overflow records stay at or below 40,672 B so 4 workgroups fit a
// CU (2 copies of 992 bins, 40,928 B in all, ran at 3: +11 % K2 time).
// Measured on C3 / C5 fused K2 (scripts/ab_inproc.py, one 32-byte overflow
// record): 1 copy 1.195 / 1.600 ms, 2 x 960 1.094 / 1.514, 4 x 480 1.102 /
// 1.559, 8 x 224 1.096 / 1.723 (narrow windows: fallbacks).  With the 16
// overflow records (640 B) the 2 copies hold 864 bins (40,512 B).
#ifndef MC_HIST_COPIES
#define MC_HIST_COPIES 2
#endif
#ifndef MC_HIST_BINS
#define MC_HIST_BINS (MC_HIST_COPIES == 1 ? 1024 : MC_HIST_COPIES == 2 ? 864 \
                      : MC_HIST_COPIES == 4 ? 480 : MC_HIST_COPIES == 8 ? 224 : 96)
#endif
// The long-read variant (C5-like deep contigs with long end ramps, whose
// quartile ranks span more values): its own copies / bins in the same LDS
#ifndef MC_HIST_COPIES_LONG
#define MC_HIST_COPIES_LONG MC_HIST_COPIES
#endif
#ifndef MC_HIST_BINS_LONG
#define MC_HIST_BINS_LONG (MC_HIST_COPIES_LONG == 1 ? 1728 : MC_HIST_BINS)
#endif
// Each copy is followed by a pad of kPad ints: it offsets the next copy by
// 32 / kCopies banks, and holds the per-lane dummy slots the branch-free
// histogram adds 0 into (hist_int4).
template <bool kLong>
struct HistCfg {
    static constexpr int kCopies = kLong ? MC_HIST_COPIES_LONG : MC_HIST_COPIES;
    static constexpr int kBins = kLong ? MC_HIST_BINS_LONG : MC_HIST_BINS;
    static constexpr int kPad = kCopies > 1 ? 32 / kCopies : 32;
    static constexpr int kStride = kBins + kPad;
    static constexpr int kLds = kCopies * kStride;   // ints of LDS
    static_assert(kBins % 32 == 0 && (kCopies & (kCopies - 1)) == 0 && kCopies <= 32,
                  "histogram bins: multiple of 32; copies: power of two");
};
constexpr int kHistBins = HistCfg<false>::kBins;          // the short-read variant's window
// values per region row of the global fused histogram
__host__ __device__ constexpr int fused_hist_vals(bool long_reads) {
    return long_reads ? HistCfg<true>::kBins : HistCfg<false>::kBins;
}

struct FusedRegions {
    int64_t n;                         // 0 = no fused statistics
    const int64_t* chunk_first;        // [n_chunks] first region ending after the chunk start
    const int64_t* gs;                 // [n] global start (sorted)
    const int64_t* ge;                 // [n] global end (clipped to the contig extent)
    const int32_t* id;                 // [n] caller's row index
    const int32_t* base;               // [n] value of histogram bin 0 (window base; direct: computed)
    const int32_t* rtid;               // [rows] each row's contig (direct path's window)
    RegionAcc* acc;                    // [rows] statistics of the values outside the window
    unsigned* hist;                    // [rows][HistCfg<kLong>::kBins]
    unsigned* low;                     // [rows] count of values below the window
};

// Statistics of the values outside the histogram window of the current
// region: kOvRecs LDS records per workgroup behind the histogram (lane L
// updates record L % kOvRecs with LDS atomics), folded at the flush.  The
// out-of-window path is cold on C3 but not at C5, where the ramps at the ends
// of deep contigs fall below the window: a wave-wide reduction per int4 there
// cost 0.1 ms a launch.  40-byte records start 10 banks apart, so the 16
// records' fields sit in distinct banks (lanes L and L + 16 share one).
struct OvLds {
    unsigned long long sum, sq;
    int vmin, vmax;
    unsigned cnt, low;                 // values outside the window / below it
    unsigned pad[2];
};
constexpr int kOvRecs = 16;
static_assert(sizeof(OvLds) == 40, "record stride: 10 banks");
constexpr int kOvInts = kOvRecs * (int)sizeof(OvLds) / 4;

__device__ __forceinline__ void ov_reset(OvLds* ov) {
    ov->sum = ov->sq = 0;
    ov->vmin = 0x7fffffff;
    ov->vmax = 0;
    ov->cnt = ov->low = 0;
}

// Out-of-window runs accumulate in each lane's registers (an OvReg, 8 VGPRs)
// while the region stays open in the chunk, and go to the lane's LDS record
// only before the region's histogram is flushed.  On C5, where the end ramps
// of deep contigs fall below the window, adding every int4's runs to the LDS
// records (6 atomics) cost 0.075 ms of a 1.13 ms fused K2.
struct OvReg {
    unsigned cnt, low;
    unsigned long long sum, sq;
    int vmin, vmax;
};

__device__ __forceinline__ void ov_reg_reset(OvReg& r) {
    r.cnt = r.low = 0;
    r.sum = r.sq = 0;
    r.vmin = 0x7fffffff;
    r.vmax = 0;
}

// a lane's accumulated out-of-window statistics into its LDS record
__device__ __attribute__((noinline)) void ov_spill(OvLds* ov, unsigned cnt, unsigned low, unsigned long long sum,
                                                   unsigned long long sq, int mn, int mx) {
    if (cnt) {
        atomicAdd(&ov->cnt, cnt);
        if (low) atomicAdd(&ov->low, low);
        atomicAdd(&ov->sum, sum);
        atomicAdd(&ov->sq, sq);
        atomicMin(&ov->vmin, mn);
        atomicMax(&ov->vmax, mx);
    }
}

// every lane of the wave calls it: the register record goes to LDS (before a
// flush's barrier) and starts over
__device__ __forceinline__ void ov_reg_spill(OvReg& r, OvLds* ovf) {
    if (__any(r.cnt != 0)) {
        ov_spill(ovf + (threadIdx.x & (kOvRecs - 1)), r.cnt, r.low, r.sum, r.sq, r.vmin, r.vmax);
        ov_reg_reset(r);
    }
}

// K2 zeroes one tile of ring slots per chunk (where the ends of reads running
// past the chunk landed), not the whole ring
static_assert(kRing == 2 * kTileW, "the ring tail is one tile (short_max = kTileW)");

// Histogram of 4 consecutive positions (y < 0: outside the region, skipped):
// one LDS atomic per run of equal values, branch-free: every slot issues its
// atomic, and a slot that is no run start, or whose value is outside the
// window, adds into the lane's own pad slot `dummy` (>= kWinBins), so its
// address is one unsigned min (y < 0 and values below the window wrap to
// large unsigned bins).  The predicated form cost ~6 SALU exec-mask
// instructions per atomic; testing in-window and in-region per slot before
// the atomic cost twice the VALU of this form.  The rare out-of-window path
// (any bin >= kWinBins in the wave: window misses, or positions outside the
// region) classifies the runs exactly (same run arithmetic as
// region_seg_kernel).
template <int kWinBins>
__device__ __forceinline__ void hist_int4(unsigned* h, int dummy, OvReg& ovr, int y0, int y1, int y2, int y3,
                                          int base) {
    const bool s1 = y1 != y0, s2 = y2 != y1, s3 = y3 != y2;
    const int l2 = s3 ? 1 : 2;
    const int l1 = s2 ? 1 : l2 + 1;
    const int l0 = s1 ? 1 : l1 + 1;
    constexpr unsigned kWin = (unsigned)kWinBins;
    const unsigned du = (unsigned)dummy;
    const unsigned d0 = (unsigned)(y0 - base), d1 = (unsigned)(y1 - base),
                   d2 = (unsigned)(y2 - base), d3 = (unsigned)(y3 - base);
    atomicAdd(&h[min(d0, du)], (unsigned)l0);
    atomicAdd(&h[s1 ? min(d1, du) : du], (unsigned)l1);
    atomicAdd(&h[s2 ? min(d2, du) : du], (unsigned)l2);
    atomicAdd(&h[s3 ? min(d3, du) : du], 1u);
    if (__builtin_expect(__any(max(max(d0, d1), max(d2, d3)) >= kWin), 0)) {
        // per position, branch-free (the per-run form took an exec-mask
        // branch per slot: 4 % of a C5 K2, where the ramps of deep contigs
        // fall below the window)
        const int y[4] = {y0, y1, y2, y3};
        const unsigned d[4] = {d0, d1, d2, d3};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool o = (y[k] >= 0) & (d[k] >= kWin);
            const unsigned v = o ? (unsigned)y[k] : 0u;
            ovr.cnt += o ? 1u : 0u;
            ovr.low += (o & (y[k] < base)) ? 1u : 0u;
            ovr.sum += v;
            ovr.sq += (unsigned long long)v * v;
            ovr.vmin = min(ovr.vmin, o ? y[k] : 0x7fffffff);
            ovr.vmax = max(ovr.vmax, (int)v);
        }
    }
}

// Block-wide AND of two predicates with one barrier: each wave's votes are
// bits 0 / 1 of a byte of a double-buffered LDS word (flip = which word; the
// next call uses the other, so a wave running ahead never overwrites a word
// another wave still reads).  __syncthreads_and compiled to three barriers
// and an LDS atomic for one predicate.
// (words: two 8-byte words; one byte per wave, up to 8 waves)
__device__ __forceinline__ void block_all2(int* words, int& flip, bool p0, bool p1, int wave, int lane,
                                           bool& all0, bool& all1) {
    const int v = (__all(p0) ? 1 : 0) | (__all(p1) ? 2 : 0);
    if (lane == 0) reinterpret_cast<unsigned char*>(words + 2 * flip)[wave] = (unsigned char)v;
    __syncthreads();
    if (kK2Waves == 4) {
        const int w = words[2 * flip];
        all0 = (w & 0x01010101) == 0x01010101;
        all1 = (w & 0x02020202) == 0x02020202;
    } else {
        const unsigned long long w = *reinterpret_cast<const unsigned long long*>(words + 2 * flip);
        all0 = (w & 0x0101010101010101ull) == 0x0101010101010101ull;
        all1 = (w & 0x0202020202020202ull) == 0x0202020202020202ull;
    }
    flip ^= 1;
}

// A batch of the chunk's long-read end events: 4 consecutive events per
// thread (chunk-relative positions), indices [e_lo, e_hi) only.
struct EvBatch {
    int rel[4];
    unsigned pending;
};

__device__ __forceinline__ void load_events(EvBatch& e, const int32_t* __restrict__ ev, int64_t base,
                                            int64_t e_lo, int64_t e_hi) {
    const int64_t i0 = base + (int64_t)threadIdx.x * 4;
    e.pending = 0;
    if (i0 < e_hi && i0 + 4 > e_lo) {   // ev is padded by one batch past its end
        const i32x4 x = *reinterpret_cast<const i32x4*>(ev + i0);
        e.rel[0] = x.x;
        e.rel[1] = x.y;
        e.rel[2] = x.z;
        e.rel[3] = x.w;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i0 + k >= e_lo && i0 + k < e_hi) e.pending |= 1u << k;
    }
}

// Every thread calls it (it holds barriers): folds the overflow statistics
// into the region's global accumulator and flushes the LDS histogram.
// kBarriers = false: the caller has just passed a barrier after the last
// atomics, and a barrier follows before the histogram is used again.
template <bool kBarriers, class HC, class RT>
__device__ __forceinline__ void flush_region(const RT& R, int id, unsigned* h, OvLds* ov) {
    // id: the region's row, loaded with its other fields (no scalar load on
    // the chunk end's path)
    if (kBarriers) __syncthreads();   // every wave's histogram and overflow atomics are in
    if (threadIdx.x < kOvRecs) {
        OvLds* o = ov + threadIdx.x;
        if (o->cnt) {
            if (o->low) atomicAdd(&R.low[id], o->low);
            atomicMin(&R.acc[id].min, o->vmin);
            atomicMax(&R.acc[id].max, o->vmax);
            atomicAdd(&R.acc[id].sum, o->sum);
            atomicAdd(&R.acc[id].sumsq, o->sq);
            ov_reset(o);
        }
    }
    unsigned* g = R.hist + (int64_t)id * HC::kBins;
    for (int k = threadIdx.x; k < HC::kBins; k += kK2Block) {
        unsigned cnt = 0;
#pragma unroll
        for (int c = 0; c < HC::kCopies; ++c) cnt += h[c * HC::kStride + k];
        if (cnt) {
            atomicAdd(&g[k], cnt);
#pragma unroll
            for (int c = 0; c < HC::kCopies; ++c) h[c * HC::kStride + k] = 0;
        }
    }
    if (kBarriers) __syncthreads();
}

// K2's chunk queue (thread 0): one counter.  (Eight queues over contiguous
// chunk ranges, one per blockIdx % 8 group = one XCD, with stealing, ran
// C3 plain +0.8 %, fused +2.0 %: K2's traffic is at its algorithmic bytes, so
// there is no L2 reuse to win.)
__device__ __forceinline__ int take_chunk(unsigned* queue, int64_t n_chunks) {
    const unsigned t = atomicAdd(queue, 1u);
    return t < (unsigned)n_chunks ? (int)t : (int)n_chunks;
}

// One workgroup walks chunks of `tiles_per_chunk` tiles of kTileW positions
// (dynamic queue).  Per chunk: the chunk's reads are applied as +1 at
// max(start, chunk start) and -1 at end into an LDS ring of kRing ints; each
// finished tile is prefix-scanned (int4 per lane, wave scan, block carry) and
// stored to HBM with 1 KiB-per-wave-instruction stores, and its ring slots
// are zeroed.  Reads longer than short_max = kRing - kTileW take the long-read
// path (see long_count_kernel).
// kStats: fold the tile into FusedRegions before it leaves the registers.
// kLong: the long-read path is compiled in (spans > short_max exist); without
// it the event stream's registers are not held (the fused variant is at its
// 128-VGPR budget).
// kDirect: the batch was not prepared: the chunk's read range comes from the
// probe's J arrays, the reads are loaded as raw (tid, pos, span), and K2
// validates them (probe_kernel); otherwise the chunk index and the packed
// read words of ingest_kernel.
// K2's pointer arguments that change only when buffers or the region set do,
// in device memory (engine.hip uploads a copy when they change): read at
// their uses by scalar loads from constant memory instead of being kernel
// arguments, which the compiler held in SGPRs for the whole launch and
// spilled (74 SGPRs into VGPR lanes on the direct fused variant: 34
// v_readlane per read batch in the apply loop reloading the read array
// pointers; 35 spills and none in that loop this way).
struct K2Consts {
    ReadArrays A;
    FusedRegions R;
    DirectArgs D;
};

template <bool kStats, bool kLong, bool kDirect>
// waves/SIMD minimum per variant (0 = unconstrained -> 1)
__global__ void __launch_bounds__(kK2Block, kStats ? (MC_WAVES_STATS ? MC_WAVES_STATS : 1)
                                                 : (MC_WAVES_PLAIN ? MC_WAVES_PLAIN : 1))
depth_kernel(ReadArrays A, const K2Consts* __restrict__ K, int64_t n,
             const int64_t* __restrict__ coff, const int64_t* __restrict__ chunk_first,
             int cstride, int64_t n_chunks, int tiles_per_chunk, int short_max,
             const int64_t* __restrict__ tile_ev_off, const int32_t* __restrict__ tile_ev,
             const int* __restrict__ chunk_carry,
             int32_t* __restrict__ depth, unsigned* __restrict__ queue,
             int* __restrict__ max_depth, unsigned long long gen, int win_parity) {
    static_assert(!(kDirect && kLong), "the direct path has no long reads");
    const auto& KC = *(const __attribute__((address_space(4))) K2Consts*)K;
    const auto& R = KC.R;
    const auto& D = KC.D;
    extern __shared__ __attribute__((aligned(16))) int lds[];
    // [0] chunk id, [4, 4 + W) wave totals, [4 + W, 4 + 2W) wave max, then the
    // block_all2 votes (kLdsHeader)
    int* hdr = lds;
    int and_flip = 0;
    int* ring = lds + kLdsHeader;
    unsigned* hist = reinterpret_cast<unsigned*>(ring + kRing);   // kStats only
    using HC = HistCfg<kLong>;
    OvLds* ovf = reinterpret_cast<OvLds*>(hist + HC::kLds);            // kStats only
    const int lane = threadIdx.x & 63;
    unsigned* hist_lane = hist + (lane & (HC::kCopies - 1)) * HC::kStride;   // this lane's copy
    // this lane's pad slot: distinct among the lanes of its copy in a half-wave
    const int hist_dummy = HC::kBins + (lane / HC::kCopies) % HC::kPad;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform per wave
    const int64_t chunk_w = (int64_t)tiles_per_chunk * kTileW;
    constexpr int kWaveSpan = kTileW / kK2Waves;       // 1024 positions per wave
    constexpr int kChunks = kWaveSpan / (64 * 4);    // int4 per lane -> 4
    // Deferred tile stores (a tile's stores issued after the next tile's
    // apply loop), plain K2 only: with 12 B/read they gained plain C3 -2.4 %,
    // C5 -4.9 %; with the packed read words the fused C3 K2 runs 1.6 % faster
    // without them (profiles/r02zz_knobs_ab.txt).
    constexpr bool kDefer = !kStats || (kLong && MC_DEFER_LONG) || (kDirect && MC_DEFER_DIRECT);
    constexpr bool kPf = kStats ? MC_PREFETCH_STATS : MC_PREFETCH;
    // The probe saw an unsorted / invalid sample or a long span: the host
    // re-runs this batch through the full prepare; nothing to do here.
    if (kDirect) {
        const unsigned long long f0 = uload(D.dres, kDresBadSample), f1 = uload(D.dres, kDresLongSample);
        if (f0 == gen || f1 == gen) return;
    }
    int my_max = 0;
    DirectAcc dacc;            // kDirect: this lane's validation counters
    OvReg ovr;                 // kStats: this lane's out-of-window runs of the open region
    ov_reg_reset(ovr);
    if (kStats) {
        for (int k = threadIdx.x; k < HC::kLds; k += kK2Block) hist[k] = 0;
        if (threadIdx.x < kOvRecs) ov_reset(ovf + threadIdx.x);   // ordered by the first barrier
    }

    // chunk ids come from an atomic queue (thread 0); everything indexed by
    // the chunk id is then loaded by every wave at a uniform index (uload).
    // kAhead (the fused long-read variant): the next chunk is reserved at the
    // start of the current one, so the queue atomic's round trip overlaps the
    // chunk instead of following its end (C5 fused -3.6 %; elsewhere the held
    // chunk worsens the tail balance: C3 plain +6.7 %, fused +3.0 %).
    constexpr bool kAhead = kStats && kLong;
    int ticket = 0;
    if (threadIdx.x == 0) hdr[0] = take_chunk(queue, n_chunks);
    // the whole ring before the first chunk; after a chunk only the tile of
    // slots after its last tile, where the ends of reads running past the
    // chunk (at most short_max = one tile) landed: every tile's own slots are
    // zeroed by its scan
    const int ring_tail = (int)(((int64_t)tiles_per_chunk * kTileW) % kRing);
    for (int k = threadIdx.x * 4; k < kRing; k += kK2Block * 4)
        *reinterpret_cast<i32x4*>(ring + k) = i32x4{0, 0, 0, 0};
    for (;;) {
        // (the barrier also orders the hdr write before the reads)
        __syncthreads();
        const int64_t c = (unsigned)__builtin_amdgcn_readfirstlane(hdr[0]);
        if (c >= n_chunks) break;
        if (kAhead && threadIdx.x == 0) ticket = take_chunk(queue, n_chunks);
        // chunk c = base chunks [c * cstride, (c + 1) * cstride)
        const int64_t b0 = c * cstride;
        int64_t cfirst, cend;
        DirectChunk dc{0, 0, 0, 0};
        int64_t far_lo = 0, far_hi = 0;
        if (kDirect) {
            // read ranges from the probe's sample counts J: lb(P) lies in
            // ((J - 1) * S, J * S]; the first chunk starts at 0, the last ends at n
            const int64_t b1 = b0 + cstride;
            auto lower = [&](int64_t J) { return J <= 0 ? (int64_t)0 : min(n, ((J - 1) << kProbeShift) + 1); };
            auto upper = [&](int64_t J) { return J <= 0 ? (int64_t)0 : min(n, J << kProbeShift); };
            const bool last = c + 1 == n_chunks;
            dc.lo = c ? lower(uload(D.jh, b0)) : 0;
            dc.vlo = c ? lower(uload(D.j0, b0)) : 0;
            dc.hi = last ? n : upper(uload(D.j0, b1));
            dc.vhi = last ? n : lower(uload(D.j0, b1));
            dc.lo = min(dc.lo, dc.vlo);   // (apart only on unsorted input, which is reported)
            dc.hi = max(dc.hi, dc.vhi);
            if (MC_FAR_HALO && c) {   // [lo, lower(J(C0 - kNearHalo))): by spans (far_halo)
                const int64_t fh = min(max(lower(uload(D.jn, b0)), dc.lo), dc.vlo);
                // (a far part under kFarHaloMin reads costs more than it saves:
                // C3 +1.4 % at 1024, neutral at 4096; C2 K2 -3 %, r05/r05ab12_*)
                if (fh - dc.lo >= kFarHaloMin) {
                    far_lo = dc.lo;
                    far_hi = fh;
                    dc.lo = fh;
                }
            }
            cfirst = dc.lo;
            cend = dc.hi;
        } else {
            // index of ingest_kernel: the chunk's reads start at the first short
            // read crossing its start, else at the first read starting in it
            cfirst = b0 ? (int64_t)min((uint64_t)uload(chunk_first, 2 * b0),
                                       (uint64_t)uload(chunk_first, 2 * b0 - 1)) : 0;
            cend = uload(chunk_first, 2 * (c + 1) * cstride - 1);
        }
        const int64_t C0 = c * chunk_w;
        int64_t rcur = 0, r_gs = 0, r_ge = 0;
        int r_base = 0, r_id = 0;
        if (kStats) {
            rcur = uload(R.chunk_first, c);
            if (rcur < R.n) {
                r_gs = uload(R.gs, rcur);
                r_ge = uload(R.ge, rcur);
                r_id = uload(R.id, rcur);
                r_base = kDirect ? direct_window_base(D.win, win_parity, uload(R.rtid, r_id)) : uload(R.base, rcur);
            }
        }
        int64_t base = cfirst & ~(int64_t)(kReadsPerThread - 1);
        bool more = base < cend;
        ReadBatch b;
        RawBatch<kDirect> nxt;
        b.pending = 0;
        auto finish = [&](const RawBatch<kDirect>& r, int64_t at) {
            if constexpr (kDirect)
                finish_batch_direct(b, r, at, C0, chunk_w, dc, coff, D, short_max, dacc);
            else
                finish_batch(b, r, at, cend, C0, cfirst);
        };
        RawBatch<kDirect> r0;
        if (more) {
            issue_raw<kDirect>(r0, base, A, cend);
            if (kPf && base + kK2Batch < cend) issue_raw<kDirect>(nxt, base + kK2Batch, A, cend);
        }
        // (after the first batches' loads are issued: one round trip for both)
        if (kDirect && MC_FAR_HALO && far_hi > far_lo) far_halo(A, D, coff, far_lo, far_hi, C0, short_max, ring);
        if (more) finish(r0, base);
        int carry = kLong ? uload(chunk_carry, c) : 0;
        // -1 end events of long reads (chunk-relative, in tile order): a
        // second stream of 1024-event batches, applied like the reads while
        // they lie before the current tile end (a dependent load chain per
        // tile was 0.24 ms of a C5 launch)
        EvBatch eb;
        eb.pending = 0;
        int64_t ev_lo = 0, ev_hi = 0, ev_base = 0;
        bool ev_more = false;
        if (kLong) {   // the chunk's range of long-read end events
            ev_lo = uload(tile_ev_off, c * tiles_per_chunk);
            ev_hi = uload(tile_ev_off, (c + 1) * tiles_per_chunk);
            ev_base = ev_lo & ~(int64_t)3;
            ev_more = ev_base < ev_hi;
            if (ev_more) load_events(eb, tile_ev, ev_base, ev_lo, ev_hi);
        }
        i32x4 v[kChunks];          // the scanned tile (this wave's span)
        int64_t pend_T0 = -1;      // kDefer: tile whose depth in v is not stored yet
        auto store_tile = [&](int64_t tile0) {
            int32_t* dst = depth + tile0 + wave * kWaveSpan + lane * 4;
#pragma unroll
            for (int j = 0; j < kChunks; ++j) {
                if (MC_NT_STORE)
                    __builtin_nontemporal_store(v[j], reinterpret_cast<i32x4*>(dst + j * 256));
                else
                    *reinterpret_cast<i32x4*>(dst + j * 256) = v[j];
            }
        };
        for (int t = 0; t < tiles_per_chunk; ++t) {
            const int64_t T0 = C0 + (int64_t)t * kTileW;
            const int64_t Tend = T0 + kTileW;
            const int tend_rel = (t + 1) * kTileW;   // C0 is a multiple of the ring size
            for (;;) {
                if (kLong) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (((eb.pending >> k) & 1u) && eb.rel[k] < tend_rel) {
                            atomicAdd(&ring[ring_slot(eb.rel[k])], -1);
                            eb.pending &= ~(1u << k);
                        }
                }
                if (MC_APPLY_SHORT && !kLong) {
                    // every pending read is short here (the direct path's masks;
                    // a packed batch without long reads): one branch per read
                    unsigned done = 0;
#pragma unroll
                    for (int k = 0; k < kReadsPerThread; ++k) {
                        const bool go = ((b.pending >> k) & 1u) && b.rs[k] < tend_rel;
                        done |= go ? 1u << k : 0u;
                        const int s = b.rs[k] > 0 ? b.rs[k] : 0, e = b.rs[k] + b.sp[k];
                        if (MC_APPLY_SHORT == 2) {
                            // no branch: a read that applies nothing adds 0 to
                            // its slots (a wave-uniform skip when no lane applies)
                            const bool ap = go && e > s;
                            if (__ballot(ap)) {
                                atomicAdd(&ring[ring_slot(s)], ap ? 1 : 0);
                                atomicAdd(&ring[ring_slot(e)], ap ? -1 : 0);
                            }
                        } else if (go && e > s) {
                            atomicAdd(&ring[ring_slot(s)], 1);
                            atomicAdd(&ring[ring_slot(e)], -1);
                        }
                    }
                    b.pending &= ~done;
                } else
#pragma unroll
                for (int k = 0; k < kReadsPerThread; ++k) {
                    if (((b.pending >> k) & 1u) && b.rs[k] < tend_rel) {
                        const int rs = b.rs[k], sp = b.sp[k];
                        if (sp <= short_max) {
                            const int s = rs > 0 ? rs : 0;
                            const int e = rs + sp;
                            if (e > s) {
                                atomicAdd(&ring[ring_slot(s)], 1);
                                atomicAdd(&ring[ring_slot(e)], -1);
                            }
                        } else if (rs >= 0) {   // long read: +1 here, -1 bucketed
                            atomicAdd(&ring[ring_slot(rs)], 1);
                        }
                        b.pending &= ~(1u << k);
                    }
                }
                bool all_done, ev_done;
                if (MC_K2_WAVE_ADVANCE) {
                    // each wave streams its own quarter of every batch (reads
                    // base + 256 w ..): it advances as soon as its lanes are
                    // done, no barrier; the tile scan's barrier orders the ring
                    all_done = __all(b.pending == 0);
                    ev_done = __all(eb.pending == 0);
                } else {
                    block_all2(hdr + 4 + 2 * kK2Waves, and_flip, b.pending == 0, eb.pending == 0, wave, lane,
                               all_done, ev_done);
                }
                const bool adv_reads = all_done && more;
                const bool adv_events = ev_done && ev_more;
                if (!adv_reads && !adv_events) break;
                if (adv_events) {
                    ev_base += kK2Batch;
                    ev_more = ev_base < ev_hi;
                    if (ev_more) load_events(eb, tile_ev, ev_base, ev_lo, ev_hi);
                }
                if (adv_reads) {
                    base += kK2Batch;
                    more = base < cend;
                    if (more) {
                        if (!kPf) issue_raw<kDirect>(nxt, base, A, cend);
                        finish(nxt, base);   // loaded one batch ago
                        if (kPf && base + kK2Batch < cend) issue_raw<kDirect>(nxt, base + kK2Batch, A, cend);
                    }
                }
            }
            // (per-wave advance: every wave's ring adds for this tile are in
            // before any wave reads its span of the tile)
            if (MC_K2_WAVE_ADVANCE) __syncthreads();
            // the previous tile's depth, held in v since its scan: its stores go
            // out only now, so a vmcnt wait in the apply loop above (batch
            // advance) found them a whole tile phase old instead of just issued
            if (kDefer && pend_T0 >= 0) {
                store_tile(pend_T0);
                pend_T0 = -1;
            }
            // ---- scan tile t: each wave owns kWaveSpan contiguous positions
            const int sb = t * kTileW + wave * kWaveSpan;   // chunk-relative start of my span
            int wave_total = 0;
#pragma unroll
            for (int j = 0; j < kChunks; ++j) {
                i32x4* slot = reinterpret_cast<i32x4*>(ring + ring_slot(sb + j * 256) + lane * 4);
                i32x4 x = *slot;
                *slot = i32x4{0, 0, 0, 0};
                x.y += x.x;
                x.z += x.y;
                x.w += x.z;
                const int incl = wave_incl_scan(x.w, lane);
                const int excl = incl - x.w + wave_total;
                x += excl;
                v[j] = x;
                wave_total += __builtin_amdgcn_readlane(incl, 63);
            }
            if (lane == 0) hdr[4 + wave] = wave_total;
            __syncthreads();
            int off = carry, tile_total = 0;
#pragma unroll
            for (int w = 0; w < kK2Waves; ++w) {
                const int tw = hdr[4 + w];
                if (w < wave) off += tw;
                tile_total += tw;
            }
            carry += tile_total;
#pragma unroll
            for (int j = 0; j < kChunks; ++j) {
                i32x4 x = v[j] + off;
                v[j] = x;
                my_max = max(my_max, max(max(x.x, x.y), max(x.z, x.w)));
            }
            if (kDefer) {
                pend_T0 = T0;   // stored after the next tile's apply loop (or at the chunk end)
            } else {
                store_tile(T0);
            }
            if (kStats) {
                // regions covering this tile, in order; the loop is uniform.
                // Only the value histogram is built here (runs of equal values
                // within a lane share one LDS atomic); min/max/sum/sumsq follow
                // from it in region_final_kernel.  Values outside the window
                // go to the lane's out-of-window record (hist_int4).
                while (rcur < R.n && r_gs < Tend) {
                    const int64_t rgs = r_gs, rge = r_ge;
                    const int lo = (int)((rgs > T0 ? rgs : T0) - T0);
                    const int hi = (int)((rge < Tend ? rge : Tend) - T0);
                    const bool full = lo == 0 && hi == kTileW;
#pragma unroll
                    for (int j = 0; j < kChunks; ++j) {
                        int y0 = v[j].x, y1 = v[j].y, y2 = v[j].z, y3 = v[j].w;
                        if (!full) {   // positions outside [lo, hi) -> -1
                            const int q0 = wave * kWaveSpan + j * 256 + lane * 4;
                            y0 = (q0 >= lo && q0 < hi) ? y0 : -1;
                            y1 = (q0 + 1 >= lo && q0 + 1 < hi) ? y1 : -1;
                            y2 = (q0 + 2 >= lo && q0 + 2 < hi) ? y2 : -1;
                            y3 = (q0 + 3 >= lo && q0 + 3 < hi) ? y3 : -1;
                        }
                        hist_int4<HC::kBins>(hist_lane, hist_dummy, ovr, y0, y1, y2, y3, r_base);
                    }
                    if (rge <= Tend) {
                        ov_reg_spill(ovr, ovf);
                        flush_region<true, HC>(R, r_id, hist, ovf);
                        ++rcur;
                        if (rcur < R.n) {
                            r_gs = uload(R.gs, rcur);
                            r_ge = uload(R.ge, rcur);
                            r_id = uload(R.id, rcur);
                            r_base = kDirect ? direct_window_base(D.win, win_parity, uload(R.rtid, r_id))
                                             : uload(R.base, rcur);
                        }
                    } else {
                        break;
                    }
                }
            }
        }
        if (kDefer && pend_T0 >= 0) store_tile(pend_T0);   // the chunk's last tile
        if (kStats) ov_reg_spill(ovr, ovf);   // ordered by the barrier below
        __syncthreads();   // everyone is past hdr / ring of this chunk (and its atomics)
        if (kStats) {
            // a region still open at the chunk end has partials here; the
            // barrier above and the one after the ring zeroing bracket it
            if (rcur < R.n && r_gs < C0 + chunk_w) flush_region<false, HC>(R, r_id, hist, ovf);
        }
        if (threadIdx.x == 0) hdr[0] = kAhead ? ticket : take_chunk(queue, n_chunks);
        for (int k = threadIdx.x * 4; k < kTileW; k += kK2Block * 4)
            *reinterpret_cast<i32x4*>(ring + ring_tail + k) = i32x4{0, 0, 0, 0};
    }
    // one atomic per workgroup (same-address atomics of every wave at the end of
    // the launch serialise); hdr[8..11] are free once the queue is drained
    my_max = wave_max(my_max);
    if (lane == 0) hdr[4 + kK2Waves + wave] = my_max;
    __syncthreads();
    if (threadIdx.x == 0) {
        int m = 0;
#pragma unroll
        for (int w = 0; w < kK2Waves; ++w) m = max(m, hdr[4 + kK2Waves + w]);
        if (m > 0) atomicMax(max_depth, m);
    }
    if (kDirect) direct_flush(dacc, D, ring);   // (ring: free now)
}

// ----------------------------------------------------------------- K3

// Statistics setup in one launch: zero the per-region histograms and
// below-window counts (low may be null), initialise the accumulators, and build
// chunk_first[c] = first region (sorted, non-overlapping: ge increasing)
// whose end lies past the chunk start c * chunk_w.
__global__ void __launch_bounds__(kBlock)
fused_init_kernel(unsigned* __restrict__ hist, int64_t hist_words, unsigned* __restrict__ low,
                  RegionAcc* __restrict__ acc, int64_t R, const int64_t* __restrict__ fge,
                  int64_t nf, int64_t chunk_w, int64_t n_chunks, int64_t* __restrict__ chunk_first,
                  unsigned* __restrict__ queue, int* __restrict__ max_depth) {
    if (blockIdx.x == 0 && threadIdx.x < 8) {   // K2's chunk queues and max depth (may be null)
        if (queue) queue[threadIdx.x] = 0;
        if (max_depth && threadIdx.x < 4) max_depth[threadIdx.x] = 0;
    }
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int64_t i0 = blockIdx.x * (int64_t)kBlock + threadIdx.x;
    for (int64_t q = i0; q * 4 < hist_words; q += stride)   // hist_words % 4 == 0
        *reinterpret_cast<i32x4*>(hist + q * 4) = i32x4{0, 0, 0, 0};
    for (int64_t r = i0; r < R; r += stride) {
        if (low) low[r] = 0;
        acc[r].sum = 0;
        acc[r].sumsq = 0;
        acc[r].min = 0x7fffffff;
        acc[r].max = 0;
    }
    for (int64_t c = i0; c < n_chunks; c += stride) {
        const int64_t C0 = c * chunk_w;
        int64_t lo = 0, hi = nf;                  // upper_bound(fge, C0)
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (fge[mid] <= C0) lo = mid + 1;
            else hi = mid;
        }
        chunk_first[c] = lo;
    }
}

// Debug check of the skipped fused_init (MC_CHECK_CLEAN=1 in the environment):
// the buffers a clean call relies on hold exactly what fused_init_kernel
// would write; every word that does not counts into *bad.
__global__ void __launch_bounds__(kBlock)
fused_clean_check_kernel(const unsigned* __restrict__ hist, int64_t hist_words, const unsigned* __restrict__ low,
                         const RegionAcc* __restrict__ acc, int64_t R, const unsigned* __restrict__ queue,
                         const int* __restrict__ max_depth, unsigned long long* __restrict__ bad) {
    unsigned long long n = 0;
    if (blockIdx.x == 0 && threadIdx.x < 8) {
        if (queue && queue[threadIdx.x] != 0) ++n;
        if (max_depth && threadIdx.x < 4 && max_depth[threadIdx.x] != 0) ++n;
    }
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int64_t i0 = blockIdx.x * (int64_t)kBlock + threadIdx.x;
    for (int64_t q = i0; q < hist_words; q += stride) n += hist[q] != 0;
    for (int64_t r = i0; r < R; r += stride) {
        n += (low && low[r] != 0) ? 1 : 0;
        n += (acc[r].sum != 0) + (acc[r].sumsq != 0) + (acc[r].min != 0x7fffffff) + (acc[r].max != 0);
    }
    n = (unsigned long long)wave_sum64((long long)n);
    if ((threadIdx.x & 63) == 0 && n) atomicAdd(bad, n);
}

// One workgroup per segment (<= kSeg positions of one region, clipped to
// the contig extent).  Builds the value histogram only (bins 0..nbins-1 cover
// every depth: nbins = max depth + 1); region_final_kernel derives min, max,
// sum and sum of squares from it.  Each thread keeps 4 int4 loads in flight;
// runs of equal values within an int4 share one atomic.
template <bool kLdsHist>
__global__ void __launch_bounds__(kBlock)
region_seg_kernel(const int32_t* __restrict__ depth, const int64_t* __restrict__ seg_gs,
                  const int64_t* __restrict__ seg_ge, const int32_t* __restrict__ seg_reg,
                  int nbins, unsigned* __restrict__ hist, RegionAcc* __restrict__ acc) {
    extern __shared__ __attribute__((aligned(16))) unsigned h[];
    const int64_t sgi = blockIdx.x;
    const int64_t gs = seg_gs[sgi], ge = seg_ge[sgi];
    const int r = seg_reg[sgi];
    unsigned* ghist = hist + (int64_t)r * nbins;
    unsigned* hh = kLdsHist ? h : ghist;
    if (kLdsHist) {   // 16-byte stores (the LDS block is rounded up to whole int4s)
        for (int k = threadIdx.x * 4; k < nbins; k += kBlock * 4)
            *reinterpret_cast<i32x4*>(h + k) = i32x4{0, 0, 0, 0};
        __syncthreads();
    }
    constexpr int kU = 4;                                // int4 loads in flight per thread
    int vmax = 0;
    unsigned vmin = 0xffffffffu;                         // (unsigned: the -1 pads never win)
    const int64_t a4 = gs & ~(int64_t)3;
    for (int64_t p0 = a4 + (int64_t)threadIdx.x * 4; p0 < ge; p0 += (int64_t)kBlock * 4 * kU) {
        i32x4 x[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t p = p0 + (int64_t)u * kBlock * 4;
            x[u] = p < ge ? __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(depth + p))
                          : i32x4{-1, -1, -1, -1};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t p = p0 + (int64_t)u * kBlock * 4;
            // positions outside [gs, ge) become -1 and are skipped
            const int y0 = (p >= gs && p < ge) ? x[u].x : -1;
            const int y1 = (p + 1 >= gs && p + 1 < ge) ? x[u].y : -1;
            const int y2 = (p + 2 >= gs && p + 2 < ge) ? x[u].z : -1;
            const int y3 = (p + 3 >= gs && p + 3 < ge) ? x[u].w : -1;
            const bool s1 = y1 != y0, s2 = y2 != y1, s3 = y3 != y2;
            const int l2 = s3 ? 1 : 2;
            const int l1 = s2 ? 1 : l2 + 1;
            const int l0 = s1 ? 1 : l1 + 1;
            if (y0 >= 0) atomicAdd(&hh[y0], (unsigned)l0);
            if (s1 && y1 >= 0) atomicAdd(&hh[y1], (unsigned)l1);
            if (s2 && y2 >= 0) atomicAdd(&hh[y2], (unsigned)l2);
            if (s3 && y3 >= 0) atomicAdd(&hh[y3], 1u);
            vmax = max(vmax, max(max(y0, y1), max(y2, y3)));
            if (kLdsHist)
                vmin = min(vmin, min(min((unsigned)y0, (unsigned)y1), min((unsigned)y2, (unsigned)y3)));
        }
    }
    vmax = wave_max(vmax);                   // bounds K3b's scan of this region's bins
    if ((threadIdx.x & 63) == 0 && vmax > 0) atomicMax(&acc[r].max, vmax);
    if (kLdsHist) {
        // flush only the segment's value range [lo, hi] (its bins are all
        // that can be non-zero; the fallback regions of the fused path have
        // ~16 Ki bins of which a segment touches a few hundred)
        __shared__ int ext[2 * kWaves];
        const int wmin = wave_min((int)min(vmin, 0x7fffffffu));
        if ((threadIdx.x & 63) == 0) {
            ext[threadIdx.x >> 6] = wmin;
            ext[kWaves + (threadIdx.x >> 6)] = vmax;
        }
        __syncthreads();
        int lo = ext[0], hi = ext[kWaves];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) {
            lo = min(lo, ext[w]);
            hi = max(hi, ext[kWaves + w]);
        }
        if (lo <= hi)   // (lo = INT_MAX when the segment has no position: lo + tid would overflow)
        for (int k = lo + (int)threadIdx.x; k <= hi && k < nbins; k += kBlock) {
            const unsigned c = h[k];
            if (c) atomicAdd(&ghist[k], c);
        }
    }
}

struct RegionOut {                     // mirrors mc_region_stat
    long long n, sum;
    unsigned long long sumsq;
    long long min, max, med_lo, med_hi, q23_sum, q23_cnt;
};

// One workgroup per region: the value histogram is walked in coalesced tiles
// of kBlock x 4 bins (a 64-bit block scan per tile gives every bin its rank
// range) for the ranks (n-1)/2, n/2 and the trimmed range [n/4, n - n/4)
// (pileup.py:21,24), and for min / max / sum / sum of squares.  Bin b holds
// the value base[r] + b (base = nullptr: 0).  Values outside the window were
// accumulated in `acc` (count below it in low[r]); with hist_stats,
// min/max/sum/sumsq are folded from the histogram and `acc`, otherwise `acc`
// holds the full statistics.  bound_by_max (K3: no window): acc[r].max, the
// region's largest depth from K3a, bounds the bins scanned.  out_row: row r
// is written to out[out_row[r]] (scattered fallback rows).  fallback[r] = 1
// when a needed rank lies outside the window: the host recomputes that region
// with the full-range K3.  Positions past the contig extent (zx) are zeros.
// One region's row from its value histogram (the body of region_final_kernel;
// every thread of the block calls it).  hr: the region's bins; a: its
// accumulator; out_p: where the row goes; fb: its fallback flag (may be null).
__device__ __forceinline__ void region_final_row(const unsigned* __restrict__ hr, int nbins, const RegionAcc& a,
                                                 long long n, long long zx, RegionOut* out_p, int* fb,
                                                 int hist_stats, long long base, long long low_in,
                                                 int bound_by_max) {
    __shared__ long long s_tot[2][kWaves];
    __shared__ long long s_red[4][kWaves];
    __shared__ long long s_med[2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // zeros past the extent land in bin 0 when the window starts at 0,
    // otherwise below the window
    const long long zx_bin = base == 0 ? zx : 0;
    const long long low = low_in + (base == 0 ? 0 : zx);
    const int nb = bound_by_max ? min(nbins, max(a.max, 0) + 1) : nbins;
    const long long r_lo = (n - 1) / 2, r_hi = n / 2;
    const long long q_lo = n / 4, q_hi = n - n / 4;
    if (threadIdx.x < 2) s_med[threadIdx.x] = 0;
    long long running = low;                 // values below the window rank first
    long long qsum = 0, s1 = 0;
    unsigned long long s2 = 0;
    int lmin = 0x7fffffff, lmax = -1;
    int buf = 0;
    for (int t0 = 0; t0 < nb; t0 += kBlock * 4, buf ^= 1) {
        const int b = t0 + (int)threadIdx.x * 4;
        long long c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            c[k] = b + k < nb ? (long long)hr[b + k] + (b + k == 0 ? zx_bin : 0) : 0;
        const long long mine = c[0] + c[1] + c[2] + c[3];
        long long incl = mine;               // 64-bit wave scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const long long y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) s_tot[buf][wave] = incl;
        __syncthreads();                     // (double-buffered: one barrier per tile)
        long long cum = running + incl - mine, tile = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const long long tw = s_tot[buf][w];
            if (w < wave) cum += tw;
            tile += tw;
        }
        running += tile;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long long cnt = c[k];
            if (cnt == 0) continue;
            const long long v = base + b + k;
            const long long e = cum + cnt;
            if (r_lo >= cum && r_lo < e) s_med[0] = v;
            if (r_hi >= cum && r_hi < e) s_med[1] = v;
            const long long lo = cum > q_lo ? cum : q_lo;
            const long long hi = e < q_hi ? e : q_hi;
            if (hi > lo) qsum += (hi - lo) * v;
            s1 += cnt * v;
            s2 += (unsigned long long)cnt * (unsigned long long)(v * v);
            lmin = min(lmin, b + k);
            lmax = max(lmax, b + k);
            cum = e;
        }
    }
    const long long in_hist = running - low;
    qsum = wave_sum64(qsum);
    s1 = wave_sum64(s1);
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) s2 += __shfl_xor(s2, d, 64);
    lmin = wave_min(lmin);
    lmax = wave_max(lmax);
    if (lane == 0) {
        s_red[0][wave] = qsum;
        s_red[1][wave] = s1;
        s_red[2][wave] = (long long)s2;
        s_red[3][wave] = ((long long)lmin << 32) | (unsigned)(lmax + 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const long long win_lo = low, win_hi = low + in_hist;   // ranks held by the window
        if (fb)
            *fb = (n > 0 && (r_lo < win_lo || r_hi >= win_hi || q_lo < win_lo || q_hi - 1 >= win_hi)) ? 1 : 0;
        long long q = 0, t1 = 0;
        unsigned long long t2 = 0;
        int hmin = 0x7fffffff, hmax = -1;
        for (int w = 0; w < kWaves; ++w) {
            q += s_red[0][w];
            t1 += s_red[1][w];
            t2 += (unsigned long long)s_red[2][w];
            hmin = min(hmin, (int)(s_red[3][w] >> 32));
            hmax = max(hmax, (int)(s_red[3][w] & 0xffffffff) - 1);
        }
        RegionOut o;
        o.n = n;
        if (hist_stats) {
            const long long high = n - win_hi;        // values above the window
            o.sum = t1 + (long long)a.sum;
            o.sumsq = t2 + a.sumsq;
            if (low > 0) {
                long long m = a.min;                   // INT_MAX when only zeros are below
                if (base > 0 && zx > 0) m = 0;
                o.min = m;
            } else {
                o.min = in_hist > 0 ? base + hmin : a.min;
            }
            o.max = high > 0 ? (long long)a.max : (in_hist > 0 ? base + hmax : (long long)a.max);
            if (o.max < 0) o.max = 0;
        } else {
            o.sum = (long long)a.sum;
            o.sumsq = a.sumsq;
            const bool any_read = n - zx > 0;
            o.min = any_read ? a.min : 0;
            if (zx > 0 && o.min > 0) o.min = 0;
            o.max = any_read ? a.max : 0;
        }
        o.med_lo = s_med[0];
        o.med_hi = s_med[1];
        o.q23_sum = q;
        o.q23_cnt = q_hi - q_lo;
        if (n == 0) {
            o.min = o.max = o.med_lo = o.med_hi = o.q23_sum = o.q23_cnt = 0;
            o.sum = 0;
            o.sumsq = 0;
        }
        *out_p = o;
    }
}

__global__ void __launch_bounds__(kBlock)
region_final_kernel(const unsigned* __restrict__ hist, int nbins,
                    const RegionAcc* __restrict__ acc, const int64_t* __restrict__ n_total,
                    const int64_t* __restrict__ n_zero_extra, RegionOut* __restrict__ out,
                    int* __restrict__ fallback, int hist_stats,
                    const int32_t* __restrict__ base_of, const unsigned* __restrict__ low_of,
                    int bound_by_max, const int64_t* __restrict__ out_row) {
    const int r = blockIdx.x;
    region_final_row(hist + (int64_t)r * nbins, nbins, acc[r], n_total[r], n_zero_extra[r],
                     out + (out_row ? out_row[r] : r), fallback ? fallback + r : nullptr, hist_stats,
                     base_of ? base_of[r] : 0, low_of ? (long long)low_of[r] : 0, bound_by_max);
}

// ---- the fused call's exact recompute on the device ----------------------
// Regions whose ranks leave their LDS window (region_final_wave_kernel flags
// them and lists them in fb_list) are recomputed in the same call from the
// depth vector K2 just wrote, without the host round trip the K3 fallback
// takes: fb_seg_kernel builds each listed region's full value histogram
// (kLdsBins values, enough while the maximum depth is below it), workgroups
// splitting the region's positions, and fb_final_kernel derives its row
// and scatters it into place.  Both leave their buffers zeroed for the next
// call.  Listed regions beyond kFbSlots, or a maximum depth >= kLdsBins, are
// left to the host's K3 fallback.
constexpr int kFbSlots = 512;

// The histogram of depth[gs, ge) into h (LDS, nb bins), runs of equal values
// within an int4 sharing one atomic; returns this thread's max and min.
__device__ __forceinline__ void seg_hist(const int32_t* __restrict__ depth, int64_t gs, int64_t ge, unsigned* h,
                                         int nb, int& vmax, unsigned& vmin) {
    constexpr int kU = 4;
    const int64_t a4 = gs & ~(int64_t)3;
    for (int64_t p0 = a4 + (int64_t)threadIdx.x * 4; p0 < ge; p0 += (int64_t)kBlock * 4 * kU) {
        i32x4 x[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t q = p0 + (int64_t)u * kBlock * 4;
            x[u] = q < ge ? *reinterpret_cast<const i32x4*>(depth + q) : i32x4{-1, -1, -1, -1};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t q = p0 + (int64_t)u * kBlock * 4;
            // (values outside [0, nb) are never there after a K2 that ran; the
            // bound keeps a stale vector from writing past the LDS histogram)
            const int y0 = (q >= gs && q < ge && x[u].x < nb) ? x[u].x : -1;
            const int y1 = (q + 1 >= gs && q + 1 < ge && x[u].y < nb) ? x[u].y : -1;
            const int y2 = (q + 2 >= gs && q + 2 < ge && x[u].z < nb) ? x[u].z : -1;
            const int y3 = (q + 3 >= gs && q + 3 < ge && x[u].w < nb) ? x[u].w : -1;
            const bool s1 = y1 != y0, s2 = y2 != y1, s3 = y3 != y2;
            const int l2 = s3 ? 1 : 2;
            const int l1 = s2 ? 1 : l2 + 1;
            const int l0 = s1 ? 1 : l1 + 1;
            if (y0 >= 0) atomicAdd(&h[y0], (unsigned)l0);
            if (s1 && y1 >= 0) atomicAdd(&h[y1], (unsigned)l1);
            if (s2 && y2 >= 0) atomicAdd(&h[y2], (unsigned)l2);
            if (s3 && y3 >= 0) atomicAdd(&h[y3], 1u);
            vmax = max(vmax, max(max(y0, y1), max(y2, y3)));
            vmin = min(vmin, min(min((unsigned)y0, (unsigned)y1), min((unsigned)y2, (unsigned)y3)));
        }
    }
}

struct FbArgs {
    const int32_t* depth;
    const int32_t* rfused;             // [R] row -> fused entry, or -1 (staged)
    const int64_t* fgs;                // [nf] entry global start / end (staged)
    const int64_t* fge;
    const int64_t* ntot;               // [R] positions / positions past the extent (staged)
    const int64_t* nzx;
    const int* max_depth;              // K2's, as region_final_wave_kernel copied it (max_out)
    int32_t* list;                     // [kFbSlots] listed rows
    unsigned* cnt;                     // [2] per call parity
    int parity;
    unsigned* hist;                    // [kFbSlots][kLdsBins]
    RegionAcc* acc;                    // [kFbSlots]
    RegionOut* out;                    // the call's rows
};

// The last workgroup of the grid to get here writes seq to *stamp (mapped
// host memory): the host learns that a call's last kernel is done without a
// stream write command after it (~13 us per call: the command's own dispatch
// and the gap before it, C2 trace r05i).  The kernel's results that others
// read (rows, host flags) are written through to memory with system-scope
// stores (store_sys), so each wave only waits for its own stores: no L2
// write-back per workgroup (a system-scope fence per workgroup cost K3b
// +1 us at C2's one workgroup and +20 us at C3's 250).  done_cnt: a device
// counter, 0 between launches (the last workgroup resets it).  Every thread
// of every workgroup calls this.
//
// The host reads, once the stamp is seen and without any stream sync:
//   RegionOut rows (out[r]), the fallback flags (fallback[r]), K2's max depth
//   copy (max_out) and the direct-path verdict copy (dres_out)
// and each of them MUST be written with store_sys when `stamp` is set (the
// `wt` paths of final_wave_row); a plain store of any of them would sit in
// its XCD's L2 and race the host's spin.  The per-wave s_waitcnt vmcnt(0)
// orders those system-scope stores before this workgroup's counter
// increment; the last workgroup then releases at system scope (one fence per
// launch, not per workgroup) before publishing the stamp, which also covers
// its own writes.
__device__ __forceinline__ void grid_done_stamp(unsigned* done_cnt, unsigned long long* stamp,
                                                unsigned long long seq) {
    if (stamp == nullptr) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores are done
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(done_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            __hip_atomic_store(done_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope, last workgroup only
            __hip_atomic_store(stamp, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <class T>
__device__ __forceinline__ void store_sys(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(kBlock)
fb_seg_kernel(FbArgs F) {
    extern __shared__ __attribute__((aligned(16))) unsigned hb[];
    const int n = (int)min(F.cnt[F.parity], (unsigned)kFbSlots);
    const int maxd = *F.max_depth;
    if (n == 0 || maxd >= kLdsBins) return;
    const int nb = maxd + 1;
    const int per = max(1, (int)gridDim.x / n);        // workgroups per region
    __shared__ int ext[2 * kWaves];
    for (int w = blockIdx.x; w < n * per; w += gridDim.x) {
        const int i = w / per, part = w % per;
        const int k = F.rfused[F.list[i]];
        if (k < 0) continue;                           // no covered position: zeros only
        const int64_t gs0 = F.fgs[k], len = F.fge[k] - gs0;
        const int64_t gs = gs0 + len * part / per, ge = gs0 + len * (part + 1) / per;
        for (int q = threadIdx.x * 4; q < nb; q += kBlock * 4)
            *reinterpret_cast<i32x4*>(hb + q) = i32x4{0, 0, 0, 0};
        __syncthreads();
        int vmax = 0;
        unsigned vmin = 0xffffffffu;
        seg_hist(F.depth, gs, ge, hb, nb, vmax, vmin);
        vmax = wave_max(vmax);
        const int wmin = wave_min((int)min(vmin, 0x7fffffffu));
        if ((threadIdx.x & 63) == 0) {
            ext[threadIdx.x >> 6] = wmin;
            ext[kWaves + (threadIdx.x >> 6)] = vmax;
        }
        __syncthreads();
        int lo = ext[0], hi = ext[kWaves];
#pragma unroll
        for (int q = 1; q < kWaves; ++q) {
            lo = min(lo, ext[q]);
            hi = max(hi, ext[kWaves + q]);
        }
        unsigned* g = F.hist + (int64_t)i * kLdsBins;
        // (an empty part leaves lo = INT_MAX > hi: nothing to flush; lo + tid would overflow)
        if (lo <= hi)
        for (int q = lo + (int)threadIdx.x; q <= hi && q < nb; q += kBlock) {
            const unsigned c = hb[q];
            if (c) atomicAdd(&g[q], c);
        }
        if (threadIdx.x == 0 && hi > 0) atomicMax(&F.acc[i].max, hi);
        __syncthreads();                               // before the next item zeroes hb
    }
}

__device__ __forceinline__ void fb_final_row(const FbArgs& F) {
    if (blockIdx.x == 0 && threadIdx.x == 0) F.cnt[F.parity ^ 1] = 0;   // the next call's counter
    const int n = (int)min(F.cnt[F.parity], (unsigned)kFbSlots);
    const int maxd = *F.max_depth;
    const int b = blockIdx.x;
    if (b >= n || maxd >= kLdsBins) return;
    const int r = F.list[b];
    unsigned* hr = F.hist + (int64_t)b * kLdsBins;
    region_final_row(hr, maxd + 1, F.acc[b], F.ntot[r], F.nzx[r], F.out + r, nullptr, 1, 0, 0, 1);
    __syncthreads();
    for (int q = threadIdx.x; q <= maxd; q += kBlock) hr[q] = 0;
    if (threadIdx.x == 0) {
        F.acc[b].sum = F.acc[b].sumsq = 0;
        F.acc[b].min = 0x7fffffff;
        F.acc[b].max = 0;
    }
}

__global__ void __launch_bounds__(kBlock)
fb_final_kernel(FbArgs F) {
    fb_final_row(F);
}

// The fused path's finalize: one wave per region (4 per workgroup) over its
// kHistBins-bin window, the same rules as region_final_kernel with base_of,
// low_of and hist_stats set and no row scatter.  A 256-thread block per
// region spent most of its time being dispatched (C5: 10,000 regions,
// 40 us).  Lane L owns bins [L * kFinPer, L * kFinPer + kFinPer).  Block 0
// also copies K2's max depth to max_out (mapped host memory: the fallback
// path needs it without a device-to-host copy).
template <int kVals>
__device__ __forceinline__ void
final_wave_row(unsigned* __restrict__ hist, int64_t R,
               RegionAcc* __restrict__ acc, const int64_t* __restrict__ n_total,
               const int64_t* __restrict__ n_zero_extra, RegionOut* __restrict__ out,
               int* __restrict__ fallback, const int32_t* __restrict__ base_of,
               unsigned* __restrict__ low_of, int* __restrict__ max_depth,
               int* __restrict__ max_out, unsigned* __restrict__ queue,
               const unsigned long long* __restrict__ dres_in, unsigned long long* __restrict__ dres_out,
               unsigned* __restrict__ fb_cnt, int32_t* __restrict__ fb_list,
               DirectWindow dwin, const int32_t* __restrict__ rtid, bool wt) {
    constexpr int kFinPer = (kVals + 63) / 64;
    const int lane = threadIdx.x & 63;
    // dres_out (mapped host memory): the direct K2's validation counters, so
    // the host reads its verdict with the flags, without a copy command
    // (wt: the call's last kernel, stamping: its host-visible results are
    // written through with system-scope stores; those cost K3b 3x at C5's
    // 10 k regions, so only then)
    if (blockIdx.x == 0 && dres_out && threadIdx.x < kDresWords) {
        if (wt) store_sys(dres_out + threadIdx.x, dres_in[threadIdx.x]);
        else dres_out[threadIdx.x] = dres_in[threadIdx.x];
    }
    // queue != null: leave the fused buffers as fused_init_kernel does (zero
    // histograms and below-window counts, initial accumulators, K2's queue
    // and max depth), so a repeated call on the same regions skips that launch
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (max_out) {
            if (wt) store_sys(max_out, *max_depth);
            else *max_out = *max_depth;
        }
        if (queue) {
            for (int k = 0; k < 4; ++k) max_depth[k] = 0;
            for (int k = 0; k < 8; ++k) queue[k] = 0;
        }
    }
    const int64_t r = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (r >= R) return;
    unsigned* hr = hist + r * kVals;
    const long long n = n_total[r];
    const long long zx = n_zero_extra[r];
    // (direct path: the window K2 used, from the probe's samples)
    const long long base = rtid ? direct_window_base(dwin, dwin.parity, __builtin_amdgcn_readfirstlane(rtid[r]))
                                : base_of[r];
    const long long zx_bin = base == 0 ? zx : 0;
    const long long low = (long long)low_of[r] + (base == 0 ? 0 : zx);
    const long long r_lo = (n - 1) / 2, r_hi = n / 2;
    const long long q_lo = n / 4, q_hi = n - n / 4;
    // bins k * 64 + lane (row k of the region's bins: one coalesced load per
    // row), a 64-bit DPP scan per row carried across rows
    long long c[kFinPer];
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
        const int b = k * 64 + lane;
        c[k] = b < kVals ? (long long)hr[b] + (b == 0 ? zx_bin : 0) : 0;
    }
    if (queue) {
#pragma unroll
        for (int k = 0; k < kFinPer; ++k)
            if (k * 64 + lane < kVals && c[k]) hr[k * 64 + lane] = 0;
    }
    long long qsum = 0, s1 = 0, med_lo = -1, med_hi = -1;
    unsigned long long s2 = 0;
    long long run = low;                      // ranks before row k
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
        const long long cnt = c[k];
        const long long incl = wave_incl_scan64(cnt);
        const long long cum = run + incl - cnt;
        run += readlane64(incl, 63);
        if (cnt == 0) continue;
        const long long v = base + k * 64 + lane;
        const long long e = cum + cnt;
        if (r_lo >= cum && r_lo < e) med_lo = v;
        if (r_hi >= cum && r_hi < e) med_hi = v;
        const long long lo = cum > q_lo ? cum : q_lo;
        const long long hi = e < q_hi ? e : q_hi;
        if (hi > lo) qsum += (hi - lo) * v;
        s1 += cnt * v;
        s2 += (unsigned long long)cnt * (unsigned long long)(v * v);
    }
    const long long in_hist = run - low;
    // the lowest and highest occupied bins
    int lmin = 0x7fffffff, lmax = -1;
#pragma unroll
    for (int k = 0; k < kFinPer; ++k) {
        const unsigned long long m = __ballot(c[k] != 0);
        if (m) {
            lmin = k * 64 + __ffsll((long long)m) - 1;
            break;
        }
    }
#pragma unroll
    for (int k = kFinPer - 1; k >= 0; --k) {
        const unsigned long long m = __ballot(c[k] != 0);
        if (m) {
            lmax = k * 64 + 63 - __builtin_clzll(m);
            break;
        }
    }
    qsum = readlane64(wave_incl_scan64(qsum), 63);
    s1 = readlane64(wave_incl_scan64(s1), 63);
    s2 = (unsigned long long)readlane64(wave_incl_scan64((long long)s2), 63);
    // the one lane holding each rank, the first / last lane holding a bin
    const unsigned long long hm_lo = __ballot(med_lo >= 0), hm_hi = __ballot(med_hi >= 0);
    med_lo = hm_lo ? readlane64(med_lo, __ffsll((long long)hm_lo) - 1) : -1;
    med_hi = hm_hi ? readlane64(med_hi, __ffsll((long long)hm_hi) - 1) : -1;
    if (lane != 0) return;
    const long long win_lo = low, win_hi = low + in_hist;   // ranks held by the window
    const bool fb = n > 0 && (r_lo < win_lo || r_hi >= win_hi || q_lo < win_lo || q_hi - 1 >= win_hi);
    if (wt) store_sys(fallback + r, fb ? 1 : 0);
    else fallback[r] = fb ? 1 : 0;
    if (fb && fb_cnt) {   // listed for the device-side recompute (fb_seg_kernel)
        const unsigned slot = atomicAdd(fb_cnt, 1u);
        if (slot < (unsigned)kFbSlots) fb_list[slot] = (int32_t)r;
    }
    const RegionAcc a = acc[r];
    if (queue) {
        acc[r].sum = 0;
        acc[r].sumsq = 0;
        acc[r].min = 0x7fffffff;
        acc[r].max = 0;
        low_of[r] = 0;
    }
    RegionOut o;
    o.n = n;
    const long long high = n - win_hi;       // values above the window
    o.sum = s1 + (long long)a.sum;
    o.sumsq = s2 + a.sumsq;
    if (low > 0) {
        long long m = a.min;                 // INT_MAX when only zeros are below
        if (base > 0 && zx > 0) m = 0;
        o.min = m;
    } else {
        o.min = in_hist > 0 ? base + lmin : a.min;
    }
    o.max = high > 0 ? (long long)a.max : (in_hist > 0 ? base + lmax : (long long)a.max);
    if (o.max < 0) o.max = 0;
    o.med_lo = med_lo < 0 ? 0 : med_lo;
    o.med_hi = med_hi < 0 ? 0 : med_hi;
    o.q23_sum = qsum;
    o.q23_cnt = q_hi - q_lo;
    if (n == 0) {
        o.min = o.max = o.med_lo = o.med_hi = o.q23_sum = o.q23_cnt = 0;
        o.sum = 0;
        o.sumsq = 0;
    }
    if (wt) {   // written through: visible to the host and other streams once stored
        unsigned long long* w = reinterpret_cast<unsigned long long*>(out + r);
        const unsigned long long* v = reinterpret_cast<const unsigned long long*>(&o);
#pragma unroll
        for (int k = 0; k < (int)(sizeof(RegionOut) / 8); ++k) store_sys(w + k, v[k]);
    } else {
        out[r] = o;
    }
}

// stamp != null (the call's last kernel): grid_done_stamp after the rows,
// flags, K2's max depth and verdict copy.
template <int kVals>
__global__ void __launch_bounds__(kBlock)
region_final_wave_kernel(unsigned* __restrict__ hist, int64_t R,
                         RegionAcc* __restrict__ acc, const int64_t* __restrict__ n_total,
                         const int64_t* __restrict__ n_zero_extra, RegionOut* __restrict__ out,
                         int* __restrict__ fallback, const int32_t* __restrict__ base_of,
                         unsigned* __restrict__ low_of, int* __restrict__ max_depth,
                         int* __restrict__ max_out, unsigned* __restrict__ queue,
                         const unsigned long long* __restrict__ dres_in, unsigned long long* __restrict__ dres_out,
                         unsigned* __restrict__ fb_cnt, int32_t* __restrict__ fb_list,
                         DirectWindow dwin, const int32_t* __restrict__ rtid,
                         unsigned* __restrict__ done_cnt, unsigned long long* __restrict__ stamp,
                         unsigned long long seq) {
    final_wave_row<kVals>(hist, R, acc, n_total, n_zero_extra, out, fallback, base_of, low_of, max_depth,
                          max_out, queue, dres_in, dres_out, fb_cnt, fb_list, dwin, rtid, stamp != nullptr);
    grid_done_stamp(done_cnt, stamp, seq);
}

}  // namespace mc
