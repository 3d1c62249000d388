// htslib's pileup read cap (pysam's max_depth, metacov/pileup.py:13) on the
// device: the same closed form as the host's mc_depth_cap_mask
// (csrc/depth_cap.cpp), one wave per pileup query.
//
// For a group of reads starting at s (the query's reads with pos == s, in
// file order): C = kept reads before the group still buffered at s (end >=
// s); the group's first read is kept; a further read j is kept while
// 1 + C + b_j <= maxcnt, b_j the group's buffered kept reads before it
// (the first one, and later ones with span > 0).  b only grows while reads
// are kept, so with b_j computed as if every earlier read of the group were
// kept the rule is unchanged: keep_j = first || 1 + C + b_j(all kept) <=
// maxcnt, a prefix of the group.
//
// The wave walks the query's reads in chunks of 64.  C comes from a ring of
// end counts in LDS (E[end mod ring], live ends lie in [ptr, ptr + max
// span]): `total` buffered reads were inserted, `removed` had ends before the
// current start.  A chunk whose every read must be kept (live + 64 <=
// maxcnt: no group in it can reach the cap) is applied in bulk — ends
// inserted, the pointer moved to its last start; otherwise its groups go in
// order, each a few ballots and LDS atomics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mc {

constexpr int kCapRing = 32768;               // LDS ints (128 KiB): max span must stay below it
constexpr int kCapRingMask = kCapRing - 1;
constexpr int kCapStage = 1024;               // reads per staged batch
constexpr int kCapPer = kCapStage / 64;
constexpr int kCapLdsBytes = (kCapRing + 6 * kCapStage) * 4;   // ring + two staged batches

struct CapWave {
    int* E;
    long long total = 0, removed = 0;         // buffered kept reads inserted / with end before ptr
    int ptr = 0;
    bool have_ptr = false;
    int lane = 0;

    // removes the ends before s (wave-uniform call)
    __device__ void advance(int s) {
        if (!have_ptr) {
            ptr = s;
            have_ptr = true;
            return;
        }
        if (s <= ptr) return;
        const long long n = (long long)s - ptr;
        if (n <= 8) {   // the usual step in a pile: a few slots, read by every lane alike (no reduction)
            int acc = 0;
            for (int x = 0; x < (int)n; ++x) {
                const int k = (ptr + x) & kCapRingMask;
                acc += E[k];
            }
            for (int x = lane; x < (int)n; x += 64) E[(ptr + x) & kCapRingMask] = 0;
            removed += __builtin_amdgcn_readfirstlane(acc);
            ptr = s;
            return;
        }
        int acc = 0;
        if (n >= kCapRing) {   // every live end lies before s
            for (int k = lane; k < kCapRing; k += 64) {
                acc += E[k];
                E[k] = 0;
            }
        } else {
            for (long long x = lane; x < n; x += 64) {
                const int k = (int)((ptr + x) & kCapRingMask);
                acc += E[k];
                E[k] = 0;
            }
        }
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        removed += acc;
        ptr = s;
    }
};

__device__ __forceinline__ int cap_lane_popc_below(unsigned long long m, int lane) {
    return __popcll(m & ((1ull << lane) - 1ull));
}

// One wave (64 threads) per query segment [seg[q], seg[q + 1]).
//   inq (optional): 0 for a read outside the query (not seen by the pileup)
//   keep (optional): 1 for a kept read of the query, else 0
//   zero_dropped: span[i] = 0 for dropped and out-of-query reads (they then
//                 add no depth: the batch keeps its order and size)
//   max_span: an upper bound of the spans (< kCapRing - 64)
__global__ void __launch_bounds__(64)
cap_walk_kernel(const int32_t* __restrict__ pos, int32_t* __restrict__ span, const uint8_t* __restrict__ inq,
                const int64_t* __restrict__ seg, int max_depth, int max_span, uint8_t* __restrict__ keep,
                int zero_dropped, unsigned long long* __restrict__ dropped_out) {
    extern __shared__ int cap_lds[];
    CapWave W;
    W.E = cap_lds;
    W.lane = threadIdx.x;
    const int lane = threadIdx.x;
    const int64_t i0 = seg[blockIdx.x], i1 = seg[blockIdx.x + 1];
    for (int k = lane; k < kCapRing; k += 64) cap_lds[k] = 0;
    __syncthreads();
    const long long maxcnt = max_depth;
    long long C = 0, b = 0;                    // the open group's C and buffered kept reads
    int last_pos = 0;
    bool have_last = false;
    unsigned long long dropped = 0;
    // reads staged through LDS in batches of kCapStage (16 chunks), the next
    // batch's loads in flight while the current one is walked (a chunk's
    // loads waited on one at a time left the walk latency-bound)
    int* st_pos = cap_lds + kCapRing;                 // [2][kCapStage]
    int* st_span = st_pos + 2 * kCapStage;            // [2][kCapStage]
    int* st_q = st_span + 2 * kCapStage;              // [2][kCapStage]
    int rp[kCapPer], rs[kCapPer], rq[kCapPer];
    auto load_batch = [&](int64_t b0) {
#pragma unroll
        for (int j = 0; j < kCapPer; ++j) {
            const int64_t i = b0 + j * 64 + lane;
            const bool ok = i < i1;
            rp[j] = ok ? pos[i] : 0;
            rs[j] = ok ? span[i] : 0;
            rq[j] = ok ? (inq ? (int)inq[i] : 1) : 0;
        }
    };
    auto stage_batch = [&](int buf) {
#pragma unroll
        for (int j = 0; j < kCapPer; ++j) {
            st_pos[buf * kCapStage + j * 64 + lane] = rp[j];
            st_span[buf * kCapStage + j * 64 + lane] = rs[j];
            st_q[buf * kCapStage + j * 64 + lane] = rq[j];
        }
    };
    if (i0 < i1) {
        load_batch(i0);
        stage_batch(0);
    }
    for (int64_t c0 = i0; c0 < i1; c0 += 64) {
        const int64_t i = c0 + lane;
        const bool valid = i < i1;
        const int64_t rel = c0 - i0;
        const int buf = (int)((rel / kCapStage) & 1);
        const int at = (int)(rel % kCapStage);
        if (at == 0 && c0 + kCapStage < i1) load_batch(c0 + kCapStage);   // the next batch, in flight
        const int p = st_pos[buf * kCapStage + at + lane], sp = st_span[buf * kCapStage + at + lane];
        const bool q = valid && st_q[buf * kCapStage + at + lane] != 0;
        const unsigned long long qm = __ballot(q);
        bool kept = false;
        if (qm) {
            // the previous in-query read of each lane: a lower lane, or the last of the walk
            const unsigned long long below = qm & ((1ull << lane) - 1ull);
            const int prev_lane = below ? 63 - __builtin_clzll(below) : lane;
            int prevp = __shfl(p, prev_lane, 64);
            const bool has_prev = below != 0 || have_last;
            if (!below) prevp = last_pos;
            const bool gstart = q && (!has_prev || p != prevp);
            const unsigned long long gm = __ballot(gstart);
            const int f_lane = gm ? __builtin_ctzll(gm) : 0;
            const int l_lane = gm ? 63 - __builtin_clzll(gm) : 0;
            const int s_first = __builtin_amdgcn_readlane(p, f_lane), s_last = __builtin_amdgcn_readlane(p, l_lane);
            const long long live = W.total - W.removed;
            // bulk: every end inserted first, then the pointer moved to the last
            // start (ends before it would have left by then anyway); the ring
            // must hold [ptr, s_last + max span] meanwhile
            const long long base = W.have_ptr ? W.ptr : s_first;
            const bool bulk = live + 64 <= maxcnt && (!gm || (long long)s_last - base + max_span + 64 < kCapRing);
            if (bulk) {
                if (gm && !W.have_ptr) W.advance(s_first);   // (the walk's first start: sets the pointer)
                const bool u = q && (gstart || sp > 0);
                if (u) atomicAdd(&cap_lds[(p + sp) & kCapRingMask], 1);
                W.total += __popcll(__ballot(u));
                kept = q;
                if (gm) {
                    W.advance(s_last);
                    // the last group stays open: its C, and its buffered reads so far
                    const unsigned long long tail = qm & ~((1ull << l_lane) - 1ull);
                    const unsigned long long tu = __ballot(u) & tail;
                    b = __popcll(tu);
                    C = W.total - W.removed - b;
                } else {
                    b += __popcll(__ballot(u));
                }
            } else {
                // groups in lane order: first the open group's continuation
                unsigned long long todo = gm;
                int first = -1;                        // the part's group-start lane (-1: continuation)
                unsigned long long part = qm & (gm ? ((gm & (~gm + 1)) - 1ull) : ~0ull);
                for (;;) {
                    if (part) {
                        const bool in = (part >> lane) & 1ull;
                        const bool u = in && (lane == first || sp > 0);
                        const unsigned long long um = __ballot(u);
                        const long long bb = b + cap_lane_popc_below(um, lane);
                        const bool k = in && (lane == first || 1 + C + bb <= maxcnt);
                        const unsigned long long km = __ballot(k);
                        if (k && u) atomicAdd(&cap_lds[(p + sp) & kCapRingMask], 1);
                        const int t = __popcll(km & um);
                        W.total += t;
                        b += t;
                        dropped += __popcll(part & ~km);
                        if (in) kept = k;
                    }
                    if (!todo) break;
                    const unsigned long long low = todo & (~todo + 1);
                    first = __builtin_ctzll(todo);
                    todo ^= low;
                    const unsigned long long next = todo & (~todo + 1);
                    part = qm & ~(low - 1ull) & (next ? next - 1ull : ~0ull);
                    W.advance(__builtin_amdgcn_readlane(p, first));
                    C = W.total - W.removed;
                    b = 0;
                }
            }
            const int hl = 63 - __builtin_clzll(qm);
            last_pos = __builtin_amdgcn_readlane(p, hl);
            have_last = true;
        }
        if (valid) {
            if (keep) keep[i] = kept ? 1 : 0;
            if (zero_dropped && !kept && sp != 0) span[i] = 0;
        }
        if (at + 64 == kCapStage && c0 + 64 < i1) stage_batch(buf ^ 1);
    }
    if (lane == 0 && dropped) atomicAdd(dropped_out, dropped);
}

// flags[i] = 1 where a new query (tid) starts; bad: an unsorted pair
__global__ void __launch_bounds__(256)
cap_seg_flags_kernel(const int32_t* __restrict__ tid, const int32_t* __restrict__ pos, int64_t n,
                     uint8_t* __restrict__ flags, unsigned* __restrict__ bad) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool f = i == 0;
        if (i > 0) {
            const int32_t t0 = tid[i - 1], t1 = tid[i];
            f = t1 != t0;
            if (t1 < t0 || (t1 == t0 && pos[i] < pos[i - 1])) atomicOr(bad, 1u);
        }
        flags[i] = f ? 1 : 0;
    }
}

// The region queries of a capped recompute: region r's reads are those of
// contig qt[r] in [lo[r], hi[r]) of the source arrays; those overlapping
// [qs[r], qe[r]) by bam_endpos (pos + max(span, 1) > qs) are in the query.
// Output slot k of region r (off[r] <= k < off[r + 1]) gets local contig r.
__global__ void __launch_bounds__(256)
cap_gather_kernel(const int32_t* __restrict__ spos, const int32_t* __restrict__ sspan,
                  const int64_t* __restrict__ lo, const int64_t* __restrict__ off, const int64_t* __restrict__ qs,
                  int32_t* __restrict__ tid_out, int32_t* __restrict__ pos_out, int32_t* __restrict__ span_out,
                  uint8_t* __restrict__ inq) {
    const int r = blockIdx.y;
    const int64_t a = off[r], n = off[r + 1] - a, src = lo[r];
    const long long start = qs[r];
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t p = spos[src + k], s = sspan[src + k];
        tid_out[a + k] = r;
        pos_out[a + k] = p;
        span_out[a + k] = s;
        inq[a + k] = (long long)p + (s > 1 ? s : 1) > start ? 1 : 0;
    }
}

// [lo, hi) of each region in the (tid, pos)-sorted source: the reads of contig
// qt with qs - max_span <= pos < qe.  One thread per region.
__global__ void __launch_bounds__(64)
cap_ranges_kernel(const int32_t* __restrict__ tid, const int32_t* __restrict__ pos, int64_t n,
                  const int32_t* __restrict__ qt, const int64_t* __restrict__ qs, const int64_t* __restrict__ qe,
                  int R, int max_span, int64_t* __restrict__ lo, int64_t* __restrict__ hi) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    auto lower = [&](int32_t t, long long p) {   // first index with (tid, pos) >= (t, p)
        int64_t a = 0, b = n;
        while (a < b) {
            const int64_t m = (a + b) >> 1;
            const int32_t tm = tid[m];
            if (tm < t || (tm == t && (long long)pos[m] < p)) a = m + 1;
            else b = m;
        }
        return a;
    };
    const long long from = qs[r] - (max_span > 1 ? max_span : 1);
    lo[r] = lower(qt[r], from);
    hi[r] = lower(qt[r], qe[r]);
}

// max span of a read array (atomicMax per workgroup)
__global__ void __launch_bounds__(256)
cap_max_span_kernel(const int32_t* __restrict__ span, int64_t n, int* __restrict__ out) {
    int m = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = max(m, span[i]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    __shared__ int red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(red[0], red[1]), max(red[2], red[3]));
        if (m > 0) atomicMax(out, m);
    }
}

}  // namespace mc
