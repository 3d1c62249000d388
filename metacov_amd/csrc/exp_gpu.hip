// pileup.experimental's read pass on the device (metacov/pileup.py:90-151),
// against the read table a reads-mode GPU decode left in HBM — the same
// aggregates as the host pass (csrc/exp_reads.cpp, one_region), computed
// without copying the table back.
//
// Per region the reference walks bam.fetch(ref, start, end) in file order:
//   secondary (0x100) and improper (!0x2) reads are counted and skipped;
//   a proper read pairs with the earlier unpaired read of the same name
//   (dict x), adding the cov2 slice and the wnf term; its k-mer correction
//   rcor gives 1/rcor for cov_cor and cor, "RCOR is ZERO" when 0; errors
//   (no SEQ, no reference length, k_cor None at a pair) end the walk.
// Here:
//   classify   every candidate read of every region (a 2-D grid: slots x
//              regions); proper reads get a 63-bit key hash(name, region)
//   sort       (key, slot) pairs (stable radix sort: equal keys stay in
//              read order), then one thread per run of equal keys pairs
//              the run's reads as the dict would (names compared exactly,
//              so a hash collision only lengthens a run)
//   per read   the pair term, 1/rcor, the zero event and the error, in the
//              reference's evaluation order; the first error's slot per
//              region (atomicMin) — events before it are kept
//   reduce     counts per region (wave-aggregated atomics); wnf = the pair
//              terms in read order of the second mate, summed in turn;
//              starts: (region, rstart) sorted, the last read per position
//              kept; cor summed in turn and as numpy's add.reduce (8192-
//              element buffers, pairwise within, exact on the sparse
//              entries); cov_cor per 8192-position block in LDS with the
//              covers applied in read order (the reference's per-position
//              float sums), then numpy's pairwise sum of the block.
// Every floating-point operation is the reference's, in its order (no FMA
// contraction in this file).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "../../include/metacov_amd.h"
#include "common.h"
#include "exp_gpu.h"

#define HIP_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            mc::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                          __FILE__, __LINE__);                                 \
            return MC_E_HIP;                                                   \
        }                                                                      \
    } while (0)

#pragma clang fp contract(off)

namespace {

constexpr uint32_t kNoKmer = 0xFFFFFFFFu;
constexpr uint8_t kNoSeq = 1, kNoRefLen = 2;
constexpr unsigned long long kNone = ~0ull;
constexpr int kBuf = 8192;        // numpy's reduction buffer
constexpr int kLeaf = 128;        // pairwise_sum's leaf
constexpr int kC = 8;             // per-region integer counters

// counters [R][kC]
enum : int { cSecondary = 0, cImproper, cNreads, cCov, cCov2, cPairs, cAnyInv, cStarts };

template <class T>
struct Buf {
    T* p = nullptr;
    size_t cap = 0;
    Buf() = default;
    Buf(const Buf&) = delete;
    Buf& operator=(const Buf&) = delete;
    ~Buf() {
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

struct Tab {
    const double* val[2];
    const uint8_t* has[2];
    int none;
};

__device__ __forceinline__ bool tab_lookup(const Tab& T, int which, uint32_t code, double* v) {
    if (T.none || code == kNoKmer || !T.has[which][code]) return false;
    *v = T.val[which][code];
    return true;
}

__device__ __forceinline__ long long slice_index(long long i, long long L) {
    if (i < 0) {
        i += L;
        return i < 0 ? 0 : i;
    }
    return i > L ? L : i;
}

// ---- table index --------------------------------------------------------

__global__ void __launch_bounds__(256)
idx_first_kernel(const int32_t* __restrict__ tid, int64_t n, int32_t n_ref, int64_t* __restrict__ first) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > n_ref) return;
    int64_t a = 0, b = n;
    while (a < b) {
        const int64_t m = (a + b) >> 1;
        if (tid[m] < t) a = m + 1;
        else b = m;
    }
    first[t] = a;
}

__global__ void __launch_bounds__(256)
idx_scan_kernel(const int32_t* __restrict__ tid, const int32_t* __restrict__ pos, const int64_t* __restrict__ end,
                int64_t n, int32_t n_ref, unsigned long long* __restrict__ max_span,
                unsigned long long* __restrict__ bad) {
    const int lane = threadIdx.x & 63;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = base + threadIdx.x;
        const bool ok = i < n;
        int32_t t = ok ? tid[i] : -1;
        const long long sp = ok ? end[i] - pos[i] : 0;
        if (ok && i > 0) {
            const int32_t t0 = tid[i - 1];
            if (t < t0 || (t == t0 && pos[i] < pos[i - 1])) atomicMin(bad, (unsigned long long)i);
        }
        if (ok && (t < 0 || t >= n_ref)) {
            atomicMin(bad, (unsigned long long)i);
            t = -1;
        }
        // one atomic per wave when its lanes share a contig (sorted input)
        const int t0 = __shfl(t, 0, 64);
        const bool same = __all(t == t0 || !ok);
        if (same) {
            long long m = t == t0 ? sp : 0;
            for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
            if (lane == 0 && t0 >= 0 && m > 0) atomicMax(max_span + t0, (unsigned long long)m);
        } else if (t >= 0 && sp > 0) {
            atomicMax(max_span + t, (unsigned long long)sp);
        }
    }
}

// ---- regions ---------------------------------------------------------------

struct Regions {
    const int32_t* t;
    const int64_t* s;
    const int64_t* L;
    int64_t* lo;          // first candidate read
    const int64_t* off;   // [R + 1] slots
};

__global__ void __launch_bounds__(64)
ranges_kernel(const int32_t* __restrict__ pos, const int64_t* __restrict__ first,
              const unsigned long long* __restrict__ max_span, Regions G, int R, int64_t* __restrict__ hi) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= R) return;
    const int32_t t = G.t[q];
    const int64_t c0 = first[t], c1 = first[t + 1];
    long long from = G.s[q] - (long long)max_span[t];
    if (from < INT32_MIN) from = INT32_MIN;
    const long long to = G.s[q] + G.L[q];
    auto lower = [&](int64_t a, long long p) {
        int64_t b = c1;
        while (a < b) {
            const int64_t m = (a + b) >> 1;
            if ((long long)pos[m] < p) a = m + 1;
            else b = m;
        }
        return a;
    };
    const int64_t lo = lower(c0, from);
    G.lo[q] = lo;
    hi[q] = lower(lo, to);
}

__device__ __forceinline__ uint64_t name_key(const ExpDevTable& T, int64_t i, int q) {
    const uint8_t* p = T.names + T.name_off[i];
    const int n = T.name_len[i];
    uint64_t h = 1469598103934665603ull;
    for (int k = 0; k < n; ++k) {
        h ^= p[k];
        h *= 1099511628211ull;
    }
    h ^= (uint64_t)(q + 1) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    return h & ~(1ull << 63);
}

__device__ __forceinline__ bool names_equal(const ExpDevTable& T, int64_t i, int64_t j) {
    const int n = T.name_len[i];
    if (n != T.name_len[j]) return false;
    const uint8_t* a = T.names + T.name_off[i];
    const uint8_t* b = T.names + T.name_off[j];
    for (int k = 0; k < n; ++k)
        if (a[k] != b[k]) return false;
    return true;
}

// wave-aggregated per-region counter add (every lane of the block is in region q)
__device__ __forceinline__ void wave_add(unsigned long long* c, long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(c, (unsigned long long)v);
}

struct Slots {
    uint8_t* cls;         // 0 outside the query, 1 secondary, 2 improper, 3 proper
    int64_t* ridx;        // read of the slot
    int32_t* sreg;        // region of the slot
    uint64_t* key;        // pairing key (proper) / unique (others)
    uint32_t* sidx;       // slot number (sort values)
    int32_t* mate;        // earlier mate slot of a pair's second read, or -1
    uint8_t* open;        // pairing scratch
    uint8_t* err;         // 0 / 1 no SEQ / 2 no reference length / 3 k_cor None
    uint8_t* ev;          // rcor == 0
    double* term;         // the pair's wnf term
    int64_t* c2;          // the pair's cov2 slice length
    double* inv;          // 1 / rcor
    int64_t* rs;          // reference-shifted read start / end (region-relative)
    int64_t* re;
};

__global__ void __launch_bounds__(256)
classify_kernel(ExpDevTable T, Regions G, Slots S, unsigned long long* __restrict__ cnt) {
    const int q = blockIdx.y;
    const int64_t k0 = G.off[q], nq = G.off[q + 1] - k0, lo = G.lo[q];
    const long long s = G.s[q];
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < nq; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t kk = base + threadIdx.x;
        const bool ok = kk < nq;
        uint8_t c = 0;
        if (ok) {
            const int64_t k = k0 + kk, i = lo + kk;
            const int f = T.flag[i];
            c = T.end[i] <= s ? 0 : (f & 0x100) ? 1 : !(f & 2) ? 2 : 3;
            S.cls[k] = c;
            S.ridx[k] = i;
            S.sreg[k] = q;
            S.key[k] = c == 3 ? name_key(T, i, q) : ((1ull << 63) | (uint64_t)k);
            S.sidx[k] = (uint32_t)k;
            S.mate[k] = -1;
            S.open[k] = 0;
        }
        wave_add(cnt + (size_t)q * kC + cSecondary, c == 1);
        wave_add(cnt + (size_t)q * kC + cImproper, c == 2);
    }
}

// one thread per run of equal keys: the dict of pileup.py:101-118 over the
// run's proper reads in read order (at most one open read per name)
__global__ void __launch_bounds__(256)
pair_kernel(ExpDevTable T, const uint64_t* __restrict__ key, const uint32_t* __restrict__ sidx, int64_t N, Slots S) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= N) return;
    const uint64_t kj = key[j];
    if ((kj >> 63) || (j > 0 && key[j - 1] == kj)) return;
    int64_t e = j + 1;
    while (e < N && key[e] == kj) ++e;
    if (e == j + 1) return;
    for (int64_t u = j; u < e; ++u) {
        const uint32_t su = sidx[u];
        const int64_t iu = S.ridx[su];
        bool paired = false;
        for (int64_t v = u - 1; v >= j; --v) {
            const uint32_t sv = sidx[v];
            if (!S.open[sv] || S.sreg[sv] != S.sreg[su] || !names_equal(T, iu, S.ridx[sv])) continue;
            S.mate[su] = (int32_t)sv;
            S.open[sv] = 0;
            paired = true;
            break;
        }
        if (!paired) S.open[su] = 1;
    }
}

// pileup.py:101-141 per proper read, in the reference's evaluation order
__global__ void __launch_bounds__(256)
read_kernel(ExpDevTable T, Tab tab, Regions G, Slots S, unsigned long long* __restrict__ err_at) {
    const int q = blockIdx.y;
    const int64_t k0 = G.off[q], nq = G.off[q + 1] - k0;
    const long long s = G.s[q], L = G.L[q];
    for (int64_t kk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; kk < nq; kk += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = k0 + kk;
        if (S.cls[k] != 3) continue;
        const int64_t i = S.ridx[k];
        const int f = T.flag[i];
        const uint8_t bi = T.bits[i];
        int err = 0;
        double term = 0;
        long long c2 = 0;
        const int32_t m = S.mate[k];
        if (m >= 0) {
            const int64_t j = S.ridx[m];
            const long long p0 = T.pos[i], p1 = T.pos[j];
            const long long a = (p0 < p1 ? p0 : p1) - s, b = (p0 < p1 ? p1 : p0) - s;
            c2 = slice_index(b + 1, L) - slice_index(a - 1, L);
            if (c2 < 0) c2 = 0;
            if (tab.none) {
                err = 3;
            } else if (bi & kNoSeq) {
                err = 1;
            } else {
                double x, y;
                if (!tab_lookup(tab, (f & 0x10) ? 1 : 0, T.kmer[i], &x)) {
                    term = 1;
                } else if (T.bits[j] & kNoSeq) {
                    err = 1;
                } else if (!tab_lookup(tab, (T.flag[j] & 0x10) ? 1 : 0, T.kmer[j], &y)) {
                    term = 1;
                } else {
                    const double p = x * y;
                    term = p == 0 ? 1.0 : 1.0 / p;
                }
            }
        }
        if (!err && (bi & kNoSeq)) err = 1;
        uint8_t ev = 0;
        double inv = 1.0;
        if (!err) {
            double rc;
            if (!tab_lookup(tab, (f & 0x40) ? 0 : 1, T.kmer[i], &rc)) rc = 1;
            if (rc == 0) {
                ev = 1;
                rc = 1;
            }
            inv = 1.0 / rc;
            if (bi & kNoRefLen) err = 2;
        }
        const long long rl = T.end[i] - T.pos[i];
        long long rs, re;
        if (f & 0x10) {
            re = (long long)T.pos[i] - s;
            rs = re - rl;
        } else {
            rs = (long long)T.pos[i] - s;
            re = rs + rl;
        }
        S.err[k] = (uint8_t)err;
        S.ev[k] = ev;
        S.term[k] = term;
        S.c2[k] = c2;
        S.inv[k] = inv;
        S.rs[k] = rs;
        S.re[k] = re;
        if (err) atomicMin(err_at + q, (unsigned long long)k);
    }
}

struct Event {
    uint32_t q;
    uint32_t k;
    uint64_t code;
};

// per proper read, once the first error of each region is known
__global__ void __launch_bounds__(256)
accum_kernel(ExpDevTable T, Regions G, Slots S, const unsigned long long* __restrict__ err_at,
             unsigned long long* __restrict__ cnt, uint8_t* __restrict__ pflag, uint64_t* __restrict__ skey,
             Event* __restrict__ events, unsigned long long* __restrict__ n_events) {
    const int q = blockIdx.y;
    const int64_t k0 = G.off[q], nq = G.off[q + 1] - k0;
    const long long L = G.L[q];
    const unsigned long long e_at = err_at[q];
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < nq; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t kk = base + threadIdx.x;
        const int64_t k = k0 + kk;
        const bool proper = kk < nq && S.cls[k] == 3;
        long long nreads = 0, cov = 0, cov2 = 0, pairs = 0, anyinv = 0;
        if (proper) {
            const bool ev_kept = S.ev[k] && ((unsigned long long)k < e_at ||
                                             ((unsigned long long)k == e_at && S.err[k] == 2));
            if (ev_kept) {
                const unsigned long long w = atomicAdd(n_events, 1ull);
                const int64_t i = S.ridx[k];
                events[w] = Event{(uint32_t)q, (uint32_t)k,
                                  ((uint64_t)((T.flag[i] & 0x40) ? 0 : 1) << 32) | T.kmer[i]};
            }
            if (e_at == kNone) {
                const long long rs = S.rs[k], re = S.re[k];
                const long long a0 = rs > 0 ? rs : 0, b0 = re < L ? re : L;
                if (b0 > a0) {
                    cov = b0 - a0;
                    anyinv = S.inv[k] != 1.0;
                }
                if (rs >= 0 && rs < L) {
                    nreads = 1;
                    skey[k] = ((uint64_t)q << 32) | (uint64_t)rs;
                }
                if (S.mate[k] >= 0) {
                    pairs = 1;
                    cov2 = S.c2[k];
                    pflag[k] = 1;
                }
            }
        }
        unsigned long long* c = cnt + (size_t)q * kC;
        wave_add(c + cNreads, nreads);
        wave_add(c + cCov, cov);
        wave_add(c + cCov2, cov2);
        wave_add(c + cPairs, pairs);
        wave_add(c + cAnyInv, anyinv);
    }
}

// distinct starts: the last read (in slot order) of each (region, rstart)
__global__ void __launch_bounds__(256)
start_runs_kernel(const uint64_t* __restrict__ skey, int64_t N, uint8_t* __restrict__ flag,
                  unsigned long long* __restrict__ cnt) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t kj = j < N ? skey[j] : kNone;
    const bool last = kj != kNone && (j + 1 == N || skey[j + 1] != kj);
    if (j < N) flag[j] = last;
    // one atomic per wave when its run ends share a region (sorted keys)
    const uint32_t q = last ? (uint32_t)(kj >> 32) : 0xFFFFFFFFu;
    const unsigned long long lm = __ballot(last);
    if (!lm) return;
    const uint32_t q0 = __shfl(q, __builtin_ctzll(lm), 64);
    if (__all(!last || q == q0)) {
        if ((threadIdx.x & 63) == 0) atomicAdd(cnt + (size_t)q0 * kC + cStarts, (unsigned long long)__popcll(lm));
    } else if (last) {
        atomicAdd(cnt + (size_t)q * kC + cStarts, 1ull);
    }
}

__global__ void __launch_bounds__(256)
start_vals_kernel(const int64_t* __restrict__ at, const uint64_t* __restrict__ skey, const uint32_t* __restrict__ sval,
                  const double* __restrict__ inv, int64_t M, int64_t* __restrict__ srs, double* __restrict__ sinv) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= M) return;
    const int64_t j = at[u];
    srs[u] = (int64_t)(skey[j] & 0xFFFFFFFFull);
    sinv[u] = inv[sval[j]];
}

// x[a, b) summed in turn from 0 (one thread per region)
__global__ void __launch_bounds__(64)
seq_sum_kernel(const double* __restrict__ x, const int64_t* __restrict__ off, int R, double* __restrict__ out) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= R) return;
    int64_t k = off[q];
    const int64_t b = off[q + 1];
    double acc = 0.0;
    for (; k + 8 <= b; k += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = x[k + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += t[u];
    }
    for (; k < b; ++k) acc += x[k];
    out[q] = acc;
}

// numpy's add.reduce total of a region's buffers: the first buffer's sum,
// then each later one added in turn
__global__ void __launch_bounds__(64)
blocks_total_kernel(const double* __restrict__ bsum, const int64_t* __restrict__ boff, int R,
                    double* __restrict__ out) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= R) return;
    const int64_t a = boff[q], b = boff[q + 1];
    double t = 0;
    for (int64_t k = a; k < b; ++k) t = k == a ? bsum[k] : t + bsum[k];
    out[q] = t;
}

// pairwise_sum over n entries of a buffer whose only non-zero entries are
// v[0, m) at sorted offsets off[0, m) (relative to base): exp_reads.cpp's
// pairwise_block, its recursion on an explicit stack
__device__ double pairwise_sparse(const int64_t* off, const double* v, int64_t m, int64_t base, int64_t n) {
    struct F {
        int64_t o, m, base, n;
        int st;
        double left;
    } f[12];
    int sp = 1;
    f[0] = F{0, m, base, n, 0, 0.0};
    double res = 0.0;
    while (sp > 0) {
        F& c = f[sp - 1];
        if (c.n < 8) {
            res = 0.0;
            for (int64_t i = 0; i < c.m; ++i) res += v[c.o + i];
            --sp;
            continue;
        }
        if (c.n <= kLeaf) {
            double r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            const int64_t body = c.n - (c.n % 8);
            int64_t i = 0;
            for (; i < c.m && off[c.o + i] - c.base < body; ++i) r[(off[c.o + i] - c.base) & 7] += v[c.o + i];
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            for (; i < c.m; ++i) res += v[c.o + i];
            --sp;
            continue;
        }
        int64_t n2 = c.n / 2;
        n2 -= n2 % 8;
        // first entry at or past base + n2
        int64_t a = 0, b = c.m;
        while (a < b) {
            const int64_t mm = (a + b) >> 1;
            if (off[c.o + mm] < c.base + n2) a = mm + 1;
            else b = mm;
        }
        if (c.st == 0) {
            c.st = 1;
            f[sp] = F{c.o, a, c.base, n2, 0, 0.0};
            ++sp;
        } else if (c.st == 1) {
            c.left = res;
            c.st = 2;
            f[sp] = F{c.o + a, c.m - a, c.base + n2, c.n - n2, 0, 0.0};
            ++sp;
        } else {
            res = c.left + res;
            --sp;
        }
    }
    return res;
}

// one thread per (region, buffer) of the sparse cor array
__global__ void __launch_bounds__(64)
cor_blocks_kernel(const int64_t* __restrict__ srs, const double* __restrict__ sinv, const int64_t* __restrict__ soff,
                  const int64_t* __restrict__ boff, const int64_t* __restrict__ L, int R, int64_t NB,
                  double* __restrict__ bsum) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= NB) return;
    int a = 0, b = R;   // region: last q with boff[q] <= g
    while (b - a > 1) {
        const int m = (a + b) >> 1;
        if (boff[m] <= g) a = m;
        else b = m;
    }
    const int q = a;
    const int64_t blk = g - boff[q];
    const int64_t c0 = blk * kBuf, n = min((long long)kBuf, L[q] - c0);
    auto lower = [&](int64_t lo, int64_t hi, int64_t p) {
        while (lo < hi) {
            const int64_t m = (lo + hi) >> 1;
            if (srs[m] < p) lo = m + 1;
            else hi = m;
        }
        return lo;
    };
    const int64_t e0 = lower(soff[q], soff[q + 1], c0), e1 = lower(e0, soff[q + 1], c0 + n);
    bsum[g] = e1 > e0 ? pairwise_sparse(srs + e0, sinv + e0, e1 - e0, c0, n) : 0.0;
}

// cov_cor of one (region, buffer): the covers of its proper reads applied in
// read order into an LDS buffer (the reference's per-position float sums),
// then numpy's pairwise sum of the buffer.  One wave per buffer.
__global__ void __launch_bounds__(64)
covc_blocks_kernel(ExpDevTable T, Regions G, Slots S, const int64_t* __restrict__ boff,
                   const unsigned long long* __restrict__ max_span, const uint8_t* __restrict__ want, int R,
                   int64_t NB, double* __restrict__ bsum) {
    __shared__ double buf[kBuf];
    const int64_t g = blockIdx.x;
    const int lane = threadIdx.x;
    if (g >= NB) return;
    int a = 0, b = R;
    while (b - a > 1) {
        const int m = (a + b) >> 1;
        if (boff[m] <= g) a = m;
        else b = m;
    }
    const int q = a;
    if (!want[q]) return;
    const long long s = G.s[q], L = G.L[q];
    const long long B0 = (g - boff[q]) * (long long)kBuf;
    const int n = (int)min((long long)kBuf, L - B0);
    const long long B1 = B0 + n;
    for (int x = lane; x < n; x += 64) buf[x] = 0.0;
    // candidate slots: read positions in [B0 + s - max span, B1 + s + max span]
    const long long ms = (long long)max_span[G.t[q]];
    const int64_t k0 = G.off[q], k1 = G.off[q + 1], lo = G.lo[q];
    auto lower = [&](long long p) {
        int64_t x = k0, y = k1;
        while (x < y) {
            const int64_t m = (x + y) >> 1;
            if ((long long)T.pos[lo + (m - k0)] < p) x = m + 1;
            else y = m;
        }
        return x;
    };
    const int64_t ka = lower(B0 + s - ms), kb = lower(B1 + s + ms + 1);
    __syncthreads();
    for (int64_t c = ka; c < kb; c += 64) {
        const int64_t k = c + lane;
        long long ca = 0, cb = 0;
        double v = 0;
        bool use = false;
        if (k < kb && S.cls[k] == 3) {
            const long long rs = S.rs[k], re = S.re[k];
            ca = rs > 0 ? rs : 0;
            cb = re < L ? re : L;
            use = cb > ca && ca < B1 && cb > B0;
            v = S.inv[k];
        }
        unsigned long long m = __ballot(use);
        while (m) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            const long long x0 = max(__shfl(ca, l, 64), B0) - B0, x1 = min(__shfl(cb, l, 64), B1) - B0;
            const double w = __shfl(v, l, 64);
            for (long long x = x0 + lane; x < x1; x += 64) buf[x] = buf[x] + w;
        }
    }
    __syncthreads();
    double r;
    if (n == kBuf) {   // 64 leaves of 128, then the aligned pair tree
        const double* p = buf + lane * kLeaf;
        double acc[8];
        for (int j = 0; j < 8; ++j) acc[j] = p[j];
        for (int i = 8; i < kLeaf; i += 8)
            for (int j = 0; j < 8; ++j) acc[j] += p[i + j];
        r = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
        for (int o = 1; o < 64; o <<= 1) {
            const double t = __shfl_xor(r, o, 64);
            r = r + t;
        }
    } else {
        // a partial buffer: the dense recursion by lane 0 (offsets = 0..n-1)
        r = 0;
        if (lane == 0) {
            struct F {
                int o, n, st;
                double left;
            } f[12];
            int sp = 1;
            f[0] = F{0, n, 0, 0.0};
            double res = 0.0;
            while (sp > 0) {
                F& c = f[sp - 1];
                if (c.n < 8) {
                    res = 0.0;
                    for (int i = 0; i < c.n; ++i) res += buf[c.o + i];
                    --sp;
                } else if (c.n <= kLeaf) {
                    double acc[8];
                    for (int j = 0; j < 8; ++j) acc[j] = buf[c.o + j];
                    int i = 8;
                    for (; i < c.n - (c.n % 8); i += 8)
                        for (int j = 0; j < 8; ++j) acc[j] += buf[c.o + i + j];
                    res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
                    for (; i < c.n; ++i) res += buf[c.o + i];
                    --sp;
                } else {
                    int n2 = c.n / 2;
                    n2 -= n2 % 8;
                    if (c.st == 0) {
                        c.st = 1;
                        f[sp++] = F{c.o, n2, 0, 0.0};
                    } else if (c.st == 1) {
                        c.left = res;
                        c.st = 2;
                        f[sp++] = F{c.o + n2, c.n - n2, 0, 0.0};
                    } else {
                        res = c.left + res;
                        --sp;
                    }
                }
            }
            r = res;
        }
    }
    if (lane == 0) bsum[g] = r;
}

__global__ void __launch_bounds__(256)
set_u64_kernel(unsigned long long* __restrict__ p, int64_t n, unsigned long long v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

inline unsigned grid_for(int64_t n, int per = 256, int64_t cap = 4096) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cap, (n + per - 1) / per));
}

}  // namespace

int exp_gpu_index(const ExpDevTable& t, int32_t n_ref, int64_t* first, int64_t* max_span, int64_t* unsorted_at) {
    HIP_TRY(hipSetDevice(t.device));
    Buf<int64_t> d_first;
    Buf<unsigned long long> d_ms, d_bad;
    HIP_TRY(d_first.reserve((size_t)n_ref + 1));
    HIP_TRY(d_ms.reserve((size_t)std::max(n_ref, 1)));
    HIP_TRY(d_bad.reserve(1));
    HIP_TRY(hipMemset(d_ms.p, 0, sizeof(unsigned long long) * std::max(n_ref, 1)));
    HIP_TRY(hipMemset(d_bad.p, 0xFF, 8));
    hipLaunchKernelGGL(idx_first_kernel, dim3(grid_for(n_ref + 1, 256, 1 << 20)), dim3(256), 0, nullptr, t.tid, t.n,
                       n_ref, d_first.p);
    HIP_TRY(hipGetLastError());
    if (t.n) {
        hipLaunchKernelGGL(idx_scan_kernel, dim3(grid_for(t.n)), dim3(256), 0, nullptr, t.tid, t.pos, t.end, t.n,
                           n_ref, d_ms.p, d_bad.p);
        HIP_TRY(hipGetLastError());
    }
    std::vector<unsigned long long> ms((size_t)std::max(n_ref, 1));
    unsigned long long bad = 0;
    HIP_TRY(hipMemcpy(first, d_first.p, ((size_t)n_ref + 1) * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(ms.data(), d_ms.p, ms.size() * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&bad, d_bad.p, 8, hipMemcpyDeviceToHost));
    for (int32_t k = 0; k < n_ref; ++k) max_span[k] = (int64_t)ms[(size_t)k];
    *unsorted_at = bad == kNone ? -1 : (int64_t)bad;
    return MC_OK;
}

struct ExpScratch {
    Buf<int64_t> d_first;
    Buf<unsigned long long> d_ms;
    Buf<double> d_val;
    Buf<uint8_t> d_has;
    Buf<int32_t> d_t;
    Buf<uint8_t> cls;
    Buf<uint8_t> open;
    Buf<uint8_t> err;
    Buf<uint8_t> ev;
    Buf<uint8_t> pflag;
    Buf<uint8_t> rflag;
    Buf<int64_t> ridx;
    Buf<int64_t> c2;
    Buf<int64_t> rs;
    Buf<int64_t> re;
    Buf<int32_t> sreg;
    Buf<int32_t> mate;
    Buf<uint64_t> key;
    Buf<uint64_t> key2;
    Buf<uint64_t> skey;
    Buf<uint64_t> skey2;
    Buf<uint32_t> sidx;
    Buf<uint32_t> sidx2;
    Buf<uint32_t> sval2;
    Buf<double> term;
    Buf<double> inv;
    Buf<unsigned long long> cnt;
    Buf<unsigned long long> err_at;
    Buf<unsigned long long> n_ev;
    Buf<Event> evs;
    Buf<unsigned char> temp;
    Buf<double> cterm;
    Buf<double> seq_out;
    Buf<int64_t> poff;
    Buf<int64_t> d_nsel;
    Buf<int64_t> runs_at;
    Buf<int64_t> srs;
    Buf<int64_t> soff;
    Buf<double> sinv;
    Buf<int64_t> boff;
    Buf<double> bsum;
    Buf<double> tot;
    Buf<uint8_t> d_want;
};

static int reads_chunk(ExpScratch& X, const ExpDevTable& t, const int64_t* first, const int64_t* max_span, const double* val1,
                       const uint8_t* has1, const double* val2, const uint8_t* has2, int64_t R, const int32_t* tid,
                       const int64_t* start, const int64_t* end, int64_t* counts, double* sums,
                       std::vector<std::vector<uint64_t>>& events) {
    events.assign((size_t)R, {});
    std::fill(counts, counts + 8 * R, 0);
    std::fill(sums, sums + 4 * R, 0.0);
    if (R == 0) return MC_OK;
    MC_REQUIRE(R < (int64_t(1) << 31) / 2, MC_E_RANGE, "too many regions");
    hipStream_t st = nullptr;
    // per-contig index on the device (first record, max span)
    int32_t n_all = 0;
    for (int64_t q = 0; q < R; ++q) n_all = std::max(n_all, tid[q] + 1);
    auto& d_first = X.d_first;
    auto& d_ms = X.d_ms;
    {
        // the caller's tables cover every contig of the header; copy what the regions index
        std::vector<unsigned long long> ms((size_t)n_all);
        for (int32_t k = 0; k < n_all; ++k) ms[(size_t)k] = (unsigned long long)max_span[k];
        HIP_TRY(d_first.reserve((size_t)n_all + 1));
        HIP_TRY(d_ms.reserve((size_t)n_all));
        HIP_TRY(hipMemcpy(d_first.p, first, ((size_t)n_all + 1) * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_ms.p, ms.data(), (size_t)n_all * 8, hipMemcpyHostToDevice));
    }
    // k-mer tables
    const bool none = !val1 || !has1 || !val2 || !has2;
    const size_t nk = (size_t)1 << (2 * t.k);
    auto& d_val = X.d_val;
    auto& d_has = X.d_has;
    Tab tab{{nullptr, nullptr}, {nullptr, nullptr}, none ? 1 : 0};
    if (!none) {
        HIP_TRY(d_val.reserve(2 * nk));
        HIP_TRY(d_has.reserve(2 * nk));
        HIP_TRY(hipMemcpy(d_val.p, val1, nk * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_val.p + nk, val2, nk * 8, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_has.p, has1, nk, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_has.p + nk, has2, nk, hipMemcpyHostToDevice));
        tab = Tab{{d_val.p, d_val.p + nk}, {d_has.p, d_has.p + nk}, 0};
    }
    // regions
    std::vector<int64_t> hL((size_t)R);
    for (int64_t q = 0; q < R; ++q) hL[(size_t)q] = end[q] - start[q];
    auto& d_t = X.d_t;
    Buf<int64_t> d_s, d_L, d_lo, d_hi, d_off;
    HIP_TRY(d_t.reserve((size_t)R));
    HIP_TRY(d_s.reserve((size_t)R));
    HIP_TRY(d_L.reserve((size_t)R));
    HIP_TRY(d_lo.reserve((size_t)R));
    HIP_TRY(d_hi.reserve((size_t)R));
    HIP_TRY(d_off.reserve((size_t)R + 1));
    HIP_TRY(hipMemcpy(d_t.p, tid, R * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_s.p, start, R * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_L.p, hL.data(), R * 8, hipMemcpyHostToDevice));
    Regions G{d_t.p, d_s.p, d_L.p, d_lo.p, d_off.p};
    hipLaunchKernelGGL(ranges_kernel, dim3(grid_for(R, 64, 1 << 20)), dim3(64), 0, st, t.pos, d_first.p, d_ms.p, G,
                       (int)R, d_hi.p);
    HIP_TRY(hipGetLastError());
    std::vector<int64_t> lo((size_t)R), hi((size_t)R), off((size_t)R + 1, 0);
    HIP_TRY(hipMemcpy(lo.data(), d_lo.p, R * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(hi.data(), d_hi.p, R * 8, hipMemcpyDeviceToHost));
    int64_t max_q = 0;
    for (int64_t q = 0; q < R; ++q) {
        const int64_t nq = std::max<int64_t>(0, hi[(size_t)q] - lo[(size_t)q]);
        off[(size_t)q + 1] = off[(size_t)q] + nq;
        max_q = std::max(max_q, nq);
    }
    const int64_t N = off[(size_t)R];
    MC_REQUIRE(N < (int64_t(1) << 31), MC_E_RANGE, "%lld candidate reads", (long long)N);
    HIP_TRY(hipMemcpy(d_off.p, off.data(), (R + 1) * 8, hipMemcpyHostToDevice));
    // slots
    auto& cls = X.cls;
    auto& open = X.open;
    auto& err = X.err;
    auto& ev = X.ev;
    auto& pflag = X.pflag;
    auto& rflag = X.rflag;
    auto& ridx = X.ridx;
    auto& c2 = X.c2;
    auto& rs = X.rs;
    auto& re = X.re;
    auto& sreg = X.sreg;
    auto& mate = X.mate;
    auto& key = X.key;
    auto& key2 = X.key2;
    auto& skey = X.skey;
    auto& skey2 = X.skey2;
    auto& sidx = X.sidx;
    auto& sidx2 = X.sidx2;
    auto& sval2 = X.sval2;
    auto& term = X.term;
    auto& inv = X.inv;
    const size_t Nz = (size_t)std::max<int64_t>(N, 1);
    for (auto* b : {&cls, &open, &err, &ev, &pflag, &rflag}) HIP_TRY(b->reserve(Nz));
    for (auto* b : {&ridx, &c2, &rs, &re}) HIP_TRY(b->reserve(Nz));
    for (auto* b : {&sreg, &mate}) HIP_TRY(b->reserve(Nz));
    for (auto* b : {&key, &key2, &skey, &skey2}) HIP_TRY(b->reserve(Nz));
    for (auto* b : {&sidx, &sidx2, &sval2}) HIP_TRY(b->reserve(Nz));
    for (auto* b : {&term, &inv}) HIP_TRY(b->reserve(Nz));
    Slots S{cls.p, ridx.p, sreg.p, key.p, sidx.p, mate.p, open.p, err.p, ev.p, term.p, c2.p, inv.p, rs.p, re.p};
    auto& cnt = X.cnt;
    auto& err_at = X.err_at;
    auto& n_ev = X.n_ev;
    HIP_TRY(cnt.reserve((size_t)R * kC));
    HIP_TRY(err_at.reserve((size_t)R));
    HIP_TRY(n_ev.reserve(1));
    HIP_TRY(hipMemset(cnt.p, 0, (size_t)R * kC * 8));
    HIP_TRY(hipMemset(err_at.p, 0xFF, (size_t)R * 8));
    HIP_TRY(hipMemset(n_ev.p, 0, 8));
    HIP_TRY(hipMemset(pflag.p, 0, Nz));
    HIP_TRY(hipMemset(skey.p, 0xFF, Nz * 8));
    auto& evs = X.evs;
    HIP_TRY(evs.reserve(Nz));
    const unsigned gx = grid_for(max_q, 256, 512);
    auto& temp = X.temp;
    auto sort_pairs = [&](const uint64_t* kin, uint64_t* kout, const uint32_t* vin, uint32_t* vout) -> int {
        size_t tb = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, (int)N, 0, 64, st));
        HIP_TRY(temp.reserve(tb));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(temp.p, tb, kin, kout, vin, vout, (int)N, 0, 64, st));
        return MC_OK;
    };
    if (N) {
        hipLaunchKernelGGL(classify_kernel, dim3(gx, (unsigned)R), dim3(256), 0, st, t, G, S, cnt.p);
        HIP_TRY(hipGetLastError());
        if (int rc = sort_pairs(key.p, key2.p, sidx.p, sidx2.p)) return rc;
        hipLaunchKernelGGL(pair_kernel, dim3(grid_for(N, 256, 1 << 30)), dim3(256), 0, st, t, key2.p, sidx2.p, N, S);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(read_kernel, dim3(gx, (unsigned)R), dim3(256), 0, st, t, tab, G, S, err_at.p);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(accum_kernel, dim3(gx, (unsigned)R), dim3(256), 0, st, t, G, S, err_at.p, cnt.p, pflag.p,
                           skey.p, evs.p, n_ev.p);
        HIP_TRY(hipGetLastError());
    }
    std::vector<unsigned long long> hc((size_t)R * kC), he((size_t)R);
    unsigned long long hn = 0;
    HIP_TRY(hipMemcpy(he.data(), err_at.p, R * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&hn, n_ev.p, 8, hipMemcpyDeviceToHost));
    // wnf: the pair terms in read order of the second mate
    auto& cterm = X.cterm;
    auto& seq_out = X.seq_out;
    auto& poff = X.poff;
    auto& d_nsel = X.d_nsel;
    HIP_TRY(cterm.reserve(Nz));
    HIP_TRY(seq_out.reserve((size_t)R));
    HIP_TRY(poff.reserve((size_t)R + 1));
    HIP_TRY(d_nsel.reserve(1));
    std::vector<double> wnf((size_t)R, 0.0), cor_seq((size_t)R, 0.0), cor_np((size_t)R, 0.0), covc((size_t)R, 0.0);
    std::vector<int64_t> hpo((size_t)R + 1, 0), hso((size_t)R + 1, 0);
    if (N) {
        size_t tb = 0;
        HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, term.p, pflag.p, cterm.p, d_nsel.p, (int)N, st));
        HIP_TRY(temp.reserve(tb));
        HIP_TRY(hipcub::DeviceSelect::Flagged(temp.p, tb, term.p, pflag.p, cterm.p, d_nsel.p, (int)N, st));
    }
    // the starts: (region, rstart) sorted, the last read of each kept
    auto& runs_at = X.runs_at;
    auto& srs = X.srs;
    auto& soff = X.soff;
    auto& sinv = X.sinv;
    if (N) {
        if (int rc = sort_pairs(skey.p, skey2.p, sidx.p, sval2.p)) return rc;
        hipLaunchKernelGGL(start_runs_kernel, dim3(grid_for(N, 256, 1 << 30)), dim3(256), 0, st, skey2.p, N, rflag.p,
                           cnt.p);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipMemcpy(hc.data(), cnt.p, (size_t)R * kC * 8, hipMemcpyDeviceToHost));
    for (int64_t q = 0; q < R; ++q) {
        hpo[(size_t)q + 1] = hpo[(size_t)q] + (int64_t)hc[(size_t)q * kC + cPairs];
        hso[(size_t)q + 1] = hso[(size_t)q] + (int64_t)hc[(size_t)q * kC + cStarts];
    }
    const int64_t M = hso[(size_t)R];
    HIP_TRY(runs_at.reserve((size_t)std::max<int64_t>(M, 1)));
    HIP_TRY(srs.reserve((size_t)std::max<int64_t>(M, 1)));
    HIP_TRY(sinv.reserve((size_t)std::max<int64_t>(M, 1)));
    HIP_TRY(soff.reserve((size_t)R + 1));
    HIP_TRY(hipMemcpy(poff.p, hpo.data(), (R + 1) * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(soff.p, hso.data(), (R + 1) * 8, hipMemcpyHostToDevice));
    if (hpo[(size_t)R]) {
        hipLaunchKernelGGL(seq_sum_kernel, dim3(grid_for(R, 64, 1 << 20)), dim3(64), 0, st, cterm.p, poff.p, (int)R,
                           seq_out.p);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpy(wnf.data(), seq_out.p, R * 8, hipMemcpyDeviceToHost));
    }
    // numpy buffers of every region (cor, cov_cor)
    std::vector<int64_t> hbo((size_t)R + 1, 0);
    for (int64_t q = 0; q < R; ++q) hbo[(size_t)q + 1] = hbo[(size_t)q] + (hL[(size_t)q] + kBuf - 1) / kBuf;
    const int64_t NB = hbo[(size_t)R];
    auto& boff = X.boff;
    auto& bsum = X.bsum;
    auto& tot = X.tot;
    HIP_TRY(boff.reserve((size_t)R + 1));
    HIP_TRY(bsum.reserve((size_t)std::max<int64_t>(NB, 1)));
    HIP_TRY(tot.reserve((size_t)R));
    HIP_TRY(hipMemcpy(boff.p, hbo.data(), (R + 1) * 8, hipMemcpyHostToDevice));
    if (M) {
        {
            size_t tb = 0;
            hipcub::CountingInputIterator<int64_t> ci(0);
            HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, ci, rflag.p, runs_at.p, d_nsel.p, (int)N, st));
            HIP_TRY(temp.reserve(tb));
            HIP_TRY(hipcub::DeviceSelect::Flagged(temp.p, tb, ci, rflag.p, runs_at.p, d_nsel.p, (int)N, st));
        }
        hipLaunchKernelGGL(start_vals_kernel, dim3(grid_for(M, 256, 1 << 30)), dim3(256), 0, st, runs_at.p, skey2.p,
                           sval2.p, inv.p, M, srs.p, sinv.p);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(seq_sum_kernel, dim3(grid_for(R, 64, 1 << 20)), dim3(64), 0, st, sinv.p, soff.p, (int)R,
                           seq_out.p);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpy(cor_seq.data(), seq_out.p, R * 8, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(cor_blocks_kernel, dim3(grid_for(NB, 64, 1 << 30)), dim3(64), 0, st, srs.p, sinv.p, soff.p,
                           boff.p, d_L.p, (int)R, NB, bsum.p);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(blocks_total_kernel, dim3(grid_for(R, 64, 1 << 20)), dim3(64), 0, st, bsum.p, boff.p,
                           (int)R, tot.p);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpy(cor_np.data(), tot.p, R * 8, hipMemcpyDeviceToHost));
    }
    // cov_cor where some 1/rcor != 1 (else it is cov's exact integer sum)
    std::vector<uint8_t> want((size_t)R, 0);
    bool any = false;
    for (int64_t q = 0; q < R; ++q) {
        want[(size_t)q] = he[(size_t)q] == kNone && hc[(size_t)q * kC + cAnyInv] > 0;
        any |= want[(size_t)q] != 0;
    }
    if (any && NB) {
        auto& d_want = X.d_want;
        HIP_TRY(d_want.reserve((size_t)R));
        HIP_TRY(hipMemcpy(d_want.p, want.data(), R, hipMemcpyHostToDevice));
        HIP_TRY(hipMemset(bsum.p, 0, (size_t)NB * 8));
        MC_REQUIRE(NB < (int64_t(1) << 31), MC_E_RANGE, "regions too long");
        hipLaunchKernelGGL(covc_blocks_kernel, dim3((unsigned)NB), dim3(64), 0, st, t, G, S, boff.p, d_ms.p,
                           d_want.p, (int)R, NB, bsum.p);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(blocks_total_kernel, dim3(grid_for(R, 64, 1 << 20)), dim3(64), 0, st, bsum.p, boff.p,
                           (int)R, tot.p);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpy(covc.data(), tot.p, R * 8, hipMemcpyDeviceToHost));
    }
    // events in read order
    std::vector<Event> hev((size_t)hn);
    if (hn) HIP_TRY(hipMemcpy(hev.data(), evs.p, hn * sizeof(Event), hipMemcpyDeviceToHost));
    HIP_TRY(hipDeviceSynchronize());
    std::sort(hev.begin(), hev.end(), [](const Event& a, const Event& b) { return a.k < b.k; });
    for (const Event& e : hev) events[e.q].push_back(e.code);
    // error slots -> status codes
    std::vector<uint8_t> err_of((size_t)R, 0);
    for (int64_t q = 0; q < R; ++q)
        if (he[(size_t)q] != kNone) HIP_TRY(hipMemcpy(&err_of[(size_t)q], err.p + he[(size_t)q], 1, hipMemcpyDeviceToHost));
    for (int64_t q = 0; q < R; ++q) {
        const unsigned long long* c = hc.data() + (size_t)q * kC;
        int64_t* o = counts + 8 * q;
        double* x = sums + 4 * q;
        o[0] = err_of[(size_t)q];   // 1 / 2 / 3: the host pass's kNoSeqError / kNoRefLenError / kNoKcorError
        o[1] = (int64_t)c[cSecondary];
        o[2] = (int64_t)c[cImproper];
        o[3] = (int64_t)c[cNreads];
        o[4] = (int64_t)c[cCov];
        o[5] = (int64_t)c[cStarts];
        o[6] = (int64_t)c[cCov2];
        o[7] = (int64_t)events[(size_t)q].size();
        x[0] = want[(size_t)q] ? covc[(size_t)q] : (double)c[cCov];
        x[1] = cor_seq[(size_t)q];
        x[2] = cor_np[(size_t)q];
        x[3] = wnf[(size_t)q];
    }
    return MC_OK;
}

int exp_gpu_reads(const ExpDevTable& t, const int64_t* first, const int64_t* max_span, const double* val1,
                  const uint8_t* has1, const double* val2, const uint8_t* has2, int64_t R, const int32_t* tid,
                  const int64_t* start, const int64_t* end, int64_t* counts, double* sums,
                  std::vector<std::vector<uint64_t>>& events, double* kernel_ms, ExpScratch** scratch) {
    const auto t_start = std::chrono::steady_clock::now();
    if (!*scratch) *scratch = new ExpScratch();
    HIP_TRY(hipSetDevice(t.device));
    events.assign((size_t)R, {});
    constexpr int64_t kChunkRegions = 32768;   // (regions are the grids' y dimension)
    for (int64_t r0 = 0; r0 < R; r0 += kChunkRegions) {
        const int64_t nr = std::min(kChunkRegions, R - r0);
        std::vector<std::vector<uint64_t>> ev;
        if (int rc = reads_chunk(**scratch, t, first, max_span, val1, has1, val2, has2, nr, tid + r0, start + r0, end + r0,
                                 counts + 8 * r0, sums + 4 * r0, ev))
            return rc;
        for (int64_t q = 0; q < nr; ++q) events[(size_t)(r0 + q)] = std::move(ev[(size_t)q]);
    }
    if (kernel_ms)
        *kernel_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return MC_OK;
}

void exp_gpu_scratch_free(ExpScratch* s) {
    delete s;
}
