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
// Layout: one lane per read (grid-stride).  A 150 bp read is ~1 KB of LDS
// atomics for BaseHist: with a lane per read a wave's 64 reads do 64
// distinct-address atomics per instruction when each lane starts its walk
// at a different offset (lane-rotated order), where a wave per read would
// leave 3/4 of its lanes idle on short reads.  BaseHist, MirrorHist and
// IsizeHist are privatised per workgroup in LDS when they fit (every read
// hits the same few hundred bins) and flushed once per workgroup; KmerHist
// (4^K+1 x NK bins per group) takes global atomics, which spread over
// its 131 K bins at K = 7.
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int kThreads = 256;
constexpr int kLdsWords = 12288;   // 48 KiB: 3 workgroups per CU
constexpr int kMaxFlags = 16;

struct ScanArgs {
    const int32_t* rlen;
    const int32_t* flag;
    const int32_t* gpos;
    const int32_t* gisize;
    const int32_t* ref_id;
    const int64_t* seq_off;
    const uint8_t* seq;
    int64_t n;
    const uint8_t* ref;       // nt4 codes, all sequences back to back
    const int64_t* ref_off;
    const int64_t* ref_len;
    int32_t n_ref;
    int32_t n_flags;
    uint32_t fmask[kMaxFlags];
    int32_t G;
    // BaseHist: [row][G][5]
    int32_t base_on, base_start, base_rows, base_lds;
    uint32_t* base;
    // KmerHist: [G][4^K + 1][NK]
    int32_t kmer_on, K, NK, STEP, OFF;
    uint32_t* kmer;
    // MirrorHist: [G][N + 1][2]
    int32_t mir_on, MOFF, MN, mir_lds;
    uint32_t* mir;
    // IsizeHist: [a][G] and max per group
    int32_t isz_on, isz_cap, isz_lds;
    uint32_t* isz;
    int32_t* isz_max;
    // LDS arena (words)
    int32_t lds_base, lds_mir, lds_isz, lds_isz_max, lds_words;
};

__device__ __forceinline__ int nt16_nt4(uint32_t v) {
    return (v != 0 && (v & (v - 1)) == 0) ? __builtin_ctz(v) : 4;
}

__device__ __forceinline__ int comp4(int n) { return n < 4 ? 3 - n : 4; }

// nt16 nibble of base j of the read whose packed bases start at s
__device__ __forceinline__ uint32_t nib(const uint8_t* s, int64_t j) {
    const uint32_t b = s[j >> 1];
    return (j & 1) ? (b & 15u) : (b >> 4);
}

struct Ref {
    const uint8_t* p;
    int64_t L;
    __device__ __forceinline__ int at(int64_t i) const {
        if (i < 0) i += L;
        return (i < 0 || i >= L) ? 4 : (int)p[i];
    }
};

__device__ __forceinline__ void inc(uint32_t* lds_or_null, uint32_t* g, int64_t i, bool in_lds) {
    if (in_lds)
        atomicAdd(lds_or_null + i, 1u);
    else
        atomicAdd(g + i, 1u);
}

__global__ __launch_bounds__(kThreads) void scan_kernel(ScanArgs a) {
    extern __shared__ uint32_t lds[];
    for (int i = threadIdx.x; i < a.lds_words; i += kThreads) lds[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x; r < a.n; r += stride) {
        const int32_t rlen = a.rlen[r], flag = a.flag[r], gpos = a.gpos[r];
        const int64_t so = a.seq_off[r];
        const uint8_t* s = a.seq + so;
        const bool rev = (flag & 0x10) != 0;
        int g = 0;
        for (int f = 0; f < a.n_flags; ++f) g = (g << 1) | ((flag & a.fmask[f]) ? 1 : 0);
        Ref ref{nullptr, 0};
        const int32_t rid = a.ref_id[r];
        if (rid >= 0 && rid < a.n_ref) ref = Ref{a.ref + a.ref_off[rid], a.ref_len[rid]};

        if (a.isz_on) {
            int32_t v = a.gisize[r];
            v = v < 0 ? -v : v;
            const int64_t bin = (int64_t)v * a.G + g;
            inc(lds + a.lds_isz, a.isz, bin, a.isz_lds);
            if (a.isz_lds)
                atomicMax(reinterpret_cast<int32_t*>(lds + a.lds_isz_max) + g, v);
            else
                atomicMax(a.isz_max + g, v);
        }

        if (a.kmer_on && rlen >= a.OFF + a.STEP * a.NK) {
            const uint32_t nbucket = 1u << (2 * a.K);
            uint32_t* kg = a.kmer + (int64_t)g * (nbucket + 1) * a.NK;
            for (int i = 0; i < a.NK; ++i) {
                uint32_t k = 0;
                for (int j = 0; j < a.K; ++j) {
                    const int64_t x = (int64_t)a.OFF + (int64_t)i * a.STEP + j;
                    int c = 4;
                    if (x >= 0 && x < rlen) {
                        c = nt16_nt4(nib(s, rev ? rlen - 1 - x : x));
                        if (rev) c = comp4(c);
                    }
                    if (c > 3) {
                        k = nbucket;
                        break;
                    }
                    k |= (uint32_t)c << (2 * j);
                }
                atomicAdd(kg + (int64_t)k * a.NK + i, 1u);
            }
        }

        if (a.mir_on) {
            const int64_t p = (int64_t)gpos + a.MOFF;
            if (p >= (int64_t)a.MN - a.MOFF) {
                int plain = 0, cmp = 0;
                for (int i = 0; i < a.MN; ++i) {
                    const int x = ref.at(p + i + 1), y = ref.at(p - i - 1);
                    plain += x != y;
                    cmp += x != comp4(y);
                }
                const int64_t b = ((int64_t)g * (a.MN + 1)) * 2;
                inc(lds + a.lds_mir, a.mir, b + plain * 2, a.mir_lds);
                inc(lds + a.lds_mir, a.mir, b + cmp * 2 + 1, a.mir_lds);
            }
        }

        if (a.base_on && gpos >= a.base_start) {
            // mismatches in BAM orientation: read[x] vs the reference, reverse
            // strand mapped back (comp is a bijection on 0..4)
            const int64_t b0 = rev ? (int64_t)gpos - rlen : (int64_t)gpos;
            int mism = 0;
            bool reject = false;
            for (int j = 0; j < rlen; ++j) {
                mism += nt16_nt4(nib(s, j)) != ref.at(b0 + j);
                if (mism * 32 > rlen) {
                    reject = true;
                    break;
                }
            }
            if (!reject) {
                const int64_t rowstride = (int64_t)a.G * 5;
                for (int x = 0; x < a.base_start; ++x) {
                    const int v = rev ? comp4(ref.at((int64_t)gpos - x - 1 + a.base_start))
                                      : ref.at((int64_t)gpos + x - a.base_start);
                    inc(lds + a.lds_base, a.base, x * rowstride + g * 5 + v, a.base_lds);
                }
                // lane-rotated walk: the wave's lanes hit different rows
                int j = rlen > 0 ? lane % rlen : 0;
                for (int t = 0; t < rlen; ++t) {
                    int v = nt16_nt4(nib(s, j));
                    int x = j;
                    if (rev) {
                        v = comp4(v);
                        x = rlen - 1 - j;
                    }
                    inc(lds + a.lds_base, a.base, (int64_t)(x + a.base_start) * rowstride + g * 5 + v,
                        a.base_lds);
                    if (++j == rlen) j = 0;
                }
            }
        }
    }
    __syncthreads();
    // flush the workgroup's private bins
    for (int i = threadIdx.x; i < a.lds_words; i += kThreads) {
        const uint32_t v = lds[i];
        if (!v) continue;
        if (i >= a.lds_isz_max && a.isz_lds && i < a.lds_isz_max + a.G) {
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
    a.ref = s->ref.p;
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
    a.lds_words = words;
    if (!a.isz_lds) a.lds_isz_max = kLdsWords;   // outside the arena: never matched by the flush
    const int64_t want = (n + kThreads - 1) / kThreads;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, s->grid));
    hipLaunchKernelGGL(scan_kernel, dim3(grid), dim3(kThreads), (size_t)words * 4, s->stream, a);
    HIP_TRY(hipGetLastError());
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
    s->grid = std::max(1, cus) * 4;
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
    HIP_TRY(s->ref.reserve((size_t)std::max<int64_t>(n_bytes, 1)));
    HIP_TRY(s->ref_off.reserve((size_t)std::max(n_seq, 1)));
    HIP_TRY(s->ref_len.reserve((size_t)std::max(n_seq, 1)));
    if (n_bytes) {
        HIP_TRY(hipMemcpy(s->ref.p, ascii, (size_t)n_bytes, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(ascii_nt4_kernel, dim3((unsigned)((n_bytes + 255) / 256)), dim3(256), 0,
                           s->stream, s->ref.p, n_bytes);
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
    const int64_t nbytes = seq_off[n];
    // staging layout: 5 int32 columns, seq_off (n+1 int64, rebased), seq
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
    uint8_t* h = static_cast<uint8_t*>(sl.host.p);
    std::memcpy(h, rlen, cols);
    std::memcpy(h + cols, flag, cols);
    std::memcpy(h + 2 * cols, gpos, cols);
    std::memcpy(h + 3 * cols, gisize, cols);
    std::memcpy(h + 4 * cols, ref_id, cols);
    std::memcpy(h + 5 * cols, seq_off, offb);
    std::memcpy(h + 5 * cols + offb, seq, (size_t)nbytes);
    HIP_TRY(hipMemcpyAsync(sl.dev.p, h, total, hipMemcpyHostToDevice, s->stream));
    uint8_t* d = sl.dev.p;
    HIP_TRY(hipEventRecord(s->t0, s->stream));
    if (int rc = launch(s, n, (const int32_t*)d, (const int32_t*)(d + cols),
                        (const int32_t*)(d + 2 * cols), (const int32_t*)(d + 3 * cols),
                        (const int32_t*)(d + 4 * cols), (const int64_t*)(d + 5 * cols),
                        d + 5 * cols + offb))
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
    const int G = s->G;
    if (base && s->cfg.base_on) {
        std::vector<uint32_t> t((size_t)(s->base_rows * G * 5));
        HIP_TRY(hipMemcpy(t.data(), s->base.p, t.size() * 4, hipMemcpyDeviceToHost));
        for (int64_t r = 0; r < s->base_rows; ++r)
            for (int g = 0; g < G; ++g)
                std::memcpy(base + ((int64_t)g * s->base_rows + r) * 5, &t[(r * G + g) * 5], 20);
    }
    if (kmer && s->cfg.kmer_on)
        HIP_TRY(hipMemcpy(kmer, s->kmer.p, (size_t)s->kmer_bins * 4, hipMemcpyDeviceToHost));
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
