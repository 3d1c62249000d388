// Expected-coverage correlation of the reference's experimental estimator
// (pileup.experimental, metacov/pileup.py:63-88), the one O(L x taps) part of
// it, as a gfx950 fp64 kernel.  Per region of length L over the reference
// sequence region = fasta[start:end].upper() (n <= L bases available):
//
//   fwd[i] = k_cor[0][region[i:i+K]]                 i < L-K, else 0  (:69-73)
//   rev[p] = k_cor[1][reversed(region[p-K+1 .. p])]  p >= K-1         (:74-78)
//            (region[i:i-K:-1] with p = L + i; missing keys -> 0)
//   revsum[i] = sum_{j < min(L-i, 900)} norm[j] * rev[i+j]            (:80-83)
//   inner     = sum_i fwd[i] * revsum[i]   (ecor = inner / L)         (:84)
//   gc / at   = counts of G+C / A+T in region (case-insensitive)      (:64-66)
//
// norm = N(450, 150).pdf(0..900) (:59-61) comes from the caller; only its
// first 900 taps are used (l <= iend - istart).  K-mer tables are dense over
// the 4^K A/C/G/T codes (first base most significant), 0 for missing keys:
// a window with any other symbol, or cut short by the region end, matches no
// key (KeyError -> 0 in the reference).
//
// Kernel layout: one 256-thread block per 2048-position tile of a region;
// thread t owns 8 consecutive outputs.  rev[i0 .. i0+2048+taps) is staged in
// LDS in a residue-transposed layout (element e at [e % 8][e / 8]) so that
// the 64 lanes' sliding-window reads are consecutive doubles (ds_read_b64,
// conflict-free); norm[j] is wave-uniform (scalar loads).  Per 8 taps a
// thread does 15 LDS reads and 64 v_fma_f64.  Tile partial sums (fixed-order
// block reduction) go to HBM and are added per region in tile order on the
// host, so results are run-to-run deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/metacov_amd.h"
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kPer = 8;                       // outputs per thread
constexpr int kTile = kThreads * kPer;        // 2048 outputs per block
constexpr int kMaxTaps = 1024;
constexpr int kRows = (kTile + kMaxTaps + 16) / 8;

__device__ __forceinline__ int base2(uint8_t c) {
    switch (c | 0x20) {   // ASCII lower-case fold (the reference upper-cases)
        case 'a': return 0;
        case 'c': return 1;
        case 'g': return 2;
        case 't': return 3;
        default: return -1;
    }
}

__global__ __launch_bounds__(kThreads) void ecor_kernel(
    const uint8_t* __restrict__ seq, const int64_t* __restrict__ reg_base,
    const int64_t* __restrict__ reg_n, const int64_t* __restrict__ reg_len,
    const int32_t* __restrict__ tile_region, const int64_t* __restrict__ tile_i0,
    const double* __restrict__ tab_fwd, const double* __restrict__ tab_rev, int k,
    const double* __restrict__ norm, int taps, double* __restrict__ tile_inner,
    int64_t* __restrict__ tile_counts) {
    __shared__ double rev_s[8][kRows];
    __shared__ double red_d[kThreads / 64];
    __shared__ int64_t red_i[2][kThreads / 64];

    const int t = threadIdx.x;
    const int q = tile_region[blockIdx.x];
    const int64_t i0 = tile_i0[blockIdx.x];
    const int64_t L = reg_len[q], n = reg_n[q];
    const uint8_t* s = seq + reg_base[q];
    const int64_t shift = L - n;              // region[i] for i = p - L is s[p - shift]

    // ---- stage rev[i0 + e], e < kTile + taps (0 past L) ----
    const int W = kTile + ((taps + 7) & ~7) + 8;
    for (int e = t; e < W; e += kThreads) {
        const int64_t p = i0 + e;
        double v = 0.0;
        const int64_t idx = p - shift;
        if (p < L && p >= k - 1 && idx - (k - 1) >= 0) {
            int code = 0;
            bool ok = true;
            for (int m = 0; m < k; ++m) {
                const int b = base2(s[idx - m]);
                ok &= b >= 0;
                code = (code << 2) | (b & 3);
            }
            if (ok) v = tab_rev[code];
        }
        rev_s[e & 7][e >> 3] = v;
    }
    __syncthreads();

    // ---- revsum for outputs o = i0 + 8t + r ----
    double acc[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) acc[r] = 0.0;
    int jb = 0;
    for (; jb + 8 <= taps; jb += 8) {
        double w[15];
        const int row = t + (jb >> 3);
#pragma unroll
        for (int m = 0; m < 15; ++m) w[m] = rev_s[m & 7][row + (m >> 3)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const double nj = norm[jb + u];
#pragma unroll
            for (int r = 0; r < kPer; ++r) acc[r] = __builtin_fma(nj, w[u + r], acc[r]);
        }
    }
    for (; jb < taps; ++jb) {                  // tail taps (taps % 8)
        const double nj = norm[jb];
#pragma unroll
        for (int r = 0; r < kPer; ++r) {
            const int e = kPer * t + r + jb;
            acc[r] = __builtin_fma(nj, rev_s[e & 7][e >> 3], acc[r]);
        }
    }

    // ---- fwd . revsum and base counts over the thread's outputs ----
    double part = 0.0;
    int64_t gc = 0, at = 0;
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
        const int64_t o = i0 + kPer * t + r;
        if (o < n) {
            const int b = base2(s[o]);
            gc += (b == 1 || b == 2);
            at += (b == 0 || b == 3);
        }
        if (o < L) {
            double fv = 0.0;
            if (o < L - k && o + k <= n) {
                int code = 0;
                bool ok = true;
                for (int m = 0; m < k; ++m) {
                    const int b = base2(s[o + m]);
                    ok &= b >= 0;
                    code = (code << 2) | (b & 3);
                }
                if (ok) fv = tab_fwd[code];
            }
            part += fv * acc[r];
        }
    }
    // fixed-order block reduction
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        part += __shfl_xor(part, off, 64);
        gc += __shfl_xor(gc, off, 64);
        at += __shfl_xor(at, off, 64);
    }
    if ((t & 63) == 0) {
        red_d[t >> 6] = part;
        red_i[0][t >> 6] = gc;
        red_i[1][t >> 6] = at;
    }
    __syncthreads();
    if (t == 0) {
        double sum = red_d[0];
        int64_t g = red_i[0][0], a = red_i[1][0];
        for (int w = 1; w < kThreads / 64; ++w) {
            sum += red_d[w];
            g += red_i[0][w];
            a += red_i[1][w];
        }
        tile_inner[blockIdx.x] = sum;
        tile_counts[2 * blockIdx.x] = g;
        tile_counts[2 * blockIdx.x + 1] = a;
    }
}

}  // namespace

#define HIP_TRY(expr)                                                          \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            mc::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                          __FILE__, __LINE__);                                 \
            return MC_E_HIP;                                                   \
        }                                                                      \
    } while (0)

struct mc_ecor {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    uint8_t* seq = nullptr;
    int64_t seq_bytes = 0;
    double* tab = nullptr;      // fwd [4^k] then rev [4^k]
    double* norm = nullptr;
    int k = 0, taps = 0;
    void* work = nullptr;       // per-call device arrays
    size_t work_cap = 0;
    ~mc_ecor() {
        if (seq) (void)hipFree(seq);
        if (tab) (void)hipFree(tab);
        if (norm) (void)hipFree(norm);
        if (work) (void)hipFree(work);
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

extern "C" int mc_ecor_create(int device, mc_ecor** out) {
    MC_REQUIRE(out, MC_E_INVALID, "null argument");
    *out = nullptr;
    int n_dev = 0;
    HIP_TRY(hipGetDeviceCount(&n_dev));
    MC_REQUIRE(device >= 0 && device < n_dev, MC_E_HIP, "no HIP device %d (%d present)", device,
               n_dev);
    HIP_TRY(hipSetDevice(device));
    mc_ecor* e = new mc_ecor();
    e->device = device;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&e->ev[0]) != hipSuccess || hipEventCreate(&e->ev[1]) != hipSuccess) {
        delete e;
        mc::set_error("HIP stream / event creation failed");
        return MC_E_HIP;
    }
    *out = e;
    return MC_OK;
}

extern "C" int mc_ecor_destroy(mc_ecor* e) {
    if (e) {
        (void)hipSetDevice(e->device);
        delete e;
    }
    return MC_OK;
}

extern "C" int mc_ecor_set_sequence(mc_ecor* e, int64_t n_bytes, const uint8_t* seq) {
    MC_REQUIRE(e && (seq || n_bytes == 0) && n_bytes >= 0, MC_E_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(e->device));
    if (e->seq) HIP_TRY(hipFree(e->seq));
    e->seq = nullptr;
    HIP_TRY(hipMalloc(&e->seq, (size_t)std::max<int64_t>(n_bytes, 1)));
    if (n_bytes) HIP_TRY(hipMemcpy(e->seq, seq, (size_t)n_bytes, hipMemcpyHostToDevice));
    e->seq_bytes = n_bytes;
    return MC_OK;
}

extern "C" int mc_ecor_set_tables(mc_ecor* e, int k_len, const double* fwd, const double* rev,
                                  int n_taps, const double* taps) {
    MC_REQUIRE(e && fwd && rev && taps, MC_E_INVALID, "null argument");
    MC_REQUIRE(k_len >= 1 && k_len <= 13, MC_E_RANGE, "k-mer length %d outside 1..13", k_len);
    MC_REQUIRE(n_taps >= 1 && n_taps <= kMaxTaps, MC_E_RANGE, "%d taps outside 1..%d", n_taps,
               kMaxTaps);
    HIP_TRY(hipSetDevice(e->device));
    const size_t nk = (size_t)1 << (2 * k_len);
    if (e->tab) HIP_TRY(hipFree(e->tab));
    if (e->norm) HIP_TRY(hipFree(e->norm));
    e->tab = nullptr;
    e->norm = nullptr;
    HIP_TRY(hipMalloc(&e->tab, 2 * nk * sizeof(double)));
    HIP_TRY(hipMalloc(&e->norm, (size_t)n_taps * sizeof(double)));
    HIP_TRY(hipMemcpy(e->tab, fwd, nk * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->tab + nk, rev, nk * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->norm, taps, (size_t)n_taps * sizeof(double), hipMemcpyHostToDevice));
    e->k = k_len;
    e->taps = n_taps;
    return MC_OK;
}

extern "C" int mc_ecor_run(mc_ecor* e, int64_t R, const int64_t* base, const int64_t* n_avail,
                           const int64_t* length, double* inner, int64_t* gc, int64_t* at,
                           float* kernel_ms) {
    MC_REQUIRE(e && base && n_avail && length && inner && gc && at, MC_E_INVALID, "null argument");
    MC_REQUIRE(e->tab && e->seq, MC_E_STATE, "mc_ecor_set_sequence / mc_ecor_set_tables first");
    MC_REQUIRE(R >= 0 && R < (int64_t)INT32_MAX, MC_E_RANGE, "%lld regions", (long long)R);
    HIP_TRY(hipSetDevice(e->device));
    // tile table (host), checking every region against the sequence buffer
    std::vector<int32_t> t_reg;
    std::vector<int64_t> t_i0;
    for (int64_t q = 0; q < R; ++q) {
        MC_REQUIRE(length[q] > 0 && n_avail[q] >= 0 && n_avail[q] <= length[q] && base[q] >= 0 &&
                       base[q] + n_avail[q] <= e->seq_bytes,
                   MC_E_INVALID, "region %lld outside the sequence buffer", (long long)q);
        for (int64_t i0 = 0; i0 < length[q]; i0 += kTile) {
            t_reg.push_back((int32_t)q);
            t_i0.push_back(i0);
        }
    }
    const int64_t T = (int64_t)t_reg.size();
    MC_REQUIRE(T < (int64_t)INT32_MAX, MC_E_RANGE, "%lld tiles", (long long)T);
    if (kernel_ms) *kernel_ms = 0;
    if (T == 0) return MC_OK;
    // device work area: regions (3 x int64), tiles (int32 + int64 + double + 2 int64)
    const size_t bytes = (size_t)R * 24 + (size_t)T * (4 + 8 + 8 + 16) + 64;
    if (bytes > e->work_cap) {
        if (e->work) HIP_TRY(hipFree(e->work));
        e->work = nullptr;
        e->work_cap = 0;
        HIP_TRY(hipMalloc(&e->work, bytes));
        e->work_cap = bytes;
    }
    char* w = (char*)e->work;
    int64_t* d_base = (int64_t*)w;
    int64_t* d_n = d_base + R;
    int64_t* d_len = d_n + R;
    int64_t* d_i0 = d_len + R;
    double* d_inner = (double*)(d_i0 + T);
    int64_t* d_cnt = (int64_t*)(d_inner + T);
    int32_t* d_reg = (int32_t*)(d_cnt + 2 * T);
    hipStream_t st = e->stream;
    HIP_TRY(hipMemcpyAsync(d_base, base, R * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_n, n_avail, R * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_len, length, R * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_i0, t_i0.data(), T * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d_reg, t_reg.data(), T * 4, hipMemcpyHostToDevice, st));
    const size_t nk = (size_t)1 << (2 * e->k);
    HIP_TRY(hipEventRecord(e->ev[0], st));
    hipLaunchKernelGGL(ecor_kernel, dim3((unsigned)T), dim3(kThreads), 0, st, e->seq, d_base, d_n,
                       d_len, d_reg, d_i0, e->tab, e->tab + nk, e->k, e->norm, e->taps, d_inner,
                       d_cnt);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e->ev[1], st));
    std::vector<double> h_inner((size_t)T);
    std::vector<int64_t> h_cnt((size_t)T * 2);
    HIP_TRY(hipMemcpyAsync(h_inner.data(), d_inner, T * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(h_cnt.data(), d_cnt, T * 16, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (kernel_ms) HIP_TRY(hipEventElapsedTime(kernel_ms, e->ev[0], e->ev[1]));
    int64_t j = 0;
    for (int64_t q = 0; q < R; ++q) {
        double sum = 0;
        int64_t g = 0, a = 0;
        for (; j < T && t_reg[j] == q; ++j) {
            sum += h_inner[j];
            g += h_cnt[2 * j];
            a += h_cnt[2 * j + 1];
        }
        inner[q] = sum;
        gc[q] = g;
        at[q] = a;
    }
    return MC_OK;
}
