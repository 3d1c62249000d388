// HBM ceiling of K2's traffic mix in K2's OWN shape (VERDICT r03 "next" #3):
// a persistent grid dequeues 128 KiB depth chunks (32768 int32 positions,
// 8 tiles of 4096) from an atomic counter; per chunk it loads the chunk's
// reads as int4 per lane from three arrays (tid, pos, span: 12 B per read,
// 1024 reads per batch) and writes the chunk's 8 tiles with 16 B per lane
// (non-temporal, 4 dwordx4 per thread per tile).  C3 sizes: 100 M reads
// (1.2 GB) over 1.005 G positions (4.02 GB) -> 5.22 GB per launch.
//
// No LDS work, no scans: only K2's memory shape and the load -> store data
// dependency, so the best variant's time is what K2's byte mix can reach.
//   wr       stores only (the write half)
//   rd       loads only (the read half)
//   seq      per chunk: all batches loaded, then the 8 tiles stored
//   inter    per tile: the batch that tile needs, then its store (K2's order:
//            next batch in flight while the tile is stored)
//   ahead    inter + the NEXT chunk's first batch issued before this chunk's
//            last tile (a queue-ahead reservation)
//   indep    seq without the load -> store dependency (stores never wait)
// Each at 512 / 1024 workgroups, with 40 KiB of LDS per workgroup (K2's
// occupancy: 4 per CU) or none.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef int i32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kChunk4 = 8192;          // int4 per chunk (128 KiB)
constexpr int kTile4 = 1024;           // int4 per tile (16 KiB)
constexpr int kBatch = 1024;           // reads per batch (one int4 per lane per array)

struct Args {
    const i32x4* tid; const i32x4* pos; const i32x4* span;
    i32x4* depth;
    int64_t n_chunks, n_reads;
    unsigned* q;
    int* sink;
};

__device__ __forceinline__ int64_t read_lo(const Args& a, int64_t c) { return c * a.n_reads / a.n_chunks; }

__device__ __forceinline__ int load_batch(const Args& a, int64_t r0, int64_t r1) {
    // int4 loads of reads [r0, r1) of three arrays, lane L: reads r0 + 4L ..
    const int64_t r = (r0 & ~3ll) + 4 * threadIdx.x;
    int acc = 0;
    if (r < r1) {
        const i32x4 t = a.tid[r >> 2], p = a.pos[r >> 2], s = a.span[r >> 2];
        acc = t.x + p.y + s.z + t.w;
    }
    return acc;
}

__device__ __forceinline__ void store_tile(const Args& a, int64_t c, int t, int v) {
    i32x4* base = a.depth + c * kChunk4 + t * kTile4 + threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) __builtin_nontemporal_store(i32x4{v, j, t, 3}, base + j * 256);
}

template <int MODE, bool LDS>
__global__ void __launch_bounds__(256, 4) k2shape(Args a) {
    __shared__ unsigned c_s[2];
    __shared__ int pad[LDS ? 10240 : 1];
    if (LDS && threadIdx.x == 0) pad[0] = 0;
    int acc = 0;
    unsigned nxt = 0;
    if (MODE == 4) {
        if (threadIdx.x == 0) c_s[0] = atomicAdd(a.q, 1u);
        __syncthreads();
        nxt = c_s[0];
        __syncthreads();
    }
    int pre = 0;                           // MODE 4: the next chunk's first batch
    for (int it = 0;; ++it) {
        unsigned cu;
        if (MODE == 4) {
            cu = nxt;
        } else {
            if (threadIdx.x == 0) c_s[0] = atomicAdd(a.q, 1u);
            __syncthreads();
            cu = c_s[0];
            __syncthreads();
        }
        const int64_t c = cu;
        if (c >= a.n_chunks) break;
        const int64_t r0 = read_lo(a, c), r1 = read_lo(a, c + 1);
        const int nb = (int)((r1 - r0 + kBatch - 1) / kBatch);
        if (MODE == 0) {                   // wr
            for (int t = 0; t < 8; ++t) store_tile(a, c, t, t);
        } else if (MODE == 1) {            // rd
            for (int b = 0; b < nb; ++b) acc += load_batch(a, r0 + (int64_t)b * kBatch, r1);
        } else if (MODE == 2 || MODE == 5) {   // seq / indep
            int v = 0;
            for (int b = 0; b < nb; ++b) v += load_batch(a, r0 + (int64_t)b * kBatch, r1);
            if (MODE == 5) acc += v;
            for (int t = 0; t < 8; ++t) store_tile(a, c, t, MODE == 5 ? t : v + t);
        } else {                           // inter / ahead
            int b = 0, v = (MODE == 4 && it > 0) ? pre : load_batch(a, r0, r1);
            b = 1;
            int nextv = b < nb ? load_batch(a, r0 + (int64_t)b * kBatch, r1) : 0;
            for (int t = 0; t < 8; ++t) {
                // tile t needs the batches up to ceil((t + 1) * nb / 8)
                const int need = ((t + 1) * nb + 7) / 8;
                while (b < need) {
                    v += nextv;
                    ++b;
                    nextv = b < nb ? load_batch(a, r0 + (int64_t)b * kBatch, r1) : 0;
                }
                if (MODE == 4 && t == 6) {
                    if (threadIdx.x == 0) c_s[1] = atomicAdd(a.q, 1u);
                    __syncthreads();
                    nxt = c_s[1];
                    __syncthreads();
                    pre = nxt < a.n_chunks ? load_batch(a, read_lo(a, nxt), read_lo(a, nxt + 1)) : 0;
                }
                store_tile(a, c, t, v + t);
            }
            acc += nextv;
        }
    }
    if (acc == 0x7fedcba9) a.sink[0] = acc;
}

// 512-thread workgroups (8 waves) on the same chunks: 2 per CU keep K2's 16
// waves per CU with half as many concurrent chunk streams (the g512 rows
// above run 2 x 256-thread workgroups per CU: 8 waves).
template <int MODE>
__global__ void __launch_bounds__(512, 2) k2shape512(Args a) {
    __shared__ unsigned c_s[2];
    __shared__ int pad[20480];
    if (threadIdx.x == 0) pad[0] = 0;
    int acc = 0;
    for (;;) {
        if (threadIdx.x == 0) c_s[0] = atomicAdd(a.q, 1u);
        __syncthreads();
        const int64_t c = c_s[0];
        __syncthreads();
        if (c >= a.n_chunks) break;
        const int64_t r0 = read_lo(a, c), r1 = read_lo(a, c + 1);
        constexpr int kB2 = 2048;
        const int nb = (int)((r1 - r0 + kB2 - 1) / kB2);
        auto load2 = [&](int64_t q0) {
            const int64_t r = (q0 & ~3ll) + 4 * threadIdx.x;
            int v = 0;
            if (r < r1) {
                const i32x4 t = a.tid[r >> 2], p = a.pos[r >> 2], s = a.span[r >> 2];
                v = t.x + p.y + s.z + t.w;
            }
            return v;
        };
        auto store2 = [&](int t, int v) {
            i32x4* base = a.depth + c * kChunk4 + t * kTile4 + threadIdx.x;
            __builtin_nontemporal_store(i32x4{v, 0, t, 3}, base);
            __builtin_nontemporal_store(i32x4{v, 1, t, 3}, base + 512);
        };
        if (MODE == 2) {
            int v = 0;
            for (int b = 0; b < nb; ++b) v += load2(r0 + (int64_t)b * kB2);
            for (int t = 0; t < 8; ++t) store2(t, v + t);
        } else {
            int b = 1, v = load2(r0);
            int nextv = b < nb ? load2(r0 + (int64_t)b * kB2) : 0;
            for (int t = 0; t < 8; ++t) {
                const int need = ((t + 1) * nb + 7) / 8;
                while (b < need) {
                    v += nextv;
                    ++b;
                    nextv = b < nb ? load2(r0 + (int64_t)b * kB2) : 0;
                }
                store2(t, v + t);
            }
            acc += nextv;
        }
    }
    if (acc == 0x7fedcba9) a.sink[0] = acc;
}

int main() {
    const int64_t n_chunks = 1005000000LL / 32768;          // 30,670 chunks (C3 genome)
    const int64_t n_reads = 100000000LL;
    const int64_t wbytes = n_chunks * kChunk4 * 16, rbytes = 3 * n_reads * 4;
    Args a;
    i32x4 *t, *p, *s, *d; unsigned* q; int* o;
    CK(hipMalloc(&t, n_reads * 4 + 64)); CK(hipMalloc(&p, n_reads * 4 + 64)); CK(hipMalloc(&s, n_reads * 4 + 64));
    CK(hipMalloc(&d, wbytes)); CK(hipMalloc(&q, 64)); CK(hipMalloc(&o, 64));
    CK(hipMemset(t, 1, n_reads * 4)); CK(hipMemset(p, 2, n_reads * 4)); CK(hipMemset(s, 3, n_reads * 4));
    a.tid = t; a.pos = p; a.span = s; a.depth = d; a.n_chunks = n_chunks; a.n_reads = n_reads; a.q = q; a.sink = o;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    printf("C3 shape: %lld chunks, %.3f GB written, %.3f GB read\n", (long long)n_chunks, wbytes / 1e9, rbytes / 1e9);
    auto run = [&](const char* nm, int g, auto kern, double bytes, int bt = 256) {
        float ms[8];
        for (int rep = 0; rep < 9; ++rep) {
            hipMemsetAsync(q, 0, 4);
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(g), dim3(bt), 0, 0, a);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float x; hipEventElapsedTime(&x, e0, e1);
            if (rep) ms[rep - 1] = x;
        }
        float best = 1e9, sum = 0; for (float x : ms) { best = x < best ? x : best; sum += x; }
        printf("%-14s g%-5d avg %.4f ms best %.4f ms  %.2f TB/s (best %.2f)\n", nm, g, sum / 8, best,
               bytes / (sum / 8 * 1e-3) / 1e12, bytes / (best * 1e-3) / 1e12);
    };
    const double mix = (double)wbytes + rbytes;
    for (int g : {512, 256}) {
        run("seq 512thr", g, k2shape512<2>, mix, 512);
        run("inter 512thr", g, k2shape512<3>, mix, 512);
    }
    for (int g : {512, 1024}) {
        run("wr", g, k2shape<0, true>, wbytes);
        run("rd", g, k2shape<1, true>, rbytes);
        run("seq", g, k2shape<2, true>, mix);
        run("inter", g, k2shape<3, true>, mix);
        run("ahead", g, k2shape<4, true>, mix);
        run("indep", g, k2shape<5, true>, mix);
        run("seq nolds", g, k2shape<2, false>, mix);
        run("inter nolds", g, k2shape<3, false>, mix);
    }
    return 0;
}
