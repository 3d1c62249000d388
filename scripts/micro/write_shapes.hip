// Write-only ceiling on one MI355X for K2's store shape: 4.02 GB of int32
// depth written once.  Variants: grid-stride, dynamic 128 KiB chunks per
// workgroup (K2's queue), workgroups per CU, plain / nt / sc1 stores.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef int i32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>
__device__ __forceinline__ void st(i32x4* p, i32x4 v) {
    if (MODE == 0) *p = v;
    else if (MODE == 1) __builtin_nontemporal_store(v, p);
    else __hip_atomic_store(reinterpret_cast<int*>(p), v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
__global__ void __launch_bounds__(256) grid_stride(i32x4* __restrict__ d, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) st<MODE>(d + i, i32x4{(int)i, 1, 2, 3});
}

// dynamic queue of chunks of CW int4 (per workgroup); inside a chunk, tiles
// of 1024 int4 (16 KiB): wave w writes int4 [w*256, w*256+256) of the tile,
// 4 instructions of 64 lanes x 16 B.
template <int MODE, int CW>
__global__ void __launch_bounds__(256) chunked(i32x4* __restrict__ d, int64_t n4, unsigned* q) {
    __shared__ unsigned c_s;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (;;) {
        if (threadIdx.x == 0) c_s = atomicAdd(q, 1u);
        __syncthreads();
        const int64_t c = c_s;
        __syncthreads();
        if (c * CW >= n4) break;
        for (int t = 0; t < CW / 1024; ++t) {
            i32x4* base = d + c * CW + t * 1024 + wave * 256 + lane;
#pragma unroll
            for (int j = 0; j < 4; ++j) st<MODE>(base + j * 64, i32x4{t, j, lane, 3});
        }
    }
}

// like chunked<0, CW>, but lane L of wave w writes the 64 contiguous bytes
// [w*4096 + 64L, +64) of the tile as 4 dwordx4 (lane stride 64 B per instruction)
template <int CW>
__global__ void __launch_bounds__(256) chunked_lane64(i32x4* __restrict__ d, int64_t n4, unsigned* q) {
    __shared__ unsigned c_s;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (;;) {
        if (threadIdx.x == 0) c_s = atomicAdd(q, 1u);
        __syncthreads();
        const int64_t c = c_s;
        __syncthreads();
        if (c * CW >= n4) break;
        for (int t = 0; t < CW / 1024; ++t) {
            i32x4* base = d + c * CW + t * 1024 + wave * 256 + lane * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) base[j] = i32x4{t, j, lane, 3};
        }
    }
}

int main() {
    const int64_t wbytes = 4020000000LL / (1 << 17) * (1 << 17);
    const int64_t n4 = wbytes / 16;
    i32x4* d; unsigned* q;
    CK(hipMalloc(&d, wbytes)); CK(hipMalloc(&q, 64));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto run = [&](const char* nm, auto launch) {
        float ms[5];
        for (int rep = 0; rep < 6; ++rep) {
            hipMemset(q, 0, 4);
            hipEventRecord(a);
            launch();
            hipEventRecord(b); hipEventSynchronize(b);
            float t; hipEventElapsedTime(&t, a, b);
            if (rep) ms[rep - 1] = t;
        }
        float best = 1e9, sum = 0; for (float t : ms) { best = t < best ? t : best; sum += t; }
        printf("%-34s avg %.4f ms  %.2f TB/s (best %.2f)\n", nm, sum / 5, wbytes / (sum / 5 * 1e-3) / 1e12,
               wbytes / (best * 1e-3) / 1e12);
    };
    for (int g : {1024, 2048}) {
        char nm[64];
        snprintf(nm, 64, "grid-stride plain g%d", g); run(nm, [&] { hipLaunchKernelGGL(grid_stride<0>, dim3(g), dim3(256), 0, 0, d, n4); });
        snprintf(nm, 64, "grid-stride nt g%d", g); run(nm, [&] { hipLaunchKernelGGL(grid_stride<1>, dim3(g), dim3(256), 0, 0, d, n4); });
    }
    for (int g : {512, 1024}) {
        char nm[64];
        snprintf(nm, 64, "chunk128K lane64B plain g%d", g); run(nm, [&] { hipLaunchKernelGGL((chunked_lane64<8192>), dim3(g), dim3(256), 0, 0, d, n4, q); });
        snprintf(nm, 64, "chunk128K coalesced plain g%d", g); run(nm, [&] { hipLaunchKernelGGL((chunked<0, 8192>), dim3(g), dim3(256), 0, 0, d, n4, q); });
    }
    for (int g : {512, 1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, 64, "chunk128K plain g%d", g); run(nm, [&] { hipLaunchKernelGGL((chunked<0, 8192>), dim3(g), dim3(256), 0, 0, d, n4, q); });
        snprintf(nm, 64, "chunk128K nt g%d", g); run(nm, [&] { hipLaunchKernelGGL((chunked<1, 8192>), dim3(g), dim3(256), 0, 0, d, n4, q); });
        snprintf(nm, 64, "chunk16K plain g%d", g); run(nm, [&] { hipLaunchKernelGGL((chunked<0, 1024>), dim3(g), dim3(256), 0, 0, d, n4, q); });
        snprintf(nm, 64, "chunk1M plain g%d", g); run(nm, [&] { hipLaunchKernelGGL((chunked<0, 65536>), dim3(g), dim3(256), 0, 0, d, n4, q); });
    }
    return 0;
}
