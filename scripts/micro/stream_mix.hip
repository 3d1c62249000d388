// Streaming ceiling for K2's traffic mix on one MI355X: 4 B/position written,
// 12 B/read loaded (C3: 1.2 GB read + 4.0 GB written per launch).
//   write-only, read-only, and the read+write mix in one persistent kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef int i32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <bool NT>
__global__ void __launch_bounds__(256) wr(i32x4* __restrict__ d, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        i32x4 v = {(int)i, 1, 2, 3};
        if (NT) __builtin_nontemporal_store(v, d + i); else d[i] = v;
    }
}
__global__ void __launch_bounds__(256) rd(const i32x4* __restrict__ s, int64_t n4, int* out) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int acc = 0;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) { i32x4 v = s[i]; acc += v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678) out[0] = acc;
}
// each block: chunks of (R reads-int4 loaded, W int4 written) in ratio 12:40 (3 read int4 per 10 written)
template <bool NT>
__global__ void __launch_bounds__(256) mix(const i32x4* __restrict__ s, int64_t rn4, i32x4* __restrict__ d, int64_t wn4, int* out) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    int acc = 0;
    int64_t ri = blockIdx.x * 256 + threadIdx.x;
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < wn4; i += stride) {
        // 3 of every 10 iterations also load
        if ((i / stride) % 10 < 3 && ri < rn4) { i32x4 v = s[ri]; acc += v.x ^ v.w; ri += stride; }
        i32x4 v = {(int)i, acc, 2, 3};
        if (NT) __builtin_nontemporal_store(v, d + i); else d[i] = v;
    }
    for (; ri < rn4; ri += stride) { i32x4 v = s[ri]; acc += v.x ^ v.w; }
    if (acc == 0x12345678) out[0] = acc;
}

int main() {
    const int64_t wbytes = 4020000000LL, rbytes = 1200000000LL;
    const int64_t wn4 = wbytes / 16, rn4 = rbytes / 16;
    i32x4 *d, *s; int* o;
    CK(hipMalloc(&d, wbytes)); CK(hipMalloc(&s, rbytes)); CK(hipMalloc(&o, 64));
    CK(hipMemset(s, 1, rbytes));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    int grids[] = {1024, 2048, 4096, 8192};
    for (int g : grids) {
        for (int k = 0; k < 5; ++k) {
            float ms[5];
            for (int rep = 0; rep < 6; ++rep) {
                CK(hipEventRecord(a));
                if (k == 0) hipLaunchKernelGGL(wr<true>, dim3(g), dim3(256), 0, 0, d, wn4);
                if (k == 1) hipLaunchKernelGGL(wr<false>, dim3(g), dim3(256), 0, 0, d, wn4);
                if (k == 2) hipLaunchKernelGGL(rd, dim3(g), dim3(256), 0, 0, s, rn4, o);
                if (k == 3) hipLaunchKernelGGL(mix<true>, dim3(g), dim3(256), 0, 0, s, rn4, d, wn4, o);
                if (k == 4) hipLaunchKernelGGL(mix<false>, dim3(g), dim3(256), 0, 0, s, rn4, d, wn4, o);
                CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
                float t; CK(hipEventElapsedTime(&t, a, b));
                if (rep) ms[rep - 1] = t;
            }
            float best = 1e9, sum = 0; for (float t : ms) { best = t < best ? t : best; sum += t; }
            const char* nm[] = {"write nt", "write", "read", "mix nt", "mix"};
            const double bytes = k < 2 ? wbytes : k == 2 ? rbytes : wbytes + rbytes;
            printf("grid %5d %-9s avg %.4f ms best %.4f ms  %.2f TB/s (best %.2f)\n", g, nm[k], sum / 5, best,
                   bytes / (sum / 5 * 1e-3) / 1e12, bytes / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
