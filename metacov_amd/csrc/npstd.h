// numpy's own float64 order for np.std(columns) (metacov/pileup.py:22).
//
// classic() rounds np.std of the float64 column vector to two decimals.  The
// exact integer row gives sqrt(exact variance), which rounds the same way
// except when the value lies on a .xx5 boundary to within numpy's rounding
// noise; for those regions the engine reproduces numpy's value bit for bit:
//
//   m  = fl(sum / n)                       (np.mean: its pairwise sum of
//                                            integers is exact)
//   a_i = fl(fl(v_i - m)^2)                 (x = arr - arrmean; x = x * x)
//   T  = ((0 + P(a[0:8192])) + P(a[8192:16384])) + ...
//                                          (umr_sum: the ufunc reduction walks
//                                            the array in buffers of 8192
//                                            elements, NPY_BUFSIZE, adding each
//                                            buffer's pairwise sum in turn)
//   P  = numpy's pairwise_sum: n < 8 a plain loop; n <= 128 eight
//        accumulators then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) and the
//        remainder; else split at n2 = n/2 - (n/2)%8
//   std = sqrt(fl(T / n))                  (computed by the caller)
//
// No FMA contraction anywhere in this file: numpy computes x*x into an
// array and sums it, each operation rounded on its own.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mc {

constexpr int kNpBuf = 8192;   // NPY_BUFSIZE: elements per reduction buffer
constexpr int kNpLeaf = 128;   // PW_BLOCKSIZE: pairwise_sum's leaf

// One numpy reduction buffer of one region: elements [0, n) at depth[gpos + i]
// for i < n_data, 0 beyond (positions past the contig's extent).
struct NpBlock {
    int64_t gpos;
    int32_t n_data;
    int32_t n;
    int32_t region;
    int32_t pad;
};

__device__ inline double np_elem(const int32_t* __restrict__ d, int n_data, int i, double m) {
#pragma clang fp contract(off)
    const double x = (double)(i < n_data ? d[i] : 0) - m;
    return x * x;
}

// pairwise_sum's leaf (n <= 128) over elements [off, off + n)
__device__ inline double np_leaf(const int32_t* __restrict__ d, int n_data, int off, int n, double m) {
#pragma clang fp contract(off)
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res += np_elem(d, n_data, off + i, m);
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = np_elem(d, n_data, off + j, m);
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += np_elem(d, n_data, off + i + j, m);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += np_elem(d, n_data, off + i, m);
    return res;
}

// pairwise_sum over [0, n) by one lane, the recursion on an explicit stack
// (n <= 8192: depth <= 7)
__device__ inline double np_pairwise_serial(const int32_t* __restrict__ d, int n_data, int n, double m) {
#pragma clang fp contract(off)
    int so[12], sn[12], st[12];
    double sl[12];
    int sp = 0;
    so[0] = 0;
    sn[0] = n;
    st[0] = 0;
    double res = 0.0;
    sp = 1;
    while (sp > 0) {
        const int f = sp - 1;
        if (sn[f] <= kNpLeaf) {
            res = np_leaf(d, n_data, so[f], sn[f], m);
            --sp;
            continue;
        }
        int n2 = sn[f] / 2;
        n2 -= n2 % 8;
        if (st[f] == 0) {          // left half
            st[f] = 1;
            so[sp] = so[f];
            sn[sp] = n2;
            st[sp] = 0;
            ++sp;
        } else if (st[f] == 1) {   // right half
            sl[f] = res;
            st[f] = 2;
            so[sp] = so[f] + n2;
            sn[sp] = sn[f] - n2;
            st[sp] = 0;
            ++sp;
        } else {
            res = sl[f] + res;
            --sp;
        }
    }
    return res;
}

// One wave per buffer.  A whole buffer (8192) is a balanced tree of 64
// leaves of 128: lane L sums leaf L, then an xor butterfly adds aligned
// pairs, fours, ... (fl(a + b) is commutative, so each lane's value is the
// subtree sum numpy forms).  A partial last buffer is summed by lane 0.
__global__ __launch_bounds__(256) void np_block_kernel(const int32_t* __restrict__ depth,
                                                       const NpBlock* __restrict__ blk, int nblk,
                                                       const double* __restrict__ mean,
                                                       double* __restrict__ bsum) {
#pragma clang fp contract(off)
    const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    if (w >= nblk) return;
    const NpBlock b = blk[w];
    const double m = mean[b.region];
    const int32_t* d = depth + b.gpos;
    if (b.n == kNpBuf) {
        double r = np_leaf(d, b.n_data, lane * kNpLeaf, kNpLeaf, m);
        for (int s = 1; s < 64; s <<= 1) {
            const double o = __shfl_xor(r, s, 64);
            r = r + o;
        }
        if (lane == 0) bsum[w] = r;
    } else if (lane == 0) {
        bsum[w] = np_pairwise_serial(d, b.n_data, b.n, m);
    }
}

// T of each region: its buffers' sums added in order, from 0.0.
__global__ void np_region_kernel(const double* __restrict__ bsum, const int32_t* __restrict__ first,
                                 int R, double* __restrict__ out) {
#pragma clang fp contract(off)
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    double t = 0.0;
    for (int k = first[r]; k < first[r + 1]; ++k) t += bsum[k];
    out[r] = t;
}

}  // namespace mc
