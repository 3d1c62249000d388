// pileup.experimental's read pass on the device (csrc/exp_gpu.hip), over the
// read table a reads-mode GPU decode leaves in HBM (mc_bam_gpu_open_reads).
// Host-side declarations only: csrc/exp_reads.cpp dispatches to it when its
// mc_reads holds a device table.
#pragma once
#include <stdint.h>

#include <vector>

struct ExpDevTable {
    int device = 0;
    int k = 0;
    int64_t n = 0;                      // placed records, file order
    const int32_t* tid = nullptr;
    const int32_t* pos = nullptr;
    const int64_t* end = nullptr;       // bam_endpos
    const int32_t* flag = nullptr;
    const uint8_t* bits = nullptr;      // 1: no SEQ, 2: no reference length
    const uint32_t* kmer = nullptr;     // the first k aligned bases (2-bit code) or ~0
    const uint8_t* name_len = nullptr;
    const int64_t* name_off = nullptr;
    const uint8_t* names = nullptr;
};

// Per contig: first[t] = the first record with tid >= t (first[n_ref] = n),
// max_span[t] = max(end - pos) of its records (0 without records).
// unsorted_at: the first record out of (tid, pos) order, or -1.
int exp_gpu_index(const ExpDevTable& t, int32_t n_ref, int64_t* first, int64_t* max_span, int64_t* unsorted_at);

// Device buffers kept between calls (one per mc_reads table).
struct ExpScratch;
void exp_gpu_scratch_free(ExpScratch* s);

// mc_experimental_reads on the device: the same counts[8 R] / sums[4 R] and
// per-region "RCOR is ZERO" events as the host pass (csrc/exp_reads.cpp).
// val / has: the two k-mer tables (null: k_cor is None).
int exp_gpu_reads(const ExpDevTable& t, const int64_t* first, const int64_t* max_span, const double* val1,
                  const uint8_t* has1, const double* val2, const uint8_t* has2, int64_t R, const int32_t* tid,
                  const int64_t* start, const int64_t* end, int64_t* counts, double* sums,
                  std::vector<std::vector<uint64_t>>& events, double* kernel_ms, ExpScratch** scratch);
