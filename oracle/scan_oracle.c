/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Linked by tests/ and by the scan
 * bench's cpu_baseline leg; never by the product.
 *
 * Plain-C restatement of the reference's `scan` read loop
 * (metacov/scan.pyx:623-672) over the same SoA batches the GPU path reads,
 * one read at a time and in the reference's per-processor shapes:
 *   get_seq         nt16 -> nt4, reverse strand reverse-complemented into a
 *                   read-orientation buffer (scan.pyx:240-259)
 *   ByFlag          group index, first flag most significant (:406-419)
 *   BaseHist        :442-470   KmerHist :482-501
 *   MirrorHist      :525-543   IsizeHist :561-579
 * Outputs are group-major: base [G][rows][5], kmer [G][4^K+1][NK], mirror
 * [G][N+1][2], isize [G][cap], isize_max [G] (uint32 counts wrap like the
 * reference's numpy uint32 arrays).  Undefined reads of the reference
 * (positions outside the sequence, no sequence, k-mer bases outside the
 * read) read as N, as in oracle/scan.py and the product.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int32_t n_flags;
    uint32_t flags[16];
    int32_t base_on, base_start;
    int32_t kmer_on, kmer_k, kmer_nk, kmer_step, kmer_offset;
    int32_t mirror_on, mirror_offset, mirror_n;
    int32_t isize_on;
} orc_scan_config;

static const uint8_t NT16_NT4[16] = {4, 0, 1, 4, 2, 4, 4, 4, 3, 4, 4, 4, 4, 4, 4, 4};

static inline uint8_t comp4(uint8_t n) { return (uint8_t)(3 - n + (((3 - n) & 4) >> 2) * 5); }

static inline int ref_at(const uint8_t* ref, int64_t L, int64_t i) {
    if (!ref) return 4;
    if (i < 0) i += L;
    return (i < 0 || i >= L) ? 4 : ref[i];
}

/* ref: nt4 codes of all sequences; ref_off / ref_len per sequence.
 * base_rows / isize_cap: the table shapes the caller allocated. */
int64_t orc_scan(const orc_scan_config* c, int64_t n, const int32_t* rlen, const int32_t* flag,
                 const int32_t* gpos, const int32_t* gisize, const int32_t* ref_id,
                 const int64_t* seq_off, const uint8_t* seq, const uint8_t* ref,
                 const int64_t* ref_off, const int64_t* ref_len, int32_t n_ref,
                 int64_t base_rows, uint32_t* base, uint32_t* kmer, uint32_t* mirror,
                 int64_t isize_cap, uint32_t* isize, int32_t* isize_max) {
    int32_t cap = 256;
    uint8_t* read = (uint8_t*)malloc((size_t)cap);
    const int64_t nbucket = (int64_t)1 << (2 * c->kmer_k);
    int64_t done = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int32_t L = rlen[r], fl = flag[r], pos0 = gpos[r];
        if (L > cap) {
            cap = L;
            read = (uint8_t*)realloc(read, (size_t)cap);
        }
        const uint8_t* s = seq + seq_off[r];
        const int rev = (fl & 0x10) != 0;
        for (int32_t i = 0; i < L; ++i) {
            const uint8_t b = (i & 1) ? (s[i >> 1] & 15) : (s[i >> 1] >> 4);
            if (rev)
                read[L - i - 1] = comp4(NT16_NT4[b]);
            else
                read[i] = NT16_NT4[b];
        }
        int g = 0;
        for (int f = 0; f < c->n_flags; ++f) {
            g <<= 1;
            if (c->flags[f] & (uint32_t)fl) g += 1;
        }
        const uint8_t* rs = NULL;
        int64_t rl = 0;
        if (ref_id[r] >= 0 && ref_id[r] < n_ref) {
            rs = ref + ref_off[ref_id[r]];
            rl = ref_len[ref_id[r]];
        }
        if (c->base_on) {
            const int sp = c->base_start;
            uint32_t* cnt = base + (int64_t)g * base_rows * 5;
            if (pos0 >= sp) {
                int mismatch = 0;
                if (rev) {
                    for (int32_t i = 0; i < L; ++i)
                        if (read[i] != comp4((uint8_t)ref_at(rs, rl, (int64_t)pos0 - i - 1)))
                            mismatch += 1;
                } else {
                    for (int32_t i = 0; i < L; ++i)
                        if (read[i] != ref_at(rs, rl, (int64_t)pos0 + i)) mismatch += 1;
                }
                if (!(mismatch * 32 > L)) {
                    for (int i = 0; i < sp; ++i) {
                        const int v = rev ? comp4((uint8_t)ref_at(rs, rl, (int64_t)pos0 - i - 1 + sp))
                                          : ref_at(rs, rl, (int64_t)pos0 + i - sp);
                        cnt[i * 5 + v] += 1;
                    }
                    for (int32_t i = 0; i < L; ++i) cnt[(int64_t)(i + sp) * 5 + read[i]] += 1;
                }
            }
        }
        if (c->kmer_on && L >= c->kmer_offset + c->kmer_step * c->kmer_nk) {
            uint32_t* cnt = kmer + (int64_t)g * (nbucket + 1) * c->kmer_nk;
            for (int i = 0; i < c->kmer_nk; ++i) {
                int64_t k = 0;
                for (int j = 0; j < c->kmer_k; ++j) {
                    const int64_t x = (int64_t)c->kmer_offset + (int64_t)i * c->kmer_step + j;
                    const int v = (x >= 0 && x < L) ? read[x] : 4;
                    if (v > 3) {
                        k = nbucket;
                        break;
                    }
                    k |= (int64_t)v << (2 * j);
                }
                cnt[k * c->kmer_nk + i] += 1;
            }
        }
        if (c->mirror_on) {
            const int64_t p = (int64_t)pos0 + c->mirror_offset;
            if (!(p < (int64_t)c->mirror_n - c->mirror_offset)) {
                int plain = 0, cmp = 0;
                for (int i = 0; i < c->mirror_n; ++i) {
                    const int a = ref_at(rs, rl, p + i + 1), b = ref_at(rs, rl, p - i - 1);
                    if (a != b) plain += 1;
                    if (a != comp4((uint8_t)b)) cmp += 1;
                }
                uint32_t* cnt = mirror + (int64_t)g * (c->mirror_n + 1) * 2;
                cnt[plain * 2] += 1;
                cnt[cmp * 2 + 1] += 1;
            }
        }
        if (c->isize_on) {
            int64_t v = gisize[r];
            if (v < 0) v = -v;
            if (v > isize_max[g]) isize_max[g] = (int32_t)v;
            if (v < isize_cap) isize[(int64_t)g * isize_cap + v] += 1;
        }
        ++done;
    }
    free(read);
    return done;
}
