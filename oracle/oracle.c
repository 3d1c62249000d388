/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Linked by tests/ and by bench.py's
 * cpu_baseline leg; never by the product (metacov_amd/), which has no CPU
 * compute path.
 *
 * A plain-C restatement of the reference's pileup path:
 *
 *  - depth as htslib's pileup engine produces it (PileupColumn.n, read by
 *    metacov/pileup.py:13-16 through pysam's default "all" stepper):
 *      orc_depth_columnwalk  the engine's own shape: a column sweep keeping
 *                            the list of active reads, visiting every active
 *                            read at every column (bam_plp_next walks its
 *                            read list per position), emitting n
 *      orc_depth_interval    the same count by a difference array
 *    Third-party algorithm (htslib bundled with pysam; version unpinned by
 *    the reference: requirements.txt:2, setup.py:45,53).
 *
 *  - the region statistics of pileup.classic (metacov/pileup.py:18-26):
 *      orc_region_stats      exact integer row (mc_region_stat layout) by a
 *                            counting sort: min, max, sum, sum of squares,
 *                            ranks (n-1)/2 and n/2, sum of ranks [n/4, n-n/4)
 *      orc_pileup_classic    classic() as the reference runs it, end to end
 *                            per region: column walk -> float64 columns
 *                            (pileup.py:11-16) -> amin/amax/median/std/mean/
 *                            sorted()-slice mean/sum (pileup.py:18-26), with
 *                            a full sort standing in for Python's sorted().
 *                            This is the CPU baseline bench.py times.
 *
 * Pinned by tests/test_oracle.py against tests/golden/*.json, whose region
 * statistics come from the reference's real pileup.classic (see
 * tests/golden/make_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t n, sum;
    uint64_t sumsq;
    int64_t min, max, med_lo, med_hi, q23_sum, q23_cnt;
} orc_region_stat;

/* contig t occupies depth[coff[t] .. coff[t] + extent[t]) */

int orc_depth_interval(int32_t nc, const int64_t* extent, const int64_t* coff, int64_t n,
                       const int32_t* tid, const int32_t* pos, const int32_t* span,
                       int32_t* depth) {
    for (int32_t t = 0; t < nc; ++t) memset(depth + coff[t], 0, (size_t)extent[t] * 4);
    /* diff array in place, one extra slot per contig kept in a side buffer */
    int32_t* tail = (int32_t*)calloc((size_t)nc + 1, 4);
    for (int64_t i = 0; i < n; ++i) {
        const int32_t t = tid[i];
        const int64_t a = pos[i], b = (int64_t)pos[i] + span[i];
        if (t < 0 || t >= nc || b <= a) continue;
        depth[coff[t] + a] += 1;
        if (b < extent[t]) depth[coff[t] + b] -= 1;
        else tail[t] -= 1;
    }
    for (int32_t t = 0; t < nc; ++t) {
        int32_t run = 0;
        int32_t* d = depth + coff[t];
        for (int64_t p = 0; p < extent[t]; ++p) {
            run += d[p];
            d[p] = run;
        }
    }
    free(tail);
    return 0;
}

/* Active-read sweep over one contig's reads [a, b) (sorted by pos), writing
 * n for every column in [lo, hi) into cols (index p - lo). */
static void column_walk(const int32_t* pos, const int32_t* span, int64_t a, int64_t b, int64_t lo,
                        int64_t hi, int64_t* act, int32_t* out_i32, double* out_f64) {
    int64_t n_act = 0, next = a;
    int64_t p = lo;
    while (p < hi) {
        if (n_act == 0) {
            if (next >= b) break;
            if (pos[next] > p) p = pos[next];
            if (p >= hi) break;
        }
        while (next < b && pos[next] <= p) {
            const int64_t e = (int64_t)pos[next] + span[next];
            if (e > p) act[n_act++] = e;
            ++next;
        }
        /* per column: visit every active read (bam_plp_next's list walk) */
        int64_t k = 0;
        for (int64_t j = 0; j < n_act; ++j)
            if (act[j] > p) act[k++] = act[j];
        n_act = k;
        if (out_i32) out_i32[p - lo] = (int32_t)n_act;
        if (out_f64) out_f64[p - lo] += (double)n_act;
        ++p;
    }
}

static int64_t lower_bound_pos(const int32_t* pos, int64_t a, int64_t b, int64_t key) {
    while (a < b) {
        const int64_t m = a + (b - a) / 2;
        if (pos[m] < key) a = m + 1;
        else b = m;
    }
    return a;
}

int orc_depth_columnwalk(int32_t nc, const int64_t* extent, const int64_t* coff, int64_t n,
                         const int32_t* tid, const int32_t* pos, const int32_t* span,
                         int32_t* depth) {
    int64_t i = 0;
    int64_t cap = 1024;
    int64_t* act = (int64_t*)malloc((size_t)cap * 8);
    for (int32_t t = 0; t < nc; ++t) {
        memset(depth + coff[t], 0, (size_t)extent[t] * 4);
        while (i < n && tid[i] < t) ++i;
        int64_t j = i;
        while (j < n && tid[j] == t) ++j;
        if (j - i > cap) {
            cap = j - i;
            act = (int64_t*)realloc(act, (size_t)cap * 8);
        }
        column_walk(pos, span, i, j, 0, extent[t], act, depth + coff[t], NULL);
        i = j;
    }
    free(act);
    return 0;
}

int orc_region_stats(const int32_t* depth, const int64_t* coff, const int64_t* extent,
                     int64_t R, const int32_t* tid, const int64_t* start, const int64_t* end,
                     orc_region_stat* out) {
    for (int64_t r = 0; r < R; ++r) {
        orc_region_stat o;
        memset(&o, 0, sizeof o);
        const int32_t t = tid[r];
        const int64_t n = end[r] - start[r];
        o.n = n;
        if (n <= 0) {
            out[r] = o;
            continue;
        }
        const int64_t a = start[r] < extent[t] ? start[r] : extent[t];
        const int64_t b = end[r] < extent[t] ? end[r] : extent[t];
        const int64_t zx = n - (b - a);
        int32_t vmax = 0;
        for (int64_t p = a; p < b; ++p)
            if (depth[coff[t] + p] > vmax) vmax = depth[coff[t] + p];
        int64_t* hist = (int64_t*)calloc((size_t)vmax + 1, 8);
        hist[0] += zx;
        for (int64_t p = a; p < b; ++p) {
            const int64_t v = depth[coff[t] + p];
            hist[v] += 1;
            o.sum += v;
            o.sumsq += (uint64_t)(v * v);
        }
        o.min = -1;
        const int64_t rlo = (n - 1) / 2, rhi = n / 2, qlo = n / 4, qhi = n - n / 4;
        int64_t cum = 0;
        for (int64_t v = 0; v <= vmax; ++v) {
            const int64_t c = hist[v];
            if (!c) continue;
            if (o.min < 0) o.min = v;
            o.max = v;
            const int64_t e = cum + c;
            if (rlo >= cum && rlo < e) o.med_lo = v;
            if (rhi >= cum && rhi < e) o.med_hi = v;
            const int64_t lo = cum > qlo ? cum : qlo, hi = e < qhi ? e : qhi;
            if (hi > lo) o.q23_sum += (hi - lo) * v;
            cum = e;
        }
        o.q23_cnt = qhi - qlo;
        free(hist);
        out[r] = o;
    }
    return 0;
}

static int cmp_f64(const void* x, const void* y) {
    const double a = *(const double*)x, b = *(const double*)y;
    return (a > b) - (a < b);
}

/* classic() end to end for R regions; reads sorted by (tid, pos), max_span
 * bounds how far before `start` an overlapping read may begin (the BAI query
 * of the real pileup).  out7[r*7 ..] = min, max, med, std, avg, q23, sum
 * (unrounded).  Returns the number of pileup columns visited. */
int64_t orc_pileup_classic(int64_t n, const int32_t* tid, const int32_t* pos, const int32_t* span,
                           int32_t max_span, int64_t R, const int32_t* rtid,
                           const int64_t* rstart, const int64_t* rend, double* out7) {
    int64_t visited = 0;
    int64_t cap = 1024;
    int64_t* act = (int64_t*)malloc((size_t)cap * 8);
    for (int64_t r = 0; r < R; ++r) {
        const int32_t t = rtid[r];
        const int64_t s = rstart[r], e = rend[r], len = e - s;
        double* o = out7 + r * 7;
        if (len <= 0) {
            for (int k = 0; k < 7; ++k) o[k] = NAN;
            continue;
        }
        /* reads of contig t: [ta, tb) */
        int64_t lo = 0, hi = n;
        while (lo < hi) { int64_t m = lo + (hi - lo) / 2; if (tid[m] < t) lo = m + 1; else hi = m; }
        const int64_t ta = lo;
        hi = n;
        while (lo < hi) { int64_t m = lo + (hi - lo) / 2; if (tid[m] <= t) lo = m + 1; else hi = m; }
        const int64_t tb = lo;
        const int64_t a = lower_bound_pos(pos, ta, tb, s - max_span);
        const int64_t b = lower_bound_pos(pos, ta, tb, e);
        if (b - a > cap) {
            cap = b - a;
            act = (int64_t*)realloc(act, (size_t)cap * 8);
        }
        double* cols = (double*)calloc((size_t)len, 8);
        column_walk(pos, span, a, b, s, e, act, NULL, cols);
        visited += len;
        double mn = cols[0], mx = cols[0], sum = 0;
        for (int64_t i = 0; i < len; ++i) {
            if (cols[i] < mn) mn = cols[i];
            if (cols[i] > mx) mx = cols[i];
            sum += cols[i];
        }
        const double mean = sum / (double)len;
        double ss = 0;
        for (int64_t i = 0; i < len; ++i) ss += (cols[i] - mean) * (cols[i] - mean);
        qsort(cols, (size_t)len, 8, cmp_f64);
        const double med = 0.5 * (cols[(len - 1) / 2] + cols[len / 2]);
        double qs = 0;
        for (int64_t i = len / 4; i < len - len / 4; ++i) qs += cols[i];
        o[0] = mn;
        o[1] = mx;
        o[2] = trunc(med);
        o[3] = sqrt(ss / (double)len);
        o[4] = mean;
        o[5] = qs / (double)(len - 2 * (len / 4));
        o[6] = sum;
        free(cols);
    }
    free(act);
    return visited;
}
