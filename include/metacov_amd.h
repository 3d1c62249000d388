/*
 * metacov_amd — MI355X (gfx950) per-base coverage engine, C ABI.
 *
 * Drop-in replacement for the arithmetic under the reference's pileup path:
 *
 *   metacov pileup (metacov/cli.py:49-108)
 *     -> pileup.classic(bam, ref, start, end)      (metacov/pileup.py:9-26)
 *        -> pysam AlignmentFile.pileup()  ->  htslib bam_plp / PileupColumn.n
 *           (called at metacov/pileup.py:13; third-party, unpinned)
 *        -> numpy min/max/median/std/mean/sorted()/sum  (pileup.py:18-26)
 *
 * and of the reference's only hand-written BAM read iterator
 * (scan.AlignmentFileIterator, metacov/scan.pyx:188-294; decl scan.pxd:6-27),
 * whose per-record callback protocol (ReadProcessor.process_read,
 * scan.pxd:30-36) is replaced by a batched struct-of-arrays interface.
 *
 * Conventions
 *  - every function returns int: 0 = ok, < 0 = error (MC_E_*); the message
 *    of the last error on the calling thread is mc_last_error().
 *  - callers own all host buffers; they are copied during the call.
 *  - the library owns device buffers, inside an opaque mc_ctx (one per GPU).
 *    A ctx is not thread-safe; distinct ctxs may be driven from distinct
 *    host threads.  There is no CPU fallback: a ctx needs a HIP device.
 *  - positions are 0-based; regions are half-open [start, end).
 */
#ifndef METACOV_AMD_H
#define METACOV_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MC_OK            0
#define MC_E_INVALID    -1   /* bad argument (null pointer, range, unsorted reads, ...) */
#define MC_E_HIP        -2   /* HIP runtime error (no device, OOM, launch failure) */
#define MC_E_IO         -3   /* file / BGZF / BAM format error */
#define MC_E_STATE      -4   /* call out of order (e.g. stats before depth) */
#define MC_E_RANGE      -5   /* value outside what the engine represents exactly */

/* Per-region statistics, exact integers.  Everything classic() reports
 * (pileup.py:18-26) follows from it:
 *   min = min, max = max, sum = sum,
 *   avg = round(sum / n, 2), std = round(sqrt((n*sumsq - sum^2) / n^2), 2),
 *   med = (med_lo + med_hi) / 2 truncated (np.median then int()),
 *   q23 = round(q23_sum / q23_cnt, 2)
 * with med_lo = sorted[(n-1)/2], med_hi = sorted[n/2] and q23_sum the sum of
 * sorted[n/4 .. n - n/4)  (pileup.py:24).  n == 0 marks an empty region
 * (classic raises ValueError there). */
typedef struct mc_region_stat {
    int64_t  n;
    int64_t  sum;
    uint64_t sumsq;
    int64_t  min;
    int64_t  max;
    int64_t  med_lo;
    int64_t  med_hi;
    int64_t  q23_sum;
    int64_t  q23_cnt;
} mc_region_stat;

/* Kernel timings of the last mc_compute_depth / mc_region_stats calls, in
 * milliseconds, from HIP events recorded on the ctx stream. */
typedef struct mc_timings {
    float cigar_ms;      /* K1: CIGAR -> span (0 when spans were given) */
    float depth_ms;      /* K2: tile depth kernel */
    float stats_ms;      /* K3: region histogram + reduction (+ finalize) */
    float prepare_ms;    /* ingest: sortedness check, extents, tile index */
    int64_t depth_launches;
    int64_t stats_launches;
    /* Sums over every mc_compute_depth_stats[_device] call of this ctx (each
     * read once its stream has drained inside the call), so a caller can
     * average many calls without a timing query between them. */
    double fused_depth_ms_total;   /* K2 */
    double fused_stats_ms_total;   /* K3b (+ fallback K3) */
    int64_t fused_calls;
    /* Batches prepared by the direct path and accepted by K2's checks, and
     * full mc_prepare passes (explicit, or a direct batch handed over). */
    int64_t direct_batches;
    int64_t full_prepares;
    double prepare_ms_total;       /* every prepare's prepare_ms (direct: the probe) */
    /* Direct batches redone with a wider halo (their spans outgrew the one
     * the previous batch set), and the halo (positions) of the last one. */
    int64_t halo_redos;
    int64_t direct_halo;
} mc_timings;

typedef struct mc_ctx mc_ctx;

const char* mc_last_error(void);
const char* mc_version(void);
/* "mc-source-sha256:<hex>": the sources and flags this library was built from
 * (metacov_amd/build.py rebuilds when the tree's hash differs). */
const char* mc_build_id(void);

/* The HIP runtime and device `device`'s context, initialised ahead of the
 * first mc_ctx_create (which does it anyway): the CLI calls it on a thread
 * while Python imports its modules, so the two start-up costs overlap
 * (nothing in the reference; pysam has no device to initialise).  A device
 * out of range initialises the runtime only. */
int mc_runtime_init(int device);

/* ---- context ------------------------------------------------------------ */
int mc_ctx_create(int device, mc_ctx** out);
int mc_ctx_destroy(mc_ctx* ctx);
/* Use an external hipStream_t (e.g. torch's current stream); NULL = own stream. */
int mc_ctx_set_stream(mc_ctx* ctx, void* hip_stream);
int mc_ctx_device(const mc_ctx* ctx, int* device);

/* ---- inputs ------------------------------------------------------------- */
/* Contig table: the BAM header's @SQ lengths (pysam bam.lengths,
 * used at util.py:64-69).  Resets reads and depth. */
int mc_set_contigs(mc_ctx* ctx, int32_t n, const int64_t* lengths);

/* Append coordinate-sorted pileup intervals (host pointers): read i covers
 * [pos[i], pos[i] + span[i]) on contig tid[i].  These are the records the
 * pileup "all" stepper keeps (flag & 0x704 == 0), span = reference length
 * of the CIGAR (ops M/D/N/=/X), 0 for a mapped read with none (1 under
 * MC_LEGACY_ENDPOS); a span-0 read adds no depth.
 * Replaces: per-record AlignmentFileIterator.cnext()/get_tid()/get_pos()
 * (scan.pyx:213-283) feeding ReadProcessor.process_read (scan.pxd:35). */
int mc_add_reads(mc_ctx* ctx, int64_t n, const int32_t* tid,
                 const int32_t* pos, const int32_t* span);

/* Same, but the copy is only enqueued on the ctx stream: with pinned host
 * buffers (hipHostMalloc / torch pin_memory) the DMA overlaps the caller's
 * next decode.  The buffers must stay unchanged until mc_synchronize(ctx)
 * (double-buffered streaming ingest: fill B, mc_synchronize, add A's
 * successor ...). */
int mc_add_reads_async(mc_ctx* ctx, int64_t n, const int32_t* tid,
                       const int32_t* pos, const int32_t* span);

/* Page-locked host buffers for mc_add_reads_async (hipHostMalloc). */
int mc_pinned_alloc(int64_t bytes, void** out);
int mc_pinned_free(void* p);

/* Same, but the three arrays are already in this ctx's device memory
 * (e.g. torch tensors); they are copied into the ctx. */
int mc_add_reads_device(mc_ctx* ctx, int64_t n, const int32_t* d_tid,
                        const int32_t* d_pos, const int32_t* d_span);

/* Long-read / raw-CIGAR mode: spans are computed on the GPU (K1) from the
 * BAM-packed CIGAR words (op in low 4 bits, length << 4) of each read,
 * read i owning cigar[cig_off[i] .. cig_off[i+1]).  Host pointers. */
int mc_add_reads_cigar(mc_ctx* ctx, int64_t n, const int32_t* tid,
                       const int32_t* pos, const int64_t* cig_off,
                       const uint32_t* cigar);

/* Same with device pointers (a batch already in HBM, e.g. torch tensors).
 * tid / pos are copied into the ctx before the call returns (the caller may
 * free or overwrite them afterwards); cig_off and cigar are BORROWED: they
 * must stay valid until the next mc_prepare (K1 reads them there), so a
 * 40 GB CIGAR batch is never duplicated.  cig_off[0] must be 0. */
int mc_add_reads_cigar_device(mc_ctx* ctx, int64_t n, const int32_t* d_tid,
                              const int32_t* d_pos, const int64_t* d_cig_off,
                              const uint32_t* d_cigar);

/* K1's span of a read whose CIGAR has no reference-consuming op: 0 (current
 * htslib bam_plp_push, the default) or 1 (legacy = 1: htslib <= 1.9
 * bam_endpos; see MC_LEGACY_ENDPOS).  Applies to later mc_add_reads_cigar*. */
int mc_set_legacy_endpos(mc_ctx* ctx, int legacy);

/* Drops the ctx's reads (the contigs stay): the next batch starts empty. */
int mc_clear_reads(mc_ctx* ctx);

/* The full prepare: validates order, computes contig extents (max of length
 * and furthest read end), the chunk index, K2's packed read words and the
 * long-read buckets.  Compute calls run it when the direct path (see
 * mc_set_direct_prepare) cannot take the batch; an explicit call builds an
 * index that later compute calls reuse. */
int mc_prepare(mc_ctx* ctx);

/* Drops the prepared index and depth (the reads stay): the next compute call
 * prepares the same device reads again, as for a fresh batch (what the
 * benchmark's per-batch step times). */
int mc_invalidate(mc_ctx* ctx);

/* Per-batch prepare of the compute calls (default on).  A compute call on a
 * batch that mc_prepare has not seen takes the DIRECT path: a sparse sample
 * of the reads (every 256th) locates each chunk's reads, K2 loads the raw
 * (tid, pos, span) and checks every read itself (range, order, end within
 * its contig, span <= 4096), so no separate pass over the batch runs before
 * K2.  A batch the direct path cannot take (unsorted / invalid reads: the
 * full prepare raises its exact error; long reads or reads past their
 * contig's end: handled by the full prepare, and later batches of the same
 * contig set go there directly) is re-run through mc_prepare inside the same
 * call, so results never depend on the path.  enable = 0: always mc_prepare. */
int mc_set_direct_prepare(mc_ctx* ctx, int enable);

/* ---- compute ------------------------------------------------------------ */
/* Per-position depth of every contig (K1 if needed, then K2). */
int mc_compute_depth(mc_ctx* ctx);

/* Copy depth[start, end) of contig tid to host (zeros past the extent). */
int mc_get_depth(mc_ctx* ctx, int32_t tid, int64_t start, int64_t end, int32_t* out);

/* Device pointer to the concatenated depth vector and each contig's offset
 * into it (for zero-copy consumers, e.g. torch). */
int mc_depth_device(mc_ctx* ctx, const int32_t** d_depth, int64_t* total_len);
int mc_contig_offset(mc_ctx* ctx, int32_t tid, int64_t* offset, int64_t* extent);

/* Region statistics (K3) for R regions; rows in input order.  Regions may
 * overlap and may run past the contig end (those positions count as 0,
 * as in pileup.py:11-16). */
int mc_region_stats(mc_ctx* ctx, int64_t R, const int32_t* tid,
                    const int64_t* start, const int64_t* end,
                    mc_region_stat* out);

/* Same, writing the R rows into device memory (for an RCCL all-gather). */
int mc_region_stats_device(mc_ctx* ctx, int64_t R, const int32_t* tid,
                           const int64_t* start, const int64_t* end,
                           mc_region_stat* d_out);

/* numpy's float64 sum of squared deviations of each region's column vector,
 * in numpy's own order, from the depth vector in HBM: with m = mean[r]
 * (= fl(sum / n), what np.mean returns), out[r] = the sum np.std forms over
 * fl(fl(v - m)^2): pairwise_sum within each 8192-element reduction buffer,
 * the buffers added in turn.  sqrt(fl(out[r] / n)) is then np.std(columns)
 * bit for bit (pileup.py:22).  classic() rounds it to two decimals; the
 * exact variance rounds the same way except within numpy's rounding noise of
 * a .xx5 boundary, and only such regions need this (metacov_amd.engine).
 * Regions must be non-empty; positions past the extent count as 0. */
int mc_region_np_sqdev(mc_ctx* ctx, int64_t R, const int32_t* tid,
                       const int64_t* start, const int64_t* end,
                       const double* mean, double* out);

/* Depth AND region statistics in one pass: K2 folds every tile into the
 * regions covering it while the depth values are still in registers, so the
 * depth vector is written once and never re-read.  Regions must not overlap
 * each other for the fused path (whole contigs, a tiling of a contig, most
 * BLAST hit lists); otherwise this runs K2 then K3.  Same rows as
 * mc_region_stats.  Each region's histogram window holds 864 values (1728 for
 * long reads) around its contig's estimated depth; a region whose median /
 * q23 ranks fall outside it is recomputed exactly from the depth vector
 * (mc_fused_recomputes / mc_fused_fallbacks). */
int mc_compute_depth_stats(mc_ctx* ctx, int64_t R, const int32_t* tid,
                           const int64_t* start, const int64_t* end,
                           mc_region_stat* out);
int mc_compute_depth_stats_device(mc_ctx* ctx, int64_t R, const int32_t* tid,
                                  const int64_t* start, const int64_t* end,
                                  mc_region_stat* d_out);
int mc_fused_fallbacks(mc_ctx* ctx, int64_t* out);
/* Regions of the last fused call whose median / q23 ranks left their LDS
 * window and were recomputed exactly ON THE DEVICE within the call (long-read
 * batches, or after a call that had such regions: the depth vector is
 * re-read for those regions only, no host round trip); mc_fused_fallbacks
 * counts the ones the host's K3 recomputed instead. */
int mc_fused_recomputes(mc_ctx* ctx, int64_t* out);

/* Aligned bases (sum of spans) of the reads added so far. */
int mc_aligned_bases(mc_ctx* ctx, int64_t* out);
int mc_max_depth(mc_ctx* ctx, int32_t* out);
int mc_get_timings(mc_ctx* ctx, mc_timings* out);
int mc_synchronize(mc_ctx* ctx);

/* ---- htslib's pileup read cap (opt-in) -----------------------------------
 * pysam's AlignmentFile.pileup(ref, start, end) (pileup.py:13) runs htslib's
 * pileup with max_depth = 8000: bam_plp_push drops a read that starts where
 * its predecessor started while the pileup's read pool holds more than
 * max_depth nodes.  keep[i] = 0 for the reads it would drop, given the
 * coordinate-sorted reads one pileup call sees (for classic(): the region's
 * overlapping records).  Host C++ (contigs on n_threads threads); the depth
 * of the kept reads is then computed as usual.  Version-dependent htslib
 * behaviour: parity unpinned (no htslib in this image); the closed form is
 * pinned by a literal restatement of the push/next loop (oracle/htslib_plp.py). */
int mc_depth_cap_mask(int64_t n, const int32_t* tid, const int32_t* pos, const int32_t* span,
                      int32_t max_depth, int n_threads, uint8_t* keep, int64_t* n_dropped);

/* The same mask on the device (csrc/capmask.h: one wave per query walks its
 * start groups in order; a chunk of 64 reads that cannot reach the cap is
 * applied in bulk).  d_*: device arrays; each distinct tid is one query.
 * MC_E_INVALID for unsorted reads, MC_E_RANGE for a span >= 32704 (the
 * wave's LDS ring of read ends; mc_depth_cap_mask takes those). */
int mc_depth_cap_mask_device(int device, int64_t n, const int32_t* d_tid, const int32_t* d_pos,
                             const int32_t* d_span, int32_t max_depth, uint8_t* d_keep,
                             int64_t* n_dropped);

/* The capped recompute's batch, built on the device (metacov_amd.depthcap):
 * from coordinate-sorted device intervals (e.g. mc_bam_gpu_intervals_device),
 * region r's query — the reads of contig qtid[r] overlapping [qstart[r],
 * qend[r]) by bam_endpos, what pysam's pileup(ref, start, end) hands htslib
 * (pileup.py:13) — with the cap applied, becomes contig r of the ctx's
 * batch.  The ctx must hold R contigs (mc_set_contigs: the regions' contig
 * lengths) and no reads.  Dropped reads (and reads of the gathered range
 * outside the query) stay in the batch with span 0, so they add no depth.
 * n_dropped: reads the cap dropped.  MC_E_RANGE for a span >= 32704. */
int mc_add_reads_capped(mc_ctx* ctx, int64_t n, const int32_t* d_tid, const int32_t* d_pos,
                        const int32_t* d_span, int64_t R, const int32_t* qtid, const int64_t* qstart,
                        const int64_t* qend, int32_t max_depth, int64_t* n_dropped);

/* ---- host BAM decoder (C++, multi-threaded BGZF inflate) ----------------
 * Replaces the pysam/htslib read path the reference uses: AlignmentFile
 * header (bam.references / bam.lengths, cli.py:80, util.py:64-69),
 * IteratorRowAll over records (scan.pyx:204), and bam_plp_push's pileup
 * interval [pos, pos + bam_cigar2rlen) (MC_LEGACY_ENDPOS: bam_endpos). */
typedef struct mc_bam mc_bam;

/* OR'd into any decoder's flag_filter (bits 0-15 are BAM flags): the pileup
 * interval of a mapped read with no reference-consuming CIGAR op is
 * [pos, pos + 1), as htslib <= 1.9 bam_plp_push set it (tail->end =
 * bam_endpos(b)).  Default (bit clear): current htslib, whose bam_plp_push
 * sets tail->end = pos + bam_cigar2rlen(...) ("raw rlen rather than
 * bam_endpos() which adjusts rlen=0 to rlen=1"), so such a read has span 0
 * and adds nothing to PileupColumn.n.  Version-dependent; parity unpinned. */
#define MC_LEGACY_ENDPOS 0x10000u

int mc_bam_open(const char* path, int n_threads, uint32_t flag_filter,
                int keep_cigar, mc_bam** out);
int mc_bam_close(mc_bam* bam);
int mc_bam_n_targets(const mc_bam* bam, int32_t* n);
int mc_bam_target(const mc_bam* bam, int32_t i, const char** name, int64_t* length);
/* records in the file / records kept by the flag filter (and tid >= 0) */
int mc_bam_counts(const mc_bam* bam, int64_t* n_records, int64_t* n_kept,
                  int64_t* n_mapped, int64_t* n_unmapped);
int mc_bam_intervals(const mc_bam* bam, int32_t* tid, int32_t* pos, int32_t* span);
/* keep_cigar only: total CIGAR words, then offsets (n_kept + 1) and words */
int mc_bam_n_cigar_words(const mc_bam* bam, int64_t* n);
int mc_bam_cigars(const mc_bam* bam, int64_t* cig_off, uint32_t* cigar);

/* ---- streaming decode -----------------------------------------------------
 * Bounded-memory variant of mc_bam_open for BAMs larger than host memory:
 * BGZF blocks are inflated a window (window_bytes inflated, 0 = 256 MiB) at
 * a time on n_threads threads and the kept records' intervals come out in
 * order, up to `cap` per mc_bam_stream_next call (*n_out = 0 at the end).
 * mc_bam_stream_header exposes the header and the running record counts
 * through the mc_bam accessors (mc_bam_n_targets, mc_bam_target,
 * mc_bam_counts); the handle stays owned by the stream. */
typedef struct mc_bam_stream mc_bam_stream;
int mc_bam_stream_open(const char* path, int n_threads, uint32_t flag_filter,
                       int64_t window_bytes, mc_bam_stream** out);
int mc_bam_stream_next(mc_bam_stream* s, int64_t cap, int32_t* tid, int32_t* pos,
                       int32_t* span, int64_t* n_out);
int mc_bam_stream_header(const mc_bam_stream* s, const mc_bam** header);
int mc_bam_stream_close(mc_bam_stream* s);

/* ---- BAI index ------------------------------------------------------------
 * The reference opens an indexed BAM (`metacov pileup` needs `samtools
 * index`: pysam AlignmentFile.pileup(ref, start, end) at pileup.py:13 is an
 * indexed query; AlignmentFile.mapped / .unmapped at cli.py:58-66 read the
 * index pseudo-bins).  mc_bam_index_build writes <bam>.bai (bai_path NULL)
 * the way htslib's hts_idx_push / hts_idx_finish do.  mc_bam_open_contigs
 * decodes only the records of the chosen contigs (one rank's shard) through
 * the index: same intervals as mc_bam_open restricted to those tids (global
 * tid values), whole-file mapped / unmapped counts from the index.
 * mc_bam_index_stats: per-reference mapped / unmapped counts and the records
 * without coordinates (sharding costs without a decode). */
int mc_bam_index_build(const char* bam_path, const char* bai_path, int n_threads);
int mc_bam_index_stats(const char* bai_path, int32_t n_ref, int64_t* n_mapped,
                       int64_t* n_unmapped, int64_t* n_no_coor);
int mc_bam_open_contigs(const char* path, const char* bai_path, int n_threads,
                        uint32_t flag_filter, int keep_cigar, int32_t n_sel,
                        const int32_t* sel, mc_bam** out);
/* Where each contig's records lie in a coordinate-sorted BAM: what a BAI's
 * per-reference pseudo-bin holds (htslib hts_idx_finish, bin 37450).
 * beg_voff / end_voff are the virtual offsets (bgzf_tell: compressed block
 * offset << 16 | offset inside the inflated block) of the contig's first
 * record and of the end of its last one; equal when it has no records.
 * n_kept: records kept under a decode's flag filter (mc_bam_gpu_extents;
 * 0 when read from an index). */
typedef struct mc_contig_extent {
    int64_t beg_voff;
    int64_t end_voff;
    int64_t n_mapped;     /* records of this tid without flag 0x4 */
    int64_t n_unmapped;   /* records of this tid with flag 0x4 */
    int64_t n_kept;
} mc_contig_extent;
/* The extents table of an index (the role of pysam's indexed
 * AlignmentFile.fetch(ref) at metacov/pileup.py:13 / :90: which bytes hold a
 * contig's reads); *n_no_coor: records without coordinates. */
int mc_bam_index_extents(const char* bai_path, int32_t n_ref, mc_contig_extent* ext,
                         int64_t* n_no_coor);

/* ---- GPU BAM decode ------------------------------------------------------
 * The records mc_bam_open keeps (same intervals in file order, same record /
 * mapped / unmapped counts, same error classes), decoded on `device`: the
 * host reads the file (n_threads pread threads into pinned staging, 0 = 16)
 * and scans the BGZF block headers; one GPU lane inflates each BGZF block,
 * and the BAM records are found and parsed per 64 KiB segment of the
 * inflated stream (csrc/bam_gpu.hip).  window_bytes: inflated bytes per
 * window (0 = 4 GiB); a record cut by a window is carried to the next.
 * The kept intervals stay in device memory owned by the handle
 * (mc_bam_gpu_intervals_device: valid until mc_bam_gpu_close; hand them to
 * mc_add_reads_device); so do the decode's window buffers (about 2.5 x the
 * window size) until mc_bam_gpu_close.  Replaces, like mc_bam_open, the record walk under
 * pysam's pileup (IteratorRowAll, scan.pyx:204-216). */
typedef struct mc_bam_gpu mc_bam_gpu;
typedef struct mc_bam_gpu_timings {
    double read_ms;      /* host: file read + upload of the compressed windows */
    double inflate_ms;   /* gz_inflate_kernel (HIP events) */
    double parse_ms;     /* record sync / walk / fill, with their host checks */
    double total_ms;     /* the whole mc_bam_gpu_open */
    int64_t windows;
    int64_t blocks;
    int64_t resyncs;     /* segment starts corrected after a walk (sync false positives) */
    int64_t compressed_bytes;
    int64_t inflated_bytes;
    double scan_ms;      /* host: BGZF block header scan */
    double upload_ms;    /* host: every file read + upload, overlapped or not */
    double kernel_ms;    /* gz_inflate_kernel launches (HIP events), summed over launches */
    double open_ms;      /* the decode inside mc_bam_gpu_open, teardown of its file mapping included */
    int64_t parse_rounds;   /* most walk / check rounds of any parsed window (1: no false sync) */
    int64_t resync_passes;  /* re-syncs with the long chain after repeated false syncs */
} mc_bam_gpu_timings;
int mc_bam_gpu_open(const char* path, int device, int n_threads, uint32_t flag_filter,
                    int64_t window_bytes, mc_bam_gpu** out);
int mc_bam_gpu_header(const mc_bam_gpu* g, const mc_bam** header);
int mc_bam_gpu_intervals_device(const mc_bam_gpu* g, int64_t* n, const int32_t** d_tid,
                                const int32_t** d_pos, const int32_t** d_span);
int mc_bam_gpu_intervals(const mc_bam_gpu* g, int32_t* tid, int32_t* pos, int32_t* span);
int mc_bam_gpu_stats(const mc_bam_gpu* g, mc_bam_gpu_timings* t);
int mc_bam_gpu_close(mc_bam_gpu* g);
/* Releases the decode's staging buffers (compressed bytes, inflated stream,
 * block and segment tables) of an open handle; its results (intervals, read
 * table or scan columns, the per-contig extents) stay valid.  For handles
 * kept between calls (metacov_amd.pileup's path cache).  freed (optional):
 * device bytes released. */
int mc_bam_gpu_trim(mc_bam_gpu* g, int64_t* freed);
/* `metacov scan` input decoded on the GPU (the BAM half of scan.pyx:188-216,
 * IteratorRowAll: every record in file order; replaces mc_scan_src_open_bam's
 * host walk): the whole file as the SoA batch mc_scan_add_batch_device takes
 * (rlen = l_seq, flag, gpos = pos [+ l_seq on the reverse strand], gisize =
 * tlen when properly paired else 0, tid, packed nt16 bases at 4-byte aligned
 * offsets seq_off[0..n]), left in device memory owned by the handle. */
int mc_bam_gpu_open_scan(const char* path, int device, int n_threads, int64_t window_bytes, mc_bam_gpu** out);
int mc_bam_gpu_scan_device(const mc_bam_gpu* g, int64_t* n, const int32_t** d_rlen, const int32_t** d_flag,
                           const int32_t** d_gpos, const int32_t** d_gisize, const int32_t** d_tid,
                           const int64_t** d_seq_off, const uint8_t** d_seq, int64_t* seq_bytes);
/* pileup.experimental's read table decoded on the GPU (the device form of
 * mc_reads_open's walk, exp_reads.cpp; replaces bam.fetch at
 * metacov/pileup.py:101): every placed record (tid >= 0) in file order, with
 * tid, pos, end (pos + reference length; pos + 1 when unmapped or 0), flag,
 * bits (1 no SEQ, 2 no reference length), the 2-bit code of the first k_len
 * bases of query_alignment_sequence (0xFFFFFFFF: none) and the query name
 * (name_len bytes at name_off in the names arena), left in device memory owned
 * by the handle.  mc_bam_gpu_reads_copy copies them to caller buffers of
 * n entries (names: name_bytes). */
int mc_bam_gpu_open_reads(const char* path, int device, int n_threads, int k_len, int64_t window_bytes,
                          mc_bam_gpu** out);
int mc_bam_gpu_reads_device(const mc_bam_gpu* g, int64_t* n, const int32_t** d_tid, const int32_t** d_pos,
                            const int64_t** d_end, const int32_t** d_flag, const uint8_t** d_bits,
                            const uint32_t** d_kmer, const uint8_t** d_name_len, const int64_t** d_name_off,
                            const uint8_t** d_names, int64_t* name_bytes);
int mc_bam_gpu_reads_copy(const mc_bam_gpu* g, int32_t* tid, int32_t* pos, int64_t* end, int32_t* flag,
                          uint8_t* bits, uint32_t* kmer, uint8_t* name_len, int64_t* name_off, uint8_t* names);
/* The same for one rank's contigs (mc_bam_gpu_open_extents' blocks and
 * extents table: only the selected contigs' BGZF blocks are read and
 * inflated); tids stay the header's.  The header counts are the table's. */
int mc_bam_gpu_open_reads_extents(const char* path, int device, int n_threads, int k_len, int32_t n_ref,
                                  const mc_contig_extent* ext, int64_t n_no_coor, int32_t n_sel, const int32_t* sel,
                                  mc_bam_gpu** out);
/* One rank's contig shard decoded on the GPU ("each rank
 * decodes only its contigs' BGZF chunks, located via BAI virtual offsets";
 * replaces the per-contig indexed query under pysam's pileup(ref, start,
 * end), metacov/pileup.py:13).  Only the BGZF blocks holding the selected
 * contigs' records are read, uploaded and inflated; the kept records are
 * those mc_bam_open keeps of those contigs, in file order.  Their device
 * tids are LOCAL ids (the rank of the header tid in the sorted, de-duplicated
 * selection: the contig ids of a ctx holding just those contigs), in
 * mc_bam_gpu_intervals_device as in mc_bam_gpu_intervals[_range].  The
 * header counts are the whole file's, from the extents (as an index reports
 * them).  mc_bam_gpu_open_contigs reads the extents from the BAI (bai_path
 * NULL: <path>.bai); mc_bam_gpu_open_extents takes them from the caller
 * (e.g. mc_bam_gpu_extents of a whole-file decode on another rank, for a BAM
 * without an index). */
int mc_bam_gpu_open_contigs(const char* path, const char* bai_path, int device, int n_threads,
                            uint32_t flag_filter, int32_t n_sel, const int32_t* sel,
                            mc_bam_gpu** out);
int mc_bam_gpu_open_extents(const char* path, int device, int n_threads, uint32_t flag_filter,
                            int32_t n_ref, const mc_contig_extent* ext, int64_t n_no_coor,
                            int32_t n_sel, const int32_t* sel, mc_bam_gpu** out);
/* The extents table of a decoded file, computed on the device during the
 * record walk (per contig: first record, end of the last record, mapped /
 * unmapped / kept counts).  For a whole-file handle it is the BAI's
 * pseudo-bin data; MC_E_INVALID if the records of a contig are not
 * contiguous (the file is not coordinate-sorted).  A contig-subset handle
 * returns the table it was opened with, with n_kept filled in for its
 * contigs. */
int mc_bam_gpu_extents(const mc_bam_gpu* g, int32_t n_ref, mc_contig_extent* ext,
                       int64_t* n_no_coor);
/* A whole-file handle turned into a contig-subset one in place: only the
 * kept intervals of the selected contigs remain, in file order, with local
 * tids (as mc_bam_gpu_open_contigs gives them); the header counts stay the
 * whole file's.  (Rank 0 of a multi-GPU run without an index decodes the
 * whole file for the extents table and keeps its own shard this way.)
 * MC_E_INVALID if the file is not coordinate-sorted. */
int mc_bam_gpu_restrict(mc_bam_gpu* g, int32_t n_sel, const int32_t* sel);
/* Kept intervals [first, first + count) of the handle, copied to the host
 * (the records of chosen contigs: offsets from the extents' n_kept). */
int mc_bam_gpu_intervals_range(const mc_bam_gpu* g, int64_t first, int64_t count, int32_t* tid,
                               int32_t* pos, int32_t* span);
/* Test hooks (no GPU): the lane decoder of the inflate kernel and the record
 * parse of the walk kernels, run on the host.  mc_gz_inflate_host: one raw
 * deflate stream into exactly isize bytes (MC_E_IO otherwise).
 * mc_bam_rec_parse_host: record body r[0, len) after block_size -> 0
 * dropped, 1 kept (out3 = tid, pos, span), 2 tid beyond n_ref, 3 CIGAR
 * overruns, 4 span exceeds int32. */
int mc_gz_inflate_host(const uint8_t* src, int64_t clen, uint8_t* dst, int64_t isize);
int mc_bam_rec_parse_host(const uint8_t* r, int64_t len, int32_t n_ref, uint32_t flag_filter,
                          int32_t* out3);
/* mc_bam_rec_chain_host: 1 if offset q of the inflated stream d[0, n) starts
 * `chain` structurally valid records in sort order (mapped records' bin
 * fields equal to reg2bin of their span), or a shorter such chain ending
 * exactly at n — the GPU record sync's rule; else 0. */
int mc_bam_rec_chain_host(const uint8_t* d, int64_t n, int64_t q, int32_t n_ref, int chain);
/* mc_bgzf_scan_host: the GPU decode's BGZF block scan (pread, n_threads
 * ranges) -> block count, inflated total, the first cap block offsets. */
int mc_bgzf_scan_host(const char* path, int n_threads, int64_t* n_blocks, int64_t* inflated,
                      int64_t* offsets, int64_t cap);

/* ---- synthetic BAM writer ------------------------------------------------
 * Writes coordinate-sorted records from SoA arrays as BGZF-compressed BAM
 * (blocks deflated on n_threads threads; level = zlib level).  The role of
 * the reference's `metacov simulate` (cli.py:288-414) for the benchmarks and
 * end-to-end tests, without ART.  Bases 'A', qualities 30, names "r<i>". */
int mc_bam_write(const char* path, int32_t n_ref, const char* const* names,
                 const int64_t* lengths, int64_t n, const int32_t* tid,
                 const int32_t* pos, const uint16_t* flag, const int64_t* cig_off,
                 const uint32_t* cigar, int32_t l_seq, int level, int n_threads);

/* ---- pileup.experimental (metacov/pileup.py:38-173, SURVEY.md §8 f) --------
 * The reference's experimental estimator, called by `metacov pileup -k`
 * (cli.py:81, :93-95) after classic() for every region.
 *
 * Read side (host C++): mc_reads_open decodes every placed record of a
 * coordinate-sorted BAM into the fields experimental() reads from pysam
 * (flags, query_name, reference_start, reference_length, the first K bases
 * of query_alignment_sequence as a 2-bit A/C/G/T code).  It replaces
 * bam.fetch(ref, start, end) at pileup.py:101.  mc_experimental_reads runs
 * the per-read loop (pileup.py:101-151) for R regions on n_threads threads:
 *   counts[8*q + 0..7] = status (0 ok, 1 read without SEQ, 2 read without
 *       reference_length, 3 k_cor None with a mate pair -- the reference
 *       raises TypeError for 1-3), secondary, improper, nreads,
 *       sum(cov), #distinct starts, sum(cov2), #"RCOR is ZERO" events
 *   sums[4*q + 0..3] = sum(cov_cor) (summation order differs from the
 *       reference), builtin sum(cor) and np.add.reduce(cor) (both exact),
 *       wnf (exact, pairing order)
 * K-mer tables: val/has [4^K] per read number (k_cor[0], k_cor[1]); pass
 * NULL tables for k_cor = None.  Events of region q (readno << 32 | code):
 * mc_experimental_events. */
typedef struct mc_reads mc_reads;
int mc_reads_open(const char* path, int n_threads, int k_len, mc_reads** out);
/* The same table with the BAM decoded on GPU `device` (mc_bam_gpu_open_reads)
 * and copied to the host; the same checks and errors. */
int mc_reads_open_gpu(const char* path, int device, int n_threads, int k_len, mc_reads** out);
/* One rank's read table: the placed records of contigs sel[0..n_sel) only,
 * decoded from their BGZF blocks (extents: a BAI's, mc_bam_index_extents, or
 * a whole-file decode's, mc_bam_gpu_extents). */
int mc_reads_open_gpu_extents(const char* path, int device, int n_threads, int k_len, int32_t n_ref,
                              const mc_contig_extent* ext, int64_t n_no_coor, int32_t n_sel, const int32_t* sel,
                              mc_reads** out);
int mc_reads_close(mc_reads* r);
int mc_reads_header(const mc_reads* r, int32_t* n_ref, int64_t* n_records, int64_t* n_placed);
int mc_reads_target(const mc_reads* r, int32_t i, const char** name, int64_t* length);
/* The table itself (views into the handle, n_placed entries; first: n_ref + 1
 * per-contig record offsets, max_span: n_ref) -- for tests and bindings that
 * read the placed records directly. */
int mc_reads_fields(const mc_reads* r, const int32_t** pos, const int64_t** end, const uint16_t** flag,
                    const uint8_t** bits, const uint32_t** kmer, const uint64_t** name_off,
                    const uint8_t** name_len, const char** names, int64_t* name_bytes,
                    const int64_t** first, const int64_t** max_span);
int mc_experimental_reads(mc_reads* r, int k_len, const double* val1, const uint8_t* has1,
                          const double* val2, const uint8_t* has2, int64_t R,
                          const int32_t* tid, const int64_t* start, const int64_t* end,
                          int n_threads, int64_t* counts, double* sums);
int mc_experimental_events(const mc_reads* r, int64_t region, int64_t cap, uint64_t* events,
                           int64_t* n);

/* Sequence side (GPU, fp64): the k-mer correction correlation of
 * pileup.py:63-88 -- fwd / rev k-mer weights over the region's bases, the
 * 900-tap normal-pdf correlation of rev and inner(fwd, revsum) -- plus the
 * G+C / A+T counts of pileup.py:64-66.  seq = all contigs' bases back to
 * back (as in the FASTA, any case); a region is (base offset of its first
 * base, bases available n <= length, length = end - start).  fwd / rev:
 * dense [4^K] tables, 0 for missing keys; taps = norm[0 .. n_taps).
 * inner[q] is ecor * length.  kernel_ms: HIP-event time of the kernel. */
typedef struct mc_ecor mc_ecor;
int mc_ecor_create(int device, mc_ecor** out);
int mc_ecor_destroy(mc_ecor* e);
int mc_ecor_set_sequence(mc_ecor* e, int64_t n_bytes, const uint8_t* seq);
int mc_ecor_set_tables(mc_ecor* e, int k_len, const double* fwd, const double* rev,
                       int n_taps, const double* taps);
int mc_ecor_run(mc_ecor* e, int64_t R, const int64_t* base, const int64_t* n_avail,
                const int64_t* length, double* inner, int64_t* gc, int64_t* at,
                float* kernel_ms);

/* ---- metacov scan: read histograms (SURVEY.md §8 f ranks 3-4) --------------
 * Replaces scan.scan_reads + the ReadProcessor plugins (metacov/scan.pyx:
 * 345-376 ReadProcessor / ReadProcessorList, 380-419 ByFlag, 422-476
 * BaseHist, 479-511 KmerHist, 514-552 MirrorHist, 555-588 IsizeHist,
 * 623-672 scan_reads) and the read iterators they are fed by
 * (AlignmentFileIterator scan.pyx:188-294, FastQFileIterator :297-340 over
 * pyfq.FastQFile / FastQFilePair, pyfq.pyx:60-270).
 *
 * Sources (host C++): every record of a BAM (file order, placed and unplaced)
 * or of one FASTQ / a FASTQ pair (plain or gzip), handed out in SoA batches
 * of the ReadIterator accessors: rlen = get_len, flag = get_flags, gpos =
 * get_pos, gisize = get_isize, tid = get_tid (int32 each), packed nt16 bases
 * (2 per byte, high nibble first; seq_off[n + 1] byte offsets).  Batch
 * arrays are borrowed until the next mc_scan_src_next. */
typedef struct mc_scan_src mc_scan_src;
int mc_scan_src_open_bam(const char* path, int n_threads, mc_scan_src** out);
int mc_scan_src_open_fastq(const char* path1, const char* path2, mc_scan_src** out);
/* SAM text (plain, gzip or BGZF), the records as htslib's sam_parse1 stores
 * them (pysam opens a .sam for `metacov scan x.sam`: cli.py:171-173,
 * scan.pyx:188-216): @SQ order for the tids, POS - 1, nt16 bases. */
int mc_scan_src_open_sam(const char* path, mc_scan_src** out);
int mc_scan_src_close(mc_scan_src* s);
int mc_scan_src_n_targets(const mc_scan_src* s, int32_t* n);
int mc_scan_src_target(const mc_scan_src* s, int32_t i, const char** name, int64_t* length);
int mc_scan_src_next(mc_scan_src* s, int64_t max_reads, int64_t max_seq_bytes, int64_t* n_out);
int mc_scan_src_batch(const mc_scan_src* s, const int32_t** rlen, const int32_t** flag,
                      const int32_t** gpos, const int32_t** gisize, const int32_t** tid,
                      const int64_t** seq_off, const uint8_t** seq, int64_t* seq_bytes);
int mc_scan_src_records(const mc_scan_src* s, int64_t* n_records);

/* Histograms (GPU).  The processor tree the CLI builds (cli.py:247-257):
 * ByFlag over any of BaseHist(base_start), KmerHist(k, nk, step, offset),
 * MirrorHist(offset, n), IsizeHist, grouped by the flag masks in order
 * (2^n_flags groups, the first flag the most significant group bit).
 * mc_scan_set_reference: FASTA sequences (ASCII) for BaseHist / MirrorHist;
 * a batch's ref_id selects one per read (-1: none; reads as N).
 * mc_scan_run drives a source through the kernel (max_reads 0 = all), with
 * tid_to_ref mapping source tids to reference sequences.  Results come back
 * group-major in the reference's layouts: base [G][rows][5] with rows =
 * max(50, longest read) + base_start, kmer [G][4^K+1][NK], mirror
 * [G][N+1][2], isize [G][isize_cap] and isize_max [G]. */
typedef struct mc_scan_config {
    int32_t n_flags;
    uint32_t flags[16];
    int32_t base_on, base_start;
    int32_t kmer_on, kmer_k, kmer_nk, kmer_step, kmer_offset;
    int32_t mirror_on, mirror_offset, mirror_n;
    int32_t isize_on;
} mc_scan_config;
typedef struct mc_scan mc_scan;
int mc_scan_create(int device, const mc_scan_config* cfg, mc_scan** out);
int mc_scan_destroy(mc_scan* s);
int mc_scan_set_reference(mc_scan* s, int32_t n_seq, const int64_t* off, const int64_t* len,
                          int64_t n_bytes, const uint8_t* ascii);
int mc_scan_add_batch(mc_scan* s, int64_t n, const int32_t* rlen, const int32_t* flag,
                      const int32_t* gpos, const int32_t* gisize, const int32_t* ref_id,
                      const int64_t* seq_off, const uint8_t* seq);
int mc_scan_add_batch_device(mc_scan* s, int64_t n, const int32_t* rlen, const int32_t* flag,
                             const int32_t* gpos, const int32_t* gisize, const int32_t* ref_id,
                             const int64_t* seq_off, const uint8_t* seq, int32_t max_rlen,
                             int64_t max_abs_isize, float* kernel_ms);
int mc_scan_run(mc_scan* s, mc_scan_src* src, int32_t n_map, const int32_t* tid_to_ref,
                int64_t max_reads, int64_t batch_reads, int64_t* n_done);
/* mc_scan_run over a BAM decoded on the GPU (mc_bam_gpu_open_scan): the same
 * reads and reference-id rule, the whole file as one device batch. */
int mc_scan_run_gpu(mc_scan* s, const mc_bam_gpu* g, int32_t n_map, const int32_t* tid_to_ref,
                    int64_t max_reads, int64_t* n_done);
int mc_scan_dims(mc_scan* s, int32_t* groups, int64_t* base_rows, int64_t* isize_cap,
                 int32_t* max_rlen, int64_t* n_reads);
int mc_scan_results(mc_scan* s, uint32_t* base, uint32_t* kmer, uint32_t* mirror,
                    uint32_t* isize, int32_t* isize_max);
int mc_scan_timing(mc_scan* s, float* last_kernel_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* METACOV_AMD_H */
