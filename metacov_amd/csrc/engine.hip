// Host side of the coverage engine: the mc_ctx C ABI (include/metacov_amd.h).
//
// Device layout (one ctx = one GPU):
//   reads   int32 tid[], pos[], span[]   SoA, coordinate-sorted, padded
//   coff    int64 contig offset into the concatenated depth vector
//           (each contig gets max(length, furthest read end), rounded up to
//           64 positions)
//   depth   int32[n_chunks * chunk_w]    all contigs back to back
//   index   int64 chunk_first[n_chunks]  first read of each chunk (with halo)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/metacov_amd.h"
#include "common.h"
#include "kernels.h"
#include "npstd.h"
#include "capmask.h"

#include <hipcub/hipcub.hpp>

using namespace mc;

#ifndef MC_PLAIN_TILES_PER_CHUNK
#define MC_PLAIN_TILES_PER_CHUNK 4
#endif
constexpr int kPlainTilesPerChunk = MC_PLAIN_TILES_PER_CHUNK;   // plain K2, short reads

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

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;   // elements
    uint64_t gen = 0; // allocations so far (a cache key: a new block may reuse the old address)
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
        }
        hipError_t e = hipMalloc(&p, n * sizeof(T));
        if (e != hipSuccess) {
            cap = 0;
            p = nullptr;
            return e;
        }
        cap = n;
        ++gen;
        return hipSuccess;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        ++gen;
    }
};

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Host memory a kernel writes directly (coherent, mapped): the fused call's
// fallback flags land here without a device-to-host copy command.
template <typename T>
struct HostMapped {
    T* h = nullptr;
    T* d = nullptr;       // device address of h
    size_t cap = 0;
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        release();
        void* p = nullptr;
        hipError_t e = hipHostMalloc(&p, n * sizeof(T), hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return e;
        void* dp = nullptr;
        e = hipHostGetDevicePointer(&dp, p, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(p);
            return e;
        }
        h = static_cast<T*>(p);
        d = static_cast<T*>(dp);
        cap = n;
        return hipSuccess;
    }
    void release() {
        if (h) (void)hipHostFree(h);
        h = d = nullptr;
        cap = 0;
    }
};

// Per-call host arrays go up in ONE copy from a pinned buffer (a pageable
// hipMemcpyAsync per array costs a staging round trip each).  The caller
// synchronises the stream before the next reuse.
struct Stage {
    void* h = nullptr;
    size_t cap = 0;
    DevBuf<unsigned char> d;
    hipError_t reserve(size_t n) {
        if (n > cap) {
            if (h) (void)hipHostFree(h);
            h = nullptr;
            cap = 0;
            hipError_t e = hipHostMalloc(&h, n, hipHostMallocDefault);
            if (e != hipSuccess) return e;
            cap = n;
        }
        return d.reserve(n);
    }
    void release() {
        if (h) (void)hipHostFree(h);
        h = nullptr;
        cap = 0;
        d.release();
    }
    unsigned char* host() const { return static_cast<unsigned char*>(h); }
};

inline size_t stage_align(size_t x) { return (x + 255) & ~size_t(255); }

// Page-locked host memory (hipHostMalloc): copies from / to it are plain
// DMAs, not staged through a bounce buffer as pageable copies are.
struct Pinned {
    void* h = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        release();
        hipError_t e = hipHostMalloc(&h, n, hipHostMallocDefault);
        if (e == hipSuccess) cap = n;
        else h = nullptr;
        return e;
    }
    void release() {
        if (h) (void)hipHostFree(h);
        h = nullptr;
        cap = 0;
    }
};

}  // namespace

struct mc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;

    std::vector<int64_t> len, extent, coff;   // coff: n_contigs + 1
    DevBuf<int64_t> d_len, d_coff;
    std::vector<int64_t> coff_dev;            // what d_coff holds (allocation coff_dev_gen)
    uint64_t coff_dev_gen = ~0ull;

    int64_t n_reads = 0;
    DevBuf<int32_t> d_tid, d_pos, d_span;
    DevBuf<uint32_t> d_gpos;              // K2's packed read words (ingest_kernel)
    // raw-CIGAR mode
    bool spans_pending = false;
    DevBuf<int64_t> d_cig_off;
    DevBuf<uint32_t> d_cigar;
    const int64_t* cig_off_ext = nullptr;   // borrowed (mc_add_reads_cigar_device)
    const uint32_t* cigar_ext = nullptr;

    bool prepared = false;
    // direct per-batch prepare (probe_kernel; K2 validates): prepared this way,
    // K2's results not checked yet, allowed for this contig set, enabled
    bool direct = false;
    bool direct_checked = false;
    bool direct_ok = true;
    bool direct_enabled = true;
    int min_span = 0;              // K1: span of a read with no reference-consuming op (mc_set_legacy_endpos)
    bool direct_retry_full = false;       // the batch K2 just refused goes to mc_prepare
    unsigned long long direct_gen = 0;
    // halo of the next direct batch (0: short_max): the previous batch's
    // maximum span and 1/8 more, so a chunk loads the reads starting up to
    // that far before it instead of short_max (C3: 4096 -> ~2400 positions)
    int direct_halo = 0;
    int direct_halo_used = 0;
    DevBuf<int32_t> d_jidx;               // [3 * (n_base + 1)]: J(k w), J(k w - halo), J(k w - kNearHalo)
    DevBuf<int32_t> d_fsamp;              // [nc + 1] first sample of each contig
    DevBuf<unsigned long long> d_dres;    // [kDresWords] probe flags + K2's counters
    DevBuf<uint32_t> d_endw;              // ingest_kernel<true>'s end words (long_fill_words_kernel)
    // K2's constant arguments (K2Consts), a few variants resident at once:
    // each launch finds its bytes in a slot or uploads them into the next one
    static constexpr int kK2Slots = 4;
    DevBuf<K2Consts> d_k2c;
    DevBuf<unsigned long long> d_bases_part;   // span_sum_kernel's per-workgroup partials
    Pinned h_k2c;
    K2Consts k2c[kK2Slots];
    bool k2c_valid[kK2Slots] = {false, false, false, false};
    hipEvent_t k2c_ev[kK2Slots] = {};   // slot i's staging copy is done
    int k2c_next = 0;
    int32_t max_span = 0;
    bool long_hint = false;               // the last full prepare of this contig set had long reads
    bool prep_pending = false;            // the last full prepare's time is not read yet
    int64_t aligned_bases = 0;
    int ring = 0;                 // LDS ring ints
    int tiles_per_chunk = 16;
    int64_t chunk_w = 0, n_chunks = 0, total_len = 0;
    DevBuf<int64_t> d_chunk_first;        // [2 * base chunks] (ingest_kernel)
    // the plain K2's chunk geometry = the index's base chunks (half-size
    // chunks for short reads); a fused chunk is cstride base chunks
    int tpc_base = 0;
    int cstride = 1;
    int64_t n_chunks_base = 0;
    // long-read path (spans > short_max)
    bool has_long = false;
    int short_max = 0;
    DevBuf<unsigned> d_tile_cnt;
    DevBuf<int64_t> d_tile_off;
    DevBuf<int32_t> d_tile_ev;
    DevBuf<int> d_chunk_carry;
    DevBuf<long long> d_scan_part;        // long_scan partial sums
    int long_grid = 0;                    // resident long_count / long_fill workgroups
    int long_grid_words = 0;              // resident long_fill_words workgroups
    DevBuf<int32_t> d_depth;
    bool depth_valid = false;
    int32_t max_depth = -1;

    // ingest results: [0, 8) counters, [8, 8 + nc) furthest ends, [8 + nc,
    // 8 + 2 nc) aligned bases per contig; one memset, one copy back
    DevBuf<unsigned long long> d_scratch;
    Pinned pin_io;                        // contig offsets up, ingest results down
    std::vector<unsigned long long> cbases;   // aligned bases per contig
    DevBuf<unsigned> d_queue;
    DevBuf<int> d_maxdepth;
    // K3 scratch
    Stage k3_stage;                       // segments + per-region counts
    DevBuf<unsigned> d_hist;
    DevBuf<RegionAcc> d_acc;
    DevBuf<RegionOut> d_out;
    // fused K2 statistics
    DevBuf<int64_t> d_fchunk;
    Stage fstage;                         // per-call region arrays + returned flags
    // the last fused call's regions: a repeated call with the same regions on
    // the same prepared reads reuses the staged (sorted) arrays on the device
    uint64_t prep_gen = 0;
    struct {
        bool valid = false;
        uint64_t gen = 0;
        std::vector<int32_t> tid;
        std::vector<int64_t> start, end;
        int64_t nf = 0;
        bool chunk_first = false;   // d_fchunk holds this region set's chunk -> region index
        // the layout the staged arrays were built on (a re-prepare that keeps
        // it keeps them, the window bases aside)
        int vals = 0;
        int64_t chunk_w = 0, n_chunks = 0;
        std::vector<int64_t> extent, coff;
    } fcache;
    DevBuf<unsigned> d_flow;
    DevBuf<unsigned> d_fhist;
    HostMapped<int> h_fflag;              // fallback flags, written by region_final_kernel
    // device-side recompute of the fused call's out-of-window regions (fb_seg_kernel)
    DevBuf<unsigned> d_fb_hist;           // [kFbSlots][kLdsBins]
    DevBuf<RegionAcc> d_fb_acc;           // [kFbSlots]
    DevBuf<int32_t> d_fb_list;            // [kFbSlots]
    DevBuf<unsigned> d_fb_cnt;            // [2] (by call parity)
    DevBuf<unsigned> d_kdone;             // [1] K3b's finished-workgroup count (0 between calls)
    int64_t fb_calls = 0;
    bool fb_recent = false;               // the last fused call had out-of-window regions
    int64_t device_recomputes = 0;
    bool fused_clean = false;             // K3b left hist / low / acc / queue initialised
    int64_t fused_clean_R = 0;
    bool check_clean = false;             // MC_CHECK_CLEAN=1: verify a skipped fused_init on the device
    DevBuf<unsigned long long> d_check;   // [1] its mismatch count
    int64_t fused_fallbacks = 0;

    hipEvent_t ev[8] = {};
    // The fused call's events, one set per call in a ring (prep start, K2
    // start, K2 end, K3b end): a call's elapsed times are read once the next
    // call has issued its launches, while the GPU runs them, not between the
    // two (3 x ~2.5 us there).  At most the previous call's set is pending.
    struct TimingSet {
        hipEvent_t e[4] = {};
        bool prep = false;      // e[0] was recorded (a direct prepare)
        bool pending = false;   // not yet added to t
    };
    static constexpr int kTimingSets = 4;
    TimingSet ts[kTimingSets];
    int ts_cur = 0;
    // completion stamp: a fused call's K3b writes done_seq into mapped host
    // memory when its last workgroup is done, and the host spins on it (a
    // stream synchronize woke ~10 us after the last kernel's end; a stream
    // write command after K3b cost ~13 us more)
    HostMapped<unsigned long long> h_done;
    unsigned long long done_seq = 0;
    bool stamp_ok = true;
    int ingest_grid[2] = {0, 0};          // resident ingest workgroups (without / with long counting)
    int k2_resident[6] = {};              // resident K2 workgroups (plain, fused) x (short, long, direct)
    size_t k2_resident_lds[6] = {};
    mc_timings t{};
    bool t_cigar = false, t_prep = false, t_depth = false, t_stats = false;
};

static int ctx_use(mc_ctx* ctx) {
    MC_REQUIRE(ctx, MC_E_INVALID, "null ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    return MC_OK;
}

static void invalidate(mc_ctx* ctx) {
    ctx->prepared = false;
    ctx->direct = false;
    ctx->direct_checked = false;
    ctx->depth_valid = false;
    ctx->max_depth = -1;
}

extern "C" int mc_ctx_create(int device, mc_ctx** out) {
    MC_REQUIRE(out, MC_E_INVALID, "null out");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    MC_REQUIRE(e == hipSuccess && n > 0, MC_E_HIP,
               "no HIP device available (hipGetDeviceCount: %s); metacov_amd has no CPU path",
               hipGetErrorString(e));
    MC_REQUIRE(device >= 0 && device < n, MC_E_INVALID, "device %d out of range [0, %d)", device, n);
    HIP_TRY(hipSetDevice(device));
    mc_ctx* c = new mc_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        mc::set_error("hipStreamCreate failed");
        return MC_E_HIP;
    }
    c->own_stream = true;
    if (const char* v = getenv("MC_CHECK_CLEAN")) c->check_clean = v[0] && v[0] != '0';
    for (auto& ev : c->ev) (void)hipEventCreate(&ev);
    for (auto& T : c->ts)
        for (auto& ev : T.e) (void)hipEventCreate(&ev);
    if (c->d_scratch.reserve(8) != hipSuccess || c->d_queue.reserve(8) != hipSuccess ||
        c->d_maxdepth.reserve(4) != hipSuccess) {
        mc_ctx_destroy(c);
        mc::set_error("hipMalloc of ctx scratch failed");
        return MC_E_HIP;
    }
    *out = c;
    return MC_OK;
}

extern "C" int mc_ctx_destroy(mc_ctx* ctx) {
    if (!ctx) return MC_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    ctx->d_len.release();
    ctx->d_coff.release();
    ctx->d_tid.release();
    ctx->d_pos.release();
    ctx->d_span.release();
    ctx->d_gpos.release();
    ctx->d_cig_off.release();
    ctx->d_cigar.release();
    ctx->d_chunk_first.release();
    ctx->d_jidx.release();
    ctx->d_fsamp.release();
    ctx->d_dres.release();
    ctx->d_endw.release();
    ctx->d_k2c.release();
    ctx->d_bases_part.release();
    ctx->h_k2c.release();
    for (hipEvent_t& e : ctx->k2c_ev)
        if (e) {
            (void)hipEventDestroy(e);
            e = nullptr;
        }
    ctx->d_tile_cnt.release();
    ctx->d_tile_off.release();
    ctx->d_tile_ev.release();
    ctx->d_chunk_carry.release();
    ctx->d_scan_part.release();
    ctx->d_depth.release();
    ctx->d_scratch.release();
    ctx->pin_io.release();
    ctx->d_queue.release();
    ctx->d_maxdepth.release();
    ctx->k3_stage.release();
    ctx->d_hist.release();
    ctx->d_acc.release();
    ctx->d_out.release();
    ctx->d_fchunk.release();
    ctx->h_fflag.release();
    ctx->fstage.release();
    ctx->fcache.valid = false;
    ctx->fcache.chunk_first = false;
    ctx->d_flow.release();
    ctx->d_fhist.release();
    ctx->d_fb_hist.release();
    ctx->d_fb_acc.release();
    ctx->d_fb_list.release();
    ctx->d_fb_cnt.release();
    ctx->d_kdone.release();
    for (auto ev : ctx->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& T : ctx->ts)
        for (auto ev : T.e)
            if (ev) (void)hipEventDestroy(ev);
    ctx->h_done.release();
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return MC_OK;
}

extern "C" int mc_ctx_set_stream(mc_ctx* ctx, void* s) {
    if (int rc = ctx_use(ctx)) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    if (s) {
        ctx->stream = (hipStream_t)s;
        ctx->own_stream = false;
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        ctx->own_stream = true;
    }
    return MC_OK;
}

extern "C" int mc_ctx_device(const mc_ctx* ctx, int* device) {
    MC_REQUIRE(ctx && device, MC_E_INVALID, "null argument");
    *device = ctx->device;
    return MC_OK;
}

extern "C" int mc_set_contigs(mc_ctx* ctx, int32_t n, const int64_t* lengths) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(n >= 0 && (n == 0 || lengths), MC_E_INVALID, "bad contig table");
    for (int32_t i = 0; i < n; ++i)
        MC_REQUIRE(lengths[i] >= 0 && lengths[i] < (int64_t(1) << 40), MC_E_INVALID,
                   "contig %d: bad length %lld", i, (long long)lengths[i]);
    ctx->len.assign(lengths, lengths + n);
    ctx->direct_ok = true;
    ctx->long_hint = false;
    ctx->n_reads = 0;
    ctx->spans_pending = false;
    ctx->cig_off_ext = nullptr;
    ctx->cigar_ext = nullptr;
    invalidate(ctx);
    HIP_TRY(ctx->d_len.reserve(std::max<int64_t>(n, 1)));
    if (n) HIP_TRY(hipMemcpy(ctx->d_len.p, lengths, n * sizeof(int64_t), hipMemcpyHostToDevice));
    return MC_OK;
}

// grow the read arrays to hold `n_total` reads (+ one batch of padding)
static int reserve_reads(mc_ctx* ctx, int64_t n_total, bool cigar_mode) {
    const size_t cap = (size_t)round_up(n_total + kPadBatch, kPadBatch);
    if (cap > ctx->d_tid.cap) {
        size_t ncap = std::max(cap, ctx->d_tid.cap * 3 / 2);
        ncap = (size_t)round_up((int64_t)ncap, kPadBatch);
        DevBuf<int32_t> t2, p2, s2;
        HIP_TRY(t2.reserve(ncap));
        HIP_TRY(p2.reserve(ncap));
        HIP_TRY(s2.reserve(ncap));
        if (ctx->n_reads) {
            HIP_TRY(hipMemcpyAsync(t2.p, ctx->d_tid.p, ctx->n_reads * 4, hipMemcpyDeviceToDevice, ctx->stream));
            HIP_TRY(hipMemcpyAsync(p2.p, ctx->d_pos.p, ctx->n_reads * 4, hipMemcpyDeviceToDevice, ctx->stream));
            HIP_TRY(hipMemcpyAsync(s2.p, ctx->d_span.p, ctx->n_reads * 4, hipMemcpyDeviceToDevice, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
        }
        ctx->d_tid.release();
        ctx->d_pos.release();
        ctx->d_span.release();
        ctx->d_tid = t2;
        ctx->d_pos = p2;
        ctx->d_span = s2;
    }
    (void)cigar_mode;
    return MC_OK;
}

static int add_reads_impl(mc_ctx* ctx, int64_t n, const int32_t* tid, const int32_t* pos,
                          const int32_t* span, hipMemcpyKind kind, bool wait = true) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(n >= 0, MC_E_INVALID, "negative read count");
    MC_REQUIRE(n == 0 || (tid && pos && span), MC_E_INVALID, "null read array");
    MC_REQUIRE(!ctx->spans_pending, MC_E_STATE,
               "cannot mix mc_add_reads with pending mc_add_reads_cigar reads; call mc_prepare first");
    if (int rc = reserve_reads(ctx, ctx->n_reads + n, false)) return rc;
    const int64_t o = ctx->n_reads;
    if (n) {
        HIP_TRY(hipMemcpyAsync(ctx->d_tid.p + o, tid, n * 4, kind, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->d_pos.p + o, pos, n * 4, kind, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->d_span.p + o, span, n * 4, kind, ctx->stream));
        if (wait) HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    ctx->n_reads += n;
    ctx->t_cigar = false;
    invalidate(ctx);
    return MC_OK;
}

extern "C" int mc_add_reads(mc_ctx* ctx, int64_t n, const int32_t* tid, const int32_t* pos,
                            const int32_t* span) {
    return add_reads_impl(ctx, n, tid, pos, span, hipMemcpyHostToDevice);
}

// Page-locked host memory for async ingest batches (hipHostMalloc).
extern "C" int mc_pinned_alloc(int64_t bytes, void** out) {
    MC_REQUIRE(out && bytes > 0, MC_E_INVALID, "bad argument");
    *out = nullptr;
    HIP_TRY(hipHostMalloc(out, (size_t)bytes, hipHostMallocDefault));
    return MC_OK;
}

extern "C" int mc_pinned_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return MC_OK;
}

// Host batch copied asynchronously on the ctx stream (pinned buffers: DMA
// overlapped with the caller's next decode); the buffers must stay unchanged
// until mc_synchronize.
extern "C" int mc_add_reads_async(mc_ctx* ctx, int64_t n, const int32_t* tid, const int32_t* pos,
                                  const int32_t* span) {
    return add_reads_impl(ctx, n, tid, pos, span, hipMemcpyHostToDevice, false);
}

extern "C" int mc_add_reads_device(mc_ctx* ctx, int64_t n, const int32_t* tid, const int32_t* pos,
                                   const int32_t* span) {
    return add_reads_impl(ctx, n, tid, pos, span, hipMemcpyDeviceToDevice);
}

extern "C" int mc_add_reads_cigar(mc_ctx* ctx, int64_t n, const int32_t* tid, const int32_t* pos,
                                  const int64_t* cig_off, const uint32_t* cigar) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(n >= 0, MC_E_INVALID, "negative read count");
    MC_REQUIRE(n == 0 || (tid && pos && cig_off), MC_E_INVALID, "null read array");
    MC_REQUIRE(ctx->n_reads == 0, MC_E_STATE,
               "mc_add_reads_cigar must be the only read source of a ctx (call mc_set_contigs to reset)");
    MC_REQUIRE(n == 0 || cig_off[0] == 0, MC_E_INVALID, "cig_off[0] must be 0");
    const int64_t nw = n ? cig_off[n] : 0;
    for (int64_t i = 0; i < n; ++i)
        MC_REQUIRE(cig_off[i + 1] >= cig_off[i], MC_E_INVALID, "cig_off not monotone at %lld",
                   (long long)i);
    MC_REQUIRE(nw == 0 || cigar, MC_E_INVALID, "null cigar array");
    if (int rc = reserve_reads(ctx, n, true)) return rc;
    HIP_TRY(ctx->d_cig_off.reserve(n + 1));
    HIP_TRY(ctx->d_cigar.reserve(std::max<int64_t>(nw, 1)));
    if (n) {
        HIP_TRY(hipMemcpyAsync(ctx->d_tid.p, tid, n * 4, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->d_pos.p, pos, n * 4, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->d_cig_off.p, cig_off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        if (nw) HIP_TRY(hipMemcpyAsync(ctx->d_cigar.p, cigar, nw * 4, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    ctx->n_reads = n;
    ctx->spans_pending = n > 0;
    ctx->cig_off_ext = nullptr;
    ctx->cigar_ext = nullptr;
    ctx->t_cigar = false;
    invalidate(ctx);
    return MC_OK;
}

extern "C" int mc_add_reads_cigar_device(mc_ctx* ctx, int64_t n, const int32_t* tid,
                                         const int32_t* pos, const int64_t* cig_off,
                                         const uint32_t* cigar) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(n >= 0, MC_E_INVALID, "negative read count");
    MC_REQUIRE(n == 0 || (tid && pos && cig_off && cigar), MC_E_INVALID, "null read array");
    MC_REQUIRE(ctx->n_reads == 0, MC_E_STATE,
               "mc_add_reads_cigar_device must be the only read source of a ctx "
               "(call mc_clear_reads to start a new batch)");
    if (int rc = reserve_reads(ctx, n, true)) return rc;
    if (n) {
        HIP_TRY(hipMemcpyAsync(ctx->d_tid.p, tid, n * 4, hipMemcpyDeviceToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->d_pos.p, pos, n * 4, hipMemcpyDeviceToDevice, ctx->stream));
        // tid/pos are the caller's (often temporaries of a dtype cast): they may be freed
        // or reused on another stream as soon as this returns, so the copies finish here.
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    ctx->cig_off_ext = cig_off;
    ctx->cigar_ext = cigar;
    ctx->n_reads = n;
    ctx->spans_pending = n > 0;
    ctx->t_cigar = false;
    invalidate(ctx);
    return MC_OK;
}

extern "C" int mc_invalidate(mc_ctx* ctx) {
    if (int rc = ctx_use(ctx)) return rc;
    invalidate(ctx);
    return MC_OK;
}

extern "C" int mc_clear_reads(mc_ctx* ctx) {
    if (int rc = ctx_use(ctx)) return rc;
    ctx->t_cigar = false;
    ctx->n_reads = 0;
    ctx->spans_pending = false;
    ctx->cig_off_ext = nullptr;
    ctx->cigar_ext = nullptr;
    ctx->fused_fallbacks = 0;
    invalidate(ctx);
    return MC_OK;
}

// MC_STEP_EVENTS 0: a fused call records no timing events (A/B of their
// cost only: its kernel times then read 0)
#ifndef MC_STEP_EVENTS
#define MC_STEP_EVENTS 1
#endif
// MC_EXT_EVENTS 1: a fused call's timing events ride on its launches
// (hipExtLaunchKernel's start / stop events) instead of four hipEventRecord
// calls (the one before the probe sits between a call's entry and its first
// launch).  Back-to-back calls ran slower that way: C2 0.0821 -> 0.0870 ms,
// C3 1.0549 -> 1.0588, one N = 8 share 0.1827 -> 0.1858
// (profiles/r06/r06w_ab_*).
#ifndef MC_EXT_EVENTS
#define MC_EXT_EVENTS 0
#endif
static float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
        (void)hipGetLastError();   // (not a stream error: keep it out of the next launch check)
        return 0.f;
    }
    return ms;
}

static float elapsed(mc_ctx* ctx, int a, int b) { return elapsed(ctx->ev[a], ctx->ev[b]); }

// The last full prepare's time (ev[2] -> ev[3]), once its events are complete
// (mc_prepare does not wait for its own kernels).
static void resolve_prepare_timing(mc_ctx* ctx) {
    if (!ctx->prep_pending || hipEventQuery(ctx->ev[3]) != hipSuccess) return;
    ctx->t.prepare_ms = elapsed(ctx, 2, 3);
    ctx->t.prepare_ms_total += ctx->t.prepare_ms;
    ctx->prep_pending = false;
}

// Adds the pending fused calls' event times to t (oldest first; the current
// set only with `all`, after the stream has drained).
static void resolve_timings(mc_ctx* ctx, bool all) {
    for (int i = 1; i <= mc_ctx::kTimingSets; ++i) {
        const int k = (ctx->ts_cur + i) % mc_ctx::kTimingSets;
        auto& T = ctx->ts[k];
        if (!T.pending || (k == ctx->ts_cur && !all)) continue;
        const float a = elapsed(T.e[1], T.e[2]), b = elapsed(T.e[2], T.e[3]);
        ctx->t.fused_depth_ms_total += a;
        ctx->t.fused_stats_ms_total += b;
        ctx->t.depth_ms = a;
        ctx->t.stats_ms = b;
        if (T.prep) {
            ctx->t.prepare_ms = elapsed(T.e[0], T.e[1]);
            ctx->t.prepare_ms_total += ctx->t.prepare_ms;
        }
        T.prep = T.pending = false;
    }
}

// ---- layout for given extents: contig offsets and chunk geometry.  One
// chunk index serves both K2 variants: its base chunks are the plain K2's,
// half-size (kPlainTilesPerChunk tiles), where the plain kernel balances
// better (C3: 0.995 -> 0.936 ms); the fused one is faster on full chunks
// (its chunk-end flushes double) and reads its chunk c as base chunks
// [c*s, c*s + s).  Long reads' end buckets and carries are per full
// chunk, so with long reads the plain K2 runs on full chunks too.
// chunks are halved while a layout would have fewer than this many.  The
// strong-scaling shard (C3 / 8: 3.8 k chunks of 8 tiles for 1024 resident
// workgroups) ran K2 2.5 % faster on 4-tile chunks in round 3
// (profiles/r03ii_min_chunks_ab.txt); on the round-6 kernel it runs 3.7 %
// faster on 8-tile chunks (floor 2048: 0.147 -> 0.142 ms; 8192 / 16384, two-
// tile chunks: 0.210 ms; profiles/r06/r06n_*, r06o_*).  C2 and C3 take the
// same chunks either way.
#ifndef MC_MIN_CHUNKS
#define MC_MIN_CHUNKS 2048
#endif
static void set_layout(mc_ctx* ctx, const std::vector<int64_t>& ext) {
    const int32_t nc = (int32_t)ctx->len.size();
    ctx->extent = ext;
    ctx->coff.resize(nc + 1);
    int64_t off = 0;
    for (int32_t i = 0; i < nc; ++i) {
        ctx->coff[i] = off;
        off += round_up(ext[i], 64);
    }
    ctx->coff[nc] = off;
    ctx->total_len = off;
    // chunks of kTilesPerChunk tiles; fewer (>= the tiles of one ring, so
    // the ring divides the chunk) when the genome is too small to fill the GPU
    const int64_t tiles = std::max<int64_t>(1, (off + kTileW - 1) / kTileW);
    const int top = ctx->long_hint ? kTilesPerChunkLong : kTilesPerChunk;
    // (one-tile chunks for C2 ran K2 at 0.077 vs 0.066 ms: profiles/r04/r04m_*)
    const int min_tpc = (kRing % kTileW == 0) ? kRing / kTileW : top;
    int tpc = top;
    while (tpc / 2 >= min_tpc && tpc % 2 == 0 && tiles / tpc < MC_MIN_CHUNKS &&
           ((int64_t)(tpc / 2) * kTileW) % kRing == 0)
        tpc /= 2;
    ctx->tiles_per_chunk = tpc;
    ctx->chunk_w = (int64_t)tpc * kTileW;
    ctx->n_chunks = std::max<int64_t>(1, (off + ctx->chunk_w - 1) / ctx->chunk_w);
    int tpc_base = tpc;
    if (tpc > kPlainTilesPerChunk && tpc % kPlainTilesPerChunk == 0 &&
        ((int64_t)kPlainTilesPerChunk * kTileW) % kRing == 0)
        tpc_base = kPlainTilesPerChunk;
    ctx->tpc_base = tpc_base;
    ctx->cstride = tpc / tpc_base;
    const int64_t wb = (int64_t)tpc_base * kTileW;
    ctx->n_chunks_base = std::max<int64_t>(1, (off + wb - 1) / wb);
}

// log2 of the base chunk width (a power of two: kTileW and the tiles per
// chunk are)
static int base_lw(const mc_ctx* ctx) {
    int lw = 0;
    while (((int64_t)1 << lw) < (int64_t)ctx->tpc_base * kTileW) ++lw;
    return lw;
}
static_assert((kTileW & (kTileW - 1)) == 0 && (kTilesPerChunk & (kTilesPerChunk - 1)) == 0 &&
                  (kTilesPerChunkLong & (kTilesPerChunkLong - 1)) == 0 &&
                  (kPlainTilesPerChunk & (kPlainTilesPerChunk - 1)) == 0,
              "chunk widths must be powers of two (ingest and the probe shift by log2 of them)");

// The contig offsets on the device, uploaded only when they changed (a new
// batch over the same contigs keeps them).  coff_up: pinned staging.
static int upload_coff(mc_ctx* ctx, int64_t* coff_up) {
    const int32_t nc = (int32_t)ctx->len.size();
    HIP_TRY(ctx->d_coff.reserve(nc + 1));
    if (ctx->coff_dev != ctx->coff || ctx->coff_dev_gen != ctx->d_coff.gen) {
        HIP_TRY(hipStreamSynchronize(ctx->stream));   // the staging buffer's last copy has drained
        std::memcpy(coff_up, ctx->coff.data(), (nc + 1) * 8);
        HIP_TRY(hipMemcpyAsync(ctx->d_coff.p, coff_up, (nc + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        ctx->coff_dev = ctx->coff;
        ctx->coff_dev_gen = ctx->d_coff.gen;
    }
    return MC_OK;
}

// K1 on a raw-CIGAR batch whose spans are still pending (CIGAR words -> span)
static int run_k1(mc_ctx* ctx) {
    // (t_cigar stays set for the batch K1 ran on: a direct batch handed over
    // to mc_prepare keeps its K1 time)
    if (!ctx->spans_pending) return MC_OK;
    hipStream_t s = ctx->stream;
    const int64_t n = ctx->n_reads;
    HIP_TRY(hipEventRecord(ctx->ev[0], s));
    const int64_t nb = (n + kBlock - 1) / kBlock;
    const size_t lds = (kBlock + 1) * 8 + 8 + kBlock * 4 + kOwnerBuckets;
    const int64_t* co = ctx->cig_off_ext ? ctx->cig_off_ext : ctx->d_cig_off.p;
    const uint32_t* cw = ctx->cigar_ext ? ctx->cigar_ext : ctx->d_cigar.p;
    hipLaunchKernelGGL(cigar_span_kernel, dim3((unsigned)nb), dim3(kBlock), lds, s, co, cw, n, ctx->min_span, ctx->d_span.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ctx->ev[1], s));
    ctx->t_cigar = true;
    ctx->spans_pending = false;
    ctx->cig_off_ext = nullptr;   // borrowed until this prepare's stream sync
    ctx->cigar_ext = nullptr;
    return MC_OK;
}

extern "C" int mc_prepare(mc_ctx* ctx) {
    if (int rc = ctx_use(ctx)) return rc;
    if (ctx->prepared) return MC_OK;
    ctx->direct_retry_full = false;
    const int32_t nc = (int32_t)ctx->len.size();
    const int64_t n = ctx->n_reads;
    hipStream_t s = ctx->stream;
    resolve_prepare_timing(ctx);   // the previous prepare's events, before ev[2] / ev[3] are reused
    const bool k1_now = ctx->spans_pending;
    if (int rc = run_k1(ctx)) return rc;
    HIP_TRY(hipEventRecord(ctx->ev[2], s));
    // K2 loads whole int4 batches past n: the tid padding must index coff
    // (zeroed by prep_clear_kernel with the first ingest pass)
    const int64_t n_pad = ctx->d_tid.cap > (size_t)n ? (int64_t)(ctx->d_tid.cap - n) : 0;
    // LDS ring of 2 tiles: reads up to short_max = ring - kTileW keep both
    // events in LDS; longer ones take the bucketed long-read path.
    ctx->ring = kRing;
    ctx->short_max = ctx->ring - kTileW;
    const size_t n_res = 8 + 2 * (size_t)nc;   // ingest results (see d_scratch)
    HIP_TRY(ctx->d_scratch.reserve(n_res));
    HIP_TRY(ctx->pin_io.reserve((n_res + nc + 1) * 8));
    unsigned long long* res = static_cast<unsigned long long*>(ctx->pin_io.h);
    int64_t* coff_up = reinterpret_cast<int64_t*>(res + n_res);
    HIP_TRY(ctx->d_coff.reserve(nc + 1));
    // (the long-read counting is known before the pass loop; see count_long)
    // ---- layout for given extents: contig offsets and chunk geometry.  One
    // chunk index serves both K2 variants: its base chunks are the plain K2's,
    // half-size (kPlainTilesPerChunk tiles), where the plain kernel balances
    // better (C3: 0.995 -> 0.936 ms); the fused one is faster on full chunks
    // (its chunk-end flushes double) and reads its chunk c as base chunks
    // [c*s, c*s + s).  Long reads' end buckets and carries are per full
    // chunk, so with long reads the plain K2 runs on full chunks too.
    // ---- ingest + chunk index in one pass over the reads, on the layout the
    // contig lengths give; a read past its contig's end grows the extent, and
    // the pass runs again on the final layout
    std::vector<int64_t> ext(ctx->len);
    set_layout(ctx, ext);
    const unsigned long long* h = res;                         // counters
    const long long* maxend = reinterpret_cast<const long long*>(res + 8);
    // the previous batch of this contig set had long reads: ingest counts
    // their end events and chunk carries itself (long_count_kernel's pass,
    // 0.2 ms of a C5 prepare, and its two fills)
    const bool count_long = ctx->long_hint && n > 0;
    int& igrid = ctx->ingest_grid[count_long ? 1 : 0];
    if (n && igrid <= 0) {
        // one resident wave per range: a second round of waves would start
        // its ranges only when the first finished
        int dev = 0, ncu = 0, per = 0;
        HIP_TRY(hipGetDevice(&dev));
        HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per, count_long ? (const void*)ingest_kernel<true> : (const void*)ingest_kernel<false>, kBlock, 0));
        igrid = std::max(1, ncu * std::max(1, per));
    }
    // The long-read end-event buckets and chunk carries on the current layout
    // (count unless ingest counted -> offsets -> fill), all on the device; the
    // bucket array is sized for every read being long.  With ingest's counts
    // they are queued behind ingest before its results are read (speculative:
    // unused if the batch has no long reads, redone if the extents grow), so
    // the host's round trip overlaps them.
    // end words (ingest's per-read end events) when global ends fit 32 bits
    bool end_words = false;
    auto launch_long = [&](bool counted) -> int {
        const int64_t alloc_len = ctx->n_chunks * ctx->chunk_w;
        const int64_t n_tiles = ctx->n_chunks * ctx->tiles_per_chunk;
        HIP_TRY(ctx->d_tile_cnt.reserve(n_tiles + 1));
        HIP_TRY(ctx->d_chunk_carry.reserve(ctx->n_chunks + 1));
        HIP_TRY(ctx->d_tile_off.reserve(n_tiles + 1));
        HIP_TRY(ctx->d_tile_ev.reserve((size_t)(n + kPadBatch)));   // K2 loads whole int4 batches
        if (!counted) {
            HIP_TRY(hipMemsetAsync(ctx->d_tile_cnt.p, 0, (n_tiles + 1) * 4, s));
            HIP_TRY(hipMemsetAsync(ctx->d_chunk_carry.p, 0, (ctx->n_chunks + 1) * 4, s));
        }
        if (ctx->long_grid <= 0) {
            int dev = 0, ncu = 0, per = 0;
            HIP_TRY(hipGetDevice(&dev));
            HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)long_fill_kernel, kBlock, 0));
            ctx->long_grid = ncu * std::max(1, per);
            HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)long_fill_words_kernel, kBlock, 0));
            ctx->long_grid_words = ncu * std::max(1, per);
        }
        LongGeo G{ctx->d_tid.p, ctx->d_pos.p, ctx->d_span.p, n, ctx->d_coff.p, ctx->short_max, alloc_len, 0, 0};
        while (((int64_t)1 << G.lcw) < ctx->chunk_w) ++G.lcw;
        const int64_t subs = (n + kLongSub - 1) / kLongSub;
        const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(subs, ctx->long_grid));
        G.per = (subs + nb - 1) / nb * kLongSub;
        if (!counted) {
            hipLaunchKernelGGL(long_count_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, G,
                               ctx->d_tile_cnt.p, ctx->d_chunk_carry.p);
            HIP_TRY(hipGetLastError());
        }
        const int bt = (int)((n_tiles + kScanSeg - 1) / kScanSeg);
        const int bc = (int)((ctx->n_chunks + kScanSeg - 1) / kScanSeg);
        HIP_TRY(ctx->d_scan_part.reserve(bt + bc));
        ScanArgs A{ctx->d_tile_cnt.p, n_tiles, ctx->d_tile_off.p, ctx->d_chunk_carry.p, ctx->n_chunks,
                   ctx->d_scan_part.p, bt};
        hipLaunchKernelGGL(long_scan_partial_kernel, dim3(bt + bc), dim3(kBlock), 0, s, A);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(long_scan_final_kernel, dim3(bt + bc), dim3(kBlock), 0, s, A);
        HIP_TRY(hipGetLastError());
        if (counted && end_words) {
            // its own resident grid (the LDS event buffer of MC_FILL_SORTED
            // lowers its occupancy); counts and fill need not share sub-ranges
            const int64_t nbw = std::max<int64_t>(1, std::min<int64_t>(subs, ctx->long_grid_words));
            const int64_t perw = (subs + nbw - 1) / nbw * kLongSub;
            hipLaunchKernelGGL(long_fill_words_kernel, dim3((unsigned)nbw), dim3(kBlock), 0, s, ctx->d_endw.p, n,
                               perw, G.lcw, ctx->d_tile_off.p, ctx->d_tile_cnt.p, ctx->d_tile_ev.p);
        } else
            hipLaunchKernelGGL(long_fill_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, G,
                               ctx->d_tile_off.p, ctx->d_tile_cnt.p, ctx->d_tile_ev.p);
        HIP_TRY(hipGetLastError());
        return MC_OK;
    };
    int lcw = 0;
    for (int pass = 0;; ++pass) {
        const int64_t n_base = ctx->n_chunks * ctx->cstride;   // every full chunk's base chunks
        const int64_t n_tiles = ctx->n_chunks * ctx->tiles_per_chunk;
        lcw = 0;
        while (((int64_t)1 << lcw) < ctx->chunk_w) ++lcw;
        HIP_TRY(ctx->d_chunk_first.reserve(2 * n_base));
        if (count_long) {
            HIP_TRY(ctx->d_tile_cnt.reserve(n_tiles + 1));
            HIP_TRY(ctx->d_chunk_carry.reserve(ctx->n_chunks + 1));
        }
        if (int rc = upload_coff(ctx, coff_up)) return rc;
        {
            const int64_t np_ = pass == 0 ? n_pad : 0, ni = 2 * n_base;
            const int64_t nt = count_long ? n_tiles + 1 : 0, ncc = count_long ? ctx->n_chunks + 1 : 0;
            const unsigned g = (unsigned)std::max<int64_t>(
                1, std::min<int64_t>(1024, (np_ + (int64_t)n_res + ni + nt + ncc + kBlock - 1) / kBlock));
            hipLaunchKernelGGL(prep_clear_kernel, dim3(g), dim3(kBlock), 0, s, ctx->d_tid.p + n, np_,
                               ctx->d_scratch.p, (int64_t)n_res,
                               reinterpret_cast<unsigned long long*>(ctx->d_chunk_first.p), ni,
                               n ? ~0ull : 0ull,   // all ones: no crossing read
                               reinterpret_cast<int32_t*>(count_long ? ctx->d_tile_cnt.p : nullptr), nt,
                               count_long ? ctx->d_chunk_carry.p : nullptr, ncc);
            HIP_TRY(hipGetLastError());
        }
        if (n) {
            HIP_TRY(ctx->d_gpos.reserve((size_t)(n + kPadBatch)));   // whole-batch loads
            end_words = count_long && ctx->n_chunks * ctx->chunk_w < (int64_t)0xffffffffll;
            if (end_words) HIP_TRY(ctx->d_endw.reserve((size_t)(n + kPadBatch)));
            IngestIndex ix{ctx->d_coff.p, base_lw(ctx), ctx->short_max, n_base, ctx->d_chunk_first.p,
                           count_long ? ctx->d_tile_cnt.p : nullptr, count_long ? ctx->d_chunk_carry.p : nullptr,
                           ctx->n_chunks * ctx->chunk_w, lcw, end_words ? ctx->d_endw.p : nullptr};
            const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((n + 4 * kBlock - 1) / (4 * kBlock),
                                                                      igrid));
            if (count_long)
                hipLaunchKernelGGL(ingest_kernel<true>, dim3((unsigned)nb), dim3(kBlock), 0, s, ctx->d_tid.p,
                                   ctx->d_pos.p, ctx->d_span.p, n, nc, ctx->d_scratch.p,
                                   reinterpret_cast<long long*>(ctx->d_scratch.p + 8),
                                   ctx->d_scratch.p + 8 + nc, ix, ctx->d_gpos.p);
            else
                hipLaunchKernelGGL(ingest_kernel<false>, dim3((unsigned)nb), dim3(kBlock), 0, s, ctx->d_tid.p,
                                   ctx->d_pos.p, ctx->d_span.p, n, nc, ctx->d_scratch.p,
                                   reinterpret_cast<long long*>(ctx->d_scratch.p + 8),
                                   ctx->d_scratch.p + 8 + nc, ix, ctx->d_gpos.p);
            HIP_TRY(hipGetLastError());
        }
        if (count_long)
            if (int rc = launch_long(true)) return rc;
        HIP_TRY(hipMemcpyAsync(res, ctx->d_scratch.p, n_res * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        MC_REQUIRE(h[0] == 0, MC_E_INVALID,
                   "%llu reads have tid outside [0, %d), negative pos or negative span", h[0], nc);
        MC_REQUIRE(h[1] == 0, MC_E_INVALID,
                   "reads are not coordinate-sorted by (tid, pos) (%llu order violations); "
                   "the reference requires a sorted, indexed BAM (cli.py:37)", h[1]);
        bool grew = false;
        for (int32_t i = 0; i < nc; ++i)
            if (maxend[i] > ext[i]) {
                ext[i] = maxend[i];
                grew = true;
            }
        if (!grew) break;
        MC_REQUIRE(pass == 0, MC_E_STATE, "contig extents changed on the second ingest pass");
        set_layout(ctx, ext);
    }
    ctx->aligned_bases = (int64_t)h[2];
    ctx->max_span = (int32_t)h[3];
    ctx->cbases.assign(res + 8 + nc, res + 8 + 2 * nc);
    if (ctx->cbases.empty()) ctx->cbases.assign(1, 0);
    HIP_TRY(ctx->d_depth.reserve((size_t)(ctx->n_chunks * ctx->chunk_w)));
    ctx->has_long = ctx->max_span > ctx->short_max;
    ctx->long_hint = ctx->has_long;
    if (ctx->has_long && !count_long)
        if (int rc = launch_long(false)) return rc;
    HIP_TRY(hipEventRecord(ctx->ev[3], s));
    if (k1_now) {
        // K1 read borrowed CIGAR arrays (mc_add_reads_cigar_device): they are
        // the caller's again once this prepare has drained
        HIP_TRY(hipStreamSynchronize(s));
        ctx->t.cigar_ms = elapsed(ctx, 0, 1);
    } else if (ctx->t_cigar) {   // K1 ran for the direct attempt this batch was handed over from
        ctx->t.cigar_ms = elapsed(ctx, 0, 1);
    }
    ctx->prep_pending = true;   // prepare_ms: read once the events are complete
    ctx->prepared = true;
    ctx->depth_valid = false;
    ++ctx->prep_gen;
    ctx->t.full_prepares += 1;
    return MC_OK;
}

// ---- the direct per-batch prepare (see probe_kernel): the layout the contig
// lengths give, the sample probe, nothing synchronous.  K2 then validates
// every read; check_direct() reads its verdict after the call's sync and
// direct_fallback() hands a batch it cannot take to mc_prepare.
static bool direct_eligible(const mc_ctx* ctx) {
    return ctx->direct_enabled && ctx->direct_ok && ctx->n_reads > 0 && !ctx->len.empty();
}

static int prepare_direct(mc_ctx* ctx) {
    const int32_t nc = (int32_t)ctx->len.size();
    const int64_t n = ctx->n_reads;
    hipStream_t s = ctx->stream;
    if (int rc = run_k1(ctx)) return rc;
    // the prepare's span: this event to K2's start event (probe + window)
    auto& T = ctx->ts[ctx->ts_cur];
    if (MC_STEP_EVENTS && !MC_EXT_EVENTS) HIP_TRY(hipEventRecord(T.e[0], s));
    T.prep = true;
    ctx->ring = kRing;
    ctx->short_max = ctx->ring - kTileW;
    const size_t n_res = 8 + 2 * (size_t)nc;   // (pin_io's layout, shared with mc_prepare)
    HIP_TRY(ctx->pin_io.reserve((n_res + nc + 1) * 8));
    int64_t* coff_up = reinterpret_cast<int64_t*>(static_cast<unsigned long long*>(ctx->pin_io.h) + n_res);
    set_layout(ctx, ctx->len);
    if (int rc = upload_coff(ctx, coff_up)) return rc;
    const int64_t n_base = ctx->n_chunks * ctx->cstride;
    HIP_TRY(ctx->d_jidx.reserve(3 * (n_base + 1)));
    HIP_TRY(ctx->d_fsamp.reserve(nc + 1));
    if (!ctx->d_dres.p) {
        HIP_TRY(ctx->d_dres.reserve(kDresWords));
        HIP_TRY(hipMemsetAsync(ctx->d_dres.p, 0, kDresWords * 8, s));   // generation stamps start below 1
    }
    // (K2's whole-batch loads read up to 3 reads of padding past n; the
    // direct K2 neither applies nor checks reads at or past n)
    ctx->direct_halo_used = ctx->direct_halo > 0 ? std::min(ctx->direct_halo, ctx->short_max) : ctx->short_max;
    ProbeArgs P{ctx->d_tid.p, ctx->d_pos.p, ctx->d_span.p, n, nc, ctx->d_coff.p, base_lw(ctx),
                ctx->short_max, ctx->direct_halo_used, n_base, ctx->d_jidx.p, ctx->d_jidx.p + (n_base + 1),
                ctx->d_jidx.p + 2 * (n_base + 1), ctx->d_fsamp.p,
                ctx->d_dres.p, ++ctx->direct_gen};
    const int64_t M = (n + kProbeStride - 1) >> kProbeShift;
    hipExtLaunchKernelGGL(probe_kernel, dim3((unsigned)std::max<int64_t>(1, (M + kBlock - 1) / kBlock)),
                          dim3(kBlock), 0, s, MC_STEP_EVENTS && MC_EXT_EVENTS ? T.e[0] : nullptr, nullptr, 0, P);
    HIP_TRY(hipGetLastError());
    HIP_TRY(ctx->d_depth.reserve((size_t)(ctx->n_chunks * ctx->chunk_w)));
    ctx->has_long = false;
    ctx->max_span = 0;
    ctx->aligned_bases = -1;   // K2 counts them
    ctx->prepared = true;
    ctx->direct = true;
    ctx->direct_checked = false;
    ctx->depth_valid = false;
    ++ctx->prep_gen;
    return MC_OK;
}

// K2's verdict on a direct batch (res: a host copy of d_dres).  True: the
// batch is exactly what the direct path computed (the counts become the
// prepare's results); false: direct_fallback + mc_prepare must redo it.
static int next_halo(unsigned long long max_span, int short_max) {
    const long long h = round_up((long long)max_span + (long long)max_span / 8, 64);
    return (int)std::max<long long>(64, std::min<long long>(h, short_max));
}

// deferred: the fused call adds the prepare's time with its other event
// times (resolve_timings); otherwise it is read here (K2 start = ev[4]).
static bool check_direct(mc_ctx* ctx, const unsigned long long* res, bool deferred = false) {
    const unsigned long long g = ctx->direct_gen;
    if (res[kDresBadSample] == g || res[kDresLongSample] == g || res[kDresFlags] ||
        res[kDresMaxSpan] > (unsigned long long)ctx->direct_halo_used)
        return false;
    ctx->max_span = (int32_t)res[kDresMaxSpan];
    ctx->direct_halo = next_halo(res[kDresMaxSpan], ctx->short_max);
    ctx->aligned_bases = -1;   // summed on request (direct_bases)
    ctx->direct_checked = true;
    ctx->t.direct_batches += 1;
    auto& T = ctx->ts[ctx->ts_cur];
    if (!deferred && T.prep) {
        ctx->t.prepare_ms = elapsed(T.e[0], ctx->ev[4]);
        ctx->t.prepare_ms_total += ctx->t.prepare_ms;
        T.prep = false;
    }
    ctx->t.cigar_ms = ctx->t_cigar ? elapsed(ctx, 0, 1) : 0.f;
    return true;
}

// A batch the direct path cannot represent: long reads or reads past their
// contig's end keep this contig set on the full prepare from now on; invalid
// or unsorted reads only get mc_prepare's exact error.  A batch whose spans
// only outgrew the halo is redone on the direct path with a halo that covers
// its (now known) maximum span.
static void direct_fallback(mc_ctx* ctx, const unsigned long long* res) {
    const unsigned long long g = ctx->direct_gen;
    const bool long_reads = res[kDresLongSample] == g || res[kDresMaxSpan] > (unsigned long long)ctx->short_max;
    if (long_reads || (res[kDresFlags] & kDirectUnfit)) ctx->direct_ok = false;
    if (long_reads || res[kDresBadSample] == g || res[kDresFlags]) {
        ctx->direct_retry_full = true;
    } else {
        ctx->direct_halo = next_halo(res[kDresMaxSpan], ctx->short_max);
        ctx->t.halo_redos += 1;
    }
    ctx->fused_clean = false;
    invalidate(ctx);
}

// Prepare for a compute call: the direct path when it may apply, else the
// full one.
static int prepare_for_compute(mc_ctx* ctx) {
    if (ctx->prepared) return MC_OK;
    if (direct_eligible(ctx) && !ctx->direct_retry_full) return prepare_direct(ctx);
    return mc_prepare(ctx);
}

extern "C" int mc_set_legacy_endpos(mc_ctx* ctx, int legacy) {
    if (int rc = ctx_use(ctx)) return rc;
    ctx->min_span = legacy ? 1 : 0;
    return MC_OK;
}

extern "C" int mc_set_direct_prepare(mc_ctx* ctx, int enable) {
    if (int rc = ctx_use(ctx)) return rc;
    ctx->direct_enabled = enable != 0;
    if (!ctx->direct_enabled && ctx->direct) invalidate(ctx);
    return MC_OK;
}

// Resident workgroups of a K2 variant (queried once per ctx and LDS size),
// at most MC_K2_PER_CU per CU (0: as many as fit).
#ifndef MC_K2_PER_CU
#define MC_K2_PER_CU 0
#endif
static int occupancy_grid(mc_ctx* ctx, int variant, const void* kernel, size_t lds, int64_t work,
                          int* grid) {
    int& cached = ctx->k2_resident[variant];
    if (cached <= 0 || ctx->k2_resident_lds[variant] != lds) {
        int dev = 0, ncu = 0, per = 0;
        HIP_TRY(hipGetDevice(&dev));
        HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kK2Block, lds));
        if (MC_K2_PER_CU > 0) per = std::min(per, (int)MC_K2_PER_CU);
        cached = ncu * std::max(1, per);
        ctx->k2_resident_lds[variant] = lds;
    }
    *grid = (int)std::max<int64_t>(1, std::min<int64_t>(work, (int64_t)cached));
    return MC_OK;
}

// Chunk geometry of a K2 launch.  The plain K2 runs on the index's base
// chunks unless long reads need full ones (their end buckets and carries are
// per full chunk).  MC_FUSED_BASE_CHUNKS: the fused K2 too.
#ifndef MC_FUSED_BASE_CHUNKS
#define MC_FUSED_BASE_CHUNKS 0
#endif
struct K2Geom {
    int tpc;
    int64_t n_chunks, chunk_w;
    int cstride;
};
static K2Geom k2_geom(const mc_ctx* ctx, bool stats) {
    const bool full = ctx->has_long || (stats && !MC_FUSED_BASE_CHUNKS);
    if (full) return {ctx->tiles_per_chunk, ctx->n_chunks, ctx->chunk_w, ctx->cstride};
    return {ctx->tpc_base, ctx->n_chunks_base, (int64_t)ctx->tpc_base * kTileW, 1};
}

#ifndef MC_WIN_BELOW
#define MC_WIN_BELOW (3 * kHistBins / 4)
#endif
constexpr int kWinBelow = MC_WIN_BELOW;   // window bins below the estimated body depth

// The direct path's window parameters (direct_window_base): this
// generation's span sums, the window placement of the short-read variant.
static DirectWindow direct_window(const mc_ctx* ctx) {
    return DirectWindow{ctx->d_fsamp.p, ctx->d_len.p, ctx->d_dres.p, (int)(ctx->direct_gen & 1),
                        (int)((int64_t)kWinBelow * fused_hist_vals(ctx->has_long) / kHistBins)};
}

// K2's constant arguments in device memory (K2Consts): the slot holding
// these bytes, else the next slot, uploaded on the ctx stream (uploads happen
// when buffers are reallocated or the region set changes).  Each slot has
// its own pinned staging; it is rewritten only once that slot's previous
// copy is done (its event), not after a drain of the whole stream.  The
// slots are matched bytewise: K2Consts has no padding but DirectArgs' one
// hole, which launch_depth keeps zeroed (memberwise stores into a zeroed
// struct).
static_assert(sizeof(DirectArgs) == 5 * 8 + 8 + sizeof(DirectWindow) && sizeof(DirectWindow) == 32 &&
                  sizeof(FusedRegions) == 10 * 8 && sizeof(ReadArrays) == 4 * 8,
              "K2Consts: padding beyond DirectArgs' 4 bytes after nc");
static int k2_consts(mc_ctx* ctx, const K2Consts& kc, const K2Consts** out) {
    for (int i = 0; i < mc_ctx::kK2Slots; ++i)
        if (ctx->k2c_valid[i] && std::memcmp(&ctx->k2c[i], &kc, sizeof kc) == 0) {
            *out = ctx->d_k2c.p + i;
            return MC_OK;
        }
    HIP_TRY(ctx->d_k2c.reserve(mc_ctx::kK2Slots));
    HIP_TRY(ctx->h_k2c.reserve(sizeof(K2Consts) * mc_ctx::kK2Slots));
    const int i = ctx->k2c_next;
    ctx->k2c_next = (i + 1) % mc_ctx::kK2Slots;
    if (ctx->k2c_ev[i]) HIP_TRY(hipEventSynchronize(ctx->k2c_ev[i]));   // the slot's previous copy is done
    else HIP_TRY(hipEventCreateWithFlags(&ctx->k2c_ev[i], hipEventDisableTiming));
    K2Consts* stage = reinterpret_cast<K2Consts*>(ctx->h_k2c.h) + i;
    std::memcpy(stage, &kc, sizeof kc);
    HIP_TRY(hipMemcpyAsync(ctx->d_k2c.p + i, stage, sizeof kc, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipEventRecord(ctx->k2c_ev[i], ctx->stream));
    ctx->k2c[i] = kc;
    ctx->k2c_valid[i] = true;
    *out = ctx->d_k2c.p + i;
    return MC_OK;
}

// K2 launch (plain or with fused region statistics)
// ea / eb: K2's start / end events (default ev[4] / ev[5], read lazily by
// mc_get_timings)
static int launch_depth(mc_ctx* ctx, const FusedRegions& fr, hipEvent_t ea = nullptr, hipEvent_t eb = nullptr) {
    hipStream_t s = ctx->stream;
    const bool stats = fr.n > 0;
    const size_t lds = (size_t)(kLdsHeader + ctx->ring +
                                (stats ? (ctx->has_long ? HistCfg<true>::kLds : HistCfg<false>::kLds) + kOvInts
                                       : 0)) * 4;
    const bool lng = ctx->has_long;
    const bool dir = ctx->direct;
    const void* kfn = stats ? (lng ? (const void*)depth_kernel<true, true, false>
                                   : dir ? (const void*)depth_kernel<true, false, true>
                                         : (const void*)depth_kernel<true, false, false>)
                            : (lng ? (const void*)depth_kernel<false, true, false>
                                   : dir ? (const void*)depth_kernel<false, false, true>
                                         : (const void*)depth_kernel<false, false, false>);
    const K2Geom geo = k2_geom(ctx, stats);
    const int tpc = geo.tpc;
    const int64_t nch = geo.n_chunks;
    const int cstride = geo.cstride;
    const int64_t* cfirst = ctx->d_chunk_first.p;
    int grid = 0;
    if (int rc = occupancy_grid(ctx, (stats ? 1 : 0) + (lng ? 2 : dir ? 4 : 0), kfn, lds, nch, &grid))
        return rc;
    if (!stats) {   // the fused path's fused_init_kernel (or the last K3b) zeroes them
        ctx->fused_clean = false;   // this K2 consumes the queue
        HIP_TRY(hipMemsetAsync(ctx->d_queue.p, 0, 32, s));
        HIP_TRY(hipMemsetAsync(ctx->d_maxdepth.p, 0, 16, s));
    }
    hipEvent_t k2_start = MC_STEP_EVENTS || !ea ? (ea ? ea : ctx->ev[4]) : nullptr;
    hipEvent_t k2_stop = MC_STEP_EVENTS || !eb ? (eb ? eb : ctx->ev[5]) : nullptr;
    if (!MC_EXT_EVENTS && k2_start) HIP_TRY(hipEventRecord(k2_start, s));
    const int64_t* toff = ctx->has_long ? ctx->d_tile_off.p : nullptr;
    const int32_t* tev = ctx->has_long ? ctx->d_tile_ev.p : nullptr;
    const int* ccar = ctx->has_long ? ctx->d_chunk_carry.p : nullptr;
    const int64_t n_base = ctx->n_chunks * ctx->cstride;
    K2Consts kc;
    std::memset(&kc, 0, sizeof kc);   // (padding too: slots are matched bytewise)
    kc.A = ReadArrays{ctx->d_gpos.p, ctx->d_tid.p, ctx->d_pos.p, ctx->d_span.p};
    kc.R = fr;
    DirectWindow w = direct_window(ctx);
    w.parity = 0;   // (K2 takes this call's parity as an argument)
    kc.D.j0 = ctx->d_jidx.p;   // (memberwise: the struct's padding stays zero)
    kc.D.jh = ctx->d_jidx.p + (n_base + 1);
    kc.D.jn = ctx->d_jidx.p + 2 * (n_base + 1);
    kc.D.len = ctx->d_len.p;
    kc.D.nc = (int32_t)ctx->len.size();
    kc.D.dres = ctx->d_dres.p;
    kc.D.win = w;
    const K2Consts* dk = nullptr;
    if (int rc = k2_consts(ctx, kc, &dk)) return rc;
    const int win_parity = (int)(ctx->direct_gen & 1);
#define MC_LAUNCH_K2(S, L, D)                                                                  \
    hipExtLaunchKernelGGL((depth_kernel<S, L, D>), dim3(grid), dim3(kK2Block), (uint32_t)lds, s,        \
                          MC_EXT_EVENTS ? k2_start : nullptr, MC_EXT_EVENTS ? k2_stop : nullptr, 0u, kc.A, dk, \
                       ctx->n_reads, ctx->d_coff.p,                                               \
                       cfirst, cstride, nch, tpc, ctx->short_max,                                \
                       toff, tev, ccar, ctx->d_depth.p, ctx->d_queue.p, ctx->d_maxdepth.p,        \
                       (unsigned long long)ctx->direct_gen, win_parity)
    if (stats) {
        if (lng) MC_LAUNCH_K2(true, true, false);
        else if (dir) MC_LAUNCH_K2(true, false, true);
        else MC_LAUNCH_K2(true, false, false);
    } else {
        if (lng) MC_LAUNCH_K2(false, true, false);
        else if (dir) MC_LAUNCH_K2(false, false, true);
        else MC_LAUNCH_K2(false, false, false);
    }
#undef MC_LAUNCH_K2
    HIP_TRY(hipGetLastError());
    if (!MC_EXT_EVENTS && k2_stop) HIP_TRY(hipEventRecord(k2_stop, s));
    ctx->t_depth = ea == nullptr;   // else the caller's set carries the time
    ctx->t.depth_launches += 1;
    ctx->depth_valid = true;
    ctx->max_depth = -1;   // read lazily
    return MC_OK;
}

extern "C" int mc_compute_depth(mc_ctx* ctx) {
    if (int rc = ctx_use(ctx)) return rc;
    // a direct batch K2 refuses is redone: on the direct path with a wider
    // halo, else on the full prepare (which K2 does not refuse)
    for (int attempt = 0; attempt < 3; ++attempt) {
        if (int rc = prepare_for_compute(ctx)) return rc;
        FusedRegions none{};
        if (int rc = launch_depth(ctx, none)) return rc;
        if (!ctx->direct || ctx->direct_checked) return MC_OK;
        unsigned long long* res = static_cast<unsigned long long*>(ctx->pin_io.h);   // K2's verdict
        HIP_TRY(hipMemcpyAsync(res, ctx->d_dres.p, kDresWords * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        if (check_direct(ctx, res)) return MC_OK;
        direct_fallback(ctx, res);
    }
    MC_REQUIRE(false, MC_E_STATE, "direct prepare refused three times");
    return MC_E_STATE;
}

static int fetch_max_depth(mc_ctx* ctx) {
    if (ctx->max_depth >= 0) return MC_OK;
    int v = 0;
    HIP_TRY(hipMemcpyAsync(&v, ctx->d_maxdepth.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->max_depth = v;
    return MC_OK;
}

extern "C" int mc_max_depth(mc_ctx* ctx, int32_t* out) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(out, MC_E_INVALID, "null out");
    MC_REQUIRE(ctx->depth_valid, MC_E_STATE, "depth not computed");
    if (int rc = fetch_max_depth(ctx)) return rc;
    *out = ctx->max_depth;
    return MC_OK;
}

extern "C" int mc_get_depth(mc_ctx* ctx, int32_t tid, int64_t start, int64_t end, int32_t* out) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(ctx->depth_valid, MC_E_STATE, "depth not computed (call mc_compute_depth)");
    MC_REQUIRE(tid >= 0 && tid < (int32_t)ctx->len.size(), MC_E_INVALID, "tid %d out of range", tid);
    MC_REQUIRE(start >= 0 && end >= start, MC_E_INVALID, "bad range [%lld, %lld)",
               (long long)start, (long long)end);
    MC_REQUIRE(end == start || out, MC_E_INVALID, "null out");
    const int64_t ext = ctx->extent[tid];
    const int64_t a = std::min(start, ext), b = std::min(end, ext);
    if (b > a)
        HIP_TRY(hipMemcpyAsync(out, ctx->d_depth.p + ctx->coff[tid] + a, (b - a) * 4,
                               hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (end > b) std::memset(out + (b - start), 0, (end - std::max(b, start)) * 4);
    return MC_OK;
}

extern "C" int mc_depth_device(mc_ctx* ctx, const int32_t** d_depth, int64_t* total_len) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(d_depth && total_len, MC_E_INVALID, "null out");
    MC_REQUIRE(ctx->depth_valid, MC_E_STATE, "depth not computed");
    *d_depth = ctx->d_depth.p;
    *total_len = ctx->total_len;
    return MC_OK;
}

extern "C" int mc_contig_offset(mc_ctx* ctx, int32_t tid, int64_t* offset, int64_t* extent) {
    MC_REQUIRE(ctx && offset && extent, MC_E_INVALID, "null argument");
    MC_REQUIRE(ctx->prepared, MC_E_STATE, "not prepared");
    MC_REQUIRE(tid >= 0 && tid < (int32_t)ctx->len.size(), MC_E_INVALID, "tid out of range");
    *offset = ctx->coff[tid];
    *extent = ctx->extent[tid];
    return MC_OK;
}

// Region statistics: K3a over segments, K3b per region.  Writes R rows of
// RegionOut (== mc_region_stat) to d_out (device).
// out_rows (host, optional): region r's row goes to d_out_final[out_rows[r]]
// instead of d_out_final[r] (the fused path's fallback regions).
static int region_stats_impl(mc_ctx* ctx, int64_t R, const int32_t* tid, const int64_t* start,
                             const int64_t* end, RegionOut* d_out_final,
                             const int64_t* out_rows = nullptr) {
    MC_REQUIRE(ctx->depth_valid, MC_E_STATE, "depth not computed (call mc_compute_depth)");
    MC_REQUIRE(R >= 0 && (R == 0 || (tid && start && end)), MC_E_INVALID, "bad region arrays");
    const int32_t nc = (int32_t)ctx->len.size();
    for (int64_t r = 0; r < R; ++r) {
        MC_REQUIRE(tid[r] >= 0 && tid[r] < nc, MC_E_INVALID, "region %lld: tid %d out of range",
                   (long long)r, tid[r]);
        MC_REQUIRE(start[r] >= 0 && end[r] >= start[r], MC_E_INVALID,
                   "region %lld: bad range [%lld, %lld)", (long long)r, (long long)start[r],
                   (long long)end[r]);
    }
    if (R == 0) return MC_OK;
    ctx->fused_clean = false;   // d_acc is shared with the fused path
    if (int rc = fetch_max_depth(ctx)) return rc;
    const int nbins = ctx->max_depth + 1;
    hipStream_t s = ctx->stream;
    // batch regions so that the histogram stays <= 256 Mi bins
    const int64_t max_hist = int64_t(1) << 28;
    const int64_t rb = std::max<int64_t>(1, std::min<int64_t>(R, max_hist / nbins));
    const bool lds_hist = nbins <= kLdsBins;
    HIP_TRY(hipEventRecord(ctx->ev[6], s));   // (a fallback's time is added to the fused K3b's)
    int64_t launches = 0;
    for (int64_t r0 = 0; r0 < R; r0 += rb) {
        const int64_t nr = std::min(rb, R - r0);
        std::vector<int64_t> sg_gs, sg_ge, ntot(nr), nzx(nr);
        std::vector<int32_t> sg_reg;
        // segment length: kSeg, halved (down to 16 Ki) while a small job
        // (the fused path's fallback regions) would leave the CUs idle
        int64_t covered = 0;
        for (int64_t k = 0; k < nr; ++k) {
            const int64_t ext = ctx->extent[tid[r0 + k]];
            covered += std::min(end[r0 + k], ext) - std::min(start[r0 + k], ext);
        }
        int64_t seg = kSeg;
        while (seg > 16384 && covered / seg < 2048) seg >>= 1;
        for (int64_t k = 0; k < nr; ++k) {
            const int64_t r = r0 + k;
            const int32_t t = tid[r];
            const int64_t ext = ctx->extent[t];
            const int64_t a = std::min(start[r], ext), b = std::min(end[r], ext);
            ntot[k] = end[r] - start[r];
            nzx[k] = ntot[k] - (b - a);
            for (int64_t p = a; p < b; p += seg) {
                sg_gs.push_back(ctx->coff[t] + p);
                sg_ge.push_back(ctx->coff[t] + std::min(b, p + seg));
                sg_reg.push_back((int32_t)k);
            }
        }
        const int64_t nseg = (int64_t)sg_gs.size();
        const size_t o_gs = 0, o_ge = o_gs + stage_align(nseg * 8),
                     o_reg = o_ge + stage_align(nseg * 8), o_ntot = o_reg + stage_align(nseg * 4),
                     o_nzx = o_ntot + stage_align(nr * 8), o_rows = o_nzx + stage_align(nr * 8),
                     total = o_rows + (out_rows ? stage_align(nr * 8) : 0);
        HIP_TRY(ctx->k3_stage.reserve(total));
        unsigned char* h = ctx->k3_stage.host();
        std::memcpy(h + o_gs, sg_gs.data(), nseg * 8);
        std::memcpy(h + o_ge, sg_ge.data(), nseg * 8);
        std::memcpy(h + o_reg, sg_reg.data(), nseg * 4);
        std::memcpy(h + o_ntot, ntot.data(), nr * 8);
        std::memcpy(h + o_nzx, nzx.data(), nr * 8);
        if (out_rows) std::memcpy(h + o_rows, out_rows + r0, nr * 8);
        unsigned char* d = ctx->k3_stage.d.p;
        const int64_t* d_seg_gs = reinterpret_cast<const int64_t*>(d + o_gs);
        const int64_t* d_seg_ge = reinterpret_cast<const int64_t*>(d + o_ge);
        const int32_t* d_seg_reg = reinterpret_cast<const int32_t*>(d + o_reg);
        HIP_TRY(ctx->d_hist.reserve((size_t)round_up(nr * nbins, 4)));
        HIP_TRY(ctx->d_acc.reserve(nr));
        HIP_TRY(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, s));
        {
            const int64_t hw = round_up(nr * nbins, 4);
            const int64_t work = std::max<int64_t>(hw / 4, nr);
            const unsigned g = (unsigned)std::min<int64_t>(4096, (work + kBlock - 1) / kBlock);
            hipLaunchKernelGGL(fused_init_kernel, dim3(std::max(g, 1u)), dim3(kBlock), 0, s,
                               ctx->d_hist.p, hw, (unsigned*)nullptr, ctx->d_acc.p, nr,
                               (const int64_t*)nullptr, (int64_t)0, (int64_t)1, (int64_t)0,
                               (int64_t*)nullptr, (unsigned*)nullptr, (int*)nullptr);
            HIP_TRY(hipGetLastError());
        }
        if (nseg) {
            if (lds_hist)
                hipLaunchKernelGGL(region_seg_kernel<true>, dim3((unsigned)nseg), dim3(kBlock),
                                   (size_t)round_up(nbins, 4) * 4, s, ctx->d_depth.p, d_seg_gs, d_seg_ge,
                                   d_seg_reg, nbins, ctx->d_hist.p, ctx->d_acc.p);
            else
                hipLaunchKernelGGL(region_seg_kernel<false>, dim3((unsigned)nseg), dim3(kBlock), 0,
                                   s, ctx->d_depth.p, d_seg_gs, d_seg_ge, d_seg_reg, nbins,
                                   ctx->d_hist.p, ctx->d_acc.p);
            HIP_TRY(hipGetLastError());
            ++launches;
        }
        hipLaunchKernelGGL(region_final_kernel, dim3((unsigned)nr), dim3(kBlock), 0, s,
                           ctx->d_hist.p, nbins, ctx->d_acc.p,
                           reinterpret_cast<const int64_t*>(d + o_ntot),
                           reinterpret_cast<const int64_t*>(d + o_nzx),
                           out_rows ? d_out_final : d_out_final + r0, (int*)nullptr, 1,
                           (const int32_t*)nullptr, (const unsigned*)nullptr, 1,
                           out_rows ? reinterpret_cast<const int64_t*>(d + o_rows) : nullptr);
        HIP_TRY(hipGetLastError());
        // the staging buffer is reused by the next batch / call
        HIP_TRY(hipStreamSynchronize(s));
    }
    HIP_TRY(hipEventRecord(ctx->ev[7], s));
    ctx->t_stats = true;
    ctx->t.stats_launches += launches;
    return MC_OK;
}

// Depth + region statistics in one K2 pass (regions folded into the tiles
// while they are in registers), then the histogram finalize.  Needs regions
// that do not overlap each other; otherwise K2 then K3.  Regions whose order
// statistics reach depths >= kHistBins are recomputed by K3.

// Staging layout of a fused call: sorted region arrays (nf), then per-region
// arrays (R).  The fallback flags come back through ctx->h_fflag.
struct FusedLayout {
    size_t gs, ge, id, base, ntot, nzx, brow, rtid, rfused, up, total;
};
static FusedLayout fused_layout(int64_t nf, int64_t R) {
    auto al = stage_align;
    FusedLayout L;
    L.gs = 0;
    L.ge = L.gs + al(nf * 8);
    L.id = L.ge + al(nf * 8);
    L.base = L.id + al(nf * 4);
    L.ntot = L.base + al(nf * 4);
    L.nzx = L.ntot + al(R * 8);
    L.brow = L.nzx + al(R * 8);
    L.rtid = L.brow + al(R * 4);        // each row's contig (the direct path's windows)
    L.rfused = L.rtid + al(R * 4);      // each row's fused entry, or -1
    L.up = L.rfused + al(R * 4);
    L.total = L.up;
    return L;
}

// Internal return code: the direct batch went back to the full prepare
// (direct_fallback); the call starts over.
constexpr int kRedo = 1;

// mapped host words after the fused call's flags: [R] fallback flags, [R]
// K2's max depth, then (8-byte aligned) a copy of d_dres
static size_t fflag_ints(int64_t R) { return (size_t)round_up(R + 1, 2) + 2 * kDresWords; }
static unsigned long long* fflag_dres(int* base, int64_t R) {
    return reinterpret_cast<unsigned long long*>(base + round_up(R + 1, 2));
}

// K2's verdict on a direct batch outside the fused call (a D2H copy + sync):
// MC_OK, or kRedo after direct_fallback.
static int direct_verdict_sync(mc_ctx* ctx) {
    if (!ctx->direct || ctx->direct_checked) return MC_OK;
    unsigned long long* res = static_cast<unsigned long long*>(ctx->pin_io.h);
    HIP_TRY(hipMemcpyAsync(res, ctx->d_dres.p, kDresWords * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (check_direct(ctx, res)) return MC_OK;
    direct_fallback(ctx, res);
    return kRedo;
}

// The launches of a fused call whose region arrays are staged in
// ctx->fstage (just now, or by an identical earlier call).
// Waits until the stream has written stamp `seq` (spinning on mapped host
// memory; a stream query every ~1k spins reports a failed stream), or, where
// the stream cannot write stamps, for the stream to drain.
// How a fused call learns that its last kernel is done (MC_DONE_MODE):
// 0 a stream write command after it writes the stamp; 1 K3b's last
// workgroup writes the stamp (grid_done_stamp) when K3b is the call's last
// kernel, else as 0; 2 the host polls the event recorded after it.
#ifndef MC_DONE_MODE
#define MC_DONE_MODE 1
#endif
static int wait_event_spin(hipEvent_t ev) {
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return MC_OK;
        if (e != hipErrorNotReady) HIP_TRY(e);
        __builtin_ia32_pause();
    }
}

static int wait_stamp(mc_ctx* ctx, unsigned long long seq) {
    if (!ctx->stamp_ok) {
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        return MC_OK;
    }
    for (unsigned k = 1;; ++k) {
        if (__atomic_load_n(ctx->h_done.h, __ATOMIC_ACQUIRE) >= seq) return MC_OK;
        __builtin_ia32_pause();
        if ((k & 1023) == 0) {
            const hipError_t e = hipStreamQuery(ctx->stream);
            if (e == hipSuccess) return MC_OK;
            if (e != hipErrorNotReady) HIP_TRY(e);
        }
    }
}

static int depth_stats_launch(mc_ctx* ctx, int64_t R, const int32_t* tid, const int64_t* start,
                              const int64_t* end, RegionOut* d_out, int64_t nf) {
    hipStream_t s = ctx->stream;
    const FusedLayout L = fused_layout(nf, R);
    const size_t o_gs = L.gs, o_ge = L.ge, o_id = L.id, o_base = L.base, o_ntot = L.ntot,
                 o_nzx = L.nzx, o_brow = L.brow;
    const K2Geom geo = k2_geom(ctx, true);
    HIP_TRY(ctx->d_fchunk.reserve(geo.n_chunks));
    HIP_TRY(ctx->d_flow.reserve(R));
    const int vals = fused_hist_vals(ctx->has_long);   // values per region row
    HIP_TRY(ctx->d_fhist.reserve((size_t)(R * vals)));
    HIP_TRY(ctx->h_fflag.reserve(fflag_ints(R)));
    const bool verdict = ctx->direct && !ctx->direct_checked;   // K3b hands K2's counters back
    HIP_TRY(ctx->d_acc.reserve(R));
    unsigned char* d = ctx->fstage.d.p;
    const int64_t* d_fge = reinterpret_cast<const int64_t*>(d + o_ge);
    // the previous call's K3b left the fused buffers initialised for this
    // region set (no fallback, nothing else used them since): no init launch
    const bool clean = ctx->fused_clean && ctx->fused_clean_R == R && ctx->fcache.chunk_first;
    ctx->fused_clean = false;
    if (!clean) {
        // the chunk -> first region index depends only on the staged region
        // set: built once per set (the binary searches are most of this
        // launch), reused by repeated calls
        const int64_t idx_chunks = ctx->fcache.chunk_first ? 0 : geo.n_chunks;
        const int64_t work = std::max<int64_t>({R * vals / 4, R, idx_chunks});
        const unsigned g = (unsigned)std::min<int64_t>(4096, (work + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(fused_init_kernel, dim3(std::max(g, 1u)), dim3(kBlock), 0, s,
                           ctx->d_fhist.p, R * vals, ctx->d_flow.p, ctx->d_acc.p, R, d_fge, nf,
                           geo.chunk_w, idx_chunks, ctx->d_fchunk.p, ctx->d_queue.p,
                           ctx->d_maxdepth.p);
        HIP_TRY(hipGetLastError());
        ctx->fcache.chunk_first = true;
    } else if (ctx->check_clean) {
        // debug: the buffers the skipped init would have written must already
        // hold its values (a path that used them without clearing the clean
        // flag shows up here as MC_E_STATE, not as silently wrong statistics)
        HIP_TRY(ctx->d_check.reserve(1));
        HIP_TRY(hipMemsetAsync(ctx->d_check.p, 0, sizeof(unsigned long long), s));
        hipLaunchKernelGGL(fused_clean_check_kernel, dim3(1024), dim3(kBlock), 0, s, ctx->d_fhist.p, R * vals,
                           ctx->d_flow.p, ctx->d_acc.p, R, ctx->d_queue.p, ctx->d_maxdepth.p, ctx->d_check.p);
        HIP_TRY(hipGetLastError());
        unsigned long long bad = 0;
        HIP_TRY(hipMemcpyAsync(&bad, ctx->d_check.p, sizeof bad, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        MC_REQUIRE(bad == 0, MC_E_STATE, "fused buffers not initialised on a clean call (%llu words differ)", bad);
    }
    FusedRegions fr{nf,
                    ctx->d_fchunk.p,
                    reinterpret_cast<const int64_t*>(d + o_gs),
                    d_fge,
                    reinterpret_cast<const int32_t*>(d + o_id),
                    reinterpret_cast<const int32_t*>(d + o_base),
                    reinterpret_cast<const int32_t*>(d + L.rtid),
                    ctx->d_acc.p,
                    ctx->d_fhist.p,
                    ctx->d_flow.p};
    if (nf == 0) fr.n = 0;
    auto& T = ctx->ts[ctx->ts_cur];
    if (int rc = launch_depth(ctx, fr, T.e[1], T.e[2])) return rc;
    // the completion stamp (MC_DONE_MODE 0 / 1)
    const unsigned long long seq = ++ctx->done_seq;
    unsigned long long* stamp = nullptr;
    if (ctx->stamp_ok) {
        if (!ctx->h_done.h) {
            if (ctx->h_done.reserve(1) != hipSuccess || ctx->d_kdone.reserve(1) != hipSuccess ||
                hipMemsetAsync(ctx->d_kdone.p, 0, sizeof(unsigned), s) != hipSuccess) {
                (void)hipGetLastError();
                ctx->stamp_ok = false;
            } else {
                __atomic_store_n(ctx->h_done.h, 0ull, __ATOMIC_RELEASE);
            }
        }
        if (ctx->stamp_ok && MC_DONE_MODE == 1) stamp = ctx->h_done.d;
    }
    // K3b: its span is timed from K2's end event (one event fewer per call)
    // the device-side recompute of out-of-window regions: on for long reads
    // (deep contigs with long end ramps) and after a call that had them
    const bool devfb = ctx->has_long || ctx->fb_recent;
    FbArgs F{};
    if (devfb) {
        if (!ctx->d_fb_cnt.p) {
            HIP_TRY(ctx->d_fb_hist.reserve((size_t)kFbSlots * kLdsBins));
            HIP_TRY(ctx->d_fb_acc.reserve(kFbSlots));
            HIP_TRY(ctx->d_fb_list.reserve(kFbSlots));
            HIP_TRY(ctx->d_fb_cnt.reserve(2));
            HIP_TRY(hipMemsetAsync(ctx->d_fb_cnt.p, 0, 8, s));
            hipLaunchKernelGGL(fused_init_kernel, dim3(1024), dim3(kBlock), 0, s, ctx->d_fb_hist.p,
                               (int64_t)kFbSlots * kLdsBins, (unsigned*)nullptr, ctx->d_fb_acc.p,
                               (int64_t)kFbSlots, (const int64_t*)nullptr, (int64_t)0, (int64_t)1, (int64_t)0,
                               (int64_t*)nullptr, (unsigned*)nullptr, (int*)nullptr);
            HIP_TRY(hipGetLastError());
        }
        F = FbArgs{ctx->d_depth.p,
                   reinterpret_cast<const int32_t*>(d + L.rfused),
                   reinterpret_cast<const int64_t*>(d + o_gs),
                   reinterpret_cast<const int64_t*>(d + o_ge),
                   reinterpret_cast<const int64_t*>(d + o_ntot),
                   reinterpret_cast<const int64_t*>(d + o_nzx),
                   // K2's max depth as K3b copied it out (K3b resets d_maxdepth for the next call)
                   ctx->h_fflag.d + R,
                   ctx->d_fb_list.p,
                   ctx->d_fb_cnt.p,
                   (int)(ctx->fb_calls & 1),
                   ctx->d_fb_hist.p,
                   ctx->d_fb_acc.p,
                   d_out};
        ctx->fb_calls += 1;
    }
    // one wave per region; flags [0, R) and K2's max depth [R] land in mapped host memory
    // the call's end event: on its last kernel (MC_EXT_EVENTS)
    hipEvent_t k3_stop = MC_STEP_EVENTS && MC_EXT_EVENTS ? T.e[3] : nullptr;
#define MC_LAUNCH_K3B(V)                                                                           \
    hipExtLaunchKernelGGL(region_final_wave_kernel<V>, dim3((unsigned)((R + kWaves - 1) / kWaves)),     \
                          dim3(kBlock), 0u, s, nullptr, devfb ? nullptr : k3_stop, 0u,                   \
                          ctx->d_fhist.p, R, ctx->d_acc.p,                                              \
                       reinterpret_cast<const int64_t*>(d + o_ntot),                                \
                       reinterpret_cast<const int64_t*>(d + o_nzx), d_out, ctx->h_fflag.d,           \
                       reinterpret_cast<const int32_t*>(d + o_brow), ctx->d_flow.p,                 \
                       ctx->d_maxdepth.p, ctx->h_fflag.d + R, ctx->d_queue.p,                       \
                       verdict ? ctx->d_dres.p : nullptr, verdict ? fflag_dres(ctx->h_fflag.d, R) : nullptr, \
                       devfb ? F.cnt + F.parity : nullptr, devfb ? F.list : nullptr,                \
                       ctx->direct ? direct_window(ctx) : DirectWindow{},                          \
                       ctx->direct ? reinterpret_cast<const int32_t*>(d + L.rtid) : nullptr,           \
                       ctx->d_kdone.p, devfb ? nullptr : stamp, seq)
    if (vals == HistCfg<false>::kBins) MC_LAUNCH_K3B(HistCfg<false>::kBins);
    else MC_LAUNCH_K3B(HistCfg<true>::kBins);
#undef MC_LAUNCH_K3B
    HIP_TRY(hipGetLastError());
    if (devfb) {
        hipLaunchKernelGGL(fb_seg_kernel, dim3(1024), dim3(kBlock), (size_t)kLdsBins * 4, s, F);
        HIP_TRY(hipGetLastError());
        hipExtLaunchKernelGGL(fb_final_kernel, dim3(kFbSlots), dim3(kBlock), 0u, s, nullptr, k3_stop, 0u, F);
        HIP_TRY(hipGetLastError());
    }
    if (MC_STEP_EVENTS && !MC_EXT_EVENTS) HIP_TRY(hipEventRecord(T.e[3], s));
    if ((MC_DONE_MODE == 0 || (MC_DONE_MODE == 1 && devfb)) && ctx->stamp_ok && hipStreamWriteValue64(s, ctx->h_done.d, seq, 0) != hipSuccess) {
        (void)hipGetLastError();
        ctx->stamp_ok = false;
    }
    ctx->t_stats = false;
    ctx->t.stats_launches += 1;
    // the flags are in host memory once K3b's stamp is (no copy command);
    // the previous call's event times are read meanwhile
    resolve_timings(ctx, false);
    if (int rc = MC_DONE_MODE == 2 ? wait_event_spin(T.e[3]) : wait_stamp(ctx, seq)) return rc;
    const int* flags = ctx->h_fflag.h;
    if (verdict && !check_direct(ctx, fflag_dres(ctx->h_fflag.h, R), true)) {
        direct_fallback(ctx, fflag_dres(ctx->h_fflag.h, R));
        T.prep = T.pending = false;   // the redo records this set again
        return kRedo;
    }
    T.pending = true;
    ctx->ts_cur = (ctx->ts_cur + 1) % mc_ctx::kTimingSets;
    ctx->max_depth = flags[R];   // a fallback's K3 sizes its histogram by it
    int64_t n_flag = 0;
    for (int64_t r = 0; r < R; ++r) n_flag += flags[r] ? 1 : 0;
    // the device recomputed them in this call unless there were too many or
    // the depth exceeds its histogram
    const bool on_device = devfb && n_flag <= kFbSlots && ctx->max_depth < kLdsBins;
    std::vector<int32_t> ft;
    std::vector<int64_t> fs, fe, fr_idx;
    if (!on_device)
        for (int64_t r = 0; r < R; ++r)
            if (flags[r]) {
                ft.push_back(tid[r]);
                fs.push_back(start[r]);
                fe.push_back(end[r]);
                fr_idx.push_back(r);
            }
    ctx->fused_fallbacks = (int64_t)ft.size();
    ctx->device_recomputes = on_device ? n_flag : 0;
    ctx->fb_recent = n_flag > 0;
    if (ft.empty()) {    // K3b reset the buffers behind it
        ctx->fused_clean = true;
        ctx->fused_clean_R = R;
    }
    if (!ft.empty()) {   // exact recompute, rows written in place
        if (int rc = region_stats_impl(ctx, (int64_t)ft.size(), ft.data(), fs.data(), fe.data(),
                                       d_out, fr_idx.data()))
            return rc;
        // the fallback recorded ev[6] / ev[7] around its launches and synced
        HIP_TRY(hipEventSynchronize(ctx->ev[7]));
        ctx->t.fused_stats_ms_total += elapsed(ctx, 6, 7);
    }
    ctx->t.fused_calls += 1;
    return MC_OK;
}

static int depth_stats_once(mc_ctx* ctx, int64_t R, const int32_t* tid, const int64_t* start,
                            const int64_t* end, RegionOut* d_out) {
    if (int rc = prepare_for_compute(ctx)) return rc;
    MC_REQUIRE(R >= 0 && (R == 0 || (tid && start && end)), MC_E_INVALID, "bad region arrays");
    auto& fc = ctx->fcache;
    // direct batch: K2 and K3b derive the windows from the probe's samples
    const bool direct = ctx->direct;
    // histogram window of each region: kHistBins values, kWinBelow of them
    // below its contig's estimated body depth
    const int vals = fused_hist_vals(ctx->has_long);
    const int64_t win_below = (int64_t)kWinBelow * vals / kHistBins;
    const double span_mean = ctx->n_reads ? (double)ctx->aligned_bases / (double)ctx->n_reads : 0.0;
    // the contig's body depth: its aligned bases over its length less one
    // mean read span (the two end ramps hold about half a span of depth
    // each); the window sits mostly below it, where the quartile ranks of a
    // contig with long-read ramps fall (C5 fallbacks: 259 at kHistBins / 2
    // below, 123 at 3 / 4)
    auto window_base = [&](int32_t t) {
        const int64_t ext = ctx->extent[t];
        const double body = ext > 2 * span_mean ? (double)ext - span_mean : (double)ext;
        const double depth_est = ext > 0 ? (double)ctx->cbases[t] / body : 0.0;
        return (int32_t)std::max<int64_t>(0, std::llround(depth_est) - win_below);
    };
    const bool same = R > 0 && fc.valid && (int64_t)fc.tid.size() == R &&
                      std::memcmp(fc.tid.data(), tid, R * 4) == 0 &&
                      std::memcmp(fc.start.data(), start, R * 8) == 0 &&
                      std::memcmp(fc.end.data(), end, R * 8) == 0;
    if (same && fc.gen == ctx->prep_gen) return depth_stats_launch(ctx, R, tid, start, end, d_out, fc.nf);
    const K2Geom geo = k2_geom(ctx, true);
    if (same && fc.vals == vals && fc.chunk_w == geo.chunk_w && fc.n_chunks == geo.n_chunks &&
        fc.extent == ctx->extent && fc.coff == ctx->coff) {
        // a new batch (or a re-prepare) over the same layout: the staged
        // regions, their order and the chunk -> region index stand; only the
        // window bases follow the new per-contig bases (one small upload)
        const FusedLayout L = fused_layout(fc.nf, R);
        if (!direct && R > 0) {   // (direct: K2 and K3b derive the windows from the probe's samples)
            // from ingest's per-contig bases, still in d_scratch, on the
            // device (the host loop over the rows and its upload were 0.05 ms
            // between C5's prepare and K2)
            const int32_t nc = (int32_t)ctx->len.size();
            unsigned char* d = ctx->fstage.d.p;
            hipLaunchKernelGGL(window_bases_kernel, dim3((unsigned)((R + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                               ctx->stream, ctx->d_scratch.p, ctx->d_scratch.p + 8 + nc, ctx->n_reads, ctx->d_len.p,
                               reinterpret_cast<const int32_t*>(d + L.rtid), reinterpret_cast<const int32_t*>(d + L.rfused),
                               R, (int)win_below, reinterpret_cast<int32_t*>(d + L.brow),
                               reinterpret_cast<int32_t*>(d + L.base));
            HIP_TRY(hipGetLastError());
        }
        fc.gen = ctx->prep_gen;
        return depth_stats_launch(ctx, R, tid, start, end, d_out, fc.nf);
    }
    fc.valid = false;
    fc.chunk_first = false;
    const int32_t nc = (int32_t)ctx->len.size();
    struct Reg { int64_t gs, ge; int32_t id, base; };
    std::vector<int32_t> base_row(std::max<int64_t>(R, 1), 0);
    std::vector<Reg> regs;
    regs.reserve(R);
    std::vector<int64_t> ntot(std::max<int64_t>(R, 1)), nzx(std::max<int64_t>(R, 1));
    for (int64_t r = 0; r < R; ++r) {
        MC_REQUIRE(tid[r] >= 0 && tid[r] < nc, MC_E_INVALID, "region %lld: tid %d out of range",
                   (long long)r, tid[r]);
        MC_REQUIRE(start[r] >= 0 && end[r] >= start[r], MC_E_INVALID,
                   "region %lld: bad range [%lld, %lld)", (long long)r, (long long)start[r],
                   (long long)end[r]);
        const int64_t ext = ctx->extent[tid[r]];
        const int64_t a = std::min(start[r], ext), b = std::min(end[r], ext);
        ntot[r] = end[r] - start[r];
        nzx[r] = ntot[r] - (b - a);
        base_row[r] = direct ? 0 : window_base(tid[r]);
        if (b > a)
            regs.push_back({ctx->coff[tid[r]] + a, ctx->coff[tid[r]] + b, (int32_t)r, base_row[r]});
    }
    std::sort(regs.begin(), regs.end(), [](const Reg& x, const Reg& y) { return x.gs < y.gs; });
    bool overlap = false;
    for (size_t k = 1; k < regs.size(); ++k) overlap |= regs[k].gs < regs[k - 1].ge;
    const bool fusable = R > 0 && !overlap && R * (int64_t)vals <= (int64_t(1) << 28);
    if (!fusable) {
        FusedRegions none{};
        if (int rc = launch_depth(ctx, none)) return rc;
        if (int rc = direct_verdict_sync(ctx)) return rc;
        return region_stats_impl(ctx, R, tid, start, end, d_out);
    }
    const int64_t nf = (int64_t)regs.size();
    const FusedLayout L = fused_layout(nf, R);
    HIP_TRY(ctx->fstage.reserve(L.total));
    unsigned char* h = ctx->fstage.host();
    for (int64_t k = 0; k < nf; ++k) {
        reinterpret_cast<int64_t*>(h + L.gs)[k] = regs[k].gs;
        reinterpret_cast<int64_t*>(h + L.ge)[k] = regs[k].ge;
        reinterpret_cast<int32_t*>(h + L.id)[k] = regs[k].id;
        reinterpret_cast<int32_t*>(h + L.base)[k] = regs[k].base;
    }
    std::memcpy(h + L.ntot, ntot.data(), R * 8);
    std::memcpy(h + L.nzx, nzx.data(), R * 8);
    std::memcpy(h + L.brow, base_row.data(), R * 4);
    std::memcpy(h + L.rtid, tid, R * 4);
    {
        int32_t* rf = reinterpret_cast<int32_t*>(h + L.rfused);
        for (int64_t r = 0; r < R; ++r) rf[r] = -1;
        for (int64_t k = 0; k < nf; ++k) rf[regs[k].id] = (int32_t)k;
    }
    HIP_TRY(hipMemcpyAsync(ctx->fstage.d.p, h, L.up, hipMemcpyHostToDevice, ctx->stream));
    fc.tid.assign(tid, tid + R);
    fc.start.assign(start, start + R);
    fc.end.assign(end, end + R);
    fc.nf = nf;
    fc.gen = ctx->prep_gen;
    fc.vals = vals;
    fc.chunk_w = geo.chunk_w;
    fc.n_chunks = geo.n_chunks;
    fc.extent = ctx->extent;
    fc.coff = ctx->coff;
    fc.valid = true;
    return depth_stats_launch(ctx, R, tid, start, end, d_out, nf);
}


static int depth_stats_impl(mc_ctx* ctx, int64_t R, const int32_t* tid, const int64_t* start,
                            const int64_t* end, RegionOut* d_out) {
    int rc = depth_stats_once(ctx, R, tid, start, end, d_out);
    // redone on the direct path with a wider halo, or on the full prepare
    for (int k = 0; k < 2 && rc == kRedo; ++k) rc = depth_stats_once(ctx, R, tid, start, end, d_out);
    MC_REQUIRE(rc != kRedo, MC_E_STATE, "direct prepare refused three times");
    return rc;
}

extern "C" int mc_compute_depth_stats(mc_ctx* ctx, int64_t R, const int32_t* tid,
                                      const int64_t* start, const int64_t* end,
                                      mc_region_stat* out) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(R == 0 || out, MC_E_INVALID, "null out");
    HIP_TRY(ctx->d_out.reserve(std::max<int64_t>(R, 1)));
    if (int rc = depth_stats_impl(ctx, R, tid, start, end, ctx->d_out.p)) return rc;
    if (R)
        HIP_TRY(hipMemcpyAsync(out, ctx->d_out.p, R * sizeof(mc_region_stat), hipMemcpyDeviceToHost,
                               ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return MC_OK;
}

extern "C" int mc_compute_depth_stats_device(mc_ctx* ctx, int64_t R, const int32_t* tid,
                                             const int64_t* start, const int64_t* end,
                                             mc_region_stat* d_out) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(R == 0 || d_out, MC_E_INVALID, "null out");
    return depth_stats_impl(ctx, R, tid, start, end, reinterpret_cast<RegionOut*>(d_out));
}

extern "C" int mc_fused_fallbacks(mc_ctx* ctx, int64_t* out) {
    MC_REQUIRE(ctx && out, MC_E_INVALID, "null argument");
    *out = ctx->fused_fallbacks;
    return MC_OK;
}

extern "C" int mc_fused_recomputes(mc_ctx* ctx, int64_t* out) {
    MC_REQUIRE(ctx && out, MC_E_INVALID, "null argument");
    *out = ctx->device_recomputes;
    return MC_OK;
}

extern "C" int mc_region_stats_device(mc_ctx* ctx, int64_t R, const int32_t* tid,
                                      const int64_t* start, const int64_t* end,
                                      mc_region_stat* d_out) {
    if (int rc = ctx_use(ctx)) return rc;
    static_assert(sizeof(RegionOut) == sizeof(mc_region_stat), "RegionOut layout");
    MC_REQUIRE(R == 0 || d_out, MC_E_INVALID, "null out");
    return region_stats_impl(ctx, R, tid, start, end, reinterpret_cast<RegionOut*>(d_out));
}

extern "C" int mc_region_stats(mc_ctx* ctx, int64_t R, const int32_t* tid, const int64_t* start,
                               const int64_t* end, mc_region_stat* out) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(R == 0 || out, MC_E_INVALID, "null out");
    if (R == 0) return MC_OK;
    HIP_TRY(ctx->d_out.reserve(R));
    if (int rc = region_stats_impl(ctx, R, tid, start, end, ctx->d_out.p)) return rc;
    HIP_TRY(hipMemcpyAsync(out, ctx->d_out.p, R * sizeof(mc_region_stat), hipMemcpyDeviceToHost,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return MC_OK;
}

extern "C" int mc_region_np_sqdev(mc_ctx* ctx, int64_t R, const int32_t* tid, const int64_t* start,
                                  const int64_t* end, const double* mean, double* out) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(ctx->depth_valid, MC_E_STATE, "depth not computed (call mc_compute_depth)");
    MC_REQUIRE(R >= 0 && (R == 0 || (tid && start && end && mean && out)), MC_E_INVALID,
               "bad region arrays");
    if (R == 0) return MC_OK;
    const int32_t nc = (int32_t)ctx->len.size();
    std::vector<NpBlock> blk;
    std::vector<int32_t> first((size_t)R + 1, 0);
    for (int64_t r = 0; r < R; ++r) {
        MC_REQUIRE(tid[r] >= 0 && tid[r] < nc, MC_E_INVALID, "region %lld: tid %d out of range",
                   (long long)r, tid[r]);
        MC_REQUIRE(start[r] >= 0 && end[r] > start[r], MC_E_INVALID,
                   "region %lld: bad range [%lld, %lld)", (long long)r, (long long)start[r],
                   (long long)end[r]);
        const int64_t ext = ctx->extent[tid[r]];
        for (int64_t p = start[r]; p < end[r]; p += kNpBuf) {
            NpBlock b{};
            b.n = (int32_t)std::min<int64_t>(kNpBuf, end[r] - p);
            b.n_data = (int32_t)std::max<int64_t>(0, std::min<int64_t>(b.n, ext - p));
            b.gpos = ctx->coff[tid[r]] + std::min(p, ext);
            b.region = (int32_t)r;
            blk.push_back(b);
        }
        MC_REQUIRE(blk.size() < (size_t(1) << 30), MC_E_RANGE, "regions too long");
        first[(size_t)r + 1] = (int32_t)blk.size();
    }
    const int64_t nb = (int64_t)blk.size();
    const size_t o_blk = 0, o_first = stage_align(nb * sizeof(NpBlock)),
                 o_mean = o_first + stage_align((R + 1) * 4), o_bsum = o_mean + stage_align(R * 8),
                 o_out = o_bsum + stage_align(nb * 8), total = o_out + stage_align(R * 8);
    HIP_TRY(ctx->k3_stage.reserve(total));
    unsigned char* h = ctx->k3_stage.host();
    std::memcpy(h + o_blk, blk.data(), nb * sizeof(NpBlock));
    std::memcpy(h + o_first, first.data(), (R + 1) * 4);
    std::memcpy(h + o_mean, mean, R * 8);
    unsigned char* d = ctx->k3_stage.d.p;
    hipStream_t s = ctx->stream;
    HIP_TRY(hipMemcpyAsync(d, h, o_bsum, hipMemcpyHostToDevice, s));
    constexpr int kWaves = kBlock / 64;
    hipLaunchKernelGGL(np_block_kernel, dim3((unsigned)((nb + kWaves - 1) / kWaves)), dim3(kBlock), 0, s,
                       ctx->d_depth.p, reinterpret_cast<const NpBlock*>(d + o_blk), (int)nb,
                       reinterpret_cast<const double*>(d + o_mean), reinterpret_cast<double*>(d + o_bsum));
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(np_region_kernel, dim3((unsigned)((R + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       reinterpret_cast<const double*>(d + o_bsum), reinterpret_cast<const int32_t*>(d + o_first),
                       (int)R, reinterpret_cast<double*>(d + o_out));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h + o_out, d + o_out, R * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::memcpy(out, h + o_out, R * 8);
    return MC_OK;
}

// ---- htslib's max_depth cap on the device (csrc/capmask.h) ----------------

static int cap_max_span(hipStream_t s, const int32_t* span, int64_t n, int* d_tmp, int* out) {
    HIP_TRY(hipMemsetAsync(d_tmp, 0, 4, s));
    if (n) {
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 255) / 256));
        hipLaunchKernelGGL(cap_max_span_kernel, dim3(g), dim3(256), 0, s, span, n, d_tmp);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipMemcpyAsync(out, d_tmp, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return MC_OK;
}

static int cap_walk(hipStream_t s, const int32_t* pos, int32_t* span, const uint8_t* inq, const int64_t* d_seg,
                    int64_t n_seg, int max_depth, int max_span, uint8_t* keep, int zero,
                    unsigned long long* d_dropped) {
    static std::atomic<bool> attr{false};   // (engines on several host threads)
    if (!attr.load(std::memory_order_acquire)) {
        HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(cap_walk_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kCapLdsBytes));
        attr.store(true, std::memory_order_release);
    }
    if (n_seg <= 0) return MC_OK;
    hipLaunchKernelGGL(cap_walk_kernel, dim3((unsigned)n_seg), dim3(64), (size_t)kCapLdsBytes, s, pos, span, inq,
                       d_seg, max_depth, max_span, keep, zero, d_dropped);
    HIP_TRY(hipGetLastError());
    return MC_OK;
}

extern "C" int mc_depth_cap_mask_device(int device, int64_t n, const int32_t* d_tid, const int32_t* d_pos,
                                        const int32_t* d_span, int32_t max_depth, uint8_t* d_keep,
                                        int64_t* n_dropped) {
    MC_REQUIRE(n >= 0 && (n == 0 || (d_tid && d_pos && d_span && d_keep)), MC_E_INVALID, "bad read arrays");
    MC_REQUIRE(max_depth >= 1, MC_E_INVALID, "max_depth must be >= 1 (got %d)", max_depth);
    HIP_TRY(hipSetDevice(device));
    if (n_dropped) *n_dropped = 0;
    if (n == 0) return MC_OK;
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct StreamGuard {
        hipStream_t s;
        ~StreamGuard() {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    } sg{s};
    DevBuf<uint8_t> flags;
    DevBuf<int64_t> segs;
    DevBuf<unsigned long long> cnt;   // [0] dropped, [1] bad (as unsigned), [2] segments, [3] max span
    DevBuf<unsigned char> temp;
    HIP_TRY(flags.reserve((size_t)n));
    HIP_TRY(segs.reserve((size_t)n + 1));
    HIP_TRY(cnt.reserve(4));
    HIP_TRY(hipMemsetAsync(cnt.p, 0, 32, s));
    unsigned* d_bad = reinterpret_cast<unsigned*>(cnt.p + 1);
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (n + 255) / 256));
    hipLaunchKernelGGL(cap_seg_flags_kernel, dim3(g), dim3(256), 0, s, d_tid, d_pos, n, flags.p, d_bad);
    HIP_TRY(hipGetLastError());
    hipcub::CountingInputIterator<int64_t> idx(0);
    int64_t* d_nsel = reinterpret_cast<int64_t*>(cnt.p + 2);
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tb, idx, flags.p, segs.p, d_nsel, (int)n, s));
    HIP_TRY(temp.reserve(std::max<size_t>(tb, 1)));
    HIP_TRY(hipcub::DeviceSelect::Flagged(temp.p, tb, idx, flags.p, segs.p, d_nsel, (int)n, s));
    unsigned long long h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(h, cnt.p, 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    MC_REQUIRE((unsigned)h[1] == 0, MC_E_INVALID, "reads are not coordinate-sorted");
    const int64_t n_seg = (int64_t)h[2];
    HIP_TRY(hipMemcpyAsync(segs.p + n_seg, &n, 8, hipMemcpyHostToDevice, s));
    int max_span = 0;
    if (int rc = cap_max_span(s, d_span, n, reinterpret_cast<int*>(cnt.p + 3), &max_span)) return rc;
    MC_REQUIRE(max_span < kCapRing - 64, MC_E_RANGE,
               "a span of %d is beyond the device cap's ring (%d); use mc_depth_cap_mask", max_span, kCapRing - 64);
    if (int rc = cap_walk(s, d_pos, const_cast<int32_t*>(d_span), nullptr, segs.p, n_seg, max_depth, max_span,
                          d_keep, 0, cnt.p))
        return rc;
    HIP_TRY(hipMemcpyAsync(h, cnt.p, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (n_dropped) *n_dropped = (int64_t)h[0];
    return MC_OK;
}

extern "C" int mc_add_reads_capped(mc_ctx* ctx, int64_t n, const int32_t* d_tid, const int32_t* d_pos,
                                   const int32_t* d_span, int64_t R, const int32_t* qtid, const int64_t* qstart,
                                   const int64_t* qend, int32_t max_depth, int64_t* n_dropped) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(n >= 0 && (n == 0 || (d_tid && d_pos && d_span)), MC_E_INVALID, "bad read arrays");
    MC_REQUIRE(R >= 0 && (R == 0 || (qtid && qstart && qend)), MC_E_INVALID, "bad region arrays");
    MC_REQUIRE(max_depth >= 1, MC_E_INVALID, "max_depth must be >= 1 (got %d)", max_depth);
    MC_REQUIRE((int64_t)ctx->len.size() == R, MC_E_STATE, "the ctx needs one contig per region (%lld, has %zu)",
               (long long)R, ctx->len.size());
    MC_REQUIRE(ctx->n_reads == 0 && !ctx->spans_pending, MC_E_STATE, "mc_add_reads_capped needs an empty batch");
    MC_REQUIRE(R < (int64_t(1) << 16), MC_E_RANGE, "at most 65535 regions per capped batch");
    for (int64_t r = 0; r < R; ++r)
        MC_REQUIRE(qstart[r] >= 0 && qend[r] >= qstart[r] && qend[r] < (int64_t(1) << 31), MC_E_INVALID,
                   "region %lld: bad range", (long long)r);
    if (n_dropped) *n_dropped = 0;
    if (R == 0) return MC_OK;
    hipStream_t s = ctx->stream;
    // staged queries: qt (int32), qs, qe, lo, hi, off (int64 each; off has R + 1)
    const size_t o_qt = 0, o_qs = stage_align(R * 4), o_qe = o_qs + stage_align(R * 8),
                 o_lo = o_qe + stage_align(R * 8), o_hi = o_lo + stage_align(R * 8),
                 o_off = o_hi + stage_align(R * 8), o_cnt = o_off + stage_align((R + 1) * 8),
                 total = o_cnt + 64;
    HIP_TRY(ctx->k3_stage.reserve(total));
    unsigned char* h = ctx->k3_stage.host();
    unsigned char* d = ctx->k3_stage.d.p;
    std::memcpy(h + o_qt, qtid, R * 4);
    std::memcpy(h + o_qs, qstart, R * 8);
    std::memcpy(h + o_qe, qend, R * 8);
    HIP_TRY(hipMemcpyAsync(d, h, o_lo, hipMemcpyHostToDevice, s));
    int* d_ms = reinterpret_cast<int*>(d + o_cnt);
    unsigned long long* d_dropped = reinterpret_cast<unsigned long long*>(d + o_cnt + 8);
    int max_span = 0;
    if (int rc = cap_max_span(s, d_span, n, d_ms, &max_span)) return rc;
    MC_REQUIRE(max_span < kCapRing - 64, MC_E_RANGE,
               "a span of %d is beyond the device cap's ring (%d)", max_span, kCapRing - 64);
    int64_t* d_lo = reinterpret_cast<int64_t*>(d + o_lo);
    int64_t* d_hi = reinterpret_cast<int64_t*>(d + o_hi);
    hipLaunchKernelGGL(cap_ranges_kernel, dim3((unsigned)((R + 63) / 64)), dim3(64), 0, s, d_tid, d_pos, n,
                       reinterpret_cast<const int32_t*>(d + o_qt), reinterpret_cast<const int64_t*>(d + o_qs),
                       reinterpret_cast<const int64_t*>(d + o_qe), (int)R, max_span, d_lo, d_hi);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h + o_lo, d_lo, o_off - o_lo, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const int64_t* lo = reinterpret_cast<const int64_t*>(h + o_lo);
    const int64_t* hi = reinterpret_cast<const int64_t*>(h + o_hi);
    int64_t* off = reinterpret_cast<int64_t*>(h + o_off);
    off[0] = 0;
    for (int64_t r = 0; r < R; ++r) off[r + 1] = off[r] + std::max<int64_t>(0, hi[r] - lo[r]);
    const int64_t N = off[R];
    MC_REQUIRE(N < (int64_t(1) << 31), MC_E_RANGE, "capped batch of %lld reads", (long long)N);
    HIP_TRY(hipMemcpyAsync(d + o_off, h + o_off, (R + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(d_dropped, 0, 8, s));
    if (int rc = reserve_reads(ctx, N, false)) return rc;
    DevBuf<uint8_t> inq;
    HIP_TRY(inq.reserve((size_t)std::max<int64_t>(N, 1)));
    if (N) {
        const int64_t per = (N + R - 1) / R;
        const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(256, (per + 255) / 256));
        hipLaunchKernelGGL(cap_gather_kernel, dim3(gx, (unsigned)R), dim3(256), 0, s, d_pos, d_span, d_lo,
                           reinterpret_cast<const int64_t*>(d + o_off), reinterpret_cast<const int64_t*>(d + o_qs),
                           ctx->d_tid.p, ctx->d_pos.p, ctx->d_span.p, inq.p);
        HIP_TRY(hipGetLastError());
        if (int rc = cap_walk(s, ctx->d_pos.p, ctx->d_span.p, inq.p, reinterpret_cast<const int64_t*>(d + o_off), R,
                              max_depth, max_span, nullptr, 1, d_dropped))
            return rc;
    }
    unsigned long long dropped = 0;
    HIP_TRY(hipMemcpyAsync(&dropped, d_dropped, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));   // (inq and the staging buffer are reused / freed next)
    ctx->n_reads = N;
    ctx->t_cigar = false;
    invalidate(ctx);
    if (n_dropped) *n_dropped = (int64_t)dropped;
    return MC_OK;
}

// The aligned bases of a direct batch K2 accepted: the sum of its spans
// (span_sum_kernel), once per batch.
static int direct_bases(mc_ctx* ctx) {
    hipStream_t s = ctx->stream;
    const int64_t n = ctx->n_reads;
    const int64_t g = std::max<int64_t>(1, std::min<int64_t>(2048, (n / 4 + kBlock - 1) / kBlock));
    HIP_TRY(ctx->d_bases_part.reserve((size_t)g));
    hipLaunchKernelGGL(span_sum_kernel, dim3((unsigned)g), dim3(kBlock), 0, s, ctx->d_span.p, n,
                       ctx->d_bases_part.p);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(span_sum_final_kernel, dim3(1), dim3(kBlock), 0, s, ctx->d_bases_part.p, (int)g,
                       ctx->d_dres.p + kDresBases);
    HIP_TRY(hipGetLastError());
    unsigned long long v = 0;
    HIP_TRY(hipMemcpyAsync(&v, ctx->d_dres.p + kDresBases, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->aligned_bases = (int64_t)v;
    return MC_OK;
}

extern "C" int mc_aligned_bases(mc_ctx* ctx, int64_t* out) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(out, MC_E_INVALID, "null out");
    if (ctx->direct && !ctx->direct_checked) invalidate(ctx);   // (only after a failed call)
    if (int rc = mc_prepare(ctx)) return rc;
    if (ctx->direct && ctx->aligned_bases < 0)
        if (int rc = direct_bases(ctx)) return rc;
    *out = ctx->aligned_bases;
    return MC_OK;
}

extern "C" int mc_synchronize(mc_ctx* ctx) {
    if (int rc = ctx_use(ctx)) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return MC_OK;
}

extern "C" int mc_get_timings(mc_ctx* ctx, mc_timings* out) {
    if (int rc = ctx_use(ctx)) return rc;
    MC_REQUIRE(out, MC_E_INVALID, "null out");
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    resolve_timings(ctx, true);
    resolve_prepare_timing(ctx);
    if (ctx->t_depth) ctx->t.depth_ms = elapsed(ctx, 4, 5);
    if (ctx->t_stats) ctx->t.stats_ms = elapsed(ctx, 6, 7);
    ctx->t.direct_halo = ctx->direct_halo_used;
    *out = ctx->t;
    return MC_OK;
}
