// GPU BAM decode: BGZF inflate and BAM record parse on the device, so the
// whole pileup path after the file read runs in HBM.
//
// The host decoder (bam_decode.cpp) follows the reference's record walk
// (IteratorRowAll, metacov/scan.pyx:204-216) with libdeflate on host threads;
// at C3 scale it is the end-to-end bound (1.56 s of 1.78 s for a 5.2 GB BAM,
// profiles/r03pp_e2e.json).  This path keeps its semantics record for record
// (same kept set, intervals, counts and error classes) and moves the work:
//
//   host    read the file in windows of BGZF blocks (pread on threads into
//           pinned staging, copied up while the next slice is read); block
//           headers scanned on the host (BSIZE hops, bgzf::scan_blocks)
//   K-gz    gz_inflate_kernel: one lane per BGZF block (inflate.h)
//   K-sync  rec_sync_kernel: one wave per 64 KiB segment of the inflated
//           stream finds the first offset that starts a chain of 8
//           structurally valid records (the host decoder's sync_at rule)
//   K-walk  rec_count_kernel: one lane per segment walks its records from its
//           start to the next segment's start, counting kept records and
//           checking each; the host then checks that every walk lands on the
//           next segment's start (segment 0 starts at the first record, so
//           consistent segments are exact) and re-walks from the landing
//           point where a sync was a false positive
//   K-fill  rec_fill_kernel: the same walk writes the kept (tid, pos, span)
//           at each segment's offset (file order, as mc_bam_open)
//
// A window's incomplete last record is carried to the front of the next
// window's inflated buffer.  The kept intervals stay in HBM
// (mc_bam_gpu_intervals_device) for mc_add_reads_device.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>

#include "bgzf.h"
#include "inflate.h"

using namespace mc::bgzf;

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

constexpr int64_t kSeg = 64 << 10;        // inflated bytes per parse segment
constexpr int kSyncChain = 8;             // records a sync candidate must chain
constexpr int kPad = 64;                  // readable bytes past a compressed window

struct GzBlock {
    int64_t cdata;    // deflate payload, relative to the window's first block
    int64_t out;      // inflated offset in the window buffer
    int32_t clen;
    int32_t isize;
};

struct SegRes {
    int64_t landing;  // first record boundary at or past the next segment's start (or where the walk stopped)
    int64_t records, mapped, kept;
    int64_t err_at;
    int64_t bytes;    // scan mode: the kept records' sequence bytes, each record's rounded up to 4
    int32_t err;      // 0, kSegIncomplete, or an error class
    int32_t pad;
};

enum : int32_t {
    kSegIncomplete = 1,   // an incomplete record at `landing` (the window's tail, or truncation)
    kSegBadSize = 2,      // block_size < 32
    kSegTid = 3,          // rec_parse 2
    kSegCigar = 4,        // rec_parse 3
    kSegSpan = 5,         // rec_parse 4
    kSegMalformed = 6,    // scan mode: l_seq < 0, SEQ past the record, or tid out of range
};

// One wave per workgroup; a wave inflates kGzLanes blocks at a time, each
// lane's primary tables and symbol lists in LDS (kGzLdsWords u16 per lane).
// A lane's symbol loop is a chain of dependent short-latency steps, and a
// window holds fewer blocks than the chip has lanes, so fewer blocks per wave
// buys waves to hide that latency (and less divergence per step).  Measured
// and dropped in round 3 (profiles/r03rc_gz_ab.txt): primary tables in the
// global scratch (230 vs 198 ms), 9 / 7 table bits (half the lanes per CU).
#ifndef MC_GZ_WAVES_PER_CU
#define MC_GZ_WAVES_PER_CU 0   // waves (workgroups) per CU the grid is sized for; 0: as many as the LDS holds
#endif
#ifndef MC_GZ_LANES
#define MC_GZ_LANES 32         // active lanes (blocks in flight) per wave: 64 100.9, 32 82.6, 16 135.6 ms (r03)
#endif
constexpr int kGzLanes = MC_GZ_LANES;
constexpr int kGzThreads = 64;
constexpr int64_t kGzSlotWords = mc::gz::kScratchWords;
constexpr int kGzLdsWords = mc::gz::kPrimaryWords + mc::gz::kSymWords + 2 * mc::gz::kRingWords + 4 * mc::gz::kQueue;
constexpr int kGzWavesPerCu = MC_GZ_WAVES_PER_CU > 0 ? MC_GZ_WAVES_PER_CU
                                                     : (160 << 10) / (kGzLanes * kGzLdsWords * 2);
static_assert(kGzWavesPerCu >= 1, "inflate LDS per wave exceeds a CU");

__global__ void __launch_bounds__(kGzThreads)
gz_inflate_kernel(const uint8_t* __restrict__ comp, const GzBlock* __restrict__ blk, int64_t nblk,
                  uint8_t* __restrict__ out, uint16_t* __restrict__ scratch, int* __restrict__ status,
                  int* __restrict__ any_err) {
    if (threadIdx.x >= kGzLanes) return;
    const int64_t lane = (int64_t)blockIdx.x * kGzLanes + threadIdx.x;
    const int64_t lanes = (int64_t)gridDim.x * kGzLanes;
    uint16_t* S = scratch + lane * kGzSlotWords;
    using lds_u16 = __attribute__((address_space(3))) uint16_t;
    __shared__ uint16_t tabs[kGzLanes * kGzLdsWords];
    lds_u16* TL = (lds_u16*)(tabs + threadIdx.x * kGzLdsWords);
    lds_u16* TD = TL + (1 << mc::gz::kLitBits);
    using lds_u8 = __attribute__((address_space(3))) uint8_t;
    lds_u8* SL = (lds_u8*)(TL + mc::gz::kPrimaryWords);
    lds_u8* SD = SL + mc::gz::kLitSyms;
    using lds_u32 = __attribute__((address_space(3))) uint32_t;
    static_assert((mc::gz::kPrimaryWords + mc::gz::kSymWords) % 2 == 0 && kGzLdsWords % 2 == 0, "ring alignment");
    lds_u32* ring = (lds_u32*)(TL + mc::gz::kPrimaryWords + mc::gz::kSymWords);
    using lds_u64 = __attribute__((address_space(3))) uint64_t;
    static_assert((mc::gz::kPrimaryWords + mc::gz::kSymWords + 2 * mc::gz::kRingWords) % 4 == 0 &&
                      kGzLdsWords % 4 == 0, "queue alignment");
    lds_u64* queue = (lds_u64*)(ring + mc::gz::kRingWords);
    for (int64_t b = lane; b < nblk; b += lanes) {
        const GzBlock g = blk[b];
        const int rc = mc::gz::inflate_block(comp + g.cdata, g.clen, out + g.out, g.isize, S, TL, TD, SL, SD, ring,
                                             queue);
        status[b] = rc;
        if (rc) atomicOr(any_err, 1);
    }
}

// One wave per segment i in [i0, nseg): found[i] = the first offset q in
// [cut_i, min(cut_i + kSeg, n)) that starts `chain` plausible records in
// sort order (or a shorter chain ending exactly at n), else n.
__global__ void __launch_bounds__(256)
rec_sync_kernel(const uint8_t* __restrict__ d, int64_t o, int64_t n, int64_t i0, int64_t nseg, int32_t n_ref,
                int chain, int64_t* __restrict__ found) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t waves = (int64_t)gridDim.x * 4;
    for (int64_t i = i0 + wave; i < nseg; i += waves) {
        const int64_t cut = o + i * kSeg;
        const int64_t lim = cut + kSeg < n ? cut + kSeg : n;
        int64_t res = n;
        for (int64_t base = cut; base < lim; base += 64) {
            const int64_t q = base + lane;
            bool ok = false;
            if (q < lim && mc::gz::rec_plausible(d, q, n, n_ref)) ok = mc::gz::rec_chain(d, q, n, n_ref, chain);
            const unsigned long long m = __ballot(ok);
            if (m) {
                res = base + __ffsll((long long)m) - 1;
                break;
            }
        }
        if (lane == 0) found[i] = res;
    }
}

// Per contig (index n_ref: the records without coordinates), accumulated by
// the fill walk: the inflated-stream offsets of its first record (stored
// complemented, so a zeroed table starts empty under atomicMax) and of the
// end of its last one, and its mapped / unmapped / kept record counts — a
// BAI's pseudo-bin once the offsets are turned into virtual offsets.
struct ExtAcc {
    unsigned long long nfirst, end, mapped, unmapped, kept;
};

// One lane per segment: walk [seg_off[i], seg_off[i+1]) (kFill: write the
// kept intervals at out_off[i]).  The walk of a segment ends at the first
// record boundary >= seg_off[i+1], at an incomplete record, or at an error.
// tid_map (optional, a contig-subset decode): a kept record's tid becomes
// tid_map[tid], and a record whose entry is negative is not kept.  ext
// (kFill, optional): the per-contig table, offsets plus `base` (the stream
// offset of d[0]), one set of atomics per run of one contig in a segment.
template <bool kFill>
__global__ void __launch_bounds__(256)
rec_walk_kernel(const uint8_t* __restrict__ d, int64_t n, const int64_t* __restrict__ seg_off, int64_t first,
                int64_t nseg, int32_t n_ref, uint32_t flag_filter, SegRes* __restrict__ res,
                const int64_t* __restrict__ out_off, int32_t* __restrict__ tid, int32_t* __restrict__ pos,
                int32_t* __restrict__ span, const int32_t* __restrict__ tid_map, ExtAcc* __restrict__ ext,
                int64_t base) {
    const int64_t i = first + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nseg) return;
    int64_t q = seg_off[i];
    const int64_t end = seg_off[i + 1];
    int64_t records = 0, mapped = 0, kept = 0, err_at = 0;
    int32_t err = 0;
    int64_t w = 0, w_end = 0;
    if (kFill) {
        w = out_off[i];
        w_end = w + res[i].kept;
    }
    // the current run of one contig (ext)
    int32_t run_t = -2;
    int64_t run_q0 = 0, run_q1 = 0;
    unsigned long long run_m = 0, run_u = 0, run_k = 0;
    auto flush = [&]() {
        if (run_t < -1) return;
        ExtAcc* e = ext + (run_t < 0 ? n_ref : run_t);
        atomicMax(&e->nfirst, ~(unsigned long long)(base + run_q0));
        atomicMax(&e->end, (unsigned long long)(base + run_q1));
        if (run_m) atomicAdd(&e->mapped, run_m);
        if (run_u) atomicAdd(&e->unmapped, run_u);
        if (run_k) atomicAdd(&e->kept, run_k);
    };
    while (q < end) {
        if (q + 4 > n) {
            err = kSegIncomplete;
            break;
        }
        const int32_t bs = mc::gz::ld_i32(d + q);
        if (bs < 32) {
            err = kSegBadSize;
            err_at = q;
            break;
        }
        if (q + 4 + (int64_t)bs > n) {
            err = kSegIncomplete;
            break;
        }
        const uint8_t* r = d + q + 4;
        mc::gz::RecOut ro;
        int rc = mc::gz::rec_parse(r, r + bs, n_ref, flag_filter, ro);
        const int64_t q0 = q;
        q += 4 + (int64_t)bs;
        ++records;
        mapped += ro.mapped ? 1 : 0;
        if (rc >= 2) {
            err = rc == 2 ? kSegTid : rc == 3 ? kSegCigar : kSegSpan;
            err_at = q;
            break;
        }
        const int32_t raw_t = mc::gz::ld_i32(r);
        if (rc == 1 && tid_map) {
            const int32_t lt = tid_map[ro.tid];
            if (lt < 0) rc = 0;
            ro.tid = lt;
        }
        if (kFill && ext && raw_t >= -1 && raw_t < n_ref) {
            if (raw_t != run_t) {
                flush();
                run_t = raw_t;
                run_q0 = q0;
                run_m = run_u = run_k = 0;
            }
            run_q1 = q;
            if (raw_t >= 0 && !(mc::gz::ld_u16(r + 14) & 4u)) ++run_m;
            else ++run_u;
            if (rc == 1) ++run_k;
        }
        if (rc == 1) {
            if (kFill && w < w_end) {
                tid[w] = ro.tid;
                pos[w] = ro.pos;
                span[w] = ro.span;
                ++w;
            }
            ++kept;
        }
    }
    if (kFill && ext) flush();
    if (!kFill) {
        SegRes s;
        s.landing = q;
        s.records = records;
        s.mapped = mapped;
        s.kept = kept;
        s.err_at = err_at;
        s.bytes = 0;
        s.err = err;
        s.pad = 0;
        res[i] = s;
    }
}

// Scan mode (`metacov scan` on BAM input, scan_src.cpp's bam_next on the
// device): every record is kept, in file order, as the SoA batch the scan
// kernels take: rlen (l_seq), flag, gpos (pos + l_seq on the reverse strand),
// gisize (tlen when properly paired, else 0), tid, and its packed nt16 bases
// at a 4-byte aligned offset (seq_off[k + 1] = the aligned end of record k).
// One lane per segment, as rec_walk_kernel.
template <bool kFill>
__global__ void __launch_bounds__(256)
scan_walk_kernel(const uint8_t* __restrict__ d, int64_t n, const int64_t* __restrict__ seg_off, int64_t first,
                 int64_t nseg, int32_t n_ref, SegRes* __restrict__ res, const int64_t* __restrict__ out_off,
                 const int64_t* __restrict__ byte_off, int32_t* __restrict__ rlen, int32_t* __restrict__ flag,
                 int32_t* __restrict__ gpos, int32_t* __restrict__ gisize, int32_t* __restrict__ tid,
                 int64_t* __restrict__ seq_off, uint8_t* __restrict__ seq) {
    const int64_t i = first + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nseg) return;
    int64_t q = seg_off[i];
    const int64_t end = seg_off[i + 1];
    int64_t records = 0, mapped = 0, bytes = 0, err_at = 0;
    int32_t err = 0;
    int64_t w = 0, w_end = 0, b = 0;
    if (kFill) {
        w = out_off[i];
        w_end = w + res[i].kept;
        b = byte_off[i];
    }
    while (q < end) {
        if (q + 4 > n) {
            err = kSegIncomplete;
            break;
        }
        const int32_t bs = mc::gz::ld_i32(d + q);
        if (bs < 32) {
            err = kSegBadSize;
            err_at = q;
            break;
        }
        if (q + 4 + (int64_t)bs > n) {
            err = kSegIncomplete;
            break;
        }
        const uint8_t* r = d + q + 4;
        const int32_t t = mc::gz::ld_i32(r), pos = mc::gz::ld_i32(r + 4);
        const uint32_t l_name = r[8], n_cigar = mc::gz::ld_u16(r + 12), fl = mc::gz::ld_u16(r + 14);
        const int32_t l_seq = mc::gz::ld_i32(r + 16), tlen = mc::gz::ld_i32(r + 28);
        const int64_t seq_at = 32 + (int64_t)l_name + 4 * (int64_t)n_cigar;
        const int64_t nbytes = ((int64_t)(l_seq > 0 ? l_seq : 0) + 1) / 2;
        if (l_seq < 0 || seq_at + nbytes > bs || t < -1 || t >= n_ref) {
            err = kSegMalformed;
            err_at = q;
            break;
        }
        q += 4 + (int64_t)bs;
        ++records;
        mapped += (t >= 0 && !(fl & 4u)) ? 1 : 0;
        const int64_t al = (nbytes + 3) & ~(int64_t)3;
        bytes += al;
        if (kFill && w < w_end) {
            rlen[w] = l_seq;
            flag[w] = (int32_t)fl;
            gpos[w] = (fl & 0x10u) ? pos + l_seq : pos;
            gisize[w] = (fl & 0x2u) ? tlen : 0;
            tid[w] = t;
            // the bases, dword by dword (the source is byte-aligned)
            const uint8_t* src = r + seq_at;
            uint32_t* dst = reinterpret_cast<uint32_t*>(seq + b);
            for (int64_t k = 0; k < al; k += 4) {
                uint32_t v = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (k + e < nbytes) v |= (uint32_t)src[k + e] << (8 * e);
                dst[k >> 2] = v;
            }
            b += al;
            seq_off[w + 1] = b;
            ++w;
        }
    }
    if (!kFill) {
        SegRes s;
        s.landing = q;
        s.records = records;
        s.mapped = mapped;
        s.kept = records;
        s.err_at = err_at;
        s.bytes = bytes;
        s.err = err;
        s.pad = 0;
        res[i] = s;
    }
}

// Reads mode (pileup.experimental's read table, exp_reads.cpp's walk on the
// device): every placed record (tid >= 0) in file order with what
// experimental() reads of it: tid, pos, end (pos + bam_cigar2rlen, pos + 1
// when unmapped or 0), flag, bits (1: no SEQ, 2: no reference length), the
// 2-bit code of the first k bases of query_alignment_sequence (0xFFFFFFFF:
// none), and its name (NUL-free bytes, name_off[w] into the names arena).
// One lane per segment, as rec_walk_kernel.  tid_map (a contig-subset
// decode): only records whose entry is >= 0 are taken; tids stay the header's.
__device__ __forceinline__ uint32_t exp_kmer(const uint8_t* cig, uint32_t n_cigar, const uint8_t* seq, int32_t l_seq,
                                             int k) {
    int64_t qs = 0, qe = l_seq;
    for (uint32_t i = 0; i < n_cigar; ++i) {   // getQueryStart
        const uint32_t cw = mc::gz::ld_u32(cig + 4ull * i), op = cw & 0xFu;
        if (op == 5) continue;
        if (op == 4) {
            qs += cw >> 4;
            continue;
        }
        break;
    }
    for (uint32_t i = n_cigar; i-- > 1;) {      // getQueryEnd (stops at op 1)
        const uint32_t cw = mc::gz::ld_u32(cig + 4ull * i), op = cw & 0xFu;
        if (op == 5) continue;
        if (op == 4) {
            qe -= cw >> 4;
            continue;
        }
        break;
    }
    if (qe - qs < k) return 0xFFFFFFFFu;
    uint32_t code = 0;
    for (int m = 0; m < k; ++m) {
        const int64_t q = qs + m;
        const uint32_t nib = (seq[q >> 1] >> ((~q & 1) << 2)) & 0xFu;
        const uint32_t b = nib == 1 ? 0u : nib == 2 ? 1u : nib == 4 ? 2u : nib == 8 ? 3u : 4u;
        if (b > 3) return 0xFFFFFFFFu;
        code = (code << 2) | b;
    }
    return code;
}

template <bool kFill>
__global__ void __launch_bounds__(256)
reads_walk_kernel(const uint8_t* __restrict__ d, int64_t n, const int64_t* __restrict__ seg_off, int64_t first,
                  int64_t nseg, int32_t n_ref, int k, SegRes* __restrict__ res, const int64_t* __restrict__ out_off,
                  const int64_t* __restrict__ byte_off, int32_t* __restrict__ tid, int32_t* __restrict__ pos,
                  int64_t* __restrict__ end_pos, int32_t* __restrict__ flag, uint8_t* __restrict__ bits,
                  uint32_t* __restrict__ kmer, uint8_t* __restrict__ name_len, int64_t* __restrict__ name_off,
                  uint8_t* __restrict__ names, const int32_t* __restrict__ tid_map) {
    const int64_t i = first + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nseg) return;
    int64_t q = seg_off[i];
    const int64_t end = seg_off[i + 1];
    int64_t records = 0, mapped = 0, placed = 0, bytes = 0, err_at = 0;
    int32_t err = 0;
    int64_t w = 0, w_end = 0, b = 0;
    if (kFill) {
        w = out_off[i];
        w_end = w + res[i].kept;
        b = byte_off[i];
    }
    while (q < end) {
        if (q + 4 > n) {
            err = kSegIncomplete;
            break;
        }
        const int32_t bs = mc::gz::ld_i32(d + q);
        if (bs < 32) {
            err = kSegBadSize;
            err_at = q;
            break;
        }
        if (q + 4 + (int64_t)bs > n) {
            err = kSegIncomplete;
            break;
        }
        const uint8_t* r = d + q + 4;
        const uint8_t* rend = r + bs;
        const int32_t t = mc::gz::ld_i32(r);
        const uint32_t l_name = r[8], fl = mc::gz::ld_u16(r + 14);
        const int32_t l_seq = mc::gz::ld_i32(r + 16);
        if (t < -1 || t >= n_ref || l_name == 0 || l_seq < 0) {
            err = kSegMalformed;
            err_at = q;
            break;
        }
        if (t >= 0 && (!tid_map || tid_map[t] >= 0)) {   // (a contig-subset decode: the selected contigs)
            uint32_t n_cigar = mc::gz::ld_u16(r + 12);
            const uint8_t* cig = r + 32 + l_name;
            const uint8_t* seq = cig + 4ull * n_cigar;
            bool ok = cig + 4ull * n_cigar <= rend && seq + ((uint64_t)l_seq + 1) / 2 <= rend;
            if (ok && n_cigar == 2 && mc::gz::ld_u32(cig) == (((uint32_t)l_seq << 4) | 4u) &&
                (mc::gz::ld_u32(cig + 4) & 0xFu) == 3u) {   // the CG:B,I placeholder
                const uint8_t* aux = seq + ((uint64_t)l_seq + 1) / 2 + (uint64_t)l_seq;
                const uint8_t* words = nullptr;
                uint32_t cnt = 0;
                if (aux <= rend && mc::gz::find_cg(aux, rend, &words, &cnt) && words) {
                    cig = words;
                    n_cigar = cnt;
                }
            }
            if (!ok) {
                err = kSegMalformed;
                err_at = q;
                break;
            }
            uint32_t nl = 0;
            while (nl < l_name && r[32 + nl]) ++nl;
            if (kFill && w < w_end) {
                const bool unmapped = fl & 4u;
                int64_t rlen = 0;
                if (!unmapped)
                    for (uint32_t c = 0; c < n_cigar; ++c) {
                        const uint32_t cw = mc::gz::ld_u32(cig + 4ull * c);
                        if ((0x18Du >> (cw & 0xFu)) & 1u) rlen += cw >> 4;
                    }
                if (rlen == 0) rlen = 1;
                const int32_t p = mc::gz::ld_i32(r + 4);
                tid[w] = t;
                pos[w] = p;
                end_pos[w] = (int64_t)p + rlen;
                flag[w] = (int32_t)fl;
                bits[w] = (uint8_t)((l_seq == 0 ? 1 : 0) | ((unmapped || n_cigar == 0) ? 2 : 0));
                kmer[w] = l_seq ? exp_kmer(cig, n_cigar, seq, l_seq, k) : 0xFFFFFFFFu;
                name_len[w] = (uint8_t)nl;
                name_off[w] = b;
                for (uint32_t c = 0; c < nl; ++c) names[b + c] = r[32 + c];
                b += nl;
                ++w;
            }
            ++placed;
            bytes += nl;
            mapped += (fl & 4u) ? 0 : 1;
        }
        q += 4 + (int64_t)bs;
        ++records;
    }
    if (!kFill) {
        SegRes s;
        s.landing = q;
        s.records = records;
        s.mapped = mapped;
        s.kept = placed;
        s.err_at = err_at;
        s.bytes = bytes;
        s.err = err;
        s.pad = 0;
        res[i] = s;
    }
}

template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t cap = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    // keep_elems: the first elements survive a reallocation
    hipError_t reserve(size_t n, hipStream_t st = nullptr, size_t keep_elems = 0) {
        if (n <= cap) return hipSuccess;
        const size_t ncap = std::max(n, cap + cap / 2);
        T* np = nullptr;
        hipError_t e = hipMalloc(&np, ncap * sizeof(T));
        if (e != hipSuccess) return e;
        if (p && keep_elems) {
            e = hipMemcpyAsync(np, p, keep_elems * sizeof(T), hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) {
                (void)hipFree(np);
                return e;
            }
        }
        if (p) (void)hipFree(p);
        p = np;
        cap = ncap;
        return hipSuccess;
    }
};

template <typename T>
struct PinnedBuf {
    T* p = nullptr;
    size_t cap = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), n * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) cap = n;
        return e;
    }
};

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct mc_bam_gpu {
    mc_bam hdr;                       // names, lengths, record counts
    std::string path;
    int device = 0;
    hipStream_t stream = nullptr;
    int nt = 16;
    uint32_t flag_filter = 0;
    DBuf<int32_t> tid, pos, span;     // kept intervals, file order (scan mode: tid, gpos, rlen)
    int64_t n_kept = 0;
    bool scan_mode = false;           // every record as scan's SoA batch (scan_walk_kernel)
    bool reads_mode = false;          // the placed records as experimental()'s read table (reads_walk_kernel)
    int reads_k = 0;
    DBuf<int64_t> rend_pos;           // reads mode: end (pos + reference length)
    DBuf<uint8_t> rbits, rnlen;       // reads mode: bits, name length
    DBuf<uint32_t> rkmer;             // reads mode: k-mer prefix code
    DBuf<int32_t> sflag, sgisize;     // scan mode: flag, gisize
    DBuf<int64_t> soff;               // scan mode: [n_kept + 1] aligned sequence offsets
    DBuf<uint8_t> sseq;               // scan mode: packed nt16 bases
    DBuf<int64_t> boff;               // scan mode: per-segment byte offsets of the fill
    int64_t n_bytes = 0;
    DBuf<uint8_t> comp[2], inflated, tail;   // comp: window k's compressed bytes in comp[k & 1]
    hipStream_t up_stream = nullptr;          // uploads of the next window (overlap the current one's kernels)
    hipStream_t kstream[3] = {};              // resident decode: inflate streams besides `stream`
    DBuf<GzBlock> blk;
    DBuf<int> status;
    DBuf<uint16_t> scratch;
    DBuf<int64_t> seg_off, found, out_off;
    DBuf<SegRes> res;
    PinnedBuf<uint8_t> stage[3];
    PinnedBuf<int64_t> h64;
    PinnedBuf<SegRes> hres;
    PinnedBuf<GzBlock> hblk;
    DBuf<ExtAcc> ext;                 // per-contig table of the walk (n_ref + 1 entries)
    DBuf<int32_t> tid_map;            // contig-subset decode: header tid -> local id (or -1)
    DBuf<uint8_t> raw;                // contig-subset decode: the inflated blocks before compaction
    std::vector<mc::bgzf::Block> blk_list;   // whole-file decode: the blocks (stream offset -> virtual offset)
    bool subset = false;
    std::vector<int32_t> sel;                // contig-subset decode: the selected header tids, sorted
    std::vector<mc_contig_extent> ext_in;    // contig-subset decode: the extents it was opened with
    int64_t n_no_coor_in = 0;
    // timings (ms)
    double t_read = 0, t_inflate = 0, t_parse = 0, t_total = 0, t_scan = 0;
    double t_upload = 0, t_kernel = 0, t_open = 0;   // every upload_file_range call; inflate launches (HIP events, summed)
    int64_t windows = 0, blocks = 0, resyncs = 0, inflated_bytes = 0, compressed_bytes = 0;
    int64_t parse_rounds = 0, resync_passes = 0;
    ~mc_bam_gpu() {
        for (hipStream_t s : {stream, up_stream, kstream[0], kstream[1], kstream[2]}) {
            if (s) {
                (void)hipStreamSynchronize(s);
                (void)hipStreamDestroy(s);
            }
        }
    }
};

namespace {

const char* seg_err_msg(int32_t e) {
    switch (e) {
        case kSegIncomplete: return "truncated record";
        case kSegBadSize: return "bad record size";
        case kSegTid: return "record tid beyond the reference list";
        case kSegCigar: return "CIGAR overruns record";
        case kSegMalformed: return "malformed record";
        default: return "reference span exceeds int32";
    }
}

const char* gz_err_msg(int e) {
    switch (e) {
        case mc::gz::kErrBlockType: return "invalid block type";
        case mc::gz::kErrStored: return "stored block length mismatch";
        case mc::gz::kErrCodes: return "invalid code lengths";
        case mc::gz::kErrSymbol: return "invalid code";
        case mc::gz::kErrDistance: return "distance too far back";
        case mc::gz::kErrOutput: return "more data than ISIZE";
        case mc::gz::kErrInput: return "payload overrun";
        default: return "fewer bytes than ISIZE";
    }
}

// File bytes [off, off + len) into device memory at dst: reader threads
// pread each slice into a pinned staging buffer (kStage buffers in rotation),
// the calling thread copies a slice up as soon as its parts are read, and a
// buffer is handed back to the readers once its copy is done.  The readers
// live for the whole range (round 3 started nt threads per slice: ~0.3 ms of
// thread starts per 64 MiB slice).
// 32 / 64 / 128 / 256 MiB slices, decode in rounds 1-2 (round 0 includes a cold
// first run): 271-288 / 273-298 / 304-307 / 323-334 ms
// (profiles/r03si_upload_slice_ab.txt): larger slices expose a longer first read
#ifndef MC_UPLOAD_SLICE_MIB
#define MC_UPLOAD_SLICE_MIB 64
#endif
// A contig-subset decode uploads only some byte ranges of the file, back to
// back: a virtual offset v lies in segment k at file offset f + (v - v_k).
// Without a map (nullptr) virtual offsets are file offsets.
struct VSeg {
    size_t v, f, len;
};
using VMap = std::vector<VSeg>;

// pread of virtual bytes [v, v + len): the part inside v's segment (the
// caller's loop continues with the rest); -1 if v is outside the map.
ssize_t pread_v(int fd, const VMap* vm, uint8_t* buf, size_t len, size_t v) {
    if (!vm) return pread(fd, buf, len, (off_t)v);
    auto it = std::upper_bound(vm->begin(), vm->end(), v, [](size_t x, const VSeg& s) { return x < s.v; });
    if (it == vm->begin()) return -1;
    --it;
    if (v >= it->v + it->len) return -1;
    return pread(fd, buf, std::min(len, it->v + it->len - v), (off_t)(it->f + (v - it->v)));
}

size_t file_off(const VMap* vm, size_t v) {
    if (!vm) return v;
    auto it = std::upper_bound(vm->begin(), vm->end(), v, [](size_t x, const VSeg& s) { return x < s.v; });
    return it == vm->begin() ? v : std::prev(it)->f + (v - std::prev(it)->v);
}

// progress (optional): virtual offset below which every byte is on the
// device (advanced as copies complete); cancel (optional): stop at the next
// slice.  off, len: a virtual range (vm: the map, nullptr: the file itself).
int upload_file_range(mc_bam_gpu* g, int fd, size_t off, size_t len, uint8_t* dst, hipStream_t st,
                      std::atomic<size_t>* progress = nullptr, const std::atomic<bool>* cancel = nullptr,
                      const VMap* vm = nullptr) {
    constexpr size_t kSlice = (size_t)MC_UPLOAD_SLICE_MIB << 20;
    constexpr int kStage = 3;
    if (len == 0) return MC_OK;
    const double t_begin = now_s();
    struct Clock {
        mc_bam_gpu* g;
        double t0;
        ~Clock() { g->t_upload += (now_s() - t0) * 1e3; }
    } clock{g, t_begin};
    // the first staging buffer now, the others while the readers fill it
    // (pinning 64 MiB takes a few ms; a new handle allocates them all)
    HIP_TRY(g->stage[0].reserve(kSlice));
    hipEvent_t done[kStage] = {};
    for (auto& e : done) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    struct Guard {
        hipEvent_t* e;
        ~Guard() {
            for (int i = 0; i < kStage; ++i)
                if (e[i]) (void)hipEventDestroy(e[i]);
        }
    } guard{done};
    const int64_t ns = (int64_t)((len + kSlice - 1) / kSlice);
    // (8 / 24 / 32 readers instead of 16: within noise, profiles/r04/r04n_e2e.json)
    const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)g->nt, std::min(len, kSlice) >> 20));
    std::mutex mu;
    std::condition_variable cv;
    int64_t free_upto = 1;                            // slices [0, free_upto) may be read
    std::vector<int> parts(ns, 0);                     // parts of each slice read
    bool bad = false, stop = false, quit = false;   // quit: a reader saw cancel
    auto reader = [&](int t) {
        for (int64_t k = 0; k < ns; ++k) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return k < free_upto || stop; });
                if (stop) return;
            }
            if (cancel && cancel->load(std::memory_order_relaxed)) {
                std::lock_guard<std::mutex> lk(mu);   // the main loop may wait for this slice
                quit = true;
                cv.notify_all();
                return;
            }
            const size_t at = (size_t)k * kSlice, n = std::min(kSlice, len - at);
            const size_t a = n * t / nt, b = n * (t + 1) / nt;
            uint8_t* buf = g->stage[k % kStage].p;
            bool ok = true;
            for (size_t got = a; got < b;) {
                const ssize_t r = pread_v(fd, vm, buf + got, b - got, off + at + got);
                if (r <= 0) {
                    ok = false;
                    break;
                }
                got += (size_t)r;
            }
            std::lock_guard<std::mutex> lk(mu);
            if (!ok) bad = true;
            parts[k] += 1;
            cv.notify_all();
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(reader, t);
    hipError_t stage_err = hipSuccess;
    for (int k = 1; k < kStage && k < ns && stage_err == hipSuccess; ++k) stage_err = g->stage[k].reserve(kSlice);
    {
        std::lock_guard<std::mutex> lk(mu);
        if (stage_err == hipSuccess) free_upto = std::min<int64_t>(ns, kStage);
        cv.notify_all();
    }
    auto finish = [&]() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& th : pool) th.join();
    };
    int rc = MC_OK;
    bool cancelled = false;
    if (stage_err != hipSuccess) {
        mc::set_error("HIP error %s allocating the upload staging", hipGetErrorString(stage_err));
        rc = MC_E_HIP;
    }
    for (int64_t k = 0; k < ns && rc == MC_OK; ++k) {
        if (cancel && cancel->load(std::memory_order_relaxed)) {
            cancelled = true;
            break;
        }
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return parts[k] == nt || bad || quit; });
            if (quit && parts[k] != nt && !bad) {
                cancelled = true;
                break;
            }
            if (bad) {
                mc::set_error("%s: read failed in [%zu, %zu)", g->path.c_str(), off, off + len);
                rc = MC_E_IO;
                break;
            }
        }
        const size_t at = (size_t)k * kSlice, n = std::min(kSlice, len - at);
        hipError_t e = hipMemcpyAsync(dst + at, g->stage[k % kStage].p, n, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventRecord(done[k % kStage], st);
        // the previous slice's buffer goes back to the readers once its copy
        // is out (slice j + kStage reuses it): the readers stay a slice ahead
        const int64_t j = k - 1;
        if (e == hipSuccess && j >= 0 && j + kStage < ns) {
            e = hipEventSynchronize(done[j % kStage]);
            if (e == hipSuccess && progress) progress->store(off + (size_t)(j + 1) * kSlice, std::memory_order_release);
            std::lock_guard<std::mutex> lk(mu);
            free_upto = j + kStage + 1;
            cv.notify_all();
        }
        if (e != hipSuccess) {
            mc::set_error("HIP error %s in the upload", hipGetErrorString(e));
            rc = MC_E_HIP;
        }
    }
    finish();
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    if (progress && !cancelled) progress->store(off + len, std::memory_order_release);
    return MC_OK;
}

// Segment starts (i0, nseg) of inflated[o, n) from a sync with chains of
// `chain` records, none before seg[i0] (seg[nseg] = n is kept).
int sync_segments(mc_bam_gpu* g, int64_t o, int64_t n, int64_t i0, int64_t nseg, int chain,
                  std::vector<int64_t>& seg) {
    hipStream_t st = g->stream;
    const int64_t todo = nseg - (i0 + 1);
    if (todo <= 0) return MC_OK;
    int64_t* h = g->h64.p;
    const int grid = (int)std::min<int64_t>((todo + 3) / 4, 65536);
    rec_sync_kernel<<<grid, 256, 0, st>>>(g->inflated.p, o, n, i0 + 1, nseg, (int32_t)g->hdr.names.size(), chain,
                                          g->found.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h + i0 + 1, g->found.p + i0 + 1, todo * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int64_t i = nseg - 1; i > i0; --i) seg[i] = std::max(seg[i0], std::min(std::min(h[i], n), seg[i + 1]));
    return MC_OK;
}

// Parses the records in inflated[o, n); partial: the window is not the
// file's last, so an incomplete last record is carried (*consumed = its
// offset).  Appends kept intervals to g->tid/pos/span; base: the stream
// offset of inflated[0] (the per-contig table's offsets).
int parse_window(mc_bam_gpu* g, int64_t o, int64_t n, bool partial, int64_t* consumed, int64_t base = 0) {
    hipStream_t st = g->stream;
    const int32_t n_ref = (int32_t)g->hdr.names.size();
    const uint8_t* d = g->inflated.p;
    const int64_t nseg = std::max<int64_t>(1, (n - o + kSeg - 1) / kSeg);
    HIP_TRY(g->seg_off.reserve(nseg + 1));
    HIP_TRY(g->found.reserve(nseg + 1));
    HIP_TRY(g->out_off.reserve(nseg + 1));
    HIP_TRY(g->res.reserve(nseg));
    HIP_TRY(g->h64.reserve(2 * (nseg + 1)));   // (scan mode: the byte offsets after the record offsets)
    HIP_TRY(g->hres.reserve(nseg));
    int64_t* h = g->h64.p;
    std::vector<int64_t> seg(nseg + 1, n);
    seg[0] = o;
    if (int rc = sync_segments(g, o, n, 0, nseg, kSyncChain, seg)) return rc;
    // walk / check rounds: segments before `first` are exact and consistent.
    // Each round verifies at least one more segment.  Repeated false syncs
    // (a record's bytes holding record-like chains) are re-synced from the
    // verified prefix with much longer chains instead of walking the rest in
    // one lane; a stream that still does not settle is refused.
    int64_t first = 0;
    SegRes* R = g->hres.p;
    bool tail_cut = false;   // a partial window's records ended early: later segments stay empty
    for (int round = 0;; ++round) {
        g->parse_rounds = std::max<int64_t>(g->parse_rounds, round + 1);
        if ((round == 3 || round == 8) && !tail_cut) {
            if (int rc = sync_segments(g, o, n, first, nseg, round == 3 ? 64 : 1024, seg)) return rc;
            ++g->resync_passes;
        }
        MC_REQUIRE(round < 16, MC_E_IO, "%s: no consistent record boundaries after %d parse rounds", g->path.c_str(),
                   round);
        std::memcpy(h, seg.data() + first, (nseg + 1 - first) * 8);
        HIP_TRY(hipMemcpyAsync(g->seg_off.p + first, h, (nseg + 1 - first) * 8, hipMemcpyHostToDevice, st));
        const int grid = (int)((nseg - first + 255) / 256);
        if (g->scan_mode)
            scan_walk_kernel<false><<<grid, 256, 0, st>>>(d, n, g->seg_off.p, first, nseg, n_ref, g->res.p, nullptr,
                                                          nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                                          nullptr, nullptr);
        else if (g->reads_mode)
            reads_walk_kernel<false><<<grid, 256, 0, st>>>(d, n, g->seg_off.p, first, nseg, n_ref, g->reads_k,
                                                           g->res.p, nullptr, nullptr, nullptr, nullptr, nullptr,
                                                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                                           g->subset ? g->tid_map.p : nullptr);
        else
            rec_walk_kernel<false><<<grid, 256, 0, st>>>(d, n, g->seg_off.p, first, nseg, n_ref, g->flag_filter,
                                                         g->res.p, nullptr, nullptr, nullptr, nullptr,
                                                         g->tid_map.p, nullptr, 0);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(R + first, g->res.p + first, (nseg - first) * sizeof(SegRes),
                               hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        // Every inconsistent landing is applied in one round, but only from a
        // walk whose start this round has not moved (a moved start's walk is
        // stale: comparing it with its successor cascaded into a "fix" of
        // every later segment, 390 k resyncs and the one-lane fallback on a
        // 2.75 GB stream).  Only the chain up to the first fix is verified
        // (`exact`): later walks may have started at a false sync, so their
        // errors are not reported, and their landings are hints the next round
        // re-checks.  The verified prefix grows every round, so the rounds end.
        int64_t redo = -1;
        int64_t moved_upto = -1;   // segments <= this one had their start moved this round
        bool exact = true;
        for (int64_t i = first; i < nseg; ++i) {
            if (i <= moved_upto) continue;
            const SegRes& r = R[i];
            const int64_t end = seg[i + 1];
            if (r.err && !exact) break;
            if (r.err == kSegIncomplete) {
                if (partial) {
                    // the window's records end here: later segments are empty
                    tail_cut = true;
                    if (end != n) {
                        for (int64_t j = i + 1; j < nseg; ++j) seg[j] = n;
                        redo = i + 1;   // (their walks are empty: nothing to redo but the copy)
                    }
                    break;
                }
                mc::set_error("%s: %s at byte %lld of the inflated stream", g->path.c_str(),
                              seg_err_msg(r.err), (long long)r.landing);
                return MC_E_IO;
            }
            if (r.err) {
                mc::set_error("%s: %s at byte %lld of the inflated stream", g->path.c_str(),
                              seg_err_msg(r.err), (long long)r.err_at);
                return MC_E_IO;
            }
            if (r.landing != end) {   // segment i+1's sync was a false positive
                int64_t j = i + 1;
                if (r.landing > end) {
                    for (; j < nseg && seg[j] < r.landing; ++j) seg[j] = r.landing;
                } else {
                    seg[j++] = r.landing;   // (a walk lands at or past its end: not reached)
                }
                moved_upto = j - 1;
                ++g->resyncs;
                if (redo < 0) redo = i + 1;
                exact = false;
            }
        }
        if (redo < 0) break;
        first = redo;
        if (first >= nseg) {
            // only the bookkeeping changed: make the remaining results empty
            break;
        }
    }
    // segments after an incomplete stop are empty; their results may be stale
    int64_t total = 0, records = 0, mapped = 0, tail = n, bytes = 0;
    std::vector<int64_t> koff(nseg + 1), bo(nseg + 1);
    for (int64_t i = 0; i < nseg; ++i) {
        SegRes& r = R[i];
        if (seg[i] >= seg[i + 1] && seg[i] == n) {   // empty tail segment
            r.kept = r.records = r.mapped = r.bytes = 0;
        }
        koff[i] = g->n_kept + total;
        bo[i] = g->n_bytes + bytes;
        total += r.kept;
        bytes += r.bytes;
        records += r.records;
        mapped += r.mapped;
        if (r.err == kSegIncomplete) {
            tail = r.landing;
            for (int64_t j = i + 1; j < nseg; ++j) {
                koff[j] = g->n_kept + total;
                bo[j] = g->n_bytes + bytes;
                R[j].kept = R[j].records = R[j].mapped = R[j].bytes = 0;
            }
            break;
        }
    }
    *consumed = partial ? tail : n;
    // device copies of the final results (kept counts bound the fill writes)
    HIP_TRY(hipMemcpyAsync(g->res.p, R, nseg * sizeof(SegRes), hipMemcpyHostToDevice, st));
    std::memcpy(h, koff.data(), nseg * 8);
    HIP_TRY(hipMemcpyAsync(g->out_off.p, h, nseg * 8, hipMemcpyHostToDevice, st));
    const size_t need = (size_t)(g->n_kept + total) + 4;
    HIP_TRY(g->tid.reserve(need, st, g->n_kept));
    HIP_TRY(g->pos.reserve(need, st, g->n_kept));
    HIP_TRY(g->span.reserve(need, st, g->n_kept));
    if (g->scan_mode || g->reads_mode) {
        HIP_TRY(g->sflag.reserve(need, st, g->n_kept));
        HIP_TRY(g->soff.reserve(need + 1, st, g->n_kept + 1));
        HIP_TRY(g->sseq.reserve((size_t)(g->n_bytes + bytes) + 16, st, (size_t)g->n_bytes));
        HIP_TRY(g->boff.reserve(nseg + 1));
        std::memcpy(h + nseg + 1, bo.data(), nseg * 8);
        HIP_TRY(hipMemcpyAsync(g->boff.p, h + nseg + 1, nseg * 8, hipMemcpyHostToDevice, st));
        const int grid = (int)((nseg + 255) / 256);
        if (g->scan_mode) {
            HIP_TRY(g->sgisize.reserve(need, st, g->n_kept));
            if (g->n_kept == 0) HIP_TRY(hipMemsetAsync(g->soff.p, 0, 8, st));
            if (total) {
                scan_walk_kernel<true><<<grid, 256, 0, st>>>(d, n, g->seg_off.p, 0, nseg, n_ref, g->res.p,
                                                             g->out_off.p, g->boff.p, g->span.p, g->sflag.p, g->pos.p,
                                                             g->sgisize.p, g->tid.p, g->soff.p, g->sseq.p);
                HIP_TRY(hipGetLastError());
            }
        } else {
            HIP_TRY(g->rend_pos.reserve(need, st, g->n_kept));
            HIP_TRY(g->rbits.reserve(need, st, g->n_kept));
            HIP_TRY(g->rkmer.reserve(need, st, g->n_kept));
            HIP_TRY(g->rnlen.reserve(need, st, g->n_kept));
            if (total) {
                reads_walk_kernel<true><<<grid, 256, 0, st>>>(d, n, g->seg_off.p, 0, nseg, n_ref, g->reads_k,
                                                              g->res.p, g->out_off.p, g->boff.p, g->tid.p, g->pos.p,
                                                              g->rend_pos.p, g->sflag.p, g->rbits.p, g->rkmer.p,
                                                              g->rnlen.p, g->soff.p, g->sseq.p,
                                                              g->subset ? g->tid_map.p : nullptr);
                HIP_TRY(hipGetLastError());
            }
        }
    } else if (total || g->ext.p) {
        const int grid = (int)((nseg + 255) / 256);
        rec_walk_kernel<true><<<grid, 256, 0, st>>>(d, n, g->seg_off.p, 0, nseg, n_ref, g->flag_filter, g->res.p,
                                                    g->out_off.p, g->tid.p, g->pos.p, g->span.p, g->tid_map.p,
                                                    g->ext.p, base);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipStreamSynchronize(st));
    g->n_kept += total;
    g->n_bytes += bytes;
    g->hdr.n_records += records;
    g->hdr.n_mapped += mapped;
    g->hdr.n_unmapped += records - mapped;
    return MC_OK;
}

// BGZF header at o of d[0, n): its total size (0 if none)
size_t bgzf_hdr(const uint8_t* d, size_t n, size_t o) {
    if (o + 18 > n || d[o] != 31 || d[o + 1] != 139 || d[o + 2] != 8 || !(d[o + 3] & 4)) return 0;
    const uint16_t xlen = rd16(d + o + 10);
    size_t bsize = 0;
    for (size_t x = o + 12; x + 4 <= o + 12 + xlen && x + 4 <= n;) {
        const uint16_t slen = rd16(d + x + 2);
        if (d[x] == 66 && d[x + 1] == 67 && slen == 2 && x + 6 <= n) bsize = (size_t)rd16(d + x + 4) + 1;
        x += 4 + slen;
    }
    return bsize >= (size_t)xlen + 20 && o + bsize <= n ? bsize : 0;
}

// BGZF header of the block at file offset o, its first bytes in h[0, hn):
// the block's total size, 0 if none (bgzf_hdr's rules; n = the file size).
size_t bgzf_hdr_at(const uint8_t* h, size_t hn, size_t o, size_t n) {
    if (hn < 18 || o + 18 > n || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return 0;
    const size_t xlen = rd16(h + 10);
    size_t bsize = 0;
    for (size_t x = 12; x + 4 <= 12 + xlen && x + 4 <= hn;) {
        const uint16_t slen = rd16(h + x + 2);
        if (h[x] == 66 && h[x + 1] == 67 && slen == 2 && x + 6 <= hn) bsize = (size_t)rd16(h + x + 4) + 1;
        x += 4 + slen;
    }
    return bsize >= xlen + 20 && o + bsize <= n ? bsize : 0;
}

bool pread_all(int fd, uint8_t* buf, size_t len, size_t off) {
    for (size_t got = 0; got < len;) {
        const ssize_t r = pread(fd, buf + got, len - got, (off_t)(off + got));
        if (r <= 0) return false;
        got += (size_t)r;
    }
    return true;
}

// A byte range of the file whose BGZF blocks a decode needs: the blocks from
// a (a block start) up to f (a block start, or the end of the file), plus the
// block at f when `extra`.
struct FileExtent {
    size_t a, f;
    bool extra;
};

// The blocks of the extents, in order, their `out` offsets continuing across
// extents from *total, through pread by nt threads (the GPU decode's scan; no
// mapping).  An extent of >= 64 MiB is cut into pieces (up to 4 nt), each
// starting at the first offset of a window that begins a chain of 4 valid
// headers (or one reaching the end of the file); one pread per block then
// takes its ISIZE and the next block's header (adjacent in the file).  The
// pieces' hops must meet exactly, else one sequential hop of the extent
// decides.  ex_first (optional): each extent's first block index.
int scan_extents_pread(int fd, size_t n, int nt, const char* path, const std::vector<FileExtent>& ex,
                       std::vector<Block>& blocks, size_t& total, std::vector<size_t>* ex_first = nullptr) {
    constexpr size_t kMaxBlock = 65536, kHdr = 96;
    std::atomic<bool> io_err{false};
    auto sync = [&](size_t from, std::vector<uint8_t>& w) -> size_t {
        const size_t wl = std::min(n - from, 5 * kMaxBlock + kHdr);
        w.resize(wl);
        if (!pread_all(fd, w.data(), wl, from)) {
            io_err = true;
            return n;
        }
        const bool to_eof = from + wl == n;
        for (size_t q = 0; q < std::min(wl, kMaxBlock); ++q) {
            size_t z = q;
            int k = 0;
            for (; k < 4 && z < wl; ++k) {
                const size_t b = bgzf_hdr(w.data(), wl, z);
                if (!b) break;
                z += b;
            }
            if (k == 4 || (to_eof && z == wl)) return from + q;
        }
        return n;   // no chain here: the pieces will not meet, the sequential hop decides
    };
    // the blocks of [a, end): false unless the hop lands exactly on end
    // (*stop: the offset it stopped at)
    auto hop = [&](size_t a, size_t end, std::vector<Block>& out, size_t* stop) -> bool {
        *stop = a;
        if (a >= n) return a == end;
        uint8_t h[4 + kHdr];   // [0, 4): the previous block's ISIZE; [4, 4 + hn): header bytes at o
        size_t hn = std::min(kHdr, n - a);
        if (!pread_all(fd, h + 4, hn, a)) {
            io_err = true;
            return false;
        }
        size_t o = a;
        while (o < end) {
            if (hn < 12) return false;
            const size_t xlen = rd16(h + 4 + 10);
            size_t b = bgzf_hdr_at(h + 4, hn, o, n);
            if (!b && 12 + xlen > hn && o + 12 + xlen <= n) {   // a long extra field: read it whole
                std::vector<uint8_t> big(12 + xlen);
                if (!pread_all(fd, big.data(), big.size(), o)) {
                    io_err = true;
                    return false;
                }
                b = bgzf_hdr_at(big.data(), big.size(), o, n);
            }
            if (!b) return false;
            Block blk;
            blk.off = o;
            blk.cdata = o + 12 + xlen;
            blk.clen = b - xlen - 20;
            blk.out = 0;
            const size_t nx = o + b;   // ISIZE is the block's last 4 bytes, the next header follows
            const size_t rl = std::min(4 + kHdr, n - (nx - 4));
            if (!pread_all(fd, h, rl, nx - 4)) {
                io_err = true;
                return false;
            }
            blk.isize = rd32(h);
            hn = rl - 4;
            out.push_back(blk);
            o = nx;
            *stop = o;
        }
        return o == end;
    };
    // pieces: [start[p], end of piece p) of extent pex[p]; pfirst[k]: extent k's first piece
    std::vector<size_t> start, pex, pfirst;
    for (size_t k = 0; k < ex.size(); ++k) {
        MC_REQUIRE(ex[k].a <= ex[k].f && ex[k].f <= n, MC_E_IO, "%s: block range [%zu, %zu) outside the file", path,
                   ex[k].a, ex[k].f);
        const size_t len = ex[k].f - ex[k].a;
        const size_t np = len < (64u << 20) ? 1
                                            : std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, nt) * 4,
                                                                                   len / (4u << 20)));
        pfirst.push_back(start.size());
        for (size_t j = 0; j < np; ++j) {
            start.push_back(ex[k].a + len / np * j);
            pex.push_back(k);
        }
    }
    pfirst.push_back(start.size());
    const size_t npc = start.size();
    auto piece_end = [&](size_t p) { return p + 1 < pfirst[pex[p] + 1] ? start[p + 1] : ex[pex[p]].f; };
    auto pool_run = [&](const std::function<void()>& w) {
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; ++t) pool.emplace_back(w);
        w();
        for (auto& t : pool) t.join();
    };
    {
        std::atomic<size_t> next{0};
        pool_run([&]() {
            std::vector<uint8_t> w;
            for (size_t p; (p = next.fetch_add(1)) < npc;)
                if (p != pfirst[pex[p]]) start[p] = std::min(sync(start[p], w), ex[pex[p]].f);
        });
    }
    for (size_t p = 1; p < npc; ++p)
        if (p != pfirst[pex[p]]) start[p] = std::max(start[p], start[p - 1]);
    std::vector<std::vector<Block>> part(npc);
    std::vector<char> ok(npc, 1);
    {
        std::atomic<size_t> next{0};
        pool_run([&]() {
            size_t stop;
            for (size_t p; (p = next.fetch_add(1)) < npc;) ok[p] = hop(start[p], piece_end(p), part[p], &stop);
        });
    }
    MC_REQUIRE(!io_err, MC_E_IO, "%s: read failed while scanning the BGZF blocks", path);
    for (size_t k = 0; k < ex.size(); ++k) {
        bool chained = true;
        for (size_t p = pfirst[k]; p < pfirst[k + 1]; ++p) chained &= ok[p] != 0;
        if (!chained) {   // one sequential hop of the extent
            for (size_t p = pfirst[k]; p < pfirst[k + 1]; ++p) part[p].clear();
            size_t stop = 0;
            MC_REQUIRE(hop(ex[k].a, ex[k].f, part[pfirst[k]], &stop), MC_E_IO,
                       "%s: no valid BGZF block at offset %zu (truncated, or not bgzip-compressed BAM)", path, stop);
            MC_REQUIRE(!io_err, MC_E_IO, "%s: read failed while scanning the BGZF blocks", path);
        }
        if (ex[k].extra) {   // the block at f
            std::vector<Block>& last = part[pfirst[k + 1] - 1];
            const size_t before = last.size();
            size_t stop = 0;
            (void)hop(ex[k].f, ex[k].f + 1, last, &stop);
            MC_REQUIRE(!io_err, MC_E_IO, "%s: read failed while scanning the BGZF blocks", path);
            MC_REQUIRE(last.size() == before + 1, MC_E_IO, "%s: no valid BGZF block at offset %zu", path, ex[k].f);
        }
    }
    for (size_t k = 0; k < ex.size(); ++k) {
        if (ex_first) ex_first->push_back(blocks.size());
        for (size_t p = pfirst[k]; p < pfirst[k + 1]; ++p)
            for (Block& b : part[p]) {
                b.out = total;
                total += b.isize;
                blocks.push_back(b);
            }
    }
    return MC_OK;
}

// The block list of the whole file (scan_extents_pread over one extent).
int scan_blocks_pread(int fd, size_t n, int nt, const char* path, std::vector<Block>& blocks, size_t& total) {
    return scan_extents_pread(fd, n, nt, path, {FileExtent{0, n, false}}, blocks, total);
}

// Header from a growing prefix of the inflated bytes [0, n): *ok = false if
// no prefix holds a complete one.
int header_from_prefix(mc_bam_gpu* g, size_t n, int64_t* o, bool* ok) {
    *ok = false;
    size_t p = std::min<size_t>(n, 1 << 20);
    std::vector<uint8_t> hb;
    for (;;) {
        hb.resize(p);
        HIP_TRY(hipMemcpy(hb.data(), g->inflated.p, p, hipMemcpyDeviceToHost));
        std::vector<std::string> names;
        std::vector<int64_t> lens;
        size_t ho = 0;
        if (parse_header(hb.data(), p, g->path.c_str(), names, lens, &ho) == MC_OK) {
            g->hdr.names = std::move(names);
            g->hdr.lens = std::move(lens);
            *o = (int64_t)ho;
            *ok = true;
            return MC_OK;
        }
        if (p >= n) return MC_OK;
        p = std::min(n, p * 4);
    }
}

// Resident decode (the default when the compressed file and its inflated
// stream fit in HBM): the inflated stream is cut into pieces (a third each),
// and each piece's inflate kernel is launched as soon as its bytes are on the
// device (uploaded by the background upload of gpu_decode, or here piece by
// piece for a small file), on alternating streams, into the piece's final
// place in one inflated buffer.  A kernel lasts at least as long as its
// slowest lane's serial decode of one block, so successive pieces' kernels
// overlap each other and the remaining uploads instead of running one window
// after another; no carry between windows, one parse at the end.  Pieces,
// end to end on the 30 M-record BAM (profiles/r04/r04z*): 8 / 6 /
// 4 / 3 / 2 pieces 0.227 / 0.211 / 0.192-0.202 / 0.184-0.193 / 0.193 s.
// Streams (round 3, profiles/r03sf_gz_pipeline_ab.txt): 2 / 3 / 4 alike.
#ifndef MC_GZ_PIECE_STREAMS
#define MC_GZ_PIECE_STREAMS 2
#endif
#ifndef MC_GZ_PIECES
#define MC_GZ_PIECES 3                 // pieces per inflated stream (each >= 256 MiB, <= 4 GiB)
#endif
static_assert(MC_GZ_PIECE_STREAMS >= 1 && MC_GZ_PIECE_STREAMS <= 4, "inflate streams: stream + kstream[]");
constexpr int kGzPieceStreams = MC_GZ_PIECE_STREAMS;

// The background upload of a file likely to decode resident: the whole file
// goes up while its blocks are scanned (the upload needs no block list, the
// scan no device); the resident pipeline launches each piece once `progress`
// has passed its bytes.
struct BgUpload {
    std::thread t;
    std::atomic<size_t> progress{0};
    std::atomic<bool> cancel{false}, finished{false};
    int rc = MC_OK;
    std::string msg;
    int join() {   // the upload's status
        if (t.joinable()) t.join();
        if (rc) mc::set_error("%s", msg.c_str());
        return rc;
    }
    ~BgUpload() {
        cancel = true;
        if (t.joinable()) t.join();
    }
};

// Inflate lanes the grid is sized for: kGzLanes per wave, as many waves per
// CU as the kernel's LDS and registers allow on this device (at most
// kGzWavesPerCu, the count for gfx950's 160 KiB of LDS per CU).
int64_t gz_max_lanes(int device) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    int per_cu = kGzWavesPerCu;
    int nb = 0;
    if (MC_GZ_WAVES_PER_CU == 0 &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gz_inflate_kernel, kGzThreads, 0) == hipSuccess && nb > 0)
        per_cu = std::min(per_cu, nb);
    return (int64_t)cus * per_cu * kGzLanes;
}

// The resident decode's device memory (compressed bytes, inflated stream,
// block table, lane scratch; `extra`: more, e.g. a compaction buffer) fits
// in half of `free_b`.
bool resident_fits(size_t comp, size_t total, size_t nblocks, int64_t max_lanes, size_t free_b, size_t extra = 0) {
    const size_t need = comp + total + extra + nblocks * (sizeof(GzBlock) + sizeof(int)) +
                        (size_t)kGzPieceStreams * (size_t)max_lanes * kGzSlotWords * sizeof(uint16_t);
    return need <= free_b / 2;
}

// The pieces' uploads and inflate launches of the resident decode: blocks
// (offsets in the virtual layout of vm, nullptr: the file) inflate into
// dst[0, total); vsize: the virtual bytes (the compressed buffer's size).
int inflate_resident(mc_bam_gpu* g, int fd, const VMap* vm, size_t vsize, const std::vector<Block>& blocks,
                     size_t total, int64_t max_lanes, BgUpload* bg, uint8_t* dst) {
    const int64_t nb = (int64_t)blocks.size();
    hipStream_t st = g->stream;
    const size_t piece = std::min<size_t>(4ull << 30, std::max<size_t>(256ull << 20, total / MC_GZ_PIECES));
    std::vector<std::pair<size_t, size_t>> pcs;
    for (size_t b0 = 0; b0 < blocks.size();) {
        size_t b1 = b0, sz = 0;
        while (b1 < blocks.size() && (b1 == b0 || sz + blocks[b1].isize <= piece)) sz += blocks[b1++].isize;
        pcs.emplace_back(b0, b1);
        b0 = b1;
    }
    HIP_TRY(g->comp[0].reserve(vsize + kPad));
    HIP_TRY(g->hblk.reserve(nb));
    for (int64_t i = 0; i < nb; ++i) {
        const Block& b = blocks[i];
        g->hblk.p[i] = GzBlock{(int64_t)b.cdata, (int64_t)b.out, (int32_t)b.clen, (int32_t)b.isize};
    }
    HIP_TRY(g->blk.reserve(nb));
    HIP_TRY(g->status.reserve(nb + 1));
    const int64_t slot = max_lanes * kGzSlotWords;   // scratch per inflate stream
    HIP_TRY(g->scratch.reserve((size_t)(kGzPieceStreams * slot)));
    HIP_TRY(hipMemcpyAsync(g->blk.p, g->hblk.p, nb * sizeof(GzBlock), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(g->status.p + nb, 0, sizeof(int), st));
    HIP_TRY(hipMemsetAsync(g->comp[0].p + vsize, 0, kPad, st));
    hipStream_t ks[kGzPieceStreams];
    ks[0] = st;
    for (int k = 1; k < kGzPieceStreams; ++k) {
        if (!g->kstream[k - 1]) HIP_TRY(hipStreamCreateWithFlags(&g->kstream[k - 1], hipStreamNonBlocking));
        ks[k] = g->kstream[k - 1];
    }
    hipEvent_t ev[2] = {nullptr, nullptr};
    for (auto& e : ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    struct EvGuard {
        hipEvent_t* e;
        ~EvGuard() {
            for (int i = 0; i < 2; ++i)
                if (e[i]) (void)hipEventDestroy(e[i]);
        }
    } evg{ev};
    HIP_TRY(hipEventRecord(ev[0], st));   // block table, status flag and pad are set
    for (int k = 1; k < kGzPieceStreams; ++k) HIP_TRY(hipStreamWaitEvent(ks[k], ev[0], 0));
    // each launch between two timing events (t_kernel: their durations summed)
    std::vector<hipEvent_t> kev(2 * pcs.size(), nullptr);
    struct KevGuard {
        std::vector<hipEvent_t>& e;
        ~KevGuard() {
            for (auto x : e)
                if (x) (void)hipEventDestroy(x);
        }
    } kevg{kev};
    for (auto& e : kev) HIP_TRY(hipEventCreate(&e));
    double t_first = now_s();
    for (size_t p = 0; p < pcs.size(); ++p) {
        const size_t b0 = pcs[p].first, b1 = pcs[p].second;
        const size_t coff = blocks[b0].off, cend = b1 < blocks.size() ? blocks[b1].off : vsize;
        const double t0 = now_s();
        if (bg) {
            // the background upload has passed the piece (its copies are
            // complete, so the bytes are visible to any stream)
            while (bg->progress.load(std::memory_order_acquire) < cend) {
                if (bg->finished.load(std::memory_order_acquire)) {
                    if (int rc = bg->join()) return rc;
                    MC_REQUIRE(bg->progress.load() >= cend, MC_E_IO, "%s: background upload stopped early",
                               g->path.c_str());
                }
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
        } else {
            // returns once the bytes are on the device (its stream synchronised)
            if (int rc = upload_file_range(g, fd, coff, cend - coff, g->comp[0].p + coff, g->up_stream, nullptr,
                                               nullptr, vm))
                return rc;
        }
        if (p == 0) {
            g->t_read += (now_s() - t0) * 1e3;   // the exposed part: the first piece
            t_first = now_s();
        }
        const int64_t n = (int64_t)(b1 - b0);
        const int64_t lanes = std::min<int64_t>(max_lanes, (n + kGzLanes - 1) / kGzLanes * kGzLanes);
        const int k = (int)(p % kGzPieceStreams);
        HIP_TRY(hipEventRecord(kev[2 * p], ks[k]));
        gz_inflate_kernel<<<(int)(lanes / kGzLanes), kGzThreads, 0, ks[k]>>>(
            g->comp[0].p, g->blk.p + b0, n, dst, g->scratch.p + k * slot, g->status.p + b0,
            g->status.p + nb);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(kev[2 * p + 1], ks[k]));
    }
    for (int k = 1; k < kGzPieceStreams; ++k) {
        HIP_TRY(hipEventRecord(ev[1], ks[k]));
        HIP_TRY(hipStreamWaitEvent(st, ev[1], 0));
    }
    int any = 0;
    HIP_TRY(hipMemcpyAsync(&any, g->status.p + nb, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    g->t_inflate = (now_s() - t_first) * 1e3;
    g->windows = (int64_t)pcs.size();
    for (size_t p = 0; p < pcs.size(); ++p) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, kev[2 * p], kev[2 * p + 1]));
        g->t_kernel += ms;
    }
    if (any) {
        std::vector<int> sv(nb);
        HIP_TRY(hipMemcpy(sv.data(), g->status.p, nb * sizeof(int), hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < nb; ++i)
            if (sv[i]) {
                mc::set_error("BGZF inflate failed in %s (block at file offset %zu: %s)", g->path.c_str(),
                              file_off(vm, blocks[i].off), gz_err_msg(sv[i]));
                return MC_E_IO;
            }
    }
    return MC_OK;
}

// The per-contig table of the record walk, zeroed (n_ref + 1 entries).
int init_ext(mc_bam_gpu* g) {
    if (g->scan_mode || g->reads_mode) return MC_OK;   // (no extents table)
    const size_t m = g->hdr.names.size() + 1;
    HIP_TRY(g->ext.reserve(m));
    HIP_TRY(hipMemsetAsync(g->ext.p, 0, m * sizeof(ExtAcc), g->stream));
    return MC_OK;
}

int gpu_decode_resident(mc_bam_gpu* g, const MappedFile& mf, const std::vector<Block>& blocks, size_t total,
                        int64_t max_lanes, BgUpload* bg) {
    HIP_TRY(g->inflated.reserve(total + 8));
    if (int rc = inflate_resident(g, mf.fd, nullptr, mf.size, blocks, total, max_lanes, bg, g->inflated.p))
        return rc;
    int64_t o = 0;
    bool ok = false;
    if (int rc = header_from_prefix(g, total, &o, &ok)) return rc;
    MC_REQUIRE(ok, MC_E_IO, "%s: no valid BAM header", g->path.c_str());
    if (int rc = init_ext(g)) return rc;
    const double t1 = now_s();
    int64_t consumed = 0;
    if (int rc = parse_window(g, o, (int64_t)total, false, &consumed)) return rc;
    g->t_parse += (now_s() - t1) * 1e3;
    MC_REQUIRE(consumed == (int64_t)total, MC_E_IO, "%s: truncated record at byte %lld of the inflated stream",
               g->path.c_str(), (long long)consumed);
    return MC_OK;
}

int gpu_decode(mc_bam_gpu* g, int64_t window_bytes) {
    const double t_start = now_s();
    MappedFile mf;
    if (int rc = mf.open(g->path.c_str(), false)) return rc;
    std::vector<Block> blocks;
    size_t total = 0;
    // A file likely to decode resident has its first bytes uploaded (the
    // first piece's worth) while the block headers are scanned: the upload
    // needs no block list, the scan no device.  (If the file turns out not to
    // be resident, the windowed decode uploads its windows itself.)
    BgUpload bg;
    // (uploading each piece only after the scan: 0.21 vs 0.17 s, profiles/r04/r04k_e2e.json)
    if (window_bytes <= 0 && mf.size >= (size_t)(256ull << 20)) {
        size_t free_b = 0, tot_b = 0;
        HIP_TRY(hipMemGetInfo(&free_b, &tot_b));
        if (mf.size * 4 <= free_b / 2) {
            HIP_TRY(g->comp[0].reserve(mf.size + kPad));
            bg.t = std::thread([&]() {
                if (hipSetDevice(g->device) != hipSuccess) {
                    bg.rc = MC_E_HIP;
                    bg.msg = "hipSetDevice failed in the upload thread";
                } else {
                    bg.rc = upload_file_range(g, mf.fd, 0, mf.size, g->comp[0].p, g->up_stream, &bg.progress,
                                              &bg.cancel);
                    if (bg.rc) bg.msg = mc::last_error();
                }
                bg.finished.store(true, std::memory_order_release);
            });
        }
    }
    if (int rc = scan_blocks_pread(mf.fd, mf.size, g->nt, g->path.c_str(), blocks, total)) return rc;
    g->t_scan = (now_s() - t_start) * 1e3;
    g->blocks = (int64_t)blocks.size();
    g->inflated_bytes = (int64_t)total;
    g->compressed_bytes = (int64_t)mf.size;
    const size_t win = (size_t)std::max<int64_t>(window_bytes > 0 ? window_bytes : (4ll << 30), 1 << 20);
    hipStream_t st = g->stream;
    hipEvent_t ev[4];
    for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
    struct EvGuard {
        hipEvent_t* e;
        ~EvGuard() {
            for (int i = 0; i < 4; ++i) (void)hipEventDestroy(e[i]);
        }
    } evg{ev};
    const int64_t max_lanes = gz_max_lanes(g->device);
    if (window_bytes <= 0 && !blocks.empty()) {
        // resident when the compressed file, its inflated stream and the
        // scratch take at most half of the device memory free before the
        // decode (the background upload's buffer, already allocated, counts
        // as free: it is the compressed file of `need`)
        size_t free_b = 0, tot_b = 0;
        HIP_TRY(hipMemGetInfo(&free_b, &tot_b));
        if (bg.t.joinable()) free_b += g->comp[0].cap;
        if (resident_fits(mf.size, total, blocks.size(), max_lanes, free_b)) {
            const int rc = gpu_decode_resident(g, mf, blocks, total, max_lanes, bg.t.joinable() ? &bg : nullptr);
            if (rc == MC_OK && bg.t.joinable()) {
                if (int urc = bg.join()) return urc;
            }
            g->blk_list = std::move(blocks);
            g->t_total = (now_s() - t_start) * 1e3;
            return rc;
        }
    }
    if (bg.t.joinable()) {   // not resident after all: the windows upload their own bytes
        bg.cancel = true;
        bg.t.join();
        g->comp[0].release();   // (the windows size their own buffers)
    }
    // windows of blocks (<= win inflated bytes each, at least one block)
    std::vector<std::pair<size_t, size_t>> wins;
    for (size_t b0 = 0; b0 < blocks.size();) {
        size_t b1 = b0, wsize = 0;
        while (b1 < blocks.size() && (b1 == b0 || wsize + blocks[b1].isize <= win)) wsize += blocks[b1++].isize;
        wins.emplace_back(b0, b1);
        b0 = b1;
    }
    MC_REQUIRE(!wins.empty(), MC_E_IO, "%s: no valid BAM header", g->path.c_str());
    auto crange = [&](size_t w, size_t* coff, size_t* clen) {
        *coff = blocks[wins[w].first].off;
        const size_t b1 = wins[w].second;
        *clen = (b1 < blocks.size() ? blocks[b1].off : mf.size) - *coff;
    };
    // window w's compressed bytes into comp[w & 1] on the upload stream (an
    // uploader thread runs it for window w + 1 while window w is inflated)
    struct Upload {
        int rc = MC_OK;
        std::string msg;
        double s = 0;
    };
    auto upload = [&](size_t w, Upload* u) {
        const double t0 = now_s();
        size_t coff, clen;
        crange(w, &coff, &clen);
        auto run = [&]() -> int {
            HIP_TRY(hipSetDevice(g->device));
            DBuf<uint8_t>& c = g->comp[w & 1];
            HIP_TRY(c.reserve(clen + kPad));
            if (int rc = upload_file_range(g, mf.fd, coff, clen, c.p, g->up_stream)) return rc;
            HIP_TRY(hipMemsetAsync(c.p + clen, 0, kPad, g->up_stream));
            HIP_TRY(hipStreamSynchronize(g->up_stream));
            return MC_OK;
        };
        u->rc = run();
        if (u->rc) u->msg = mc::last_error();
        u->s = now_s() - t0;
    };
    // up_next before the joiner: locals die in reverse order, so an early
    // return joins the uploader thread before the Upload it writes is gone
    Upload up_next;
    struct Joiner {
        std::thread t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } uploader;
    size_t carry = 0;
    bool have_header = false;
    int64_t o = 0;
    for (size_t w = 0; w < wins.size(); ++w) {
        const size_t b0 = wins[w].first, b1 = wins[w].second;
        size_t wsize = 0;
        for (size_t b = b0; b < b1; ++b) wsize += blocks[b].isize;
        const bool last = w + 1 == wins.size();
        size_t coff, clen;
        crange(w, &coff, &clen);
        // this window's upload: done now (the first) or by the uploader
        const double t0 = now_s();
        Upload cur;
        if (w == 0) {
            upload(0, &cur);
        } else {
            uploader.t.join();
            cur = up_next;
        }
        if (cur.rc) {
            mc::set_error("%s", cur.msg.c_str());
            return cur.rc;
        }
        g->t_read += (now_s() - t0) * 1e3;   // the part not hidden behind the previous window
        if (!last) {
            up_next = Upload();
            uploader.t = std::thread(upload, w + 1, &up_next);
        }
        uint8_t* comp = g->comp[w & 1].p;
        const int64_t nb = (int64_t)(b1 - b0);
        HIP_TRY(g->hblk.reserve(nb));
        for (int64_t i = 0; i < nb; ++i) {
            const Block& b = blocks[b0 + i];
            g->hblk.p[i] = GzBlock{(int64_t)(b.cdata - coff), (int64_t)(carry + (b.out - blocks[b0].out)),
                                   (int32_t)b.clen, (int32_t)b.isize};
        }
        HIP_TRY(g->blk.reserve(nb));
        HIP_TRY(hipMemcpyAsync(g->blk.p, g->hblk.p, nb * sizeof(GzBlock), hipMemcpyHostToDevice, st));
        // inflated buffer: carry (already at the front) + this window
        const size_t n = carry + wsize;
        if (n + 8 > g->inflated.cap) {
            HIP_TRY(g->tail.reserve(std::max<size_t>(carry, 1)));
            if (carry) HIP_TRY(hipMemcpyAsync(g->tail.p, g->inflated.p, carry, hipMemcpyDeviceToDevice, st));
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(g->inflated.reserve(n + 8));
            if (carry) HIP_TRY(hipMemcpyAsync(g->inflated.p, g->tail.p, carry, hipMemcpyDeviceToDevice, st));
        }
        HIP_TRY(g->status.reserve(nb + 1));
        HIP_TRY(hipMemsetAsync(g->status.p + nb, 0, sizeof(int), st));
        // a multiple of the workgroup: every launched lane owns a scratch slot
        // a multiple of the lanes per workgroup: every launched lane owns a scratch slot
        const int64_t lanes = std::min<int64_t>(max_lanes, (nb + kGzLanes - 1) / kGzLanes * kGzLanes);
        HIP_TRY(g->scratch.reserve((size_t)lanes * kGzSlotWords));
        HIP_TRY(hipEventRecord(ev[0], st));
        gz_inflate_kernel<<<(int)(lanes / kGzLanes), kGzThreads, 0, st>>>(
            comp, g->blk.p, nb, g->inflated.p, g->scratch.p, g->status.p, g->status.p + nb);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(ev[1], st));
        int any = 0;
        HIP_TRY(hipMemcpyAsync(&any, g->status.p + nb, sizeof(int), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, ev[0], ev[1]));
        g->t_inflate += ms;
        g->t_kernel += ms;
        if (any) {
            std::vector<int> s(nb);
            HIP_TRY(hipMemcpy(s.data(), g->status.p, nb * sizeof(int), hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < nb; ++i)
                if (s[i]) {
                    mc::set_error("BGZF inflate failed in %s (block at file offset %zu: %s)", g->path.c_str(),
                                  blocks[b0 + i].off, gz_err_msg(s[i]));
                    return MC_E_IO;
                }
        }
        if (!have_header) {
            // header from a growing prefix of the inflated bytes
            size_t p = std::min<size_t>(n, 1 << 20);
            std::vector<uint8_t> hb;
            for (;;) {
                hb.resize(p);
                HIP_TRY(hipMemcpy(hb.data(), g->inflated.p, p, hipMemcpyDeviceToHost));
                std::vector<std::string> names;
                std::vector<int64_t> lens;
                size_t ho = 0;
                if (parse_header(hb.data(), p, g->path.c_str(), names, lens, &ho) == MC_OK) {
                    g->hdr.names = std::move(names);
                    g->hdr.lens = std::move(lens);
                    o = (int64_t)ho;
                    have_header = true;
                    if (int rc = init_ext(g)) return rc;
                    break;
                }
                if (p >= n) break;
                p = std::min(n, p * 4);
            }
            if (!have_header) {
                // the header continues in the next window: keep everything
                MC_REQUIRE(!last, MC_E_IO, "%s: no valid BAM header", g->path.c_str());
                carry = n;
                ++g->windows;
                continue;
            }
        }
        const double t1 = now_s();
        int64_t consumed = 0;
        if (int rc = parse_window(g, o, (int64_t)n, !last, &consumed, (int64_t)(blocks[b0].out - carry)))
            return rc;
        g->t_parse += (now_s() - t1) * 1e3;
        carry = n - (size_t)consumed;
        if (last) {
            MC_REQUIRE(carry == 0, MC_E_IO, "%s: truncated record at byte %lld of the inflated stream",
                       g->path.c_str(), (long long)consumed);
        } else if (carry) {
            HIP_TRY(g->tail.reserve(carry));
            HIP_TRY(hipMemcpyAsync(g->tail.p, g->inflated.p + consumed, carry, hipMemcpyDeviceToDevice, st));
            HIP_TRY(hipMemcpyAsync(g->inflated.p, g->tail.p, carry, hipMemcpyDeviceToDevice, st));
        }
        o = 0;
        ++g->windows;
    }
    HIP_TRY(hipStreamSynchronize(st));
    g->blk_list = std::move(blocks);
    g->t_total = (now_s() - t_start) * 1e3;
    return MC_OK;
}

// The BAM header through pread of the leading blocks (inflated on the host).
int read_header_pread(int fd, size_t n, const char* path, std::vector<std::string>& names,
                      std::vector<int64_t>& lens) {
    std::vector<uint8_t> buf, blk(65536);
    size_t off = 0;
    for (;;) {
        MC_REQUIRE(off < n, MC_E_IO, "%s: truncated BAM header", path);
        const size_t hn = std::min<size_t>(n - off, blk.size());
        MC_REQUIRE(pread_all(fd, blk.data(), hn, off), MC_E_IO, "%s: read failed", path);
        const size_t b = bgzf_hdr(blk.data(), hn, 0);
        MC_REQUIRE(b, MC_E_IO, "%s: no valid BGZF block at offset %zu", path, off);
        const size_t xlen = rd16(blk.data() + 10), isize = rd32(blk.data() + b - 4);
        const size_t at = buf.size();
        buf.resize(at + isize);
        MC_REQUIRE(isize == 0 || inflate_block(blk.data() + 12 + xlen, b - xlen - 20, buf.data() + at, isize), MC_E_IO,
                   "BGZF inflate failed in %s", path);
        off += b;
        names.clear();
        lens.clear();
        size_t o = 0;
        if (buf.size() >= 12 && parse_header(buf.data(), buf.size(), path, names, lens, &o) == MC_OK) return MC_OK;
        MC_REQUIRE(buf.size() < (size_t(1) << 31), MC_E_IO, "%s: no valid BAM header", path);
    }
}

// Size of the BGZF block at file offset o (0 if none).
size_t block_size_at(int fd, size_t n, size_t o) {
    uint8_t h[96];
    const size_t hn = std::min<size_t>(sizeof h, n - std::min(n, o));
    if (hn < 18 || !pread_all(fd, h, hn, o)) return 0;
    return bgzf_hdr_at(h, hn, o, n);
}

// Block i of `blocks` (file offsets, sorted) in [b0, b1) at file offset off.
int64_t block_at(const std::vector<Block>& blocks, size_t b0, size_t b1, size_t off) {
    auto it = std::lower_bound(blocks.begin() + b0, blocks.begin() + b1, off,
                               [](const Block& b, size_t x) { return b.off < x; });
    return it != blocks.begin() + b1 && it->off == off ? (int64_t)(it - blocks.begin()) : -1;
}

// One rank's contigs (sel) decoded on the GPU from the extents table: only
// the BGZF blocks holding their records are read (the extents' byte ranges,
// back to back in a virtual layout), uploaded and inflated; each contig's
// inflated range [first record, end of the last) is copied into one compact
// record stream, which one parse walks with a tid map (header tid -> local
// id).  The header counts are the whole file's, from the table.
int gpu_decode_extents(mc_bam_gpu* g, int32_t n_ref_in, const mc_contig_extent* ext, int64_t n_no_coor,
                       int32_t n_sel, const int32_t* sel_in) {
    const double t_start = now_s();
    const char* path = g->path.c_str();
    MappedFile mf;
    if (int rc = mf.open(path, false)) return rc;
    if (int rc = read_header_pread(mf.fd, mf.size, path, g->hdr.names, g->hdr.lens)) return rc;
    const int32_t n_ref = (int32_t)g->hdr.names.size();
    MC_REQUIRE(n_ref_in == n_ref, MC_E_INVALID, "%s: the extents table has %d contigs, the BAM header %d", path,
               n_ref_in, n_ref);
    g->subset = true;
    g->sel.assign(sel_in, sel_in + n_sel);
    std::sort(g->sel.begin(), g->sel.end());
    g->sel.erase(std::unique(g->sel.begin(), g->sel.end()), g->sel.end());
    for (int32_t t : g->sel) MC_REQUIRE(t >= 0 && t < n_ref, MC_E_INVALID, "contig %d out of range", t);
    g->ext_in.assign(ext, ext + n_ref);
    g->n_no_coor_in = n_no_coor;
    for (const mc_contig_extent& e : g->ext_in) {
        g->hdr.n_mapped += e.n_mapped;
        g->hdr.n_unmapped += e.n_unmapped;
    }
    g->hdr.n_unmapped += n_no_coor;
    g->hdr.n_records = g->hdr.n_mapped + g->hdr.n_unmapped;
    // the selected contigs with records, in file order, and their file extents
    struct Cr {
        int32_t tid;
        uint64_t beg, end;
        size_t ext = 0;
        int64_t q0 = 0, q1 = 0;
    };
    std::vector<Cr> crs;
    for (int32_t t : g->sel) {
        const mc_contig_extent& e = ext[t];
        if ((uint64_t)e.end_voff <= (uint64_t)e.beg_voff) continue;
        MC_REQUIRE(((uint64_t)e.beg_voff >> 16) < mf.size && ((uint64_t)e.end_voff >> 16) <= mf.size, MC_E_IO,
                   "%s: the extent of contig %d lies outside the file", path, t);
        crs.push_back(Cr{t, (uint64_t)e.beg_voff, (uint64_t)e.end_voff});
    }
    std::sort(crs.begin(), crs.end(), [](const Cr& a, const Cr& b) { return a.beg < b.beg; });
    std::vector<FileExtent> fx;
    for (Cr& c : crs) {
        const size_t a = c.beg >> 16, f = c.end >> 16;
        const bool extra = (c.end & 0xffff) != 0;
        if (!fx.empty() && a <= fx.back().f) {   // shares (or starts at) the previous extent's last block
            FileExtent& b = fx.back();
            if (f > b.f) {
                b.f = f;
                b.extra = extra;
            } else if (f == b.f) {
                b.extra |= extra;
            }
        } else {
            fx.push_back(FileExtent{a, f, extra});
        }
        c.ext = fx.size() - 1;
    }
    // the virtual layout: the extents' bytes back to back
    VMap vm;
    size_t vsize = 0;
    for (const FileExtent& x : fx) {
        size_t e = x.f;
        if (x.extra) {
            const size_t b = block_size_at(mf.fd, mf.size, x.f);
            MC_REQUIRE(b, MC_E_IO, "%s: no valid BGZF block at offset %zu (index offsets do not match the BAM)", path,
                       x.f);
            e += b;
        }
        vm.push_back(VSeg{vsize, x.a, e - x.a});
        vsize += e - x.a;
    }
    // the upload runs beside the block scan
    BgUpload bg;
    if (vsize >= (size_t)(64ull << 20)) {
        size_t free_b = 0, tot_b = 0;
        HIP_TRY(hipMemGetInfo(&free_b, &tot_b));
        if (vsize * 4 <= free_b / 2) {
            HIP_TRY(g->comp[0].reserve(vsize + kPad));
            bg.t = std::thread([&]() {
                if (hipSetDevice(g->device) != hipSuccess) {
                    bg.rc = MC_E_HIP;
                    bg.msg = "hipSetDevice failed in the upload thread";
                } else {
                    bg.rc = upload_file_range(g, mf.fd, 0, vsize, g->comp[0].p, g->up_stream, &bg.progress,
                                              &bg.cancel, &vm);
                    if (bg.rc) bg.msg = mc::last_error();
                }
                bg.finished.store(true, std::memory_order_release);
            });
        }
    }
    std::vector<Block> blocks;
    std::vector<size_t> ex_first;
    size_t total = 0;
    if (int rc = scan_extents_pread(mf.fd, mf.size, g->nt, path, fx, blocks, total, &ex_first)) return rc;
    ex_first.push_back(blocks.size());
    g->t_scan = (now_s() - t_start) * 1e3;
    g->blocks = (int64_t)blocks.size();
    g->inflated_bytes = (int64_t)total;
    g->compressed_bytes = (int64_t)vsize;
    // each contig's range of the inflated stream
    for (Cr& c : crs) {
        const size_t k = c.ext, b0 = ex_first[k], b1 = ex_first[k + 1];
        const int64_t i0 = block_at(blocks, b0, b1, c.beg >> 16);
        MC_REQUIRE(i0 >= 0 && (c.beg & 0xffff) <= blocks[i0].isize, MC_E_IO,
                   "%s: the index's first offset of contig %d does not match the BAM blocks", path, c.tid);
        c.q0 = (int64_t)(blocks[i0].out + (c.beg & 0xffff));
        const int64_t i1 = block_at(blocks, b0, b1, c.end >> 16);
        if (i1 >= 0) {
            MC_REQUIRE((c.end & 0xffff) <= blocks[i1].isize, MC_E_IO,
                       "%s: the index's end offset of contig %d does not match the BAM blocks", path, c.tid);
            c.q1 = (int64_t)(blocks[i1].out + (c.end & 0xffff));
        } else {   // the end is the start of the block after the extent
            MC_REQUIRE((c.end & 0xffff) == 0 && (c.end >> 16) == fx[k].f && b1 > b0, MC_E_IO,
                       "%s: the index's end offset of contig %d does not match the BAM blocks", path, c.tid);
            c.q1 = (int64_t)(blocks[b1 - 1].out + blocks[b1 - 1].isize);
        }
        MC_REQUIRE(c.q0 <= c.q1, MC_E_IO, "%s: contig %d's index offsets are reversed", path, c.tid);
    }
    // blocks into the virtual layout
    for (size_t k = 0; k < fx.size(); ++k)
        for (size_t i = ex_first[k]; i < ex_first[k + 1]; ++i) {
            blocks[i].off = vm[k].v + (blocks[i].off - fx[k].a);
            blocks[i].cdata = vm[k].v + (blocks[i].cdata - fx[k].a);
        }
    // compact ranges (neighbours merged)
    std::vector<std::pair<int64_t, int64_t>> cpy;
    int64_t n_comp = 0;
    for (const Cr& c : crs) {
        if (c.q1 == c.q0) continue;
        if (!cpy.empty() && cpy.back().second == c.q0) cpy.back().second = c.q1;
        else cpy.emplace_back(c.q0, c.q1);
        n_comp += c.q1 - c.q0;
    }
    const int64_t max_lanes = gz_max_lanes(g->device);
    {
        size_t free_b = 0, tot_b = 0;
        HIP_TRY(hipMemGetInfo(&free_b, &tot_b));
        if (bg.t.joinable()) free_b += g->comp[0].cap;
        MC_REQUIRE(resident_fits(vsize, total, blocks.size(), max_lanes, free_b, (size_t)n_comp), MC_E_RANGE,
                   "%s: the selected contigs' %zu inflated bytes do not fit in device memory (decode them on the "
                   "host: mc_bam_open_contigs)", path, total);
    }
    hipStream_t st = g->stream;
    HIP_TRY(g->raw.reserve(total + 8));
    HIP_TRY(g->inflated.reserve((size_t)n_comp + 8));
    if (!blocks.empty()) {
        const int rc = inflate_resident(g, mf.fd, &vm, vsize, blocks, total, max_lanes,
                                        bg.t.joinable() ? &bg : nullptr, g->raw.p);
        if (rc) return rc;
        if (bg.t.joinable())
            if (int urc = bg.join()) return urc;
    }
    int64_t at = 0;
    for (const auto& c : cpy) {
        HIP_TRY(hipMemcpyAsync(g->inflated.p + at, g->raw.p + c.first, c.second - c.first, hipMemcpyDeviceToDevice,
                               st));
        at += c.second - c.first;
    }
    std::vector<int32_t> map(n_ref, -1);
    for (size_t i = 0; i < g->sel.size(); ++i) map[g->sel[i]] = (int32_t)i;
    HIP_TRY(g->tid_map.reserve(std::max<size_t>(1, map.size())));
    if (!map.empty()) HIP_TRY(hipMemcpyAsync(g->tid_map.p, map.data(), map.size() * 4, hipMemcpyHostToDevice, st));
    if (int rc = init_ext(g)) return rc;
    HIP_TRY(hipStreamSynchronize(st));   // (map is a host temporary)
    const int64_t rec = g->hdr.n_records, m = g->hdr.n_mapped, u = g->hdr.n_unmapped;
    if (n_comp > 0) {
        const double t1 = now_s();
        int64_t consumed = 0;
        if (int rc = parse_window(g, 0, n_comp, false, &consumed)) return rc;
        g->t_parse += (now_s() - t1) * 1e3;
        MC_REQUIRE(consumed == n_comp, MC_E_IO, "%s: truncated record at byte %lld of the selected ranges", path,
                   (long long)consumed);
    }
    g->hdr.n_records = rec;   // the whole file's counts, not the parsed ranges'
    g->hdr.n_mapped = m;
    g->hdr.n_unmapped = u;
    g->t_total = (now_s() - t_start) * 1e3;
    return MC_OK;
}

// Virtual offset (bgzf_tell) of inflated-stream offset q of a whole-file
// decode, as the index builder's VoffWalker (bam_index.cpp) and htslib give
// it: inside the first non-empty block that ends at or after q, or, when q
// is that block's end, at the start of the next block (htslib moves on once
// a block is used up; the file's end when there is none).  nz: the indices
// of the non-empty blocks.
uint64_t voff_of(const std::vector<Block>& b, const std::vector<size_t>& nz, size_t q, size_t file_size) {
    auto it = std::partition_point(nz.begin(), nz.end(), [&](size_t k) { return b[k].out + b[k].isize < q; });
    const size_t k = it != nz.end() ? *it : b.size() - 1;
    if (q >= b[k].out && q < b[k].out + b[k].isize) return ((uint64_t)b[k].off << 16) | (uint64_t)(q - b[k].out);
    return k + 1 < b.size() ? (uint64_t)b[k + 1].off << 16 : (uint64_t)file_size << 16;
}

int open_common(const char* path, int device, int n_threads, uint32_t flag_filter,
                std::unique_ptr<mc_bam_gpu>& g) {
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    MC_REQUIRE(device >= 0 && device < ndev, MC_E_INVALID, "no HIP device %d", device);
    HIP_TRY(hipSetDevice(device));
    g.reset(new mc_bam_gpu());
    g->path = path;
    g->device = device;
    g->nt = n_threads > 0 ? n_threads : std::min(16, n_threads_or_all(0));   // file reads only
    g->flag_filter = flag_filter;
    HIP_TRY(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&g->up_stream, hipStreamNonBlocking));
    return MC_OK;
}

}  // namespace

extern "C" int mc_bam_gpu_open(const char* path, int device, int n_threads, uint32_t flag_filter,
                               int64_t window_bytes, mc_bam_gpu** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<mc_bam_gpu> g;
    if (int rc = open_common(path, device, n_threads, flag_filter, g)) return rc;
    const double t0 = now_s();
    if (int rc = gpu_decode(g.get(), window_bytes)) return rc;
    g->t_open = (now_s() - t0) * 1e3;   // total_ms + the mapping's teardown
    // (the staging and parse buffers go with the handle: a hipFree of the
    // multi-GB windows here sat on the open's critical path)
    *out = g.release();
    return MC_OK;
}

extern "C" int mc_bam_gpu_open_scan(const char* path, int device, int n_threads, int64_t window_bytes,
                                    mc_bam_gpu** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<mc_bam_gpu> g;
    if (int rc = open_common(path, device, n_threads, 0, g)) return rc;
    g->scan_mode = true;
    const double t0 = now_s();
    if (int rc = gpu_decode(g.get(), window_bytes)) return rc;
    g->t_open = (now_s() - t0) * 1e3;
    *out = g.release();
    return MC_OK;
}

extern "C" int mc_bam_gpu_scan_device(const mc_bam_gpu* g, int64_t* n, const int32_t** d_rlen,
                                      const int32_t** d_flag, const int32_t** d_gpos, const int32_t** d_gisize,
                                      const int32_t** d_tid, const int64_t** d_seq_off, const uint8_t** d_seq,
                                      int64_t* seq_bytes) {
    MC_REQUIRE(g && n && d_rlen && d_flag && d_gpos && d_gisize && d_tid && d_seq_off && d_seq && seq_bytes,
               MC_E_INVALID, "null argument");
    MC_REQUIRE(g->scan_mode, MC_E_STATE, "not a scan-mode decode (mc_bam_gpu_open_scan)");
    *n = g->n_kept;
    *d_rlen = g->span.p;
    *d_flag = g->sflag.p;
    *d_gpos = g->pos.p;
    *d_gisize = g->sgisize.p;
    *d_tid = g->tid.p;
    *d_seq_off = g->soff.p;
    *d_seq = g->sseq.p;
    *seq_bytes = g->n_bytes;
    return MC_OK;
}

extern "C" int mc_bam_gpu_open_reads(const char* path, int device, int n_threads, int k, int64_t window_bytes,
                                     mc_bam_gpu** out) {
    MC_REQUIRE(path && out, MC_E_INVALID, "null argument");
    MC_REQUIRE(k >= 1 && k <= 16, MC_E_INVALID, "k-mer length %d outside [1, 16]", k);
    *out = nullptr;
    std::unique_ptr<mc_bam_gpu> g;
    if (int rc = open_common(path, device, n_threads, 0, g)) return rc;
    g->reads_mode = true;
    g->reads_k = k;
    const double t0 = now_s();
    if (int rc = gpu_decode(g.get(), window_bytes)) return rc;
    g->t_open = (now_s() - t0) * 1e3;
    *out = g.release();
    return MC_OK;
}

extern "C" int mc_bam_gpu_open_reads_extents(const char* path, int device, int n_threads, int k, int32_t n_ref,
                                             const mc_contig_extent* ext, int64_t n_no_coor, int32_t n_sel,
                                             const int32_t* sel, mc_bam_gpu** out) {
    MC_REQUIRE(path && out && (ext || n_ref == 0) && n_ref >= 0 && n_sel >= 0 && (sel || n_sel == 0) &&
                   n_no_coor >= 0,
               MC_E_INVALID, "bad argument");
    MC_REQUIRE(k >= 1 && k <= 16, MC_E_INVALID, "k-mer length %d outside [1, 16]", k);
    *out = nullptr;
    std::unique_ptr<mc_bam_gpu> g;
    if (int rc = open_common(path, device, n_threads, 0, g)) return rc;
    g->reads_mode = true;
    g->reads_k = k;
    const double t0 = now_s();
    if (int rc = gpu_decode_extents(g.get(), n_ref, ext, n_no_coor, n_sel, sel)) return rc;
    g->t_open = (now_s() - t0) * 1e3;
    *out = g.release();
    return MC_OK;
}

extern "C" int mc_bam_gpu_reads_device(const mc_bam_gpu* g, int64_t* n, const int32_t** d_tid,
                                       const int32_t** d_pos, const int64_t** d_end, const int32_t** d_flag,
                                       const uint8_t** d_bits, const uint32_t** d_kmer, const uint8_t** d_name_len,
                                       const int64_t** d_name_off, const uint8_t** d_names, int64_t* name_bytes) {
    MC_REQUIRE(g && n && d_tid && d_pos && d_end && d_flag && d_bits && d_kmer && d_name_len && d_name_off &&
                   d_names && name_bytes,
               MC_E_INVALID, "null argument");
    MC_REQUIRE(g->reads_mode, MC_E_STATE, "not a reads-mode decode (mc_bam_gpu_open_reads)");
    *n = g->n_kept;
    *d_tid = g->tid.p;
    *d_pos = g->pos.p;
    *d_end = g->rend_pos.p;
    *d_flag = g->sflag.p;
    *d_bits = g->rbits.p;
    *d_kmer = g->rkmer.p;
    *d_name_len = g->rnlen.p;
    *d_name_off = g->soff.p;
    *d_names = g->sseq.p;
    *name_bytes = g->n_bytes;
    return MC_OK;
}

extern "C" int mc_bam_gpu_reads_copy(const mc_bam_gpu* g, int32_t* tid, int32_t* pos, int64_t* end, int32_t* flag,
                                     uint8_t* bits, uint32_t* kmer, uint8_t* name_len, int64_t* name_off,
                                     uint8_t* names) {
    MC_REQUIRE(g && ((tid && pos && end && flag && bits && kmer && name_len && name_off) || !g->n_kept) &&
                   (names || !g->n_bytes),
               MC_E_INVALID, "null argument");   // (an empty table: no buffers needed)
    MC_REQUIRE(g->reads_mode, MC_E_STATE, "not a reads-mode decode (mc_bam_gpu_open_reads)");
    HIP_TRY(hipSetDevice(g->device));
    const size_t n = (size_t)g->n_kept;
    hipStream_t st = g->stream;
    if (n) {
        HIP_TRY(hipMemcpyAsync(tid, g->tid.p, n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(pos, g->pos.p, n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(end, g->rend_pos.p, n * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(flag, g->sflag.p, n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(bits, g->rbits.p, n, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(kmer, g->rkmer.p, n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(name_len, g->rnlen.p, n, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(name_off, g->soff.p, n * 8, hipMemcpyDeviceToHost, st));
    }
    if (g->n_bytes) HIP_TRY(hipMemcpyAsync(names, g->sseq.p, (size_t)g->n_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return MC_OK;
}

extern "C" int mc_bam_gpu_header(const mc_bam_gpu* g, const mc_bam** header) {
    MC_REQUIRE(g && header, MC_E_INVALID, "null argument");
    *header = &g->hdr;
    return MC_OK;
}

extern "C" int mc_bam_gpu_intervals_device(const mc_bam_gpu* g, int64_t* n, const int32_t** d_tid,
                                           const int32_t** d_pos, const int32_t** d_span) {
    MC_REQUIRE(g && n && d_tid && d_pos && d_span, MC_E_INVALID, "null argument");
    *n = g->n_kept;
    *d_tid = g->tid.p;
    *d_pos = g->pos.p;
    *d_span = g->span.p;
    return MC_OK;
}

extern "C" int mc_bam_gpu_intervals(const mc_bam_gpu* g, int32_t* tid, int32_t* pos, int32_t* span) {
    MC_REQUIRE(g && tid && pos && span, MC_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(g->device));
    if (g->n_kept) {
        HIP_TRY(hipMemcpy(tid, g->tid.p, g->n_kept * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(pos, g->pos.p, g->n_kept * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(span, g->span.p, g->n_kept * 4, hipMemcpyDeviceToHost));
    }
    return MC_OK;
}

extern "C" int mc_bam_gpu_stats(const mc_bam_gpu* g, mc_bam_gpu_timings* t) {
    MC_REQUIRE(g && t, MC_E_INVALID, "null argument");
    t->read_ms = g->t_read;
    t->inflate_ms = g->t_inflate;
    t->parse_ms = g->t_parse;
    t->total_ms = g->t_total;
    t->windows = g->windows;
    t->blocks = g->blocks;
    t->resyncs = g->resyncs;
    t->compressed_bytes = g->compressed_bytes;
    t->inflated_bytes = g->inflated_bytes;
    t->scan_ms = g->t_scan;
    t->upload_ms = g->t_upload;
    t->kernel_ms = g->t_kernel;
    t->open_ms = g->t_open;
    t->parse_rounds = g->parse_rounds;
    t->resync_passes = g->resync_passes;
    return MC_OK;
}

extern "C" int mc_bam_gpu_close(mc_bam_gpu* g) {
    delete g;
    return MC_OK;
}

extern "C" int mc_bam_gpu_trim(mc_bam_gpu* g, int64_t* freed) {
    MC_REQUIRE(g, MC_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(g->device));
    for (hipStream_t s : {g->stream, g->up_stream, g->kstream[0], g->kstream[1], g->kstream[2]})
        if (s) HIP_TRY(hipStreamSynchronize(s));
    int64_t bytes = 0;
    auto drop = [&](auto& b) {
        bytes += (int64_t)(b.cap * sizeof(*b.p));
        b.release();
    };
    // the decode's staging: compressed bytes, inflated stream, raw blocks,
    // block / segment tables, scan-mode fill offsets; the results (the kept
    // intervals, reads / scan columns, the per-contig table) stay
    drop(g->comp[0]);
    drop(g->comp[1]);
    drop(g->inflated);
    drop(g->tail);
    drop(g->raw);
    drop(g->blk);
    drop(g->status);
    drop(g->scratch);
    drop(g->seg_off);
    drop(g->found);
    drop(g->out_off);
    drop(g->res);
    drop(g->boff);
    if (freed) *freed = bytes;
    return MC_OK;
}

extern "C" int mc_bam_gpu_open_extents(const char* path, int device, int n_threads, uint32_t flag_filter,
                                       int32_t n_ref, const mc_contig_extent* ext, int64_t n_no_coor, int32_t n_sel,
                                       const int32_t* sel, mc_bam_gpu** out) {
    MC_REQUIRE(path && out && (ext || n_ref == 0) && n_ref >= 0 && n_sel >= 0 && (sel || n_sel == 0) &&
                   n_no_coor >= 0,
               MC_E_INVALID, "bad argument");
    *out = nullptr;
    std::unique_ptr<mc_bam_gpu> g;
    if (int rc = open_common(path, device, n_threads, flag_filter, g)) return rc;
    const double t0 = now_s();
    if (int rc = gpu_decode_extents(g.get(), n_ref, ext, n_no_coor, n_sel, sel)) return rc;
    g->t_open = (now_s() - t0) * 1e3;
    *out = g.release();
    return MC_OK;
}

extern "C" int mc_bam_gpu_open_contigs(const char* path, const char* bai_path, int device, int n_threads,
                                       uint32_t flag_filter, int32_t n_sel, const int32_t* sel, mc_bam_gpu** out) {
    MC_REQUIRE(path && out && n_sel >= 0 && (sel || n_sel == 0), MC_E_INVALID, "bad argument");
    *out = nullptr;
    int n_ref = 0;
    {
        MappedFile mf;
        if (int rc = mf.open(path, false)) return rc;
        std::vector<std::string> names;
        std::vector<int64_t> lens;
        if (int rc = read_header_pread(mf.fd, mf.size, path, names, lens)) return rc;
        n_ref = (int)names.size();
    }
    const std::string bai = bai_path && *bai_path ? std::string(bai_path) : std::string(path) + ".bai";
    std::vector<mc_contig_extent> ext((size_t)n_ref);
    int64_t n_no_coor = 0;
    if (int rc = mc_bam_index_extents(bai.c_str(), n_ref, ext.data(), &n_no_coor)) return rc;
    return mc_bam_gpu_open_extents(path, device, n_threads, flag_filter, n_ref, ext.data(), n_no_coor, n_sel, sel,
                                   out);
}

extern "C" int mc_bam_gpu_extents(const mc_bam_gpu* g, int32_t n_ref, mc_contig_extent* ext, int64_t* n_no_coor) {
    MC_REQUIRE(g && (ext || n_ref == 0) && n_no_coor, MC_E_INVALID, "null argument");
    MC_REQUIRE(n_ref == (int32_t)g->hdr.names.size(), MC_E_INVALID, "the file has %zu contigs, not %d",
               g->hdr.names.size(), n_ref);
    HIP_TRY(hipSetDevice(g->device));
    std::vector<ExtAcc> acc((size_t)n_ref + 1);
    if (g->ext.p) HIP_TRY(hipMemcpy(acc.data(), g->ext.p, acc.size() * sizeof(ExtAcc), hipMemcpyDeviceToHost));
    if (g->subset) {
        for (int32_t t = 0; t < n_ref; ++t) {
            ext[t] = g->ext_in[t];
            ext[t].n_kept = std::binary_search(g->sel.begin(), g->sel.end(), t) ? (int64_t)acc[t].kept : 0;
        }
        *n_no_coor = g->n_no_coor_in;
        return MC_OK;
    }
    std::vector<std::pair<uint64_t, uint64_t>> spans;   // (first, end) stream offsets of contigs with records
    std::vector<size_t> nz;
    for (size_t k = 0; k < g->blk_list.size(); ++k)
        if (g->blk_list[k].isize) nz.push_back(k);
    for (int32_t t = 0; t < n_ref; ++t) {
        const ExtAcc& a = acc[t];
        mc_contig_extent& e = ext[t];
        e.n_mapped = (int64_t)a.mapped;
        e.n_unmapped = (int64_t)a.unmapped;
        e.n_kept = (int64_t)a.kept;
        e.beg_voff = e.end_voff = 0;
        if (a.nfirst == 0) continue;
        const uint64_t q0 = ~a.nfirst, q1 = a.end;
        spans.emplace_back(q0, q1);
        e.beg_voff = (int64_t)voff_of(g->blk_list, nz, (size_t)q0, (size_t)g->compressed_bytes);
        e.end_voff = (int64_t)voff_of(g->blk_list, nz, (size_t)q1, (size_t)g->compressed_bytes);
    }
    std::sort(spans.begin(), spans.end());
    for (size_t i = 1; i < spans.size(); ++i)
        MC_REQUIRE(spans[i - 1].second <= spans[i].first, MC_E_INVALID,
                   "%s: a contig's records are not contiguous (the BAM is not coordinate-sorted)", g->path.c_str());
    const ExtAcc& nc = acc[n_ref];
    if (nc.nfirst && !spans.empty())
        MC_REQUIRE(spans.back().second <= ~nc.nfirst, MC_E_INVALID,
                   "%s: records without coordinates are not all at the end of the file", g->path.c_str());
    *n_no_coor = (int64_t)(nc.mapped + nc.unmapped);
    return MC_OK;
}

extern "C" int mc_bam_gpu_restrict(mc_bam_gpu* g, int32_t n_sel, const int32_t* sel) {
    MC_REQUIRE(g && n_sel >= 0 && (sel || n_sel == 0), MC_E_INVALID, "bad argument");
    MC_REQUIRE(!g->subset, MC_E_STATE, "the handle already holds a contig subset");
    const int32_t n_ref = (int32_t)g->hdr.names.size();
    std::vector<mc_contig_extent> ext((size_t)n_ref);
    int64_t n_no_coor = 0;
    if (int rc = mc_bam_gpu_extents(g, n_ref, ext.data(), &n_no_coor)) return rc;   // (checks contiguity)
    std::vector<int32_t> keep(sel, sel + n_sel);
    std::sort(keep.begin(), keep.end());
    keep.erase(std::unique(keep.begin(), keep.end()), keep.end());
    for (int32_t t : keep) MC_REQUIRE(t >= 0 && t < n_ref, MC_E_INVALID, "contig %d out of range", t);
    // each contig's slice of the kept intervals (file order = order of first offsets)
    std::vector<int32_t> order;
    for (int32_t t = 0; t < n_ref; ++t)
        if (ext[t].n_kept) order.push_back(t);
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return ext[a].beg_voff < ext[b].beg_voff; });
    std::vector<int64_t> first((size_t)n_ref, 0);
    int64_t at = 0;
    for (int32_t t : order) {
        first[t] = at;
        at += ext[t].n_kept;
    }
    MC_REQUIRE(at == g->n_kept, MC_E_STATE, "kept counts per contig (%lld) differ from the kept records (%lld)",
               (long long)at, (long long)g->n_kept);
    std::vector<int32_t> picked;   // selected contigs with records, in file order
    for (int32_t t : order)
        if (std::binary_search(keep.begin(), keep.end(), t)) picked.push_back(t);
    int64_t n = 0;
    for (int32_t t : picked) n += ext[t].n_kept;
    HIP_TRY(hipSetDevice(g->device));
    hipStream_t st = g->stream;
    DBuf<int32_t> tid, pos, span;
    HIP_TRY(tid.reserve((size_t)n + 4));
    HIP_TRY(pos.reserve((size_t)n + 4));
    HIP_TRY(span.reserve((size_t)n + 4));
    int64_t w = 0;
    for (int32_t t : picked) {
        const int64_t k = ext[t].n_kept, f = first[t];
        const int32_t local = (int32_t)(std::lower_bound(keep.begin(), keep.end(), t) - keep.begin());
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(tid.p + w), local, (size_t)k, st));
        HIP_TRY(hipMemcpyAsync(pos.p + w, g->pos.p + f, k * 4, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemcpyAsync(span.p + w, g->span.p + f, k * 4, hipMemcpyDeviceToDevice, st));
        w += k;
    }
    HIP_TRY(hipStreamSynchronize(st));
    std::swap(g->tid.p, tid.p);
    std::swap(g->tid.cap, tid.cap);
    std::swap(g->pos.p, pos.p);
    std::swap(g->pos.cap, pos.cap);
    std::swap(g->span.p, span.p);
    std::swap(g->span.cap, span.cap);
    g->n_kept = n;
    // the per-contig table keeps the whole file's extents; kept counts only for the subset
    g->subset = true;
    g->sel = keep;
    g->ext_in = ext;
    for (mc_contig_extent& e : g->ext_in) e.n_kept = 0;
    g->n_no_coor_in = n_no_coor;
    return MC_OK;
}

extern "C" int mc_bam_gpu_intervals_range(const mc_bam_gpu* g, int64_t first, int64_t count, int32_t* tid,
                                          int32_t* pos, int32_t* span) {
    MC_REQUIRE(g && tid && pos && span, MC_E_INVALID, "null argument");
    MC_REQUIRE(first >= 0 && count >= 0 && first + count <= g->n_kept, MC_E_RANGE,
               "intervals [%lld, %lld) outside the %lld kept", (long long)first, (long long)(first + count),
               (long long)g->n_kept);
    HIP_TRY(hipSetDevice(g->device));
    if (count) {
        HIP_TRY(hipMemcpy(tid, g->tid.p + first, count * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(pos, g->pos.p + first, count * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(span, g->span.p + first, count * 4, hipMemcpyDeviceToHost));
    }
    return MC_OK;
}

// The lane decoder of gz_inflate_kernel run on the host (unit tests: the
// same inflate.h code against zlib without a GPU).  Not a product path.
extern "C" int mc_gz_inflate_host(const uint8_t* src, int64_t clen, uint8_t* dst, int64_t isize) {
    MC_REQUIRE(src && dst && clen >= 0 && isize >= 0, MC_E_INVALID, "bad argument");
    std::vector<uint8_t> padded((size_t)clen + kPad + 32, 0);
    std::memcpy(padded.data(), src, (size_t)clen);
    std::vector<uint16_t> scratch(mc::gz::kScratchWords + kGzLdsWords);
    uint16_t* TL = scratch.data() + mc::gz::kScratchWords;
    uint8_t* SL = reinterpret_cast<uint8_t*>(TL + mc::gz::kPrimaryWords);
    uint32_t ring[mc::gz::kRingWords];
    uint64_t queue[mc::gz::kQueue];
    const int rc = mc::gz::inflate_block(padded.data(), clen, dst, isize, scratch.data(), TL,
                                         TL + (1 << mc::gz::kLitBits), SL, SL + mc::gz::kLitSyms, ring, queue);
    MC_REQUIRE(rc == 0, MC_E_IO, "inflate failed: %s", gz_err_msg(rc));
    return MC_OK;
}

// The GPU decode's BGZF block scan on the host (unit tests): block count,
// inflated total and up to cap block offsets.
extern "C" int mc_bgzf_scan_host(const char* path, int n_threads, int64_t* n_blocks, int64_t* inflated,
                                 int64_t* offsets, int64_t cap) {
    MC_REQUIRE(path && n_blocks && inflated && cap >= 0 && (offsets || cap == 0), MC_E_INVALID, "bad argument");
    MappedFile f;
    if (int rc = f.open(path, false)) return rc;
    std::vector<Block> blocks;
    size_t total = 0;
    if (int rc = scan_blocks_pread(f.fd, f.size, std::max(1, n_threads), path, blocks, total)) return rc;
    *n_blocks = (int64_t)blocks.size();
    *inflated = (int64_t)total;
    for (int64_t i = 0; i < std::min<int64_t>(cap, (int64_t)blocks.size()); ++i) offsets[i] = (int64_t)blocks[i].off;
    return MC_OK;
}

// rec_chain on the host: q of d[0, n) starts `chain` plausible records in
// sort order (the record sync's rule; unit tests)
extern "C" int mc_bam_rec_chain_host(const uint8_t* d, int64_t n, int64_t q, int32_t n_ref, int chain) {
    MC_REQUIRE(d && n >= 0 && q >= 0 && chain >= 1, MC_E_INVALID, "bad argument");
    return mc::gz::rec_chain(d, q, n, n_ref, chain) ? 1 : 0;
}

// rec_parse on the host for one record body (unit tests)
extern "C" int mc_bam_rec_parse_host(const uint8_t* r, int64_t len, int32_t n_ref, uint32_t flag_filter,
                                     int32_t* out3) {
    MC_REQUIRE(r && out3 && len >= 32, MC_E_INVALID, "bad argument");
    mc::gz::RecOut ro{};
    const int rc = mc::gz::rec_parse(r, r + len, n_ref, flag_filter, ro);
    out3[0] = ro.tid;
    out3[1] = ro.pos;
    out3[2] = ro.span;
    return rc;
}
