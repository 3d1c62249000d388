// BAI index: build (the role of `samtools index`, which the reference needs
// before `metacov pileup`: pysam's AlignmentFile.pileup(ref, start, end) at
// metacov/pileup.py:13 is an indexed region query) and use it to decode only
// the records of chosen contigs (one rank's LPT shard: SURVEY.md §8e).
//
// The index follows htslib's hts_idx_push / hts_idx_finish for BAM
// (min_shift 14, 5 levels): record chunks per bin with the virtual offsets
// bgzf_tell reports, the 16 kbp linear index, the per-reference pseudo-bin
// 37450 {(first record, end), (mapped, unmapped)} and the trailing count of
// records without coordinates.  Bins are written in ascending order (htslib
// writes them in hash order; readers do not care).
#include <cstdio>
#include <map>
#include <memory>

#include "bgzf.h"

using namespace mc::bgzf;

namespace {

constexpr int kMinShift = 14, kLevels = 5;
constexpr uint32_t kNBins = ((1u << 18) - 1) / 7;   // 37449
constexpr uint32_t kMetaBin = kNBins + 1;            // 37450
constexpr uint64_t kMinMarkerDist = 0x10000;
constexpr uint64_t kUnset = ~uint64_t(0);

typedef std::pair<uint64_t, uint64_t> Chunk;

struct RefIndex {
    std::map<uint32_t, std::vector<Chunk>> bins;
    std::vector<uint64_t> lin;
    bool seen = false;
};

int reg2bin(int64_t beg, int64_t end) {   // hts_reg2bin
    int s = kMinShift, t = ((1 << (kLevels * 3)) - 1) / 7;
    --end;
    for (int l = kLevels; l > 0; --l, s += 3, t -= 1 << (l * 3)) {
        if (beg >> s == end >> s) return t + (int)(beg >> s);
    }
    return 0;
}

uint32_t bin_first(int l) { return ((1u << (l * 3)) - 1) / 7; }

// Virtual offset (bgzf_tell) of inflated-stream position q, walking forward:
// k is the block holding byte q - 1; at the exact end of a block the offset is
// the next block's start (htslib moves block_address once a block is used up).
struct VoffWalker {
    const std::vector<Block>& b;
    size_t k = 0;
    explicit VoffWalker(const std::vector<Block>& blocks) : b(blocks) {}
    uint64_t at(size_t q) {
        while (k + 1 < b.size() && (b[k].isize == 0 || b[k].out + b[k].isize < q)) ++k;
        const Block& x = b[k];
        if (q < x.out + x.isize) return ((uint64_t)x.off << 16) | (uint64_t)(q - x.out);
        return k + 1 < b.size() ? (uint64_t)b[k + 1].off << 16 : kUnset;
    }
};

struct Builder {   // hts_idx_t's z state
    std::vector<RefIndex> refs;
    uint64_t n_no_coor = 0;
    int64_t last_tid = -2, save_tid = -1;
    uint32_t last_bin = 0xffffffffu, save_bin = 0xffffffffu;
    int64_t last_coor = -1;
    uint64_t last_off, save_off, off_beg, off_end;
    uint64_t n_mapped = 0, n_unmapped = 0;
    bool first_tid = true;

    Builder(size_t n_ref, uint64_t off0)
        : refs(n_ref), last_off(off0), save_off(off0), off_beg(off0), off_end(off0) {}

    void insert_b(int64_t tid, uint32_t bin, uint64_t u, uint64_t v) {
        refs[tid].bins[bin].push_back(Chunk(u, v));
    }
    void insert_l(int64_t tid, int64_t beg, int64_t end, uint64_t off) {
        std::vector<uint64_t>& l = refs[tid].lin;
        const int64_t b = beg >> kMinShift, e = (end - 1) >> kMinShift;
        if ((int64_t)l.size() < e + 1) l.resize(e + 1, kUnset);
        for (int64_t i = b; i <= e; ++i)
            if (l[i] == kUnset) l[i] = off;
    }
    int push(int64_t tid, int64_t beg, int64_t end, uint64_t offset, bool mapped) {
        if (tid < 0) beg = -1, end = 0;
        if (first_tid || last_tid != tid || (last_tid >= 0 && tid < 0)) {   // change of chromosome
            MC_REQUIRE(!(tid >= 0 && n_no_coor), MC_E_INVALID,
                       "records without coordinates are not all at the end of the file");
            MC_REQUIRE(!(tid >= 0 && refs[tid].seen), MC_E_INVALID,
                       "BAM is not coordinate-sorted (reference %lld appears twice)", (long long)tid);
            last_tid = tid;
            last_bin = 0xffffffffu;
            first_tid = false;
        } else if (tid >= 0 && last_coor > beg) {
            MC_REQUIRE(false, MC_E_INVALID, "BAM is not coordinate-sorted (reference %lld, position %lld)",
                       (long long)tid, (long long)beg);
        }
        if (tid >= 0) {
            refs[tid].seen = true;
            if (mapped) {
                if (beg < 0) beg = 0;
                if (end <= 0) end = 1;
                insert_l(tid, beg, end, last_off);   // last_off = start of this record
            }
        } else {
            ++n_no_coor;
        }
        const uint32_t bin = (uint32_t)reg2bin(beg, end);
        if (last_bin != bin) {
            if (save_bin != 0xffffffffu) insert_b(save_tid, save_bin, save_off, last_off);
            if (last_bin == 0xffffffffu && save_bin != 0xffffffffu) {   // chromosome changed
                off_end = last_off;
                insert_b(save_tid, kMetaBin, off_beg, off_end);
                insert_b(save_tid, kMetaBin, n_mapped, n_unmapped);
                n_mapped = n_unmapped = 0;
                off_beg = off_end;
            }
            save_off = last_off;
            save_bin = last_bin = bin;
            save_tid = tid;
        }
        if (mapped) ++n_mapped;
        else ++n_unmapped;
        last_off = offset;
        last_coor = beg;
        return MC_OK;
    }
    void finish(uint64_t final_offset) {
        if (save_tid >= 0) {
            insert_b(save_tid, save_bin, save_off, final_offset);
            insert_b(save_tid, kMetaBin, off_beg, final_offset);
            insert_b(save_tid, kMetaBin, n_mapped, n_unmapped);
        }
        for (RefIndex& r : refs) {
            // linear index: leading gaps take the reference's first offset,
            // later gaps the previous window's (update_loff)
            auto meta = r.bins.find(kMetaBin);
            const uint64_t off0 = meta != r.bins.end() ? meta->second[0].first : 0;
            size_t l = 0;
            for (; l < r.lin.size() && r.lin[l] == kUnset; ++l) r.lin[l] = off0;
            for (; l < r.lin.size(); ++l)
                if (r.lin[l] == kUnset) r.lin[l] = r.lin[l - 1];
            // compress_binning: fold small bins into their parent, then merge
            // chunks that start in the block where the previous one ends
            for (int lv = kLevels; lv > 0; --lv) {
                const uint32_t start = bin_first(lv);
                for (auto it = r.bins.begin(); it != r.bins.end();) {
                    const uint32_t key = it->first;
                    if (key >= kNBins || key < start) {
                        ++it;
                        continue;
                    }
                    std::vector<Chunk>& p = it->second;
                    if (lv < kLevels && p.size() > 1) std::sort(p.begin(), p.end());
                    if ((p.back().second >> 16) - (p.front().first >> 16) < kMinMarkerDist) {
                        auto par = r.bins.find((key - 1) >> 3);
                        if (par == r.bins.end()) {
                            ++it;
                            continue;
                        }
                        par->second.insert(par->second.end(), p.begin(), p.end());
                        it = r.bins.erase(it);
                        continue;
                    }
                    ++it;
                }
            }
            for (auto& kv : r.bins) {
                if (kv.first >= kNBins) continue;
                std::vector<Chunk>& p = kv.second;
                std::sort(p.begin(), p.end());
                size_t m = 0;
                for (size_t i = 1; i < p.size(); ++i) {
                    if ((p[m].second >> 16) >= (p[i].first >> 16)) {
                        if (p[m].second < p[i].second) p[m].second = p[i].second;
                    } else {
                        p[++m] = p[i];
                    }
                }
                p.resize(m + 1);
            }
        }
    }
};

void put32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
void put64(std::string& s, uint64_t v) { s.append(reinterpret_cast<const char*>(&v), 8); }

// A parsed .bai: per reference, the pseudo-bin (first / end virtual offsets,
// mapped / unmapped counts) and the overall chunk extent.
struct Bai {
    struct Ref {
        bool has_meta = false, has_bins = false;
        uint64_t beg = kUnset, end = 0, n_mapped = 0, n_unmapped = 0;
    };
    std::vector<Ref> refs;
    uint64_t n_no_coor = 0;
};

int read_bai(const char* path, Bai& out) {
    MappedFile mf;
    if (int rc = mf.open(path)) return rc;
    const uint8_t* d = mf.data;
    const size_t n = mf.size;
    MC_REQUIRE(n >= 8 && std::memcmp(d, "BAI\1", 4) == 0, MC_E_IO, "%s: not a BAI index", path);
    size_t o = 4;
    const int32_t n_ref = rdi32(d + o);
    o += 4;
    MC_REQUIRE(n_ref >= 0, MC_E_IO, "%s: bad n_ref", path);
    out.refs.assign(n_ref, Bai::Ref());
    for (int32_t t = 0; t < n_ref; ++t) {
        Bai::Ref& r = out.refs[t];
        MC_REQUIRE(o + 4 <= n, MC_E_IO, "%s: truncated", path);
        const int32_t n_bin = rdi32(d + o);
        o += 4;
        for (int32_t b = 0; b < n_bin; ++b) {
            MC_REQUIRE(o + 8 <= n, MC_E_IO, "%s: truncated", path);
            const uint32_t bin = rd32(d + o);
            const int32_t n_chunk = rdi32(d + o + 4);
            o += 8;
            MC_REQUIRE(n_chunk >= 0 && o + 16 * (size_t)n_chunk <= n, MC_E_IO, "%s: truncated", path);
            if (bin == kMetaBin && n_chunk == 2) {
                r.has_meta = true;
                r.beg = rd64(d + o);
                r.end = rd64(d + o + 8);
                r.n_mapped = rd64(d + o + 16);
                r.n_unmapped = rd64(d + o + 24);
            } else if (n_chunk > 0 && !r.has_meta) {
                r.has_bins = true;
                for (int32_t c = 0; c < n_chunk; ++c) {
                    r.beg = std::min(r.beg, rd64(d + o + 16 * c));
                    r.end = std::max(r.end, rd64(d + o + 16 * c + 8));
                }
            }
            o += 16 * (size_t)n_chunk;
        }
        MC_REQUIRE(o + 4 <= n, MC_E_IO, "%s: truncated", path);
        const int32_t n_intv = rdi32(d + o);
        o += 4 + 8 * (size_t)std::max(0, n_intv);
        MC_REQUIRE(o <= n, MC_E_IO, "%s: truncated linear index", path);
    }
    if (o + 8 <= n) out.n_no_coor = rd64(d + o);
    return MC_OK;
}

std::string bai_path_for(const char* bam_path, const char* bai_path) {
    return bai_path && *bai_path ? std::string(bai_path) : std::string(bam_path) + ".bai";
}

}  // namespace

extern "C" int mc_bam_index_build(const char* bam_path, const char* bai_path, int n_threads) {
    MC_REQUIRE(bam_path, MC_E_INVALID, "null path");
    MappedFile mf;
    if (int rc = mf.open(bam_path)) return rc;
    std::vector<Block> blocks;
    size_t total = 0;
    if (int rc = scan_blocks(mf.data, mf.size, 0, SIZE_MAX, blocks, total)) return rc;
    std::unique_ptr<uint8_t[]> buf(new (std::nothrow) uint8_t[total + 8]);
    MC_REQUIRE(buf, MC_E_IO, "cannot allocate %zu bytes for %s", total, bam_path);
    MC_REQUIRE(inflate_blocks(mf.data, blocks, buf.get(), n_threads_or_all(n_threads)), MC_E_IO,
               "BGZF inflate failed in %s", bam_path);
    const uint8_t* d = buf.get();
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    size_t q = 0;
    if (int rc = parse_header(d, total, bam_path, names, lens, &q)) return rc;
    const int64_t n_ref = (int64_t)names.size();
    VoffWalker vw(blocks);
    Builder ix((size_t)n_ref, vw.at(q));
    while (q < total) {
        MC_REQUIRE(q + 4 <= total, MC_E_IO, "%s: truncated record at byte %zu", bam_path, q);
        const int32_t bs = rdi32(d + q);
        MC_REQUIRE(bs >= 32 && q + 4 + (size_t)bs <= total, MC_E_IO,
                   "%s: bad record size at byte %zu", bam_path, q);
        const uint8_t* r = d + q + 4;
        const uint8_t* rend = r + bs;
        q += 4 + (size_t)bs;
        const int32_t tid = rdi32(r), pos = rdi32(r + 4);
        const uint16_t flag = rd16(r + 14);
        MC_REQUIRE(tid >= -1 && tid < n_ref, MC_E_IO, "%s: record tid %d out of range", bam_path, tid);
        int64_t rlen = 0;
        if (!(flag & 4)) {   // bam_endpos: unmapped or no reference-consuming op -> pos + 1
            const uint8_t* cig;
            uint32_t n_cigar;
            MC_REQUIRE(cigar_of(r, rend, &cig, &n_cigar), MC_E_IO, "%s: CIGAR overruns record",
                       bam_path);
            rlen = cigar_rlen(cig, n_cigar);
        }
        if (rlen <= 0) rlen = 1;
        if (int rc = ix.push(tid, pos, (int64_t)pos + rlen, vw.at(q), !(flag & 4))) return rc;
    }
    ix.finish(vw.at(total));
    std::string s("BAI\1", 4);
    put32(s, (uint32_t)n_ref);
    for (const RefIndex& r : ix.refs) {
        put32(s, (uint32_t)r.bins.size());
        for (const auto& kv : r.bins) {
            put32(s, kv.first);
            put32(s, (uint32_t)kv.second.size());
            for (const Chunk& c : kv.second) {
                put64(s, c.first);
                put64(s, c.second);
            }
        }
        put32(s, (uint32_t)r.lin.size());
        for (uint64_t v : r.lin) put64(s, v);
    }
    put64(s, ix.n_no_coor);
    const std::string out = bai_path_for(bam_path, bai_path);
    FILE* f = std::fopen(out.c_str(), "wb");
    MC_REQUIRE(f, MC_E_IO, "cannot write %s", out.c_str());
    const bool ok = std::fwrite(s.data(), 1, s.size(), f) == s.size();
    MC_REQUIRE(std::fclose(f) == 0 && ok, MC_E_IO, "write to %s failed", out.c_str());
    return MC_OK;
}

extern "C" int mc_bam_index_stats(const char* bai_path, int32_t n_ref, int64_t* n_mapped,
                                  int64_t* n_unmapped, int64_t* n_no_coor) {
    MC_REQUIRE(bai_path && n_mapped && n_unmapped && n_no_coor, MC_E_INVALID, "null argument");
    Bai bai;
    if (int rc = read_bai(bai_path, bai)) return rc;
    MC_REQUIRE((int32_t)bai.refs.size() == n_ref, MC_E_INVALID,
               "%s indexes %zu references, expected %d", bai_path, bai.refs.size(), n_ref);
    for (int32_t t = 0; t < n_ref; ++t) {
        n_mapped[t] = (int64_t)bai.refs[t].n_mapped;
        n_unmapped[t] = (int64_t)bai.refs[t].n_unmapped;
    }
    *n_no_coor = (int64_t)bai.n_no_coor;
    return MC_OK;
}

extern "C" int mc_bam_index_extents(const char* bai_path, int32_t n_ref, mc_contig_extent* ext,
                                    int64_t* n_no_coor) {
    MC_REQUIRE(bai_path && (ext || n_ref == 0) && n_no_coor && n_ref >= 0, MC_E_INVALID, "bad argument");
    Bai bai;
    if (int rc = read_bai(bai_path, bai)) return rc;
    MC_REQUIRE((int32_t)bai.refs.size() == n_ref, MC_E_INVALID,
               "%s indexes %zu references, the BAM header has %d", bai_path, bai.refs.size(), n_ref);
    for (int32_t t = 0; t < n_ref; ++t) {
        const Bai::Ref& r = bai.refs[t];
        const bool has = (r.has_meta || r.has_bins) && r.end > r.beg;
        ext[t].beg_voff = has ? (int64_t)r.beg : 0;
        ext[t].end_voff = has ? (int64_t)r.end : 0;
        ext[t].n_mapped = (int64_t)r.n_mapped;
        ext[t].n_unmapped = (int64_t)r.n_unmapped;
        ext[t].n_kept = 0;
    }
    *n_no_coor = (int64_t)bai.n_no_coor;
    return MC_OK;
}

extern "C" int mc_bam_open_contigs(const char* path, const char* bai_path, int n_threads,
                                   uint32_t flag_filter, int keep_cigar, int32_t n_sel,
                                   const int32_t* sel, mc_bam** out) {
    MC_REQUIRE(path && out && (n_sel == 0 || sel) && n_sel >= 0, MC_E_INVALID, "bad argument");
    *out = nullptr;
    MappedFile mf;
    if (int rc = mf.open(path)) return rc;
    const std::string bp = bai_path_for(path, bai_path);
    Bai bai;
    if (int rc = read_bai(bp.c_str(), bai)) return rc;
    // header: inflate leading blocks until the reference list is complete
    std::vector<Block> hb;
    size_t htotal = 0;
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    {
        size_t next_off = 0;
        std::vector<uint8_t> hbuf;
        for (;;) {
            MC_REQUIRE(next_off < mf.size, MC_E_IO, "%s: truncated BAM header", path);
            const size_t first = hb.size();
            if (int rc = scan_blocks(mf.data, mf.size, next_off, next_off, hb, htotal)) return rc;
            const Block& b = hb[first];
            next_off = b.off + (b.cdata - b.off) + b.clen + 8;
            hbuf.resize(htotal + 8);
            MC_REQUIRE(inflate_block(mf.data + b.cdata, b.clen, hbuf.data() + b.out, b.isize), MC_E_IO,
                       "BGZF inflate failed in %s", path);
            names.clear();
            lens.clear();
            size_t o = 0;
            if (htotal >= 12 && parse_header(hbuf.data(), htotal, path, names, lens, &o) == MC_OK) break;
            MC_REQUIRE(htotal < (size_t(1) << 31), MC_E_IO, "%s: no valid BAM header", path);
        }
    }
    const int32_t n_ref = (int32_t)names.size();
    MC_REQUIRE((int32_t)bai.refs.size() == n_ref, MC_E_IO,
               "%s indexes %zu references, the BAM header has %d", bp.c_str(), bai.refs.size(), n_ref);
    std::vector<int32_t> tids(sel, sel + n_sel);
    std::sort(tids.begin(), tids.end());
    tids.erase(std::unique(tids.begin(), tids.end()), tids.end());
    for (int32_t t : tids) MC_REQUIRE(t >= 0 && t < n_ref, MC_E_INVALID, "contig %d out of range", t);
    // the compressed extent of each chosen contig, then one flat block list
    struct Range { int32_t tid; size_t b0, b1; uint64_t beg, end; size_t q0 = 0, q1 = 0; };
    std::vector<Range> ranges;
    std::vector<Block> blocks;
    size_t total = 0;
    for (int32_t t : tids) {
        const Bai::Ref& r = bai.refs[t];
        if (!(r.has_meta || r.has_bins) || r.end <= r.beg) continue;
        Range g;
        g.tid = t;
        g.beg = r.beg;
        g.end = r.end;
        g.b0 = blocks.size();
        if (int rc = scan_blocks(mf.data, mf.size, (size_t)(r.beg >> 16), (size_t)(r.end >> 16), blocks,
                                 total))
            return rc;
        g.b1 = blocks.size();
        MC_REQUIRE(g.b1 > g.b0 && blocks[g.b0].off == (r.beg >> 16) &&
                       blocks[g.b1 - 1].off == (r.end >> 16),
                   MC_E_IO, "%s: index offsets of contig %d do not match the BAM blocks", bp.c_str(), t);
        g.q0 = blocks[g.b0].out + (size_t)(r.beg & 0xffff);
        g.q1 = blocks[g.b1 - 1].out + (size_t)(r.end & 0xffff);
        ranges.push_back(g);
    }
    std::unique_ptr<uint8_t[]> buf(new (std::nothrow) uint8_t[total + 8]);
    MC_REQUIRE(buf, MC_E_IO, "cannot allocate %zu bytes for %s", total, path);
    const int nt = n_threads_or_all(n_threads);
    MC_REQUIRE(blocks.empty() || inflate_blocks(mf.data, blocks, buf.get(), nt), MC_E_IO,
               "BGZF inflate failed in %s", path);
    const uint8_t* d = buf.get();
    // parse the ranges in parallel (one contig per task)
    struct Part { std::vector<int32_t> tid, pos, span; std::vector<int64_t> nw; std::vector<uint32_t> cig; int err = 0; size_t at = 0; };
    std::vector<Part> parts(ranges.size());
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t g; (g = next.fetch_add(1)) < ranges.size();) {
            const Range& rg = ranges[g];
            Part& p = parts[g];
            for (size_t q = rg.q0; q < rg.q1;) {
                if (q + 4 > total) { p.err = 1; p.at = q; break; }
                const int32_t bs = rdi32(d + q);
                if (bs < 32 || q + 4 + (size_t)bs > total) { p.err = 1; p.at = q; break; }
                const uint8_t* r = d + q + 4;
                const uint8_t* rend = r + bs;
                q += 4 + (size_t)bs;
                const int32_t tid = rdi32(r);
                const uint16_t flag = rd16(r + 14);
                if (tid != rg.tid || (flag & flag_filter)) continue;
                const uint8_t* cig;
                uint32_t n_cigar;
                if (!cigar_of(r, rend, &cig, &n_cigar)) { p.err = 2; p.at = q; break; }
                int64_t rlen = cigar_rlen(cig, n_cigar);
                if (rlen <= 0 && (flag_filter & MC_LEGACY_ENDPOS)) rlen = 1;   // else raw (bam_plp_push)
                if (rlen > INT32_MAX) { p.err = 3; p.at = q; break; }
                p.tid.push_back(tid);
                p.pos.push_back(rdi32(r + 4));
                p.span.push_back((int32_t)rlen);
                if (keep_cigar) {
                    p.cig.insert(p.cig.end(), reinterpret_cast<const uint32_t*>(cig),
                                 reinterpret_cast<const uint32_t*>(cig) + n_cigar);
                    p.nw.push_back(n_cigar);
                }
            }
        }
    };
    {
        std::vector<std::thread> pool;
        for (int i = 1; i < std::min<int>(nt, (int)ranges.size()); ++i) pool.emplace_back(work);
        work();
        for (auto& th : pool) th.join();
    }
    for (const Part& p : parts)
        MC_REQUIRE(!p.err, MC_E_IO, "%s: %s at byte %zu of the inflated ranges", path,
                   p.err == 1 ? "bad record size" : p.err == 2 ? "CIGAR overruns record"
                                                  : "reference span exceeds int32",
                   p.at);
    mc_bam* bam = new mc_bam();
    bam->names = std::move(names);
    bam->lens = std::move(lens);
    bam->keep_cigar = keep_cigar != 0;
    // whole-file counts as the index reports them (pysam AlignmentFile.mapped
    // / .unmapped, used at metacov/cli.py:58-66, read the same pseudo-bins)
    for (const Bai::Ref& r : bai.refs) {
        bam->n_mapped += (int64_t)r.n_mapped;
        bam->n_unmapped += (int64_t)r.n_unmapped;
    }
    bam->n_unmapped += (int64_t)bai.n_no_coor;
    bam->n_records = bam->n_mapped + bam->n_unmapped;
    size_t nk = 0, nw = 0;
    for (const Part& p : parts) {
        nk += p.tid.size();
        nw += p.cig.size();
    }
    bam->tid.reserve(nk);
    bam->pos.reserve(nk);
    bam->span.reserve(nk);
    if (keep_cigar) {
        bam->cigar.reserve(nw);
        bam->cig_off.assign(1, 0);
    }
    for (const Part& p : parts) {
        bam->tid.insert(bam->tid.end(), p.tid.begin(), p.tid.end());
        bam->pos.insert(bam->pos.end(), p.pos.begin(), p.pos.end());
        bam->span.insert(bam->span.end(), p.span.begin(), p.span.end());
        if (keep_cigar) {
            bam->cigar.insert(bam->cigar.end(), p.cig.begin(), p.cig.end());
            for (int64_t w : p.nw) bam->cig_off.push_back(bam->cig_off.back() + w);
        }
    }
    *out = bam;
    return MC_OK;
}
