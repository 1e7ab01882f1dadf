// plan.cpp — stripe plans: a batch of stripes of mixed shard lengths coded in
// one launch (stripes.hip).  A stripe is ecSplit's databuf layout
// (objectserver/ecutils.go:31-35,55-58): k+m shards of shard_len bytes back
// to back, data first.  Stripes the tiled kernel cannot take (unaligned:
// S % 16 != 0 for 15 object sizes in 16; every object of an object plan with
// k > 8) are coded by one more launch per pass of gf_apply_unaligned_plan over
// their own records; stripe plans with k > 8 run the tiled kernel in
// accumulate passes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/hbec.h"
#include "gf256.h"
#include "internal.h"
#include "kernels.h"

using hbec::fail;
using hbec::hip_fail;

struct hbec_plan {
    int k = 0, m = 0;
    int tile_bytes = 0;
    hbec::TileRec* d_tiles = nullptr;
    uint64_t n_tiles = 0;
    std::vector<hbec_stripe> tiled;     // stripes covered by d_tiles
    std::vector<hbec_stripe> fallback;  // stripes coded one by one
    // object plans (hbec_plan_objects): data shards and parity shards in
    // separate regions; tiles carry base A = data, base B = parity
    bool objects = false;
    std::vector<hbec_object> obj_tiled, obj_fallback;
    uint64_t shard_bytes = 0;           // sum of shard_len over all stripes
    // stripes / objects the tiled kernel cannot take: unaligned-kernel records
    hbec::URec* d_urecs = nullptr;
    uint64_t n_urecs = 0;
    // gf_odd: one edge record per such stripe / object (its guard-band bytes)
    hbec::URec* d_erecs = nullptr;
    uint64_t n_erecs = 0;
    // shards of 2^31 bytes or more (gf_odd positions are 32-bit), or all of
    // them with HBEC_ODD=0: round-2 gf_apply_unaligned_plan records
    hbec::URec* d_brecs = nullptr;
    uint64_t n_brecs = 0;
    // gf_odd_rec: one record per stripe / object with a main-kernel part,
    // and the tile lists the record kernels walk (one per tile span)
    hbec::URec* d_orecs = nullptr;
    uint32_t* d_lists[hbec::kOddSpans] = {};
    hbec::OddStripeRecs orecs;
    std::unique_ptr<hbec::OddRecCache> rec_cache;
};

// The gf_odd_rec records of a plan pass depend only on the plan's stripes and
// on which shards the pass reads and writes, not on its coefficients: a
// plan keeps those it built (the encode pass, recurring erasure patterns)
// instead of rebuilding them on every call (gf_odd_planrec: 13-15 us of a
// 16384-stripe 8+3 plan's 250 us, r6_trace_mid).  Built on the first
// caller's stream; a caller on another stream waits for that build's event.
struct hbec::OddRecCache {
    static constexpr size_t kMaxEntries = 16;
    struct Entry {
        std::vector<uint32_t> key;
        uint32_t* d = nullptr;
        hipEvent_t ev = nullptr;
        hipStream_t stream = nullptr;
    };
    std::mutex mu;
    std::vector<Entry> entries;
    ~OddRecCache() {
        for (auto& x : entries) {
            if (x.ev) (void)hipEventDestroy(x.ev);
            if (x.d) (void)hipFree(x.d);
        }
    }
};

namespace {

bool aligned_stripe(const hbec_stripe& s) {
    return (reinterpret_cast<uintptr_t>(s.base) & 15u) == 0 && (s.shard_len % 16) == 0 &&
           s.shard_len < (1ull << 32);
}

bool aligned_object(const hbec_object& o) {
    return ((reinterpret_cast<uintptr_t>(o.data) | reinterpret_cast<uintptr_t>(o.parity)) & 15u) == 0 &&
           (o.shard_len % 16) == 0 && o.shard_len < (1ull << 32);
}

std::mutex g_occ_mu;

void add_urecs(std::vector<hbec::URec>& recs, std::vector<hbec::URec>& erecs, std::vector<hbec::URec>& brecs,
               std::vector<hbec::URec>& orecs, const void* a, const void* b, uint64_t s, int k) {
    const uint64_t ua = reinterpret_cast<uint64_t>(a), ub = reinterpret_cast<uint64_t>(b);
    if (!hbec::odd_enabled() || !hbec::pos32_shard(s)) {
        const uint64_t tile = (uint64_t)hbec::unaligned_tile_bytes();
        for (uint64_t p0 = 0; p0 < s; p0 += tile) brecs.push_back({ua, ub, s, p0});
        return;
    }
    const uint64_t tile = hbec::urec_tile_for(std::min(k, hbec::kOddMaxK), false), span = hbec::urec_span(s);
    for (uint64_t p0 = 0; p0 < span; p0 += tile) recs.push_back({ua, ub, s, p0});
    erecs.push_back({ua, ub, s, 0});
    if (span > 0) orecs.push_back({ua, ub, s, 0});
}

// Tile lists of the per-stripe records: for each record-kernel tile span,
// tile t of stripe e for t < odd_frame_tiles(S_e, span), stripe by stripe,
// as {e, t, S_e | flags << 30, 0} (kernels.h kOddListWords): flag 1 the
// stripe's first tile, 2 its last (apply passes code the guard band there,
// HBEC_ODD_EDGE_FUSE; bits 0-29 hold S when S < 2^30, else the stripe's edges
// go to gf_odd_edges_plan).  A one-tile stripe has two entries, {e, 0, S | 1 <<
// 30} and {e, 0, S | 2 << 30 | 1 << 29}: bit 29 = guard-band bytes only.
int build_tile_lists(hbec_plan* p, const std::vector<hbec::URec>& orecs) {
    p->orecs = hbec::OddStripeRecs{};
    if (orecs.empty()) return HBEC_OK;
    uint32_t spans[hbec::kOddSpans];
    hbec::odd_plan_spans(spans);
    uint64_t s_max = 0;
    for (const auto& r : orecs) s_max = std::max<uint64_t>(s_max, r.shard_len);
    for (int i = 0; i < hbec::kOddSpans; ++i) {
        std::vector<uint32_t> l;
        for (size_t e = 0; e < orecs.size(); ++e) {
            const uint64_t S = orecs[e].shard_len;
            const uint64_t nt = hbec::odd_frame_tiles(S, spans[i]);
            const bool small = S < (1ull << 30);
            auto put = [&](uint64_t t, uint32_t fl, uint32_t only) {
                l.push_back((uint32_t)e);
                l.push_back((uint32_t)t);
                l.push_back(small && fl ? (uint32_t)S | (fl << 30) | only : 0u);
                l.push_back(0u);
            };
            for (uint64_t t = 0; t < nt; ++t) put(t, t == 0 ? 1u : (t + 1 == nt ? 2u : 0u), 0u);
            if (nt == 1 && small) put(0, 2u, 1u << 29);
        }
        if (l.size() / hbec::kOddListWords >= (1ull << 31))
            return fail(HBEC_ERR_INVALID_ARG, "plan too large (>= 2^31 record tiles)");
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&p->d_lists[i]), l.size() * 4);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc plan tile list");
        e = hipMemcpy(p->d_lists[i], l.data(), l.size() * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpy plan tile list");
        p->orecs.lists[i] = hbec::OddTileList{spans[i], p->d_lists[i], l.size() / hbec::kOddListWords};
    }
    p->rec_cache = std::make_unique<hbec::OddRecCache>();
    p->orecs.cache = p->rec_cache.get();
    p->orecs.recs = p->d_orecs;
    p->orecs.n = orecs.size();
    p->orecs.s_max = s_max;
    return HBEC_OK;
}

template <class T>
int upload(const std::vector<T>& recs, T** dst, const char* what) {
    if (recs.empty()) return HBEC_OK;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(dst), recs.size() * sizeof(T));
    if (e != hipSuccess) return hip_fail(e, what);
    e = hipMemcpy(*dst, recs.data(), recs.size() * sizeof(T), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(*dst);
        *dst = nullptr;
        return hip_fail(e, what);
    }
    return HBEC_OK;
}

// One pass of a plan over per-stripe records: the records of every stripe in
// one launch (stream-ordered scratch), then one gf_odd_rec launch over the
// tile list of the span the pass's kernel uses.
int odd_stripe_rec_pass(int K, int R, int mode, const hbec::UPlanArgs& a, const hbec::OddStripeRecs& o, int cus,
                        int max_blocks, hipStream_t stream, bool one_pass, bool* fused) {
    const uint64_t rw = hbec::odd_rec_words(K, R, mode);
    const int xs = hbec::odd_bp_schedule(K, R, mode, a.tab, true);
    const uint32_t span = hbec::odd_rec_tile_span(K, mode, xs);
    const hbec::OddTileList* tl = nullptr;
    for (const auto& l : o.lists)
        if (l.span == span) tl = &l;
    if (!tl || !tl->d) return fail(HBEC_ERR_INVALID_ARG, "plan has no tile list for this pass");
    uint32_t* recs = nullptr;
    bool cached = false;
    hipError_t e = hipSuccess;
    if (o.cache) {
        std::vector<uint32_t> key{(uint32_t)K, (uint32_t)R, (uint32_t)mode, a.in_sel, a.out_sel};
        key.insert(key.end(), a.in_idx, a.in_idx + K);
        key.insert(key.end(), a.out_idx, a.out_idx + R);
        std::lock_guard<std::mutex> lk(o.cache->mu);
        for (const auto& x : o.cache->entries) {
            if (x.key != key) continue;
            if (x.stream != stream) {
                e = hipStreamWaitEvent(stream, x.ev, 0);
                if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent (plan records)");
            }
            recs = x.d;
            cached = true;
        }
        if (!cached && o.cache->entries.size() < hbec::OddRecCache::kMaxEntries) {
            hbec::OddRecCache::Entry x;
            x.key = std::move(key);
            x.stream = stream;
            if (hipMalloc(reinterpret_cast<void**>(&x.d), o.n * rw * 4) == hipSuccess) {
                e = hbec::launch_odd_planrec(K, R, mode, a, o.recs, (uint32_t)o.n, x.d, stream);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&x.ev, hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventRecord(x.ev, stream);
                if (e != hipSuccess) {
                    if (x.ev) (void)hipEventDestroy(x.ev);
                    (void)hipFree(x.d);
                    return hip_fail(e, "launch gf_odd_planrec (plan records)");
                }
                recs = x.d;
                cached = true;
                o.cache->entries.push_back(std::move(x));
            } else {
                (void)hipGetLastError();  // HBM full: per-call scratch records below
            }
        }
    }
    if (!cached) {
        int rc = hbec::scratch_alloc(o.n * rw * 4, stream, reinterpret_cast<void**>(&recs));
        if (rc) return rc;
        e = hbec::launch_odd_planrec(K, R, mode, a, o.recs, (uint32_t)o.n, recs, stream);
        if (e != hipSuccess) {
            hbec::scratch_free(recs, stream);
            return hip_fail(e, "launch gf_odd_planrec");
        }
    }
    hbec::PassArgs c;
    std::memset(&c, 0, sizeof(c));
    std::memcpy(c.tab, a.tab, sizeof(c.tab));
    c.n_obj = o.n;
    c.shard_len = o.s_max;
    c.tiles_per_obj = 1;
    c.n_tiles = (uint32_t)tl->n;
    c.list = tl->d;
    // the record kernel codes the guard band of the stripes it covers (the
    // tile list's edge flags) when this pass's inputs are all of them
    *fused = one_pass && o.s_max < (1ull << 30) && hbec::odd_edge_fuse(K, R, mode, true, xs, true, o.s_max);
    c.fuse = *fused ? 1u : 0u;
    const uint64_t wpb = hbec::odd_waves_per_block(xs);
    const uint64_t want = (c.n_tiles + wpb - 1) / wpb;
    uint64_t cap = (uint64_t)cus * (uint64_t)hbec::odd_blocks_per_cu(mode, K, R, false, true, xs);
    if (max_blocks > 0) cap = std::min<uint64_t>(cap, (uint64_t)max_blocks);
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, cap));
    e = hbec::launch_odd(K, R, mode, c, nullptr, recs, grid, stream, xs);
    if (!cached) hbec::scratch_free(recs, stream);
    if (e != hipSuccess) return hip_fail(e, "launch gf_odd_rec (plan)");
    return HBEC_OK;
}

}  // namespace

// out rows (^)= rows x in over unaligned-kernel records, in passes of <= 4
// outputs x <= kMaxK inputs (later input passes accumulate).  sel_k > 0:
// object records (shard indices >= sel_k are parity, base b).
int hbec::launch_unaligned_passes(const URec* recs, uint64_t n_recs, const std::vector<int>& in_idx,
                                  const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, int sel_k,
                                  hipStream_t stream, int max_blocks, const URec* erecs, uint64_t n_erecs,
                                  bool mirror, bool round2, const OddStripeRecs* orecs) {
    const int K_all = (int)in_idx.size(), R_all = (int)out_idx.size();
    if ((n_recs == 0 && n_erecs == 0) || R_all == 0) return HBEC_OK;
    if (mirror && (!hbec::odd_enabled() || sel_k > 0 || round2))
        return fail(HBEC_ERR_INVALID_ARG, "mirrored unaligned plans need gf_odd and stripe records");
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return hip_fail(e, "hipDeviceGetAttribute");
    if (hbec::odd_enabled() && !round2) {
        // per-stripe records over the plan's tile lists (unmirrored plans)
        const bool use_orecs = orecs && orecs->n > 0 && !mirror;
        // gf_odd_plan: launches of <= 4 outputs x <= kOddMaxK inputs, later input
        // launches accumulating; one 4-wave block per CU
        for (int r0 = 0; r0 < R_all; r0 += hbec::kMaxR) {
            const int R = std::min(hbec::kMaxR, R_all - r0);
            for (int c0 = 0; c0 < K_all; c0 += hbec::kOddMaxK) {
                const int K = std::min(hbec::kOddMaxK, K_all - c0);
                hbec::UPlanArgs a;
                std::memset(&a, 0, sizeof(a));
                a.recs = recs;
                a.n_recs = (uint32_t)n_recs;
                a.accumulate = c0 > 0 ? 1u : 0u;
                // mirror: each pass's inputs once (first output group), the
                // outputs when one input pass makes them final
                if (mirror) a.mirror = (r0 == 0 ? 1u : 0u) | (K_all <= hbec::kOddMaxK ? 2u : 0u);
                // records built as carried tiles (K_all <= 4, not mirrored) take the carry kernel
                a.carry = (!mirror && K <= 4 &&
                           hbec::urec_tile_for(std::min(K_all, hbec::kOddMaxK), false) != hbec::urec_tile_for(K, true))
                              ? 1u : 0u;
                for (int j = 0; j < K; ++j) {
                    int i = in_idx[c0 + j];
                    if (sel_k > 0 && i >= sel_k) {
                        a.in_sel |= 1u << j;
                        i -= sel_k;
                    }
                    a.in_idx[j] = (uint32_t)i;
                }
                for (int r = 0; r < R; ++r) {
                    int i = out_idx[r0 + r];
                    if (sel_k > 0 && i >= sel_k) {
                        a.out_sel |= 1u << r;
                        i -= sel_k;
                    }
                    a.out_idx[r] = (uint32_t)i;
                    for (int j = 0; j < K; ++j)
                        hbec::perm_table(rows[(size_t)(r0 + r) * K_all + c0 + j], a.tab[r][j]);
                }
                const uint64_t want = (n_recs + 3) / 4;  // 4 waves per block
                uint64_t cap = (uint64_t)cus * (uint64_t)hbec::odd_blocks_per_cu(c0 > 0 ? 1 : 0, K, R, mirror);
                if (max_blocks > 0) cap = std::min<uint64_t>(cap, (uint64_t)max_blocks);
                const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, cap));
                const int mode = c0 > 0 ? 1 : 0;
                bool fused = false;
                if (use_orecs) {
                    int rc = odd_stripe_rec_pass(K, R, mode, a, *orecs, cus, max_blocks, stream, K == K_all, &fused);
                    if (rc) return rc;
                } else if (n_recs > 0) {
                    e = hbec::launch_odd_plan(K, R, mode, a, grid, stream);
                    if (e != hipSuccess) return hip_fail(e, "launch gf_odd_plan");
                }
                // guard-band bytes of every stripe, this pass's inputs (fused:
                // only the stripes of S <= odd_min_main(), which have no main
                // tiles; the edge records list them first)
                const uint64_t ne = fused ? orecs->n_short_edges : n_erecs;
                e = hbec::launch_odd_edges_plan(K, R, c0 > 0 ? 1 : 0, a, erecs, (uint32_t)ne, stream,
                                                !fused && orecs && orecs->edges_long);
                if (e != hipSuccess) return hip_fail(e, "launch gf_odd_edges_plan");
            }
        }
        if (mirror && n_erecs > 0) {
            // the bytes the main kernel did not mirror, read back from the
            // (final) stripes: guard bands of every shard, and whole outputs
            // when k > kOddMaxK made them final only after the last pass
            std::vector<int> all(in_idx);
            all.insert(all.end(), out_idx.begin(), out_idx.end());
            for (int pass = 0; pass < 2; ++pass) {
                const bool full = pass == 1;
                if (full && K_all <= hbec::kOddMaxK) break;
                const std::vector<int>& idx = full ? out_idx : all;
                for (size_t t0 = 0; t0 < idx.size(); t0 += hbec::kMirrorMaxIdx) {
                    hbec::MirrorCopyArgs m;
                    std::memset(&m, 0, sizeof(m));
                    m.n_idx = (uint32_t)std::min<size_t>(hbec::kMirrorMaxIdx, idx.size() - t0);
                    for (uint32_t t = 0; t < m.n_idx; ++t) m.idx[t] = (uint32_t)idx[t0 + t];
                    m.full = full ? 1u : 0u;
                    e = hbec::launch_odd_mirror_copy(erecs, (uint32_t)n_erecs, m, stream);
                    if (e != hipSuccess) return hip_fail(e, "launch gf_odd_mirror_copy");
                }
            }
        }
        return HBEC_OK;
    }
    for (int r0 = 0; r0 < R_all; r0 += hbec::kMaxR) {
        const int R = std::min(hbec::kMaxR, R_all - r0);
        e = hbec::unaligned_occupancy(R, &per_cu);
        if (e != hipSuccess) return hip_fail(e, "unaligned occupancy");
        if (const long long v = hbec::tune_knob("HBEC_UNALIGNED_BPC", 0); v > 0) per_cu = std::min(per_cu, (int)v);
        for (int c0 = 0; c0 < K_all; c0 += hbec::kMaxK) {
            const int K = std::min(hbec::kMaxK, K_all - c0);
            hbec::UPlanArgs a;
            std::memset(&a, 0, sizeof(a));
            a.recs = recs;
            a.n_recs = (uint32_t)n_recs;
            a.accumulate = c0 > 0 ? 1u : 0u;
            for (int j = 0; j < K; ++j) {
                int i = in_idx[c0 + j];
                if (sel_k > 0 && i >= sel_k) {
                    a.in_sel |= 1u << j;
                    i -= sel_k;
                }
                a.in_idx[j] = (uint32_t)i;
            }
            for (int r = 0; r < R; ++r) {
                int i = out_idx[r0 + r];
                if (sel_k > 0 && i >= sel_k) {
                    a.out_sel |= 1u << r;
                    i -= sel_k;
                }
                a.out_idx[r] = (uint32_t)i;
                for (int j = 0; j < K; ++j) hbec::perm_table(rows[(size_t)(r0 + r) * K_all + c0 + j], a.tab[r][j]);
            }
            const uint64_t want = (n_recs + 3) / 4;  // 4 waves per block
            uint64_t cap = (uint64_t)cus * std::max(1, per_cu);
            if (max_blocks > 0) cap = std::min<uint64_t>(cap, (uint64_t)max_blocks);
            const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, cap));
            e = hbec::launch_unaligned_plan(K, R, a, grid, stream);
            if (e != hipSuccess) return hip_fail(e, "launch gf_apply_unaligned_plan");
        }
    }
    return HBEC_OK;
}

int hbec::stripes_grid(int k, int r, uint64_t n_tiles, int* grid, int blocks_per_cu, int max_blocks) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    static int cus[64] = {0};
    static int occ[64][9][4] = {};
    std::lock_guard<std::mutex> g(g_occ_mu);
    if (dev < 0 || dev >= 64) return fail(HBEC_ERR_DEVICE, "device index out of range");
    if (cus[dev] == 0) {
        hipDeviceProp_t p;
        e = hipGetDeviceProperties(&p, dev);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
        cus[dev] = p.multiProcessorCount;
    }
    if (occ[dev][k][r] == 0) {
        int b = 0;
        e = hbec::stripes_occupancy(k, r, &b);
        if (e != hipSuccess) return hip_fail(e, "stripes occupancy");
        b = std::max(1, b);
        if (hbec::kPipeBlocksPerCu > 0) b = std::min(b, hbec::kPipeBlocksPerCu);  // same HBM sweet spot
        if (const long long v = hbec::tune_knob("HBEC_STRIPE_BLOCKS_PER_CU", 0); v > 0) b = std::max(1, std::min(b, (int)v));
        occ[dev][k][r] = b;
    }
    const uint64_t want = (n_tiles + 3) / 4;  // 4 waves per block
    int bpc = occ[dev][k][r];
    if (blocks_per_cu > 0) {  // caller's choice (zero-copy over PCIe), within what fits
        int fit = 1;
        if (hbec::stripes_occupancy(k, r, &fit) != hipSuccess) fit = 1;
        bpc = std::max(1, std::min(fit, blocks_per_cu));
    }
    uint64_t cap = (uint64_t)cus[dev] * (uint64_t)bpc;
    if (max_blocks > 0) cap = std::min<uint64_t>(cap, (uint64_t)max_blocks);
    *grid = (int)std::max<uint64_t>(1, std::min(want, cap));
    return HBEC_OK;
}

// out[r] (^)= XOR_j rows[r][j] * in[j] over every tile record: launches of
// <= 3 outputs x <= kStripeMaxK inputs; a shape with more inputs (k > 8)
// runs in passes, the later ones accumulating into the outputs.  sel_k > 0
// marks an object plan (split bases: shard indices >= sel_k are parity).
int hbec::launch_stripe_passes(const TileRec* tiles, uint64_t n_tiles, const std::vector<int>& in_idx,
                               const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, int sel_k,
                               hipStream_t stream, int blocks_per_cu, bool mirror, int max_blocks) {
    const int K_all = (int)in_idx.size(), R_all = (int)out_idx.size();
    if (n_tiles == 0 || R_all == 0) return HBEC_OK;
    if (sel_k > 0 && K_all > kStripeMaxK) return fail(HBEC_ERR_INVALID_ARG, "object plans take <= 8 inputs per pass");
    if (sel_k > 0 && mirror) return fail(HBEC_ERR_INVALID_ARG, "object plans are not mirrored");
    for (int r0 = 0; r0 < R_all; r0 += 3) {
        const int R = std::min(3, R_all - r0);
        for (int c0 = 0; c0 < K_all; c0 += kStripeMaxK) {
            const int K = std::min(kStripeMaxK, K_all - c0);
            StripeArgs a;
            std::memset(&a, 0, sizeof(a));
            a.tiles = tiles;
            a.n_tiles = (uint32_t)n_tiles;
            a.split = sel_k > 0 ? 1u : 0u;
            a.accumulate = c0 > 0 ? 1u : 0u;
            a.mirror = mirror ? 1u : 0u;
            for (int j = 0; j < K; ++j) {
                a.in_idx[j] = (uint32_t)in_idx[c0 + j];
                if (sel_k > 0 && in_idx[c0 + j] >= sel_k) {  // parity shard: base B
                    a.in_sel |= 1u << j;
                    a.in_idx[j] -= (uint32_t)sel_k;
                }
            }
            for (int r = 0; r < R; ++r) {
                a.out_idx[r] = (uint32_t)out_idx[r0 + r];
                if (sel_k > 0) {
                    if (out_idx[r0 + r] < sel_k) a.out_sel |= 1u << r;  // data shard: base A
                    else a.out_idx[r] -= (uint32_t)sel_k;
                }
                for (int j = 0; j < K; ++j) perm_table(rows[(size_t)(r0 + r) * K_all + c0 + j], a.tab[r][j]);
            }
            int grid = 0;
            int rc = stripes_grid(K, R, n_tiles, &grid, blocks_per_cu, max_blocks);
            if (rc) return rc;
            hipError_t e = launch_stripes(K, R, a, grid, stream);
            if (e != hipSuccess) return hip_fail(e, "launch gf_apply_stripes");
        }
    }
    return HBEC_OK;
}

namespace {

// out rows (given as shard indices + coefficient rows over in_idx) for every stripe
int run_plan(const hbec_plan* p, const std::vector<int>& in_idx, const std::vector<int>& out_idx,
             const std::vector<uint8_t>& rows, hipStream_t stream) {
    const int K = (int)in_idx.size();
    const int R_all = (int)out_idx.size();
    if (R_all == 0 || p->shard_bytes == 0) return HBEC_OK;
    // stripe plans take any k (inputs beyond 8 accumulate in later passes);
    // object plans keep the tiled kernel to k <= 8
    const bool tiled_ok = p->objects ? K <= hbec::kStripeMaxK : true;
    if (tiled_ok && p->n_tiles > 0) {
        int rc = hbec::launch_stripe_passes(p->d_tiles, p->n_tiles, in_idx, out_idx, rows, p->objects ? p->k : 0,
                                            stream);
        if (rc) return rc;
    }
    // with k > 8 every object is in the unaligned records (hbec_plan_objects)
    const int sel_k = p->objects ? p->k : 0;
    int rc = hbec::launch_unaligned_passes(p->d_urecs, p->n_urecs, in_idx, out_idx, rows, sel_k, stream, 0,
                                           p->d_erecs, p->n_erecs, false, false, &p->orecs);
    if (rc || p->n_brecs == 0) return rc;
    return hbec::launch_unaligned_passes(p->d_brecs, p->n_brecs, in_idx, out_idx, rows, sel_k, stream, 0, nullptr, 0,
                                         false, true);
}

}  // namespace

extern "C" {

int hbec_plan_stripes(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n, hbec_plan** out) {
    return hbec::guarded("hbec_plan_stripes", [&]() -> int {
        if (!codec || !out || (n && !stripes)) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        *out = nullptr;
        const int k = hbec_data_shards(codec), m = hbec_parity_shards(codec);
        std::unique_ptr<hbec_plan> p(new (std::nothrow) hbec_plan());
        if (!p) return fail(HBEC_ERR_NOMEM, "plan allocation");
        p->k = k;
        p->m = m;
        p->tile_bytes = hbec::stripes_tile_bytes(std::min(k, hbec::kStripeMaxK));
        std::vector<hbec::TileRec> recs;
        std::vector<hbec::URec> urecs, erecs, brecs, orecs;
        for (uint64_t i = 0; i < n; ++i) {
            const hbec_stripe& s = stripes[i];
            if (s.shard_len == 0) continue;
            if (!s.base) return fail(HBEC_ERR_INVALID_ARG, "stripe with null base");
            p->shard_bytes += s.shard_len;
            // (aligned stripes the record kernels code faster join them, hbec.cpp rec_route)
            if (!aligned_stripe(s) ||
                hbec::plan_rec_route(codec, s.shard_len, (reinterpret_cast<uintptr_t>(s.base) & 127u) == 0 && s.shard_len % 128 == 0)) {
                p->fallback.push_back(s);
                add_urecs(urecs, erecs, brecs, orecs, s.base, nullptr, s.shard_len, k);
                continue;
            }
            p->tiled.push_back(s);
            for (uint64_t off = 0; off < s.shard_len; off += (uint64_t)p->tile_bytes) {
                hbec::TileRec r;
                r.in_addr = r.out_addr = reinterpret_cast<uint64_t>(s.base) + off;
                r.in_stride = r.out_stride = (uint32_t)s.shard_len;
                r.valid = (uint32_t)std::min<uint64_t>((uint64_t)p->tile_bytes, s.shard_len - off);
                r.pad_ = 0;
                recs.push_back(r);
            }
        }
        // both record counts are checked before anything is allocated on the device
        if (recs.size() >= (1ull << 31) || urecs.size() >= (1ull << 31) || erecs.size() >= (1ull << 31) ||
            brecs.size() >= (1ull << 31))
            return fail(HBEC_ERR_INVALID_ARG, "plan too large (>= 2^31 tiles)");
        p->n_tiles = recs.size();
        if (!recs.empty()) {
            hipError_t e = hipMalloc(&p->d_tiles, recs.size() * sizeof(hbec::TileRec));
            if (e != hipSuccess) return hip_fail(e, "hipMalloc plan tiles");
            e = hipMemcpy(p->d_tiles, recs.data(), recs.size() * sizeof(hbec::TileRec), hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                (void)hipFree(p->d_tiles);
                p->d_tiles = nullptr;
                return hip_fail(e, "hipMemcpy plan tiles");
            }
        }
        // edge records of the stripes with no main tiles (S <= odd_min_main()) first
        const auto short_end = std::stable_partition(erecs.begin(), erecs.end(), [](const hbec::URec& e) {
            return e.shard_len <= hbec::odd_min_main();
        });
        const uint64_t n_short = (uint64_t)(short_end - erecs.begin());
        int urc = upload(urecs, &p->d_urecs, "plan unaligned records");
        if (!urc) urc = upload(erecs, &p->d_erecs, "plan edge records");
        if (!urc) urc = upload(brecs, &p->d_brecs, "plan large-shard records");
        if (!urc) urc = upload(orecs, &p->d_orecs, "plan stripe records");
        if (!urc) urc = build_tile_lists(p.get(), orecs);
        if (urc) {
            hbec_plan_free(p.release());
            return urc;
        }
        p->n_urecs = urecs.size();
        p->n_erecs = erecs.size();
        p->orecs.edges_long = n_short == 0;
        p->orecs.n_short_edges = n_short;
        p->n_brecs = brecs.size();
        *out = p.release();
        return HBEC_OK;
    });
}

int hbec_plan_objects(hbec_codec* codec, const hbec_object* objects, uint64_t n, hbec_plan** out) {
    return hbec::guarded("hbec_plan_objects", [&]() -> int {
        if (!codec || !out || (n && !objects)) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        *out = nullptr;
        const int k = hbec_data_shards(codec), m = hbec_parity_shards(codec);
        std::unique_ptr<hbec_plan> p(new (std::nothrow) hbec_plan());
        if (!p) return fail(HBEC_ERR_NOMEM, "plan allocation");
        p->k = k;
        p->m = m;
        p->objects = true;
        p->tile_bytes = hbec::stripes_tile_bytes(std::min(k, hbec::kStripeMaxK));
        std::vector<hbec::TileRec> recs;
        std::vector<hbec::URec> urecs, erecs, brecs, orecs;
        for (uint64_t i = 0; i < n; ++i) {
            const hbec_object& o = objects[i];
            if (o.shard_len == 0) continue;
            if (!o.data || (m > 0 && !o.parity)) return fail(HBEC_ERR_INVALID_ARG, "object with null data or parity");
            p->shard_bytes += o.shard_len;
            const bool line = ((reinterpret_cast<uintptr_t>(o.data) | reinterpret_cast<uintptr_t>(o.parity)) & 127u) == 0 &&
                              o.shard_len % 128 == 0;
            if (!aligned_object(o) || (k <= hbec::kStripeMaxK && hbec::plan_rec_route(codec, o.shard_len, line))) {
                p->obj_fallback.push_back(o);
                add_urecs(urecs, erecs, brecs, orecs, o.data, o.parity, o.shard_len, k);
                continue;
            }
            if (k > hbec::kStripeMaxK) {
                // the object-plan tiled kernel takes <= 8 inputs: every object goes to
                // the unaligned kernel's records (one launch per pass, not one per object)
                add_urecs(urecs, erecs, brecs, orecs, o.data, o.parity, o.shard_len, k);
                continue;
            }
            p->obj_tiled.push_back(o);
            for (uint64_t off = 0; off < o.shard_len; off += (uint64_t)p->tile_bytes) {
                hbec::TileRec r;
                r.in_addr = reinterpret_cast<uint64_t>(o.data) + off;
                r.out_addr = reinterpret_cast<uint64_t>(o.parity) + off;
                r.in_stride = r.out_stride = (uint32_t)o.shard_len;
                r.valid = (uint32_t)std::min<uint64_t>((uint64_t)p->tile_bytes, o.shard_len - off);
                r.pad_ = 0;
                recs.push_back(r);
            }
        }
        // both record counts are checked before anything is allocated on the device
        if (recs.size() >= (1ull << 31) || urecs.size() >= (1ull << 31) || erecs.size() >= (1ull << 31) ||
            brecs.size() >= (1ull << 31))
            return fail(HBEC_ERR_INVALID_ARG, "plan too large (>= 2^31 tiles)");
        p->n_tiles = recs.size();
        if (!recs.empty()) {
            hipError_t e = hipMalloc(&p->d_tiles, recs.size() * sizeof(hbec::TileRec));
            if (e != hipSuccess) return hip_fail(e, "hipMalloc plan tiles");
            e = hipMemcpy(p->d_tiles, recs.data(), recs.size() * sizeof(hbec::TileRec), hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                (void)hipFree(p->d_tiles);
                p->d_tiles = nullptr;
                return hip_fail(e, "hipMemcpy plan tiles");
            }
        }
        // edge records of the stripes with no main tiles (S <= odd_min_main()) first
        const auto short_end = std::stable_partition(erecs.begin(), erecs.end(), [](const hbec::URec& e) {
            return e.shard_len <= hbec::odd_min_main();
        });
        const uint64_t n_short = (uint64_t)(short_end - erecs.begin());
        int urc = upload(urecs, &p->d_urecs, "plan unaligned records");
        if (!urc) urc = upload(erecs, &p->d_erecs, "plan edge records");
        if (!urc) urc = upload(brecs, &p->d_brecs, "plan large-shard records");
        if (!urc) urc = upload(orecs, &p->d_orecs, "plan stripe records");
        if (!urc) urc = build_tile_lists(p.get(), orecs);
        if (urc) {
            hbec_plan_free(p.release());
            return urc;
        }
        p->n_urecs = urecs.size();
        p->n_erecs = erecs.size();
        p->orecs.edges_long = n_short == 0;
        p->orecs.n_short_edges = n_short;
        p->n_brecs = brecs.size();
        *out = p.release();
        return HBEC_OK;
    });
}

void hbec_plan_free(hbec_plan* plan) {
    if (!plan) return;
    if (plan->d_tiles) (void)hipFree(plan->d_tiles);
    if (plan->d_urecs) (void)hipFree(plan->d_urecs);
    if (plan->d_erecs) (void)hipFree(plan->d_erecs);
    if (plan->d_brecs) (void)hipFree(plan->d_brecs);
    if (plan->d_orecs) (void)hipFree(plan->d_orecs);
    for (uint32_t* l : plan->d_lists)
        if (l) (void)hipFree(l);
    delete plan;
}

int hbec_plan_info(const hbec_plan* plan, uint64_t* n_tiles, int* tile_bytes, uint64_t* n_fallback,
                   uint64_t* shard_bytes) {
    return hbec::guarded("hbec_plan_info", [&]() -> int {
        if (!plan) return fail(HBEC_ERR_INVALID_ARG, "null plan");
        if (n_tiles) *n_tiles = plan->n_tiles;
        if (tile_bytes) *tile_bytes = plan->tile_bytes;
        if (n_fallback) *n_fallback = plan->objects ? plan->obj_fallback.size() : plan->fallback.size();
        if (shard_bytes) *shard_bytes = plan->shard_bytes;
        return HBEC_OK;
    });
}

int hbec_encode_plan(hbec_codec* codec, const hbec_plan* plan, void* hip_stream) {
    return hbec::guarded("hbec_encode_plan", [&]() -> int {
        if (!codec || !plan) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        const int k = hbec_data_shards(codec), m = hbec_parity_shards(codec);
        if (k != plan->k || m != plan->m) return fail(HBEC_ERR_INVALID_ARG, "plan built for another (k, m)");
        if (m == 0) return HBEC_OK;
        std::vector<uint8_t> mat((size_t)(k + m) * k);
        hbec_matrix(codec, mat.data());
        std::vector<uint8_t> rows(mat.begin() + (size_t)k * k, mat.end());
        std::vector<int> in_idx(k), out_idx(m);
        for (int j = 0; j < k; ++j) in_idx[j] = j;
        for (int r = 0; r < m; ++r) out_idx[r] = k + r;
        return run_plan(plan, in_idx, out_idx, rows, static_cast<hipStream_t>(hip_stream));
    });
}

int hbec_reconstruct_plan(hbec_codec* codec, const hbec_plan* plan, const uint8_t* present, int data_only,
                          void* hip_stream) {
    return hbec::guarded("hbec_reconstruct_plan", [&]() -> int {
        if (!codec || !plan || !present) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        const int k = hbec_data_shards(codec), m = hbec_parity_shards(codec), n = k + m;
        if (k != plan->k || m != plan->m) return fail(HBEC_ERR_INVALID_ARG, "plan built for another (k, m)");
        int n_present = 0, data_present = 0;
        for (int i = 0; i < n; ++i) {
            n_present += present[i] ? 1 : 0;
            if (i < k) data_present += present[i] ? 1 : 0;
        }
        if (n_present == n || (data_only && data_present == k)) return HBEC_OK;
        if (n_present < k) return fail(HBEC_ERR_TOO_FEW_SHARDS, "too few shards given");
        std::vector<int> surv(k), outs(n);
        std::vector<uint8_t> rows((size_t)n * k);
        int n_out = 0;
        int rc = hbec_decode_rows(codec, present, data_only, surv.data(), outs.data(), &n_out, rows.data());
        if (rc) return rc;
        outs.resize(n_out);
        rows.resize((size_t)n_out * k);
        return run_plan(plan, surv, outs, rows, static_cast<hipStream_t>(hip_stream));
    });
}

}  // extern "C"
