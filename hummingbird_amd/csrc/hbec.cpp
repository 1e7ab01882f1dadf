// hbec.cpp — the codec (klauspost Encoder mirror) and the device batch API
// behind include/hbec.h.
//
// Reference semantics restated here (klauspost/reedsolomon, reached from
// objectserver/ecutils.go:27,59,77,111,135,168):
//   New:            k <= 0 || m < 0 -> ErrInvShardNum; k+m > 256 -> ErrMaxShardNum
//   Encode:         len(shards) != k+m -> ErrTooFewShards; checkShards(nilok=false)
//   Reconstruct(*): checkShards(nilok=true); nothing to do if all present (or all
//                   data present for ReconstructData); < k present -> ErrTooFewShards;
//                   survivors = first k present shards; missing data = inv(sub) rows;
//                   missing parity = M_p x data.  Parity rows are fused with the
//                   inverse (M_p x inv(sub)), which is the same linear map for
//                   every input (DESIGN.md "Reconstruct").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hbec.h"
#include "gf256.h"
#include "internal.h"
#include "kernels.h"

namespace hbec {

static thread_local std::string t_last_error;

int fail(int code, const std::string& msg) {
    t_last_error = msg;
    return code;
}

// A failed runtime call also leaves its code in the thread's last-error slot,
// where the next successful launch's hipGetLastError() check would find it
// and fail a call that did nothing wrong: clear it here.  Out of memory is
// HBEC_ERR_NOMEM (the caller may retry smaller or fall back), anything else
// HBEC_ERR_DEVICE.
int hip_fail(hipError_t e, const char* what) {
    (void)hipGetLastError();
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return fail(e == hipErrorOutOfMemory ? HBEC_ERR_NOMEM : HBEC_ERR_DEVICE, m);
}

long long hbec::env_knob(const char* name, long long dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::atoll(e) : dflt;
}

static std::atomic<int> g_force_stream{0};
// Views that are not all 16-B aligned (or shards not a multiple of 16 B):
// gf_odd (k <= 12), gf_wide (k > 16), gf_apply_unaligned (13..16, S > 2^31).
// Tuning knob: resident blocks per CU for the unaligned kernels' grids (0 = occupancy).
static const int g_unaligned_bpc = (int)tune_knob("HBEC_UNALIGNED_BPC", 0);
// Tuning knob: cap on resident blocks per CU used to size vec-kernel grids
// (0 = the occupancy the compiler's register allocation allows).
static const int g_blocks_per_cu_override = (int)tune_knob("HBEC_BLOCKS_PER_CU", 0);
// Tuning knob: absolute cap on vec-kernel grids (0 = none), to run fewer CUs.
static const int g_grid_cap_env = (int)tune_knob("HBEC_GRID_CAP", 0);
// Per-thread grid cap set by a caller that shares the GPU with its own side
// work (the encode + ShardHash pipeline); 0 = none.
thread_local int t_grid_cap = 0;
void set_thread_grid_cap(int blocks) { t_grid_cap = blocks; }
#define g_grid_cap (t_grid_cap > 0 ? (g_grid_cap_env > 0 ? std::min(t_grid_cap, g_grid_cap_env) : t_grid_cap) : g_grid_cap_env)
// Tiles per launch of the pipelined / packed kernels (HBEC_CHUNK_TILES):
// a batch is split into launches of whole objects of at most this many
// tiles.  Over one very long launch the blocks' grid-stride fronts drift
// apart and HBM streams less well: 65 536 x 1 MiB 4+2 in one launch ran at
// 72.6 % of 8 TB/s, in 16 launches of 4096 objects at 76.0 %
// (profiles/r02_config5_tune.jsonl).
static const uint64_t g_chunk_tiles = [] {
    const long long v = tune_knob("HBEC_CHUNK_TILES", 0);
    return (uint64_t)(v > 0 ? v : (1ll << 20));
}();
// test hook (hbec_set_odd_chunk_tiles): the odd strided kernels' launch size
static std::atomic<uint64_t> g_odd_chunk_override{0};
static uint64_t odd_chunk_tiles() {
    const uint64_t v = g_odd_chunk_override.load(std::memory_order_relaxed);
    return v ? v : g_chunk_tiles;
}
// the aligned strided (vec / pipelined) kernels' launches (tuning.h
// HBEC_VEC_CHUNK_TILES; a tuning build's HBEC_CHUNK_TILES overrides both)
static const uint64_t g_vec_chunk_tiles = [] {
    const long long v = tune_knob("HBEC_VEC_CHUNK_TILES", tune_knob("HBEC_CHUNK_TILES", 0));
    return (uint64_t)(v > 0 ? v : HBEC_VEC_CHUNK_TILES);
}();

// ---------------------------------------------------------------------------
// Per-device facts (CU count, occupancy per kernel shape)
// ---------------------------------------------------------------------------
struct DeviceInfo {
    int cus = 0;
    std::map<std::pair<int, int>, int> blocks_per_cu;
};

static std::mutex g_dev_mu;
static std::map<int, DeviceInfo> g_devs;

// Occupancy ceiling of the verify kernel (for the tuning override).
static int bpc_occ_cap(int k, int r) {
    int b = 1;
    if (verify_occupancy(k, r, &b) != hipSuccess) return 1;
    return b;
}

static int current_device(int* dev) {
    hipError_t e = hipGetDevice(dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    return HBEC_OK;
}

static int device_blocks(int dev, int k, int r, int pipe, int force_stream, int* cus, int* per_cu) {
    std::lock_guard<std::mutex> g(g_dev_mu);
    DeviceInfo& d = g_devs[dev];
    if (d.cus == 0) {
        hipDeviceProp_t p;
        hipError_t e = hipGetDeviceProperties(&p, dev);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
        d.cus = p.multiProcessorCount;
    }
    // pipe: 1 = pipelined kernel, 2 = packed kernel (short shards), 3 = unaligned kernel
    const int key_k = pipe == 3 ? 3000 : (force_stream ? -k : (pipe == 2 ? 2000 + k : (pipe ? 1000 + k : k)));
    auto it = d.blocks_per_cu.find({key_k, r});
    if (it == d.blocks_per_cu.end()) {
        int b = 0;
        hipError_t e = pipe == 3   ? unaligned_occupancy(r, &b)
                       : pipe == 2 ? packed_occupancy(k, r, &b)
                                   : vec_occupancy(k, r, pipe, force_stream, &b);
        if (e != hipSuccess) return hip_fail(e, "occupancy query");
        if (b < 1) b = 1;
        it = d.blocks_per_cu.emplace(std::make_pair(key_k, r), b).first;
    }
    *cus = d.cus;
    *per_cu = it->second;
    return HBEC_OK;
}

// ---------------------------------------------------------------------------
// Shards at any alignment (gf_odd, odd.hip)
// ---------------------------------------------------------------------------
static int cu_count(int dev, int* cus) {
    std::lock_guard<std::mutex> g(g_dev_mu);
    DeviceInfo& d = g_devs[dev];
    if (d.cus == 0) {
        hipDeviceProp_t p;
        hipError_t e = hipGetDeviceProperties(&p, dev);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
        d.cus = p.multiProcessorCount;
    }
    *cus = d.cus;
    return HBEC_OK;
}

// Per-object records of a strided record pass depend only on the views (bases
// and strides), the object count, S and the pass shape, never on the data or
// the coefficients.  Views coded again (a service reusing its batch buffers,
// bench loops) get the records built the first time instead of a
// gf_odd_objrec launch per call (10 us of a 16 384-object 8+3 call).  A key
// is cached on its second sighting, so one-off views (per-call entries) never
// allocate; at most kObjRecMax entries / kObjRecMaxBytes, never evicted (a
// full cache codes new views with per-call scratch records).  Built on the
// first caller's stream; another stream waits for the build's event.
namespace {
struct ObjRecCache {
    struct Entry {
        std::vector<uint64_t> key;
        uint32_t* d = nullptr;
        hipEvent_t ev = nullptr;
        hipStream_t stream = nullptr;
    };
    std::mutex mu;
    std::vector<Entry> entries;
    std::deque<std::vector<uint64_t>> seen;  // keys seen once
    uint64_t bytes = 0, hits = 0;
};
constexpr size_t kObjRecMax = 16, kObjRecSeen = 64;
constexpr uint64_t kObjRecMaxBytes = 64ull << 20;
ObjRecCache& objrec_cache() {
    static ObjRecCache* c = new ObjRecCache;  // process lifetime (no teardown against the HIP runtime)
    return *c;
}
}  // namespace

// *out = the cached records of this launch's views, or nullptr (build them)
static int objrec_cached(const PassArgs& c, int K, int R, int m, int dev, uint64_t rw, hipStream_t stream,
                         uint32_t** out) {
    *out = nullptr;
    static const bool on = tune_knob("HBEC_ODD_REC_CACHE", 1) != 0;  // tuning builds: 0 = rebuild every call
    if (!on) return HBEC_OK;
    std::vector<uint64_t> key{(uint64_t)dev, (uint64_t)K, (uint64_t)R, (uint64_t)m, c.n_obj, c.shard_len};
    for (int j = 0; j < K; ++j) {
        key.push_back(reinterpret_cast<uintptr_t>(c.in[j]));
        key.push_back(c.in_stride[j]);
    }
    for (int r = 0; r < R; ++r) {
        key.push_back(reinterpret_cast<uintptr_t>(c.out[r]));
        key.push_back(c.out_stride[r]);
    }
    ObjRecCache& C = objrec_cache();
    std::lock_guard<std::mutex> lk(C.mu);
    for (const auto& x : C.entries) {
        if (x.key != key) continue;
        if (x.stream != stream) {
            hipError_t e = hipStreamWaitEvent(stream, x.ev, 0);
            if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent (object records)");
        }
        *out = x.d;
        ++C.hits;
        return HBEC_OK;
    }
    const auto it = std::find(C.seen.begin(), C.seen.end(), key);
    if (it == C.seen.end()) {
        C.seen.push_back(std::move(key));
        if (C.seen.size() > kObjRecSeen) C.seen.pop_front();
        return HBEC_OK;
    }
    C.seen.erase(it);
    const uint64_t bytes = c.n_obj * rw * 4;
    if (C.entries.size() >= kObjRecMax || C.bytes + bytes > kObjRecMaxBytes) return HBEC_OK;
    ObjRecCache::Entry x;
    x.key = std::move(key);
    x.stream = stream;
    if (hipMalloc(reinterpret_cast<void**>(&x.d), bytes) != hipSuccess) {
        (void)hipGetLastError();  // HBM full: scratch records
        return HBEC_OK;
    }
    hipError_t e = launch_odd_objrec(K, R, m, c, x.d, stream);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&x.ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(x.ev, stream);
    if (e != hipSuccess) {
        if (x.ev) (void)hipEventDestroy(x.ev);
        (void)hipFree(x.d);
        return hip_fail(e, "launch gf_odd_objrec (cached)");
    }
    C.bytes += bytes;
    *out = x.d;
    C.entries.push_back(std::move(x));
    return HBEC_OK;
}

// One pass of a (K <= kMaxK inputs, R <= kMaxR outputs) over strided views at
// any alignment, as launches of <= kOddMaxK inputs: the first accumulates
// only when `accumulate`, the later ones always.  mode 2 (verify) flags
// objects instead of writing (K <= kOddMaxK).  One 4-wave block per CU (the
// pipelined kernels' HBM sweet spot), launches of <= g_chunk_tiles tiles.
static int odd_launches(const PassArgs& a, int K, int R, int mode, bool accumulate, uint64_t n_obj,
                        uint64_t shard_len, uint32_t* flags, int dev, hipStream_t stream) {
    int cus = 0;
    int rc = cu_count(dev, &cus);
    if (rc) return rc;
    // the main kernel codes the guard band too (HBEC_ODD_EDGE_FUSE): one
    // apply launch group whose shards span >= 2 tiles (the edge tiles are
    // each shard's first and last)
    bool fused = false;
    if (shard_len > odd_min_main()) {
        for (int c1 = 0; c1 < K; c1 += kOddMaxK) {
            const int K1 = std::min(kOddMaxK, K - c1);
            PassArgs b = a;
            for (int j = 0; j < K1; ++j) {
                b.in[j] = a.in[c1 + j];
                b.in_stride[j] = a.in_stride[c1 + j];
                for (int r = 0; r < R; ++r)
                    for (int q = 0; q < 5; ++q) b.tab[r][j][q] = a.tab[r][c1 + j][q];
            }
            const int m = mode == 2 ? 2 : ((accumulate || c1 > 0) ? 1 : 0);
            // Verify with register tables (K <= 8) stays on gf_odd: the record
            // kernel's 8+3 Verify ran at the same speed with the same traffic
            // (1.11 vs 1.10 x, bench.py's leg); K > 8 needs its LDS tables
            // fixed encode matrices of a compiled shape: the bit-plane record kernel
            const int xs = odd_bp_schedule(K1, R, m, b.tab, false);
            const bool use_rec = xs >= 0 || ((m != 2 || K1 > 8) && odd_uses_records(K1, R));
            const uint64_t tpo = odd_tiles_per_obj(K1, m, shard_len, use_rec, xs);
            const uint64_t max_obj = std::max<uint64_t>(1, std::min<uint64_t>((1ull << 31), odd_chunk_tiles()) / tpo);
            // per-object records of one launch's objects (stream-ordered
            // scratch of at most max_obj records, rebuilt per launch, freed
            // after the pass): device memory bounded by the chunk, not the batch
            uint32_t* recs = nullptr;  // scratch, allocated when a launch's records are not cached
            const uint64_t rw = odd_rec_words(K1, R, m);
            for (uint64_t o0 = 0; o0 < n_obj; o0 += max_obj) {
                const uint64_t no = std::min(max_obj, n_obj - o0);
                PassArgs c = b;
                for (int j = 0; j < K1; ++j) c.in[j] = b.in[j] + o0 * b.in_stride[j];
                for (int r = 0; r < R; ++r) c.out[r] = b.out[r] + o0 * b.out_stride[r];
                c.n_obj = no;
                c.shard_len = shard_len;
                uint32_t* lrecs = nullptr;
                if (use_rec) {
                    rc = objrec_cached(c, K1, R, m, dev, rw, stream, &lrecs);
                    if (rc) {
                        if (recs) scratch_free(recs, stream);
                        return rc;
                    }
                    if (!lrecs) {
                        if (!recs) {
                            rc = scratch_alloc(std::min(n_obj, max_obj) * rw * 4, stream, reinterpret_cast<void**>(&recs));
                            if (rc) return rc;
                        }
                        hipError_t e = launch_odd_objrec(K1, R, m, c, recs, stream);
                        if (e != hipSuccess) {
                            scratch_free(recs, stream);
                            return hip_fail(e, "launch gf_odd_objrec");
                        }
                        lrecs = recs;
                    }
                }
                c.tiles_per_obj = (uint32_t)tpo;
                c.n_tiles = (uint32_t)(no * tpo);
                c.fuse = odd_edge_fuse(K1, R, m, use_rec, xs, false, shard_len) && K <= kOddMaxK && tpo >= 2 &&
                                 shard_len < (1ull << 30) ? 1u : 0u;
                fused = c.fuse != 0u;
                const uint64_t wpb = odd_waves_per_block(xs);
                const uint64_t want = (c.n_tiles + wpb - 1) / wpb;
                const uint64_t cap = (uint64_t)cus * (uint64_t)odd_blocks_per_cu(m, K1, R, false, use_rec, xs);
                int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, cap));
                if (g_grid_cap > 0) grid = std::min(grid, g_grid_cap);
                hipError_t e = launch_odd(K1, R, m, c, flags ? flags + o0 : nullptr, lrecs, grid, stream, xs);
                if (e != hipSuccess) {
                    if (recs) scratch_free(recs, stream);
                    return hip_fail(e, "launch gf_odd");
                }
            }
            if (recs) scratch_free(recs, stream);
        }
    }
    // the guard-band bytes of every shard, all K inputs of the pass at once
    // (on a second stream beside the main kernel this ran 0.6-3 points
    // slower, the scattered edge lines disturbing the main stream; before the
    // main kernel, within +-1: r05_ab_edges.jsonl)
    if (fused) return HBEC_OK;
    PassArgs g = a;
    g.n_obj = n_obj;
    g.shard_len = shard_len;
    hipError_t e = launch_odd_edges(K, R, mode == 2 ? 2 : (accumulate ? 1 : 0), g, flags, stream);
    if (e != hipSuccess) return hip_fail(e, "launch gf_odd_edges");
    return HBEC_OK;
}

static int apply_odd(const PassArgs& a, int K, int R, bool accumulate, uint64_t n_obj, uint64_t shard_len, int dev,
                     hipStream_t stream) {
    return odd_launches(a, K, R, 0, accumulate, n_obj, shard_len, nullptr, dev, stream);
}

// ---------------------------------------------------------------------------
// Generic pass planner: out[R] (^)= C[R][K] x in[K] over strided views
// ---------------------------------------------------------------------------
static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
static bool vec_len(uint64_t v) { return v % 16 == 0; }
// 16-B-aligned views the record kernels (gf_odd_rec) code faster than the
// aligned ones, interleaved A/B over 40 shapes (profiles/r05_ab_route.jsonl):
//  * 9 <= k <= 12 at any pitch: one bit-plane / record pass against the
//    tables at 1-KiB tiles, encode +2 to +9 points, 12+4 reconstruct +3;
//  * 5 <= k <= 8 when a base, object stride or S is not a multiple of the
//    128-B line (+0.4 to +9: the aligned kernels lose 4-10 points there, the
//    record kernels with their per-tile block barrier do not), or with 4
//    output rows (6+4 / 8+4 +7 / +10, their plans +22 to +27: the stripe
//    kernels take 3 rows per pass), as long as a pass is K R <= 24 or has a
//    compiled bit-plane schedule (7+4 on tables: -8);
//  * k <= 4, line-aligned 5 <= k <= 8 with <= 3 rows, and short shards
//    (tuning.h HBEC_REC_ROUTE_MIN_S*) stay on the aligned kernels.
// Tuning builds: HBEC_REC_ROUTE=0 keeps every 16-B-aligned view there.
static const int g_rec_route = (int)tune_knob("HBEC_REC_ROUTE", 1);
bool rec_route(int cols, int rows, uint64_t shard_len, bool line_aligned, bool bitplane) {
    if (!g_rec_route || !odd_enabled() || cols < 5 || cols > kOddMaxK || !pos32_shard(shard_len)) return false;
    if (cols > 8) return shard_len >= HBEC_REC_ROUTE_MIN_S_BIG;
    const int r = std::min(rows, kMaxR);
    return shard_len >= HBEC_REC_ROUTE_MIN_S && (!line_aligned || r >= 4) && (cols * r <= 24 || bitplane);
}
// the first pass's rows (<= kMaxR of `rows`, coefficients row-major with
// `cols` per row) have a compiled bit-plane schedule
static bool bitplane_rows(int k, int rows, const uint8_t* coeffs, int cols, bool plan) {
    if (k > kMaxK) return false;
    uint32_t tab[kMaxR][kMaxK][5] = {};
    const int r = std::min(rows, kMaxR);
    for (int q = 0; q < r; ++q)
        for (int j = 0; j < k; ++j) tab[q][j][0] = (uint32_t)coeffs[(size_t)q * cols + j] << 8;  // byte 1 = c * 1
    return odd_bp_schedule(k, r, 0, tab, plan) >= 0;
}
static bool line_aligned(const void* p, uint64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 127u) == 0 && stride % 128 == 0;
}

static int apply_wide(int rows, int cols, const uint8_t* coeffs, const hbec_view* in, const hbec_view* out,
                      uint64_t n_obj, uint64_t shard_len, hipStream_t stream);

int apply_views(int rows, int cols, const uint8_t* coeffs, const hbec_view* in, const hbec_view* out,
                uint64_t n_obj, uint64_t shard_len, hipStream_t stream) {
    if (rows <= 0 || n_obj == 0 || shard_len == 0) return HBEC_OK;
    if (cols <= 0 || !coeffs || !in || !out) return fail(HBEC_ERR_INVALID_ARG, "apply: bad arguments");
    bool vec = vec_len(shard_len);
    for (int c = 0; c < cols && vec; ++c) vec = aligned16(in[c].base) && vec_len(in[c].obj_stride);
    for (int r = 0; r < rows && vec; ++r) vec = aligned16(out[r].base) && vec_len(out[r].obj_stride);
    bool line = vec && shard_len % 128 == 0;
    for (int c = 0; c < cols && line; ++c) line = line_aligned(in[c].base, in[c].obj_stride);
    for (int r = 0; r < rows && line; ++r) line = line_aligned(out[r].base, out[r].obj_stride);
    // the schedule match only where it can change the route (rec_route with and without it differ)
    const bool to_rec = vec && rec_route(cols, rows, shard_len, line, true) &&
                        (rec_route(cols, rows, shard_len, line, false) || bitplane_rows(cols, rows, coeffs, cols, false));
    for (int c = 0; c < cols; ++c)
        if (!in[c].base) return fail(HBEC_ERR_INVALID_ARG, "apply: null input view");
    for (int r = 0; r < rows; ++r)
        if (!out[r].base) return fail(HBEC_ERR_INVALID_ARG, "apply: null output view");
    int dev = 0;
    int rc = current_device(&dev);
    if (rc) return rc;
    const int force_stream = g_force_stream.load();
    // k > 16 at any alignment: one gf_wide pass instead of accumulate passes
    // (9..12 take gf_odd, 13..16 the round-2 one-pass gf_apply_unaligned)
    if (!vec && cols > kMaxK && cols <= 256 && pos32_shard(shard_len))
        return apply_wide(rows, cols, coeffs, in, out, n_obj, shard_len, stream);

    for (int r0 = 0; r0 < rows; r0 += kMaxR) {
        const int R = std::min(kMaxR, rows - r0);
        for (int c0 = 0; c0 < cols; c0 += kMaxK) {
            const int K = std::min(kMaxK, cols - c0);
            PassArgs a;
            std::memset(&a, 0, sizeof(a));
            for (int j = 0; j < K; ++j) {
                a.in[j] = static_cast<const uint8_t*>(in[c0 + j].base);
                a.in_stride[j] = in[c0 + j].obj_stride;
            }
            for (int r = 0; r < R; ++r) {
                a.out[r] = static_cast<uint8_t*>(out[r0 + r].base);
                a.out_stride[r] = out[r0 + r].obj_stride;
                for (int j = 0; j < K; ++j) perm_table(coeffs[(size_t)(r0 + r) * cols + c0 + j], a.tab[r][j]);
            }
            a.shard_len = shard_len;
            a.accumulate = c0 > 0 ? 1u : 0u;
            if (vec && is_packed_shape(K, R, shard_len, c0 > 0, force_stream)) {
                // short shards: wave tiles across objects (gf_apply_packed)
                int cus = 0, per_cu = 0;
                rc = device_blocks(dev, K, R, 2, 0, &cus, &per_cu);
                if (rc) return rc;
                const uint64_t spo = shard_len / 16;
                const uint64_t te = (uint64_t)packed_tile_elems(K);
                uint64_t max_obj = std::max<uint64_t>(1, ((1ull << 31) - te) / spo);  // n_elems < 2^31
                max_obj = std::min(max_obj, std::max<uint64_t>(1, g_chunk_tiles * te / spo));
                for (uint64_t o0 = 0; o0 < n_obj; o0 += max_obj) {
                    const uint64_t no = std::min(max_obj, n_obj - o0);
                    PassArgs b = a;
                    for (int j = 0; j < K; ++j) b.in[j] = a.in[j] + o0 * a.in_stride[j];
                    for (int r = 0; r < R; ++r) b.out[r] = a.out[r] + o0 * a.out_stride[r];
                    b.n_obj = no;
                    b.elems_per_obj = (uint32_t)spo;
                    b.n_elems = (uint32_t)(no * spo);
                    b.n_tiles = (uint32_t)((no * spo + te - 1) / te);
                    const uint64_t wpb = (uint64_t)kPipeBlockThreads / 64;
                    const uint64_t want_blocks = (b.n_tiles + wpb - 1) / wpb;
                    const uint64_t cap = (uint64_t)cus * (uint64_t)(g_blocks_per_cu_override > 0
                                                                         ? g_blocks_per_cu_override
                                                                         : per_cu);
                    int grid = (int)std::max<uint64_t>(1, std::min(want_blocks, cap));
                    if (g_grid_cap > 0) grid = std::min(grid, g_grid_cap);
                    hipError_t e = launch_packed(K, R, b, grid, stream);
                    if (e != hipSuccess) return hip_fail(e, "launch gf_apply_packed");
                }
            } else if (vec && !to_rec) {
                int cus = 0, per_cu = 0;
                rc = device_blocks(dev, K, R, is_pipe_shape(K, R, shard_len, force_stream) && c0 == 0, force_stream,
                                   &cus, &per_cu);
                if (rc) return rc;
                const uint64_t tile = (uint64_t)vec_tile_bytes(K, R, shard_len, c0 > 0, force_stream);
                const uint64_t tpo = (shard_len + tile - 1) / tile;
                // keep n_tiles < 2^31 (and <= g_vec_chunk_tiles) per launch: split the batch by objects
                const uint64_t max_obj = std::max<uint64_t>(1, std::min<uint64_t>((1ull << 31), g_vec_chunk_tiles) / tpo);
                for (uint64_t o0 = 0; o0 < n_obj; o0 += max_obj) {
                    const uint64_t no = std::min(max_obj, n_obj - o0);
                    PassArgs b = a;
                    for (int j = 0; j < K; ++j) b.in[j] = a.in[j] + o0 * a.in_stride[j];
                    for (int r = 0; r < R; ++r) b.out[r] = a.out[r] + o0 * a.out_stride[r];
                    b.n_obj = no;
                    b.tiles_per_obj = (uint32_t)tpo;
                    b.n_tiles = (uint32_t)(no * tpo);
                    const uint64_t wpb = (uint64_t)vec_block_threads(K, R, shard_len, c0 > 0, force_stream) / 64;
                    const uint64_t want_blocks = (b.n_tiles + wpb - 1) / wpb;
                    const uint64_t cap = (uint64_t)cus * (uint64_t)(g_blocks_per_cu_override > 0
                                                                         ? g_blocks_per_cu_override
                                                                         : per_cu);
                    int grid = (int)std::max<uint64_t>(1, std::min(want_blocks, cap));
                    if (g_grid_cap > 0) grid = std::min(grid, g_grid_cap);
                    hipError_t e = launch_vec(K, R, b, grid, stream, force_stream);
                    if (e != hipSuccess) return hip_fail(e, "launch gf_apply_vec");
                }
            } else if (odd_enabled() && cols <= kOddMaxK && pos32_shard(shard_len)) {
                // any alignment / length: gf_odd (odd.hip), passes of <= 8 inputs,
                // later ones accumulating into the outputs
                rc = apply_odd(a, K, R, c0 > 0, n_obj, shard_len, dev, stream);
                if (rc) return rc;
            } else {
                // any alignment: aligned 16-B accesses with in-register shifts (gf_apply_unaligned)
                int cus = 0, per_cu = 0;
                rc = device_blocks(dev, K, R, 3, 0, &cus, &per_cu);
                if (rc) return rc;
                if (g_unaligned_bpc > 0) per_cu = std::min(per_cu, g_unaligned_bpc);
                const uint64_t tpo = unaligned_tiles_per_obj(shard_len);
                const uint64_t max_obj = std::max<uint64_t>(1, std::min<uint64_t>((1ull << 31), g_chunk_tiles) / tpo);
                for (uint64_t o0 = 0; o0 < n_obj; o0 += max_obj) {
                    const uint64_t no = std::min(max_obj, n_obj - o0);
                    PassArgs b = a;
                    for (int j = 0; j < K; ++j) b.in[j] = a.in[j] + o0 * a.in_stride[j];
                    for (int r = 0; r < R; ++r) b.out[r] = a.out[r] + o0 * a.out_stride[r];
                    b.n_obj = no;
                    b.tiles_per_obj = (uint32_t)tpo;
                    b.n_tiles = (uint32_t)(no * tpo);
                    const uint64_t want_blocks = (b.n_tiles + kBlockThreads / 64 - 1) / (kBlockThreads / 64);
                    int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want_blocks, (uint64_t)cus * per_cu));
                    if (g_grid_cap > 0) grid = std::min(grid, g_grid_cap);
                    hipError_t e = launch_unaligned(K, R, b, grid, stream);
                    if (e != hipSuccess) return hip_fail(e, "launch gf_apply_unaligned");
                }
            }
        }
    }
    return HBEC_OK;
}

// ---------------------------------------------------------------------------
// Staging pool for the host-memory API (one stream + device buffer each)
// ---------------------------------------------------------------------------
struct Staging {
    int dev = 0;
    hipStream_t stream = nullptr;
    uint8_t* dbuf = nullptr;
    size_t dcap = 0;
    // pinned, device-mapped host bounce buffer (per-call host path, "mapped" mode)
    uint8_t* hbuf = nullptr;
    uint64_t hbuf_dev = 0;
    size_t hcap = 0;
    // one event per column piece of a pipelined per-call apply (created on first use)
    std::vector<hipEvent_t> ev;
};

// Per-call host path for pageable shards (tuning knob HBEC_PERCALL_DMA):
//   "mapped" (default): the calling thread copies the inputs into a pinned,
//     device-mapped bounce buffer, the kernel reads them and writes the
//     outputs there over PCIe, and the thread copies the outputs back;
//   "dma": one hipMemcpyAsync per shard through a device buffer (the runtime
//     stages each pageable copy itself).
// One 1 MiB 4+2 Encode: 87 us mapped vs 131 us dma (profiles/r01_host_path.jsonl).
static const bool g_percall_mapped = tune_knob("HBEC_PERCALL_DMA", 0) == 0;

// Column pieces of one per-call apply in mapped mode (HBEC_PERCALL_PIECES,
// default 2; shards shorter than 64 KiB are one piece): the calling thread
// copies piece p+1 into the bounce buffer while the kernel codes piece p over
// PCIe, then copies each piece's outputs back as soon as its kernel is done.
// 1 MiB 4+2 Encode from pageable memory, one caller: 77 us in one piece,
// 66 us in 2, 86 us in 4 (per-piece launch cost; profiles/r02_percall_pieces.jsonl).
static const int g_percall_pieces = (int)std::max(1LL, std::min(16LL, tune_knob("HBEC_PERCALL_PIECES", 2)));

// Per-call applies running at once (HBEC_PERCALL_CONCURRENCY, default 16;
// 0 = no limit).  Callers past the limit block on a condition variable
// instead of joining the copy / launch / wait: with 64-128 concurrent callers
// on a 16-core share, the extra threads' bounce-buffer copies and stream
// waits only steal cores from the ones that can make progress.  1 MiB 4+2
// pageable Encode, 128 callers: 6.3 GiB/s unlimited, 26-31 GiB/s at 16
// (profiles/r02_percall_gate.jsonl).
class PercallGate {
  public:
    explicit PercallGate(int limit) : limit_(limit) {}
    // FIFO with direct hand-off: a leaving call gives its slot to the oldest
    // waiter, so a caller that returns and calls again cannot starve threads
    // already queued.  Throughput matched a barging semaphore within run-to-run
    // noise (profiles/r02_percall_gate.jsonl); the hand-off bounds each
    // caller's wait.
    void enter() {
        if (limit_ <= 0) return;
        std::unique_lock<std::mutex> lk(mu_);
        if (running_ < limit_ && waiters_.empty()) {
            ++running_;
            return;
        }
        Waiter w;
        waiters_.push_back(&w);
        w.cv.wait(lk, [&] { return w.granted; });
    }
    void leave() {
        if (limit_ <= 0) return;
        std::lock_guard<std::mutex> g(mu_);
        if (waiters_.empty()) {
            --running_;
            return;
        }
        Waiter* w = waiters_.front();
        waiters_.pop_front();
        w->granted = true;
        w->cv.notify_one();
    }

  private:
    struct Waiter {
        bool granted = false;
        std::condition_variable cv;
    };
    const int limit_;
    int running_ = 0;
    std::deque<Waiter*> waiters_;
    std::mutex mu_;
};

static PercallGate g_percall_gate([] {
    return (int)std::max(0LL, env_knob("HBEC_PERCALL_CONCURRENCY", 16));
}());

struct PercallSlot {
    PercallSlot() { g_percall_gate.enter(); }
    ~PercallSlot() { g_percall_gate.leave(); }
    PercallSlot(const PercallSlot&) = delete;
    PercallSlot& operator=(const PercallSlot&) = delete;
};

static int staging_events(Staging* s, size_t n) {
    while (s->ev.size() < n) {
        hipEvent_t e = nullptr;
        hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (r != hipSuccess) return hip_fail(r, "hipEventCreate");
        s->ev.push_back(e);
    }
    return HBEC_OK;
}

static int staging_host(Staging* s, size_t bytes) {
    if (s->hcap >= bytes) return HBEC_OK;
    if (s->hbuf) (void)hipHostFree(s->hbuf);
    s->hbuf = nullptr;
    s->hbuf_dev = 0;
    s->hcap = 0;
    const size_t cap = std::max<size_t>(bytes, 2 << 20);
    void* h = nullptr;
    hipError_t e = hipHostMalloc(&h, cap, hipHostMallocMapped);
    if (e != hipSuccess) return hip_fail(e, "hipHostMalloc bounce");
    void* d = nullptr;
    e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        return hip_fail(e, "hipHostGetDevicePointer bounce");
    }
    s->hbuf = static_cast<uint8_t*>(h);
    s->hbuf_dev = reinterpret_cast<uint64_t>(d);
    s->hcap = cap;
    return HBEC_OK;
}

static std::mutex g_pool_mu;
static std::vector<Staging*> g_pool;

static int staging_acquire(size_t bytes, Staging** out) {
    int dev = 0;
    int rc = current_device(&dev);
    if (rc) return rc;
    Staging* s = nullptr;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); ++i)
            if (g_pool[i]->dev == dev) {
                s = g_pool[i];
                g_pool.erase(g_pool.begin() + i);
                break;
            }
    }
    if (!s) {
        s = new Staging();
        s->dev = dev;
        hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete s;
            return hip_fail(e, "hipStreamCreate");
        }
    }
    if (s->dcap < bytes) {
        if (s->dbuf) (void)hipFree(s->dbuf);
        s->dbuf = nullptr;
        s->dcap = 0;
        size_t cap = std::max<size_t>(bytes, 1 << 20);
        hipError_t e = hipMalloc(&s->dbuf, cap);
        if (e != hipSuccess) {
            std::lock_guard<std::mutex> g(g_pool_mu);
            g_pool.push_back(s);
            return hip_fail(e, "hipMalloc staging");
        }
        s->dcap = cap;
    }
    *out = s;
    return HBEC_OK;
}

static void staging_release(Staging* s) {
    std::lock_guard<std::mutex> g(g_pool_mu);
    g_pool.push_back(s);
}

}  // namespace hbec

// ---------------------------------------------------------------------------
// Codec
// ---------------------------------------------------------------------------
struct hbec_codec {
    int k = 0, m = 0;
    std::vector<uint8_t> matrix;  // (k+m) x k
    std::mutex mu;
    std::map<std::vector<int>, std::vector<uint8_t>> inv_cache;  // survivors -> inv(sub)
    bool bp_plan = false;  // the parity rows have a compiled bit-plane plan schedule (set by hbec_new)
};

namespace hbec {

bool plan_rec_route(const hbec_codec* c, uint64_t shard_len, bool line_aligned) {
    return rec_route(c->k, c->m, shard_len, line_aligned, c->bp_plan);  // once per stripe: no per-call matching
}

// Decode rows for a present mask: survivors = first k present shards.
static int decode_rows(hbec_codec* c, const std::vector<uint8_t>& present, bool data_only,
                       std::vector<int>& survivors, std::vector<int>& outputs, std::vector<uint8_t>& rows) {
    const int k = c->k, n = c->k + c->m;
    survivors.clear();
    for (int i = 0; i < n && (int)survivors.size() < k; ++i)
        if (present[i]) survivors.push_back(i);
    if ((int)survivors.size() < k) return fail(HBEC_ERR_TOO_FEW_SHARDS, "too few shards given");
    outputs.clear();
    for (int i = 0; i < n; ++i)
        if (!present[i] && (i < k || !data_only)) outputs.push_back(i);
    std::vector<uint8_t> inv;
    {
        std::lock_guard<std::mutex> g(c->mu);
        auto it = c->inv_cache.find(survivors);
        if (it != c->inv_cache.end()) {
            inv = it->second;
        } else {
            std::vector<uint8_t> sub((size_t)k * k);
            for (int r = 0; r < k; ++r)
                std::memcpy(&sub[(size_t)r * k], &c->matrix[(size_t)survivors[r] * k], k);
            inv.resize((size_t)k * k);
            if (!invert(k, sub.data(), inv.data())) return fail(HBEC_ERR_SINGULAR, "matrix is singular");
            c->inv_cache.emplace(survivors, inv);
        }
    }
    const Field& F = field();
    rows.assign(outputs.size() * (size_t)k, 0);
    for (size_t o = 0; o < outputs.size(); ++o) {
        const int i = outputs[o];
        uint8_t* row = &rows[o * k];
        if (i < k) {
            std::memcpy(row, &inv[(size_t)i * k], k);
        } else {  // parity row fused with the inverse: M[i] x inv
            for (int t = 0; t < k; ++t) {
                const uint8_t mc = c->matrix[(size_t)i * k + t];
                if (!mc) continue;
                for (int j = 0; j < k; ++j) row[j] ^= F.mul(mc, inv[(size_t)t * k + j]);
            }
        }
    }
    return HBEC_OK;
}

// klauspost checkShards: size of first non-empty shard, then equality.
static int check_shards(const size_t* lens, int n, bool nilok, size_t* size) {
    size_t s = 0;
    for (int i = 0; i < n; ++i)
        if (lens[i] != 0) {
            s = lens[i];
            break;
        }
    if (s == 0) return fail(HBEC_ERR_SHARD_NO_DATA, "no shard data");
    for (int i = 0; i < n; ++i)
        if (lens[i] != s && (lens[i] != 0 || !nilok)) return fail(HBEC_ERR_SHARD_SIZE, "shard sizes do not match");
    *size = s;
    return HBEC_OK;
}

static uint64_t round16(uint64_t v) { return (v + 15) & ~uint64_t(15); }

// Host-memory apply: copy inputs in, run one object, copy outputs back.
static int host_apply(int rows, int cols, const uint8_t* coeffs, const uint8_t* const* in, uint8_t* const* out,
                      size_t len) {
    if (rows == 0) return HBEC_OK;
    const uint64_t pad = round16(len);
    // Zero-copy: every shard in pinned, device-mapped memory -> the kernel
    // reads and writes them in place over PCIe (no staging copies).
    std::vector<hbec_view> zin(cols), zout(rows);
    // (odd lengths / offsets too: apply_views takes them to gf_apply_unaligned)
    bool zero_copy = len > 0 && (len % 16 == 0 || (zero_copy_any_alignment()));
    for (int j = 0; j < cols && zero_copy; ++j) {
        const uint64_t d = pinned_device_addr(in[j], len);
        zero_copy = d != 0;
        zin[j] = {reinterpret_cast<uint8_t*>(d), 0};
    }
    for (int r = 0; r < rows && zero_copy; ++r) {
        const uint64_t d = pinned_device_addr(out[r], len);
        zero_copy = d != 0;
        zout[r] = {reinterpret_cast<uint8_t*>(d), 0};
    }
    PercallSlot slot;
    Staging* s = nullptr;
    int rc = staging_acquire(zero_copy || g_percall_mapped ? 16 : (size_t)pad * (cols + rows), &s);
    if (rc) return rc;
    if (zero_copy) {
        rc = apply_views(rows, cols, coeffs, zin.data(), zout.data(), 1, len, s->stream);
        hipError_t e = hipStreamSynchronize(s->stream);
        staging_release(s);
        if (rc) return rc;
        if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
        return HBEC_OK;
    }
    std::vector<hbec_view> vin(cols), vout(rows);
    if (g_percall_mapped) {
        rc = staging_host(s, (size_t)pad * (cols + rows));
        if (rc) {
            staging_release(s);
            return rc;
        }
        // column pieces, 4 KiB-aligned, the last one padded to 16 B
        const uint64_t want = len >= (64u << 10) ? (uint64_t)g_percall_pieces : 1u;
        const uint64_t step = ((pad + want - 1) / want + 4095) & ~uint64_t(4095);
        std::vector<uint64_t> cut;
        for (uint64_t c0 = 0; c0 < pad; c0 += step) cut.push_back(c0);
        cut.push_back(pad);
        const size_t np = cut.size() - 1;
        rc = staging_events(s, np);
        hipError_t es = hipSuccess;
        size_t launched = 0;
        for (size_t p = 0; p < np && !rc; ++p, ++launched) {
            const uint64_t c0 = cut[p], c1 = cut[p + 1];
            const uint64_t copy = std::min<uint64_t>(c1, len) - c0;  // caller bytes in this piece
            for (int j = 0; j < cols; ++j) {
                uint8_t* dst = s->hbuf + (size_t)j * pad + c0;
                std::memcpy(dst, in[j] + c0, copy);
                if (c1 > len) std::memset(dst + copy, 0, c1 - c0 - copy);  // deterministic pad bytes
                vin[j] = {reinterpret_cast<uint8_t*>(s->hbuf_dev + (size_t)j * pad + c0), 0};
            }
            for (int r = 0; r < rows; ++r)
                vout[r] = {reinterpret_cast<uint8_t*>(s->hbuf_dev + (size_t)(cols + r) * pad + c0), 0};
            rc = apply_views(rows, cols, coeffs, vin.data(), vout.data(), 1, c1 - c0, s->stream);
            if (!rc) {
                es = hipEventRecord(s->ev[p], s->stream);
                if (es != hipSuccess) rc = hip_fail(es, "hipEventRecord");
            }
        }
        for (size_t p = 0; p < launched; ++p) {  // outputs back, piece by piece as each completes
            es = hipEventSynchronize(s->ev[p]);
            if (es != hipSuccess) {
                if (!rc) rc = hip_fail(es, "hipEventSynchronize");
                break;
            }
            if (rc) continue;
            const uint64_t c0 = cut[p], copy = std::min<uint64_t>(cut[p + 1], len) - c0;
            for (int r = 0; r < rows; ++r) std::memcpy(out[r] + c0, s->hbuf + (size_t)(cols + r) * pad + c0, copy);
        }
        es = hipStreamSynchronize(s->stream);
        staging_release(s);
        if (rc) return rc;
        if (es != hipSuccess) return hip_fail(es, "hipStreamSynchronize");
        return HBEC_OK;
    }
    hipError_t e = hipSuccess;
    for (int j = 0; j < cols && e == hipSuccess; ++j) {
        vin[j] = {s->dbuf + (size_t)j * pad, 0};
        e = hipMemcpyAsync(vin[j].base, in[j], len, hipMemcpyHostToDevice, s->stream);
    }
    for (int r = 0; r < rows; ++r) vout[r] = {s->dbuf + (size_t)(cols + r) * pad, 0};
    if (e != hipSuccess) {
        staging_release(s);
        return hip_fail(e, "hipMemcpyAsync H2D");
    }
    // process the padded length: bytes past len are don't-care in, don't-care out
    rc = apply_views(rows, cols, coeffs, vin.data(), vout.data(), 1, pad, s->stream);
    for (int r = 0; r < rows && rc == HBEC_OK && e == hipSuccess; ++r)
        e = hipMemcpyAsync(out[r], vout[r].base, len, hipMemcpyDeviceToHost, s->stream);
    hipError_t e2 = hipStreamSynchronize(s->stream);
    staging_release(s);
    if (rc) return rc;
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync D2H");
    if (e2 != hipSuccess) return hip_fail(e2, "hipStreamSynchronize");
    return HBEC_OK;
}

// Shards are the consecutive s-byte slots of one buffer (ecutils.go's databuf).
static bool consecutive(uint8_t* const* shards, int n, size_t s) {
    for (int i = 1; i < n; ++i)
        if (shards[i] != shards[0] + (size_t)i * s) return false;
    return true;
}

// Per-call paths over a databuf (no coalescing): a coalesced group of one.
static int direct_encode(hbec_codec* c, uint8_t* base, uint64_t s) {
    std::vector<uint8_t*> p((size_t)(c->k + c->m));
    for (size_t i = 0; i < p.size(); ++i) p[i] = base + i * s;
    return host_apply(c->m, c->k, c->matrix.data() + (size_t)c->k * c->k, p.data(), p.data() + c->k, s);
}

static int direct_reconstruct(hbec_codec* c, uint8_t* base, uint64_t s, const uint8_t* present, int data_only) {
    const int n = c->k + c->m;
    std::vector<uint8_t> p(present, present + n);
    std::vector<int> surv, outs;
    std::vector<uint8_t> rows;
    int rc = decode_rows(c, p, data_only != 0, surv, outs, rows);
    if (rc) return rc;
    std::vector<const uint8_t*> in(surv.size());
    std::vector<uint8_t*> out(outs.size());
    for (size_t j = 0; j < surv.size(); ++j) in[j] = base + (size_t)surv[j] * s;
    for (size_t o = 0; o < outs.size(); ++o) out[o] = base + (size_t)outs[o] * s;
    return host_apply((int)outs.size(), c->k, rows.data(), in.data(), out.data(), s);
}

static const DirectFns kDirect = {direct_encode, direct_reconstruct};

}  // namespace hbec

using namespace hbec;

extern "C" {

const char* hbec_strerror(int code) {
    switch (code) {
        case HBEC_OK: return "ok";
        case HBEC_ERR_INV_SHARD_NUM: return "cannot create Encoder with zero or less data/parity shards";
        case HBEC_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
        case HBEC_ERR_TOO_FEW_SHARDS: return "too few shards given";
        case HBEC_ERR_SHARD_NO_DATA: return "no shard data";
        case HBEC_ERR_SHARD_SIZE: return "shard sizes do not match";
        case HBEC_ERR_SINGULAR: return "matrix is singular";
        case HBEC_ERR_INVALID_ARG: return "invalid argument";
        case HBEC_ERR_DEVICE: return "device error";
        case HBEC_ERR_NOMEM: return "out of memory";
        case HBEC_ERR_UNEXPECTED_EOF: return "unexpected EOF";
        case HBEC_ERR_IO: return "i/o error";
        case HBEC_ERR_SCHEME: return "invalid EC scheme";
    }
    return "unknown error";
}

const char* hbec_last_error(void) { return t_last_error.c_str(); }

int hbec_version(void) { return HBEC_VERSION; }

int hbec_new(int data_shards, int parity_shards, hbec_codec** out) {
    return hbec::guarded("hbec_new", [&]() -> int {
        if (!out) return fail(HBEC_ERR_INVALID_ARG, "out is NULL");
        *out = nullptr;
        if (data_shards <= 0 || parity_shards < 0)
            return fail(HBEC_ERR_INV_SHARD_NUM, "cannot create Encoder with zero or less data/parity shards");
        if (data_shards + parity_shards > 256)
            return fail(HBEC_ERR_MAX_SHARD_NUM, "cannot create Encoder with more than 256 data+parity shards");
        std::unique_ptr<hbec_codec> c(new (std::nothrow) hbec_codec());
        if (!c) return fail(HBEC_ERR_NOMEM, "codec allocation");
        c->k = data_shards;
        c->m = parity_shards;
        if (!build_matrix(c->k, c->m, c->matrix)) return fail(HBEC_ERR_SINGULAR, "matrix is singular");
        c->bp_plan = c->m > 0 && hbec::bitplane_rows(c->k, c->m, c->matrix.data() + (size_t)c->k * c->k, c->k, true);
        *out = c.release();
        return HBEC_OK;
    });
}

void hbec_free(hbec_codec* codec) { delete codec; }

int hbec_data_shards(const hbec_codec* c) { return c ? c->k : HBEC_ERR_INVALID_ARG; }
int hbec_parity_shards(const hbec_codec* c) { return c ? c->m : HBEC_ERR_INVALID_ARG; }

int hbec_matrix(const hbec_codec* c, uint8_t* out) {
    return hbec::guarded("hbec_matrix", [&]() -> int {
        if (!c || !out) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        std::memcpy(out, c->matrix.data(), c->matrix.size());
        return HBEC_OK;
    });
}

int hbec_encode(hbec_codec* c, uint8_t* const* shards, const size_t* lens, int n_shards) {
    return hbec::guarded("hbec_encode", [&]() -> int {
        if (!c || !shards || !lens) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        if (n_shards != c->k + c->m) return fail(HBEC_ERR_TOO_FEW_SHARDS, "too few shards given");
        size_t s = 0;
        int rc = check_shards(lens, n_shards, false, &s);
        if (rc) return rc;
        for (int i = 0; i < n_shards; ++i)
            if (!shards[i]) return fail(HBEC_ERR_INVALID_ARG, "null shard pointer");
        // one databuf's consecutive slots (every ecutils.go call site): join
        // concurrent callers (coalesce.cpp)
        if (coalesce_enabled() && consecutive(shards, n_shards, s))
            return coalesced_call(c, 0, shards[0], s, nullptr, n_shards, 0, kDirect);
        return host_apply(c->m, c->k, c->matrix.data() + (size_t)c->k * c->k, shards, shards + c->k, s);
    });
}

int hbec_reconstruct(hbec_codec* c, uint8_t* const* shards, size_t* lens, int n_shards, int data_only) {
    return hbec::guarded("hbec_reconstruct", [&]() -> int {
        if (!c || !shards || !lens) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        if (n_shards != c->k + c->m) return fail(HBEC_ERR_TOO_FEW_SHARDS, "too few shards given");
        size_t s = 0;
        int rc = check_shards(lens, n_shards, true, &s);
        if (rc) return rc;
        std::vector<uint8_t> present(n_shards);
        int n_present = 0, data_present = 0;
        for (int i = 0; i < n_shards; ++i) {
            present[i] = lens[i] != 0;
            n_present += present[i];
            if (i < c->k) data_present += present[i];
        }
        if (n_present == n_shards || (data_only && data_present == c->k)) return HBEC_OK;
        if (n_present < c->k) return fail(HBEC_ERR_TOO_FEW_SHARDS, "too few shards given");
        std::vector<int> surv, outs;
        std::vector<uint8_t> rows;
        rc = decode_rows(c, present, data_only != 0, surv, outs, rows);
        if (rc) return rc;
        for (int o : outs)
            if (!shards[o]) return fail(HBEC_ERR_INVALID_ARG, "missing shard has no buffer");
        if (coalesce_enabled() && consecutive(shards, n_shards, s)) {
            rc = coalesced_call(c, 1, shards[0], s, present.data(), n_shards, data_only, kDirect);
        } else {
            std::vector<const uint8_t*> in(surv.size());
            std::vector<uint8_t*> out(outs.size());
            for (size_t j = 0; j < surv.size(); ++j) in[j] = shards[surv[j]];
            for (size_t o = 0; o < outs.size(); ++o) out[o] = shards[outs[o]];
            rc = host_apply((int)outs.size(), c->k, rows.data(), in.data(), out.data(), s);
        }
        if (rc) return rc;
        for (int i : outs) lens[i] = s;
        return HBEC_OK;
    });
}

int hbec_encode_batch(hbec_codec* c, const hbec_view* views, uint64_t n_objects, uint64_t shard_len,
                      void* hip_stream) {
    return hbec::guarded("hbec_encode_batch", [&]() -> int {
        if (!c || !views) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        return apply_views(c->m, c->k, c->matrix.data() + (size_t)c->k * c->k, views, views + c->k, n_objects,
                           shard_len, static_cast<hipStream_t>(hip_stream));
    });
}

int hbec_decode_rows(hbec_codec* c, const uint8_t* present, int data_only, int* survivors, int* outputs,
                     int* n_outputs, uint8_t* rows) {
    return hbec::guarded("hbec_decode_rows", [&]() -> int {
        if (!c || !present || !survivors || !outputs || !n_outputs || !rows)
            return fail(HBEC_ERR_INVALID_ARG, "null argument");
        std::vector<uint8_t> p(present, present + c->k + c->m);
        for (auto& v : p) v = v ? 1 : 0;
        std::vector<int> surv, outs;
        std::vector<uint8_t> r;
        int rc = decode_rows(c, p, data_only != 0, surv, outs, r);
        if (rc) return rc;
        std::copy(surv.begin(), surv.end(), survivors);
        std::copy(outs.begin(), outs.end(), outputs);
        *n_outputs = (int)outs.size();
        std::copy(r.begin(), r.end(), rows);
        return HBEC_OK;
    });
}

int hbec_reconstruct_batch(hbec_codec* c, const hbec_view* views, const uint8_t* present, uint64_t n_objects,
                           uint64_t shard_len, int data_only, void* hip_stream) {
    return hbec::guarded("hbec_reconstruct_batch", [&]() -> int {
        if (!c || !views || !present) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        const int n = c->k + c->m;
        std::vector<uint8_t> p(present, present + n);
        int n_present = 0, data_present = 0;
        for (int i = 0; i < n; ++i) {
            p[i] = p[i] ? 1 : 0;
            n_present += p[i];
            if (i < c->k) data_present += p[i];
        }
        if (n_present == n || (data_only && data_present == c->k)) return HBEC_OK;
        if (n_present < c->k) return fail(HBEC_ERR_TOO_FEW_SHARDS, "too few shards given");
        std::vector<int> surv, outs;
        std::vector<uint8_t> rows;
        int rc = decode_rows(c, p, data_only != 0, surv, outs, rows);
        if (rc) return rc;
        std::vector<hbec_view> vin(surv.size()), vout(outs.size());
        for (size_t j = 0; j < surv.size(); ++j) vin[j] = views[surv[j]];
        for (size_t o = 0; o < outs.size(); ++o) vout[o] = views[outs[o]];
        return apply_views((int)outs.size(), c->k, rows.data(), vin.data(), vout.data(), n_objects, shard_len,
                           static_cast<hipStream_t>(hip_stream));
    });
}

int hbec_apply_batch(int rows, int cols, const uint8_t* coeffs, const hbec_view* in, const hbec_view* out,
                     uint64_t n_objects, uint64_t shard_len, void* hip_stream) {
    return hbec::guarded("hbec_apply_batch", [&]() -> int {
        return apply_views(rows, cols, coeffs, in, out, n_objects, shard_len, static_cast<hipStream_t>(hip_stream));
    });
}

int hbec_fill_splitmix(void* dst, uint64_t n_objects, uint64_t obj_len, uint64_t obj_stride, uint64_t base_seed,
                       uint64_t first, void* hip_stream) {
    return hbec::guarded("hbec_fill_splitmix", [&]() -> int {
        if (!dst) return fail(HBEC_ERR_INVALID_ARG, "null dst");
        if (n_objects == 0 || obj_len == 0) return HBEC_OK;
        const uint64_t words = ((obj_len + 7) / 8) * n_objects;
        const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((words + kBlockThreads - 1) / kBlockThreads, 16384));
        hipError_t e = launch_fill(static_cast<uint8_t*>(dst), n_objects, obj_len, obj_stride, base_seed, first, grid,
                                   static_cast<hipStream_t>(hip_stream));
        if (e != hipSuccess) return hip_fail(e, "launch fill_splitmix");
        return HBEC_OK;
    });
}

// ---- Encoder.Verify ------------------------------------------------------
// Verify of k > 8 data shards: gf_verify_wide in one read-only pass; shards
// beyond the 32-bit kernels' range take gf_verify_unaligned (k <= 16) or the
// scratch recompute (k > 16).

// gf_wide launches over n_obj objects of k input views: per group of <= 8
// rows one device blob {in_base[k], in_stride[k], tables[k][words]} (the
// input bases are re-uploaded, shifted, for each chunk of objects), then
// launch(args, first object) per chunk of < 2^31 (and <= g_chunk_tiles) tiles.
}  // extern "C"

namespace hbec {  // gf_wide host side (templates need C++ linkage)

template <class Launch>
static int wide_launches(const hbec_view* in, int k, const uint8_t* coeffs, int rows, const hbec_view* out,
                         uint64_t n_obj, uint64_t shard_len, uint64_t tpo, hipStream_t stream, Launch launch) {
    for (int r0 = 0; r0 < rows; r0 += kWideMaxR) {
        const int R = std::min(kWideMaxR, rows - r0);
        const uint32_t tw = wide_tab_words(R);
        const size_t words = (size_t)k * tw;
        std::vector<uint64_t> blob((size_t)2 * k + (words + 1) / 2, 0);
        for (int j = 0; j < k; ++j) {
            blob[j] = reinterpret_cast<uint64_t>(in[j].base);
            blob[(size_t)k + j] = in[j].obj_stride;
        }
        uint32_t* tab = reinterpret_cast<uint32_t*>(blob.data() + 2 * k);
        for (int j = 0; j < k; ++j)
            for (int r = 0; r < R; ++r) perm_table(coeffs[(size_t)(r0 + r) * k + j], tab + (size_t)j * tw + 5 * r);
        void* d = nullptr;
        int rc = scratch_alloc(blob.size() * 8, stream, &d);
        if (rc) return rc;
        hipError_t e = launch_put_words(d, blob.data(), blob.size() * 8, stream);
        WideArgs a;
        std::memset(&a, 0, sizeof(a));
        a.in_base = static_cast<const uint64_t*>(d);
        a.in_stride = static_cast<const uint64_t*>(d) + k;
        a.tab = reinterpret_cast<const uint32_t*>(static_cast<const uint64_t*>(d) + 2 * k);
        a.K = (uint32_t)k;
        a.shard_len = shard_len;
        a.tiles_per_obj = (uint32_t)tpo;
        const uint64_t max_obj = tpo ? std::max<uint64_t>(1, std::min<uint64_t>((1ull << 31), g_chunk_tiles) / tpo) : n_obj;
        for (uint64_t o0 = 0; o0 < n_obj && e == hipSuccess; o0 += max_obj) {
            const uint64_t no = std::min(max_obj, n_obj - o0);
            WideArgs b = a;
            for (int r = 0; r < R; ++r) {
                b.out[r] = reinterpret_cast<uint64_t>(out[r0 + r].base) + o0 * out[r0 + r].obj_stride;
                b.out_stride[r] = out[r0 + r].obj_stride;
            }
            b.n_obj = no;
            b.n_tiles = (uint32_t)(no * tpo);
            if (o0 > 0) {
                std::vector<uint64_t> base(k);
                for (int j = 0; j < k; ++j) base[j] = blob[j] + o0 * blob[(size_t)k + j];
                e = launch_put_words(d, base.data(), (size_t)k * 8, stream);
                if (e != hipSuccess) break;
            }
            e = launch(b, R, o0);
        }
        scratch_free(d, stream);
        if (e != hipSuccess) return hip_fail(e, "launch gf_wide");
    }
    return HBEC_OK;
}

// 4-wave blocks per CU of the gf_wide grids (HBEC_WIDE_BPC overrides): the
// kernel keeps HBEC_WIDE_D loads in flight per lane, so it needs several waves
// per SIMD; verify 8 (10+4 46 -> 49 %, r3b5), apply 4 (r3b6)
static int wide_grid(uint64_t n_tiles, int dflt) {
    static const int env = (int)tune_knob("HBEC_WIDE_BPC", 0);
    const int bpc = env > 0 ? env : dflt;
    int dev = 0, cus = 256;
    if (current_device(&dev) == HBEC_OK) (void)cu_count(dev, &cus);
    return (int)std::max<uint64_t>(1, std::min<uint64_t>((n_tiles + 3) / 4, (uint64_t)cus * bpc));
}

static int verify_wide(const hbec_view* views, int k, int m, const uint8_t* prow, uint64_t n_obj,
                       uint64_t shard_len, uint32_t* flags, hipStream_t stream) {
    const uint64_t tpo = (wide_main_len(shard_len) + wide_tile_bytes() - 1) / wide_tile_bytes();
    return wide_launches(views, k, prow, m, views + k, n_obj, shard_len, tpo, stream,
                         [&](const WideArgs& b, int R, uint64_t o0) {
                             return launch_verify_wide(R, b, flags + o0, wide_grid(b.n_tiles, 8), stream);
                         });
}

// Apply of k > 16 inputs at any alignment in one pass (gf_wide apply).

static int apply_wide(int rows, int cols, const uint8_t* coeffs, const hbec_view* in, const hbec_view* out,
                      uint64_t n_obj, uint64_t shard_len, hipStream_t stream) {
    const uint64_t tpo = wide_apply_tiles_per_obj(shard_len);
    return wide_launches(in, cols, coeffs, rows, out, n_obj, shard_len, tpo, stream,
                         [&](const WideArgs& b, int R, uint64_t) {
                             return launch_apply_wide(R, b, wide_grid(b.n_tiles, 4), stream);
                         });
}

}  // namespace hbec

extern "C" {

static int verify_views(hbec_codec* c, const hbec_view* views, uint64_t n_obj, uint64_t shard_len, uint32_t* flags,
                        hipStream_t stream) {
    const int k = c->k, m = c->m;
    if (m == 0 || n_obj == 0 || shard_len == 0) return HBEC_OK;
    bool vec = vec_len(shard_len);
    for (int i = 0; i < k + m && vec; ++i) vec = aligned16(views[i].base) && vec_len(views[i].obj_stride);
    const uint8_t* prow = c->matrix.data() + (size_t)k * k;
    if (vec && is_verify_packed_shape(k, m, shard_len)) {
        // short shards: wave tiles across objects (gf_verify_packed)
        PassArgs a;
        std::memset(&a, 0, sizeof(a));
        for (int j = 0; j < k; ++j) {
            a.in[j] = static_cast<const uint8_t*>(views[j].base);
            a.in_stride[j] = views[j].obj_stride;
        }
        for (int r = 0; r < m; ++r) {
            a.out[r] = static_cast<uint8_t*>(views[k + r].base);
            a.out_stride[r] = views[k + r].obj_stride;
            for (int j = 0; j < k; ++j) perm_table(prow[(size_t)r * k + j], a.tab[r][j]);
        }
        a.shard_len = shard_len;
        int dev = 0, cus = 0, bpc = 1;
        int rc = current_device(&dev);
        if (rc) return rc;
        hipDeviceProp_t p;
        hipError_t e = hipGetDeviceProperties(&p, dev);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
        cus = p.multiProcessorCount;
        e = verify_packed_occupancy(k, m, &bpc);
        if (e != hipSuccess) return hip_fail(e, "verify occupancy");
        bpc = std::max(1, bpc);
        if (g_blocks_per_cu_override > 0) bpc = g_blocks_per_cu_override;
        const uint64_t spo = shard_len / 16;
        const uint64_t te = (uint64_t)verify_packed_tile_elems(k);
        uint64_t max_obj = std::max<uint64_t>(1, ((1ull << 31) - te) / spo);  // n_elems < 2^31
        max_obj = std::min(max_obj, std::max<uint64_t>(1, g_chunk_tiles * te / spo));
        for (uint64_t o0 = 0; o0 < n_obj; o0 += max_obj) {
            const uint64_t no = std::min(max_obj, n_obj - o0);
            PassArgs b = a;
            for (int j = 0; j < k; ++j) b.in[j] = a.in[j] + o0 * a.in_stride[j];
            for (int r = 0; r < m; ++r) b.out[r] = a.out[r] + o0 * a.out_stride[r];
            b.n_obj = no;
            b.elems_per_obj = (uint32_t)spo;
            b.n_elems = (uint32_t)(no * spo);
            b.n_tiles = (uint32_t)((no * spo + te - 1) / te);
            const uint64_t wpb = (uint64_t)kPipeBlockThreads / 64;
            const uint64_t want = (b.n_tiles + wpb - 1) / wpb;
            const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cus * bpc));
            e = launch_verify_packed(k, m, b, flags + o0, grid, stream);
            if (e != hipSuccess) return hip_fail(e, "launch gf_verify_packed");
        }
        return HBEC_OK;
    }
    // 16-B-aligned Verify stays on gf_verify_pipe (2-4 points ahead of the
    // record kernels from 5+3 to 8+3 at any pitch) except where its tables
    // run out of issue slots: K R > 24 with a compiled bit-plane Verify
    // (8+4: 59.8-62.1 -> 74.3-75.5 %, profiles/r05_ab_route.jsonl r5_vroute).
    // Tuning builds: HBEC_VERIFY_ROUTE=0 keeps them all there.
    static const bool verify_route = tune_knob("HBEC_VERIFY_ROUTE", 1) != 0;
    bool v_to_rec = vec && verify_route && odd_enabled() && k >= 5 && k <= 8 && m <= kMaxR && k * m > 24 &&
                    shard_len >= HBEC_REC_ROUTE_MIN_S && pos32_shard(shard_len);
    if (v_to_rec) {
        uint32_t tab[kMaxR][kMaxK][5] = {};
        for (int r = 0; r < m; ++r)
            for (int j = 0; j < k; ++j) tab[r][j][0] = (uint32_t)prow[(size_t)r * k + j] << 8;  // byte 1 = c * 1
        v_to_rec = odd_bp_schedule(k, m, 2, tab, false) >= 0;
    }
    if (vec && verify_supported(k, m) && !v_to_rec) {
        PassArgs a;
        std::memset(&a, 0, sizeof(a));
        for (int j = 0; j < k; ++j) {
            a.in[j] = static_cast<const uint8_t*>(views[j].base);
            a.in_stride[j] = views[j].obj_stride;
        }
        for (int r = 0; r < m; ++r) {
            a.out[r] = static_cast<uint8_t*>(views[k + r].base);
            a.out_stride[r] = views[k + r].obj_stride;
            for (int j = 0; j < k; ++j) perm_table(prow[(size_t)r * k + j], a.tab[r][j]);
        }
        a.shard_len = shard_len;
        const uint64_t tile = (uint64_t)verify_tile_bytes(k);
        const uint64_t tpo = (shard_len + tile - 1) / tile;
        int dev = 0, cus = 0, bpc = 1;
        int rc = current_device(&dev);
        if (rc) return rc;
        {
            hipDeviceProp_t p;
            hipError_t e = hipGetDeviceProperties(&p, dev);
            if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
            cus = p.multiProcessorCount;
            e = verify_occupancy(k, m, &bpc);
            if (e != hipSuccess) return hip_fail(e, "verify occupancy");
            bpc = std::max(1, kPipeBlocksPerCu > 0 ? std::min(bpc, kPipeBlocksPerCu) : bpc);
            if (g_blocks_per_cu_override > 0) bpc = std::min(std::max(1, bpc_occ_cap(k, m)), g_blocks_per_cu_override);
        }
        const uint64_t max_obj = std::max<uint64_t>(1, (1ull << 31) / tpo);
        for (uint64_t o0 = 0; o0 < n_obj; o0 += max_obj) {
            const uint64_t no = std::min(max_obj, n_obj - o0);
            PassArgs b = a;
            for (int j = 0; j < k; ++j) b.in[j] = a.in[j] + o0 * a.in_stride[j];
            for (int r = 0; r < m; ++r) b.out[r] = a.out[r] + o0 * a.out_stride[r];
            b.n_obj = no;
            b.tiles_per_obj = (uint32_t)tpo;
            b.n_tiles = (uint32_t)(no * tpo);
            const uint64_t want = (b.n_tiles + 3) / 4;
            const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cus * bpc));
            hipError_t e = launch_verify(k, m, b, flags + o0, grid, stream);
            if (e != hipSuccess) return hip_fail(e, "launch gf_verify_pipe");
        }
        return HBEC_OK;
    }
    // k <= 8: gf_odd verify; 9 <= k <= 12 with 3 or 4 parity rows: the record
    // kernel with LDS tables in one pass (10+4 54.1 -> 64.5 %, 12+4 45.7 ->
    // 53.6 % over gf_verify_wide, profiles/r04_ab_odd.jsonl batch N).  Other
    // 9 <= k <= 12 shapes (1-2 rows: the register-table gf_odd, m > 4: the
    // data read once per 4 rows) and k > 12 take gf_verify_wide, one
    // read-only pass per <= 8 rows.
    bool odd_verify = k <= 8 || (k <= kOddMaxK && m >= 3 && m <= kMaxR);
    if (!odd_verify && k <= kOddMaxK && m <= kMaxR) {
        // 9 <= k <= 12 with 1-2 rows: the one-pass bit-plane Verify when the
        // rows have a compiled schedule (10+2, 12+2)
        uint32_t tab[kMaxR][kMaxK][5];
        for (int r = 0; r < m; ++r)
            for (int j = 0; j < k; ++j) perm_table(prow[(size_t)r * k + j], tab[r][j]);
        odd_verify = odd_bp_schedule(k, m, 2, tab, false) >= 0;
    }
    if (odd_enabled() && odd_verify && pos32_shard(shard_len)) {
        // any alignment: recompute and compare in one pass (gf_odd verify), <= 4 rows per launch
        int dev = 0;
        int rc = current_device(&dev);
        if (rc) return rc;
        for (int r0 = 0; r0 < m; r0 += kMaxR) {
            const int R = std::min(kMaxR, m - r0);
            PassArgs a;
            std::memset(&a, 0, sizeof(a));
            for (int j = 0; j < k; ++j) {
                a.in[j] = static_cast<const uint8_t*>(views[j].base);
                a.in_stride[j] = views[j].obj_stride;
            }
            for (int r = 0; r < R; ++r) {
                a.out[r] = static_cast<uint8_t*>(views[k + r0 + r].base);
                a.out_stride[r] = views[k + r0 + r].obj_stride;
                for (int j = 0; j < k; ++j) perm_table(prow[(size_t)(r0 + r) * k + j], a.tab[r][j]);
            }
            rc = odd_launches(a, k, R, 2, false, n_obj, shard_len, flags, dev, stream);
            if (rc) return rc;
        }
        return HBEC_OK;
    }
    if (k > 8 && k <= 256 && pos32_shard(shard_len)) {
        // k > 8 at any alignment (k > 16 included): one read-only pass per <= 8
        // rows (gf_verify_wide, wide.hip), coefficient tables in LDS
        return verify_wide(views, k, m, prow, n_obj, shard_len, flags, stream);
    }
    if (k <= kMaxK) {
        // any alignment: recompute and compare in one pass (gf_verify_unaligned), <= 4 rows per launch
        int dev = 0, cus = 0;
        int rc = current_device(&dev);
        if (rc) return rc;
        const uint64_t tpo = unaligned_tiles_per_obj(shard_len);
        const uint64_t max_obj = std::max<uint64_t>(1, std::min<uint64_t>((1ull << 31), g_chunk_tiles) / tpo);
        for (int r0 = 0; r0 < m; r0 += kMaxR) {
            const int R = std::min(kMaxR, m - r0);
            int per_cu = 0;
            rc = device_blocks(dev, k, R, 3, 0, &cus, &per_cu);
            if (rc) return rc;
            if (g_unaligned_bpc > 0) per_cu = std::min(per_cu, g_unaligned_bpc);
            PassArgs a;
            std::memset(&a, 0, sizeof(a));
            for (int j = 0; j < k; ++j) {
                a.in[j] = static_cast<const uint8_t*>(views[j].base);
                a.in_stride[j] = views[j].obj_stride;
            }
            for (int r = 0; r < R; ++r) {
                a.out[r] = static_cast<uint8_t*>(views[k + r0 + r].base);
                a.out_stride[r] = views[k + r0 + r].obj_stride;
                for (int j = 0; j < k; ++j) perm_table(prow[(size_t)(r0 + r) * k + j], a.tab[r][j]);
            }
            a.shard_len = shard_len;
            for (uint64_t o0 = 0; o0 < n_obj; o0 += max_obj) {
                const uint64_t no = std::min(max_obj, n_obj - o0);
                PassArgs b = a;
                for (int j = 0; j < k; ++j) b.in[j] = a.in[j] + o0 * a.in_stride[j];
                for (int r = 0; r < R; ++r) b.out[r] = a.out[r] + o0 * a.out_stride[r];
                b.n_obj = no;
                b.tiles_per_obj = (uint32_t)tpo;
                b.n_tiles = (uint32_t)(no * tpo);
                const uint64_t want = (b.n_tiles + kBlockThreads / 64 - 1) / (kBlockThreads / 64);
                const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cus * per_cu));
                hipError_t e = launch_verify_unaligned(k, R, b, flags + o0, grid, stream);
                if (e != hipSuccess) return hip_fail(e, "launch gf_verify_unaligned");
            }
        }
        return HBEC_OK;
    }
    // generic: recompute parity into scratch, then compare bytewise
    uint8_t* scratch = nullptr;
    const size_t bytes = (size_t)n_obj * m * shard_len;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&scratch), bytes, stream);
    if (e != hipSuccess) return hip_fail(e, "hipMallocAsync verify scratch");
    std::vector<hbec_view> out(m);
    for (int r = 0; r < m; ++r) out[r] = {scratch + (size_t)r * shard_len, (uint64_t)m * shard_len};
    int rc = apply_views(m, k, prow, views, out.data(), n_obj, shard_len, stream);
    for (int r0 = 0; r0 < m && rc == HBEC_OK; r0 += kMaxR) {
        const int R = std::min(kMaxR, m - r0);
        PassArgs a;
        std::memset(&a, 0, sizeof(a));
        for (int r = 0; r < R; ++r) {
            a.in[r] = static_cast<const uint8_t*>(out[r0 + r].base);
            a.in_stride[r] = out[r0 + r].obj_stride;
            a.out[r] = static_cast<uint8_t*>(views[k + r0 + r].base);
            a.out_stride[r] = views[k + r0 + r].obj_stride;
        }
        a.shard_len = shard_len;
        a.n_obj = n_obj;
        const uint64_t want = (shard_len * n_obj + kBlockThreads - 1) / kBlockThreads;
        const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, 16384));
        e = launch_compare(R, a, flags, grid, stream);
        if (e != hipSuccess) rc = hip_fail(e, "launch compare_views");
    }
    hipError_t e2 = hipFreeAsync(scratch, stream);
    if (rc) return rc;
    if (e2 != hipSuccess) return hip_fail(e2, "hipFreeAsync verify scratch");
    return HBEC_OK;
}

int hbec_verify_batch(hbec_codec* c, const hbec_view* views, uint64_t n_objects, uint64_t shard_len,
                      uint32_t* d_flags, void* hip_stream) {
    return hbec::guarded("hbec_verify_batch", [&]() -> int {
        if (!c || !views || (!d_flags && n_objects)) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        return verify_views(c, views, n_objects, shard_len, d_flags, static_cast<hipStream_t>(hip_stream));
    });
}

int hbec_verify(hbec_codec* c, uint8_t* const* shards, const size_t* lens, int n_shards, int* ok) {
    return hbec::guarded("hbec_verify", [&]() -> int {
        if (!c || !shards || !lens || !ok) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        *ok = 0;
        if (n_shards != c->k + c->m) return fail(HBEC_ERR_TOO_FEW_SHARDS, "too few shards given");
        size_t s = 0;
        int rc = check_shards(lens, n_shards, false, &s);
        if (rc) return rc;
        if (c->m == 0) {
            *ok = 1;
            return HBEC_OK;
        }
        const uint64_t pad = round16(s);
        const int n = c->k + c->m;
        Staging* st = nullptr;
        rc = staging_acquire((size_t)pad * n + 16, &st);
        if (rc) return rc;
        std::vector<hbec_view> v(n);
        hipError_t e = hipSuccess;
        for (int i = 0; i < n && e == hipSuccess; ++i) {
            v[i] = {st->dbuf + (size_t)i * pad, 0};
            e = hipMemcpyAsync(v[i].base, shards[i], s, hipMemcpyHostToDevice, st->stream);
            // padding bytes must compare equal: zero both sides' tails
            if (e == hipSuccess && pad > s)
                e = hipMemsetAsync(static_cast<uint8_t*>(v[i].base) + s, 0, pad - s, st->stream);
        }
        uint32_t* d_flag = reinterpret_cast<uint32_t*>(st->dbuf + (size_t)pad * n);
        if (e == hipSuccess) e = hipMemsetAsync(d_flag, 0, sizeof(uint32_t), st->stream);
        if (e != hipSuccess) {
            staging_release(st);
            return hip_fail(e, "verify staging");
        }
        rc = verify_views(c, v.data(), 1, pad, d_flag, st->stream);
        uint32_t h_flag = 1;
        if (rc == HBEC_OK) e = hipMemcpyAsync(&h_flag, d_flag, sizeof(h_flag), hipMemcpyDeviceToHost, st->stream);
        hipError_t e2 = hipStreamSynchronize(st->stream);
        staging_release(st);
        if (rc) return rc;
        if (e != hipSuccess) return hip_fail(e, "verify D2H");
        if (e2 != hipSuccess) return hip_fail(e2, "hipStreamSynchronize");
        *ok = h_flag == 0 ? 1 : 0;
        return HBEC_OK;
    });
}

// ---- databuf entry points: ONE base pointer + scalars ----------------------
// Every ecutils.go call site hands klauspost slices of one contiguous databuf:
// shard i at databuf + i*S (ecSplit :31-35,55-58; ecReconstruct :94-101;
// ecGlue :151-159).  Passing that base instead of a [][]byte lets a cgo shim
// call in with no array of Go pointers (so no runtime.Pinner: Go 1.10's cgo
// pointer rules allow a Go pointer to memory that holds no Go pointers).
static void databuf_shards(const hbec_codec* c, uint8_t* databuf, size_t s, std::vector<uint8_t*>& p) {
    p.resize((size_t)(c->k + c->m));
    for (size_t i = 0; i < p.size(); ++i) p[i] = databuf + i * s;
}

int hbec_encode_databuf(hbec_codec* c, uint8_t* databuf, size_t shard_len) {
    return hbec::guarded("hbec_encode_databuf", [&]() -> int {
        if (!c || !databuf) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        if (shard_len == 0) return fail(HBEC_ERR_SHARD_NO_DATA, "no shard data");  // checkShards: all empty
        if (coalesce_enabled()) return coalesced_call(c, 0, databuf, shard_len, nullptr, c->k + c->m, 0, kDirect);
        return direct_encode(c, databuf, shard_len);
    });
}

int hbec_reconstruct_databuf(hbec_codec* c, uint8_t* databuf, size_t shard_len, const uint8_t* present,
                             int data_only) {
    return hbec::guarded("hbec_reconstruct_databuf", [&]() -> int {
        if (!c || !databuf || !present) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        std::vector<uint8_t*> p;
        databuf_shards(c, databuf, shard_len, p);
        // a missing shard is a zero-length slice whose capacity is its slot
        // (ecutils.go:98-100): klauspost fills it in place
        std::vector<size_t> lens(p.size());
        for (size_t i = 0; i < p.size(); ++i) lens[i] = present[i] ? shard_len : 0;
        return hbec_reconstruct(c, p.data(), lens.data(), (int)p.size(), data_only);
    });
}

int hbec_verify_databuf(hbec_codec* c, const uint8_t* databuf, size_t shard_len, int* ok) {
    return hbec::guarded("hbec_verify_databuf", [&]() -> int {
        if (!c || !databuf || !ok) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        *ok = 0;
        if (shard_len == 0) return fail(HBEC_ERR_SHARD_NO_DATA, "no shard data");
        std::vector<uint8_t*> p;
        databuf_shards(c, const_cast<uint8_t*>(databuf), shard_len, p);
        std::vector<size_t> lens(p.size(), shard_len);
        return hbec_verify(c, p.data(), lens.data(), (int)p.size(), ok);
    });
}

int hbec_coalesce_stats(uint64_t* groups, uint64_t* calls) {
    return hbec::guarded("hbec_coalesce_stats", [&]() -> int {
        coalesce_stats(groups, calls);
        return HBEC_OK;
    });
}

int hbec_set_odd_chunk_tiles(uint64_t tiles) {
    g_odd_chunk_override.store(tiles, std::memory_order_relaxed);
    return HBEC_OK;
}

int hbec_set_force_stream(int on) {
    return hbec::guarded("hbec_set_force_stream", [&]() -> int {
        g_force_stream.store(on ? 1 : 0);
        return HBEC_OK;
    });
}

int hbec_kernel_info(int k, int r, uint64_t shard_len, int* tile_bytes, int* kind, int* blocks_per_cu) {
    return hbec::guarded("hbec_kernel_info", [&]() -> int {
        if (k < 1 || k > kMaxK || r < 1 || r > kMaxR) return fail(HBEC_ERR_INVALID_ARG, "shape out of range");
        const int fs = g_force_stream.load();
        const bool packed = r <= 3 && is_packed_shape(k, r, shard_len, 0, fs);
        const bool rec = !packed && shard_len % 16 == 0 && rec_route(k, r, shard_len, shard_len % 128 == 0, false);
        const int pipe = packed ? 2 : is_pipe_shape(k, r, shard_len, fs);
        if (tile_bytes)
            *tile_bytes = packed ? packed_tile_elems(k) * 16
                                 : (rec ? (int)odd_rec_tile_span(k, 0, -1) : vec_tile_bytes(k, r, shard_len, 0, fs));
        if (kind) *kind = packed ? 3 : (rec ? 4 : (is_streaming_shape(k, r, fs) ? 2 : (pipe ? 1 : 0)));
        if (blocks_per_cu) {
            int dev = 0, cus = 0;
            int rc = current_device(&dev);
            if (rc) return rc;
            rc = device_blocks(dev, k, r, pipe, packed ? 0 : fs, &cus, blocks_per_cu);
            if (rc) return rc;
            if (rec) *blocks_per_cu = odd_blocks_per_cu(0, k, r, false, true);
            if (g_blocks_per_cu_override > 0) *blocks_per_cu = g_blocks_per_cu_override;
        }
        return HBEC_OK;
    });
}

}  // extern "C"

extern "C" int hbec_odd_record_cache(int clear, uint64_t* entries, uint64_t* hits) {
    return hbec::guarded("hbec_odd_record_cache", [&]() -> int {
        ObjRecCache& C = objrec_cache();
        std::lock_guard<std::mutex> lk(C.mu);
        if (clear) {
            hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize (record cache)");
            for (auto& x : C.entries) {
                if (x.ev) (void)hipEventDestroy(x.ev);
                if (x.d) (void)hipFree(x.d);
            }
            C.entries.clear();
            C.seen.clear();
            C.bytes = 0;
            C.hits = 0;
        }
        if (entries) *entries = C.entries.size();
        if (hits) *hits = C.hits;
        return HBEC_OK;
    });
}
