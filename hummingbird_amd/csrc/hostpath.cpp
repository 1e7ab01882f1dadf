// hostpath.cpp — streaming host path: code a batch of
// HOST-resident stripes (ecSplit databuf layout, objectserver/ecutils.go:31-35,
// 55-58) through a pinned staging ring.  Per chunk of stripes:
//
//   CPU gather (thread pool) caller memory -> pinned IN slot
//   H2D IN slot -> device IN region            (copy stream)
//   gf_apply_stripes over the chunk's tiles    (compute stream)
//   D2H device OUT region -> pinned OUT slot   (copy-back stream)
//   CPU scatter pinned OUT slot -> caller memory
//
// with three slots in flight, so the CPU copies of one chunk overlap the DMA
// and kernel work of the others.  Stripes wider than a slot are cut into
// column pieces.  Everything is synchronous for the caller: when the call
// returns, parity (encode) or the rebuilt shards (reconstruct) are in the
// caller's buffers.
//
// Zero-copy: stripes that live in pinned, device-mapped host memory
// (hbec_host_alloc, or any hipHostMalloc / hipHostRegister buffer) skip the
// ring entirely.  The stripe kernel reads their data shards and writes their
// parity in place over PCIe, so there is no CPU copy and no DMA call per
// chunk; only 32-B tile records travel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hbec.h"
#include "gf256.h"
#include "internal.h"
#include "kernels.h"
#include "pool.h"

using hbec::fail;
using hbec::hip_fail;

namespace {

// One column piece of one stripe: columns [col, col+len) of its K inputs / R outputs.
struct Piece {
    uint64_t stripe;
    uint64_t col;
    uint64_t len;   // bytes (<= shard_len - col)
    uint64_t lpad;  // len rounded up to 16
    uint64_t in_off, out_off;  // offsets of this piece in the slot's IN / OUT regions
};

constexpr int kSlots = 3;

struct Ring {
    int dev = -1;
    int cus = 0;  // compute units of dev (grid sizing), read once
    size_t in_cap = 0, out_cap = 0, tile_cap = 0;
    hipStream_t s_h2d = nullptr, s_cmp = nullptr, s_d2h = nullptr;
    uint8_t* pin_in[kSlots] = {};
    uint8_t* pin_out[kSlots] = {};
    uint8_t* dev_in[kSlots] = {};
    uint8_t* dev_out[kSlots] = {};
    hbec::TileRec* pin_tiles[kSlots] = {};
    hbec::TileRec* dev_tiles[kSlots] = {};
    hipEvent_t ev_h2d[kSlots] = {}, ev_cmp[kSlots] = {}, ev_done[kSlots] = {};
    // ShardHash (hbec_encode_host_md5), created on first use: n_arenas device
    // hash arenas (HBEC_HASH_ARENAS, default 2, of HBEC_HASH_ARENA_MB, default
    // 1024; 2 x 3 GiB: pinned 4+2 encode+hash 1.14 x encode alone instead of
    // 1.21 x, profiles/r02_host_md5_arenas.jsonl).  A chunk's shards land in the current arena (copied D2D after the
    // ring's kernel, or written by the mirrored zero-copy kernel); a full
    // arena is hashed by ONE md5_list launch on its own stream while the next
    // arenas fill, so hashing hides behind the PCIe stream, and the hashes of
    // several arenas may run at once.
    static constexpr int kArenas = 8;
    int n_arenas = 0;
    hipStream_t s_md5[kArenas] = {};
    uint8_t* arena[kArenas] = {};
    size_t arena_cap = 0, arena_rec_cap = 0;
    uint64_t* pin_md5rec[kArenas] = {};
    uint64_t* dev_md5rec[kArenas] = {};
    hipEvent_t ev_arena_copied[kArenas] = {}, ev_arena_hashed[kArenas] = {};
    std::unique_ptr<hbec::Pool> pool;

    ~Ring() {
        for (int i = 0; i < kSlots; ++i) {
            if (pin_in[i]) (void)hipHostFree(pin_in[i]);
            if (pin_out[i]) (void)hipHostFree(pin_out[i]);
            if (pin_tiles[i]) (void)hipHostFree(pin_tiles[i]);
            if (dev_in[i]) (void)hipFree(dev_in[i]);
            if (dev_out[i]) (void)hipFree(dev_out[i]);
            if (dev_tiles[i]) (void)hipFree(dev_tiles[i]);
            if (ev_h2d[i]) (void)hipEventDestroy(ev_h2d[i]);
            if (ev_cmp[i]) (void)hipEventDestroy(ev_cmp[i]);
            if (ev_done[i]) (void)hipEventDestroy(ev_done[i]);
        }
        for (int a = 0; a < kArenas; ++a) {
            if (arena[a]) (void)hipFree(arena[a]);
            if (pin_md5rec[a]) (void)hipHostFree(pin_md5rec[a]);
            if (dev_md5rec[a]) (void)hipFree(dev_md5rec[a]);
            if (ev_arena_copied[a]) (void)hipEventDestroy(ev_arena_copied[a]);
            if (ev_arena_hashed[a]) (void)hipEventDestroy(ev_arena_hashed[a]);
        }
        for (int a = 0; a < kArenas; ++a)
            if (s_md5[a]) (void)hipStreamDestroy(s_md5[a]);
        if (s_h2d) (void)hipStreamDestroy(s_h2d);
        if (s_cmp) (void)hipStreamDestroy(s_cmp);
        if (s_d2h) (void)hipStreamDestroy(s_d2h);
    }
};

size_t env_size(const char* name, size_t dflt) {
    const long long v = hbec::env_knob(name, 0);
    return v > 0 ? (size_t)v : dflt;
}
size_t tune_size(const char* name, size_t dflt) {
    const long long v = hbec::tune_knob(name, 0);
    return v > 0 ? (size_t)v : dflt;
}

int ring_init(Ring& r, int dev) {
    r.dev = dev;
    {
        hipDeviceProp_t prop;
        hipError_t pe = hipGetDeviceProperties(&prop, dev);
        if (pe != hipSuccess) return hip_fail(pe, "hipGetDeviceProperties");
        r.cus = prop.multiProcessorCount;
    }
    const size_t slot = env_size("HBEC_HOST_SLOT_MB", 64) << 20;  // IN bytes per slot
    r.in_cap = slot;
    r.out_cap = slot;  // outputs per piece <= inputs (R <= K) except tiny K: sized below per call
    r.tile_cap = slot / 1024 + 1024;
    hipError_t e;
#define HB_CHECK(x, what)                       \
    do {                                        \
        e = (x);                                \
        if (e != hipSuccess) return hip_fail(e, what); \
    } while (0)
    HB_CHECK(hipStreamCreateWithFlags(&r.s_h2d, hipStreamNonBlocking), "stream");
    HB_CHECK(hipStreamCreateWithFlags(&r.s_cmp, hipStreamNonBlocking), "stream");
    HB_CHECK(hipStreamCreateWithFlags(&r.s_d2h, hipStreamNonBlocking), "stream");
    for (int i = 0; i < kSlots; ++i) {
        HB_CHECK(hipHostMalloc(reinterpret_cast<void**>(&r.pin_tiles[i]), r.tile_cap * sizeof(hbec::TileRec),
                               hipHostMallocDefault),
                 "pinned tiles");
        HB_CHECK(hipMalloc(&r.dev_tiles[i], r.tile_cap * sizeof(hbec::TileRec)), "device tiles");
        HB_CHECK(hipEventCreateWithFlags(&r.ev_h2d[i], hipEventDisableTiming), "event");
        HB_CHECK(hipEventCreateWithFlags(&r.ev_cmp[i], hipEventDisableTiming), "event");
        HB_CHECK(hipEventCreateWithFlags(&r.ev_done[i], hipEventDisableTiming), "event");
    }
#undef HB_CHECK
    return HBEC_OK;
}

// The staging slots and copy threads, made on the first call that stages
// (zero-copy calls only need the tile records).
int ring_staging_init(Ring& r) {
    if (r.pool) return HBEC_OK;  // set last: everything below exists
    hipError_t e = hipSuccess;
    for (int i = 0; i < kSlots && e == hipSuccess; ++i) {  // a failed earlier attempt keeps what it got
        if (!r.pin_in[i]) e = hipHostMalloc(reinterpret_cast<void**>(&r.pin_in[i]), r.in_cap, hipHostMallocDefault);
        if (e == hipSuccess && !r.pin_out[i])
            e = hipHostMalloc(reinterpret_cast<void**>(&r.pin_out[i]), r.out_cap, hipHostMallocDefault);
        if (e == hipSuccess && !r.dev_in[i]) e = hipMalloc(&r.dev_in[i], r.in_cap);
        if (e == hipSuccess && !r.dev_out[i]) e = hipMalloc(&r.dev_out[i], r.out_cap);
    }
    if (e != hipSuccess) return hip_fail(e, "staging slots");
    r.pool.reset(new hbec::Pool(hbec::host_threads() - 1));  // + the calling thread
    return HBEC_OK;
}

int ring_md5_init(Ring& r) {
    if (r.n_arenas > 0) return HBEC_OK;  // set last: everything below exists
    const size_t cap = env_size("HBEC_HASH_ARENA_MB", 1024) << 20;
    const int n_arenas = (int)std::min<size_t>(Ring::kArenas, std::max<size_t>(2, tune_size("HBEC_HASH_ARENAS", 2)));
    r.arena_cap = std::max(cap, r.in_cap + r.out_cap);
    // MD5 records per arena (32 B pinned each; HBEC_HASH_ARENA_RECS, default
    // 256 K = 8 MiB): an arena is hashed early when its records run out, so
    // this bounds pinned memory, not batch size (one record per 16-B shard
    // would pin 2 GiB per arena)
    r.arena_rec_cap = std::min<size_t>(r.arena_cap / 16 + 1024, tune_size("HBEC_HASH_ARENA_RECS", 1u << 18));
    hipError_t e = hipSuccess;
    for (int a = 0; a < n_arenas && e == hipSuccess; ++a) {  // a failed earlier attempt keeps what it got
        if (!r.s_md5[a]) e = hipStreamCreateWithFlags(&r.s_md5[a], hipStreamNonBlocking);
        if (e == hipSuccess && !r.arena[a]) e = hipMalloc(&r.arena[a], r.arena_cap);
        if (e == hipSuccess && !r.pin_md5rec[a])
            e = hipHostMalloc(reinterpret_cast<void**>(&r.pin_md5rec[a]), r.arena_rec_cap * 32, hipHostMallocDefault);
        if (e == hipSuccess && !r.dev_md5rec[a])
            e = hipMalloc(reinterpret_cast<void**>(&r.dev_md5rec[a]), r.arena_rec_cap * 32);
        if (e == hipSuccess && !r.ev_arena_copied[a])
            e = hipEventCreateWithFlags(&r.ev_arena_copied[a], hipEventDisableTiming);
        if (e == hipSuccess && !r.ev_arena_hashed[a])
            e = hipEventCreateWithFlags(&r.ev_arena_hashed[a], hipEventDisableTiming);
    }
    if (e != hipSuccess) return hip_fail(e, "hash arena");
    r.n_arenas = n_arenas;
    return HBEC_OK;
}

// The hash arenas of one hbec_encode_host_md5 call.  Shards are appended to
// the current arena and a record per shard to its pinned record list; a full
// arena is hashed by one md5_list launch on the arena's stream, ordered after
// the work `producer` queued to fill it, and the call moves on to the next
// arena once that arena's previous hash has finished (its memory and pinned
// records are then free).
struct ArenaCursor {
    Ring* ring;
    hipStream_t producer;
    uint8_t* d_digest;
    int cur = 0;
    uint64_t used = 0, recs = 0;

    uint64_t base() const { return reinterpret_cast<uint64_t>(ring->arena[cur]) + used; }
    bool fits(uint64_t bytes, uint64_t n_recs) const {
        return used + bytes <= ring->arena_cap && recs + n_recs <= ring->arena_rec_cap;
    }
    void add(uint64_t addr, uint64_t len, uint64_t slot) {
        uint64_t* r = ring->pin_md5rec[cur] + 4 * recs++;
        r[0] = addr;
        r[1] = len;
        r[2] = slot;
        r[3] = 0;
    }
    int flush() {  // hash the current arena, move to the next free one
        if (recs == 0) return HBEC_OK;
        const int a = cur;
        hipStream_t hs = ring->s_md5[a];
        hipError_t e = hipEventRecord(ring->ev_arena_copied[a], producer);
        if (e == hipSuccess) e = hipStreamWaitEvent(hs, ring->ev_arena_copied[a], 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ring->dev_md5rec[a], ring->pin_md5rec[a], recs * 32, hipMemcpyHostToDevice, hs);
        if (e == hipSuccess) e = hbec::launch_md5_list(ring->dev_md5rec[a], recs, d_digest, true, hs);
        if (e == hipSuccess) e = hipEventRecord(ring->ev_arena_hashed[a], hs);
        if (e != hipSuccess) return hip_fail(e, "hash arena launch");
        cur = (cur + 1) % ring->n_arenas;
        used = recs = 0;
        e = hipEventSynchronize(ring->ev_arena_hashed[cur]);  // may still hash its last fill
        if (e != hipSuccess) return hip_fail(e, "hash arena wait");
        return HBEC_OK;
    }
    int finish() {  // hash the last partial arena and wait for every hash
        int rc = flush();
        if (rc) return rc;
        for (int a = 0; a < ring->n_arenas; ++a) {
            hipError_t e = hipStreamSynchronize(ring->s_md5[a]);
            if (e != hipSuccess) return hip_fail(e, "hash drain");
        }
        return HBEC_OK;
    }
};

// Rings per device are bounded (HBEC_HOST_RINGS, default 8): each staged
// ring pins 384 MiB of host memory and runs a copy pool of host_threads()
// threads, so one ring per concurrent caller (a busy object server has
// hundreds) would pin tens of GiB and spawn thousands of threads; the first
// 64-thread soak spent minutes creating them.  Callers beyond the bound wait,
// in arrival order, for a ring to come back.  No caller holds a ring while
// waiting for another, so the bound cannot deadlock.
std::mutex g_rings_mu;
std::condition_variable g_rings_cv;
std::vector<Ring*> g_free_rings;
std::map<int, int> g_rings_made;  // per device

int ring_limit() {
    static const int v = (int)env_size("HBEC_HOST_RINGS", 8);
    return v;
}

// Pooled non-blocking streams per device for short per-call work (creating
// and destroying a stream per call costs more than a small batch's copies).
std::mutex g_streams_mu;
std::vector<std::pair<int, hipStream_t>> g_free_streams;

int stream_acquire(hipStream_t* out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    {
        std::lock_guard<std::mutex> g(g_streams_mu);
        for (size_t i = 0; i < g_free_streams.size(); ++i)
            if (g_free_streams[i].first == dev) {
                *out = g_free_streams[i].second;
                g_free_streams.erase(g_free_streams.begin() + (long)i);
                return HBEC_OK;
            }
    }
    e = hipStreamCreateWithFlags(out, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
    return HBEC_OK;
}

void stream_release(hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> g(g_streams_mu);
    g_free_streams.emplace_back(dev, s);
}

int ring_acquire(Ring** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    {
        std::unique_lock<std::mutex> lk(g_rings_mu);
        for (;;) {
            for (size_t i = 0; i < g_free_rings.size(); ++i)
                if (g_free_rings[i]->dev == dev) {
                    *out = g_free_rings[i];
                    g_free_rings.erase(g_free_rings.begin() + (long)i);
                    return HBEC_OK;
                }
            if (g_rings_made[dev] < ring_limit()) break;
            g_rings_cv.wait(lk);
        }
        ++g_rings_made[dev];  // reserved: made below, outside the lock
    }
    std::unique_ptr<Ring> r(new (std::nothrow) Ring());
    int rc = r ? ring_init(*r, dev) : fail(HBEC_ERR_NOMEM, "ring allocation");
    if (rc) {
        {
            std::lock_guard<std::mutex> g(g_rings_mu);
            --g_rings_made[dev];
        }
        g_rings_cv.notify_one();
        return rc;
    }
    *out = r.release();
    return HBEC_OK;
}

void ring_release(Ring* r) {
    {
        std::lock_guard<std::mutex> g(g_rings_mu);
        g_free_rings.push_back(r);
    }
    g_rings_cv.notify_all();  // waiters may be on different devices
}

// ---- pinned host memory (zero-copy host path) ----
struct PinnedRange {
    uint64_t len;
    uint64_t dev;  // device address of the range's first byte
};
std::mutex g_pin_mu;
std::map<uint64_t, PinnedRange> g_pinned;  // host base -> range (hbec_host_alloc)

// Blocks per CU of the zero-copy stripes kernel (HBEC_ZC_BLOCKS_PER_CU):
// it streams over PCIe, whose latency wants more requests in flight than
// HBM's sweet spot of one 4-wave block per CU.
int zero_copy_blocks_per_cu() {
    // 1: 45.9, 2: 46.7, 4: 46.6, 8: 46.8 GiB/s (profiles/r02_zc_bpc.jsonl)
    static const int v = (int)tune_size("HBEC_ZC_BLOCKS_PER_CU", 2);
    return v;
}

// Pinned stripes that are not 16-B aligned (or S % 16 != 0): zero-copy through
// the unaligned kernel (a tuning build's HBEC_ZC_UNALIGNED=0: the staged ring).
bool zero_copy_unaligned_enabled() {
    static const bool on = hbec::tune_knob("HBEC_ZC_UNALIGNED", 1) != 0;
    return on;
}

// Grid cap of the zero-copy stripes kernel (HBEC_ZC_GRID blocks, 0 = CUs x
// blocks per CU).  64 blocks of 4 waves keep ~1 MiB of PCIe reads in flight,
// plenty for the link, where the whole chip (512 blocks) kept ~8 MiB queued
// and streamed slower: 4096 x 1 MiB 4+2 pinned stripes 48.4-48.8 -> 52.2-52.5
// GiB/s, 4 KiB stripes 42.2 -> 45.1 GiB/s; 32 and 128 blocks tie with 64
// (profiles/r02_zc_grid.jsonl).
int zero_copy_max_blocks() {
    static const int v = (int)std::max(0LL, hbec::tune_knob("HBEC_ZC_GRID", 64));
    return v;
}

bool zero_copy_enabled() {
    static const bool on = hbec::env_knob("HBEC_ZEROCOPY", 1) != 0;
    return on;
}

}  // namespace

// Device address of host range [p, p + len) when all of it lies in one
// pinned, device-mapped allocation; 0 otherwise.  hbec_host_alloc ranges are
// looked up in the registry; other pinned memory is asked of the runtime at
// both ends of the range.
bool hbec::zero_copy_any_alignment() { return zero_copy_unaligned_enabled(); }

uint64_t hbec::pinned_device_addr(const void* p, uint64_t len) {
    if (!zero_copy_enabled()) return 0;
    const uint64_t h = reinterpret_cast<uint64_t>(p);
    if (!p || len == 0) return 0;
    {
        std::lock_guard<std::mutex> g(g_pin_mu);
        auto it = g_pinned.upper_bound(h);
        if (it != g_pinned.begin()) {
            --it;
            if (h >= it->first && h + len <= it->first + it->second.len) return it->second.dev + (h - it->first);
        }
    }
    hipPointerAttribute_t a0, a1;
    if (hipPointerGetAttributes(&a0, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (a0.type != hipMemoryTypeHost || !a0.devicePointer) return 0;
    // memory pinned elsewhere is only trusted on the device it was pinned for
    // (hbec_host_alloc memory is portable: every device)
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || a0.device != cur) {
        (void)hipGetLastError();
        return 0;
    }
    if (hipPointerGetAttributes(&a1, reinterpret_cast<const uint8_t*>(p) + (len - 1)) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    const uint64_t d0 = reinterpret_cast<uint64_t>(a0.devicePointer);
    const uint64_t d1 = reinterpret_cast<uint64_t>(a1.devicePointer);
    if (a1.type != hipMemoryTypeHost || d1 != d0 + (len - 1)) return 0;
    return d0;
}

namespace {
using hbec::pinned_device_addr;

struct ZcStripe {
    uint64_t dev;  // device address of the stripe base
    uint64_t shard_len;
};

// Code pinned stripes in place: tile records (rings of kSlots pinned/device
// buffers) are the only host->device traffic; the kernel streams the shards
// over PCIe.  One stream, so records, kernels and their reuse are ordered.
int zero_copy_run(Ring* ring, const std::vector<ZcStripe>& zs, const std::vector<int>& in_idx,
                  const std::vector<int>& out_idx, const std::vector<uint8_t>& rows) {
    const int K = (int)in_idx.size();
    const uint64_t tile = (uint64_t)hbec::stripes_tile_bytes(std::min(K, hbec::kStripeMaxK));
    size_t si = 0;
    uint64_t off = 0;
    hipError_t e = hipSuccess;
    for (int c = 0; si < zs.size(); ++c) {
        const int slot = c % kSlots;
        e = hipEventSynchronize(ring->ev_cmp[slot]);  // the slot's previous records are consumed
        if (e != hipSuccess) return hip_fail(e, "zero-copy slot wait");
        hbec::TileRec* rec = ring->pin_tiles[slot];
        uint64_t nt = 0;
        while (si < zs.size() && nt < ring->tile_cap) {
            const ZcStripe& z = zs[si];
            hbec::TileRec& t = rec[nt++];
            t.in_addr = t.out_addr = z.dev + off;
            t.in_stride = t.out_stride = (uint32_t)z.shard_len;
            t.valid = (uint32_t)std::min<uint64_t>(tile, z.shard_len - off);
            t.pad_ = 0;
            off += tile;
            if (off >= z.shard_len) {
                off = 0;
                ++si;
            }
        }
        e = hipMemcpyAsync(ring->dev_tiles[slot], rec, nt * sizeof(hbec::TileRec), hipMemcpyHostToDevice,
                           ring->s_cmp);
        if (e != hipSuccess) return hip_fail(e, "zero-copy records H2D");
        int rc = hbec::launch_stripe_passes(ring->dev_tiles[slot], nt, in_idx, out_idx, rows, 0, ring->s_cmp,
                                            zero_copy_blocks_per_cu(), false, zero_copy_max_blocks());
        if (rc) return rc;
        e = hipEventRecord(ring->ev_cmp[slot], ring->s_cmp);
        if (e != hipSuccess) return hip_fail(e, "zero-copy event");
    }
    e = hipStreamSynchronize(ring->s_cmp);
    if (e != hipSuccess) return hip_fail(e, "zero-copy drain");
    return HBEC_OK;
}

// Pinned stripes at any alignment / shard length (S % 16 != 0 for most object
// sizes): the same in-place PCIe coding through gf_apply_unaligned_plan
// records (URec and TileRec are both 32 B, so the slot buffers are shared).
int zero_copy_unaligned_run(Ring* ring, const std::vector<ZcStripe>& zs, const std::vector<int>& in_idx,
                            const std::vector<int>& out_idx, const std::vector<uint8_t>& rows) {
    static_assert(sizeof(hbec::URec) == sizeof(hbec::TileRec), "record slots are shared");
    const uint64_t tile = hbec::urec_tile_for(std::min((int)in_idx.size(), hbec::kOddMaxK), false);
    size_t si = 0;
    uint64_t off = 0;
    hipError_t e = hipSuccess;
    for (int c = 0; si < zs.size(); ++c) {
        const int slot = c % kSlots;
        e = hipEventSynchronize(ring->ev_cmp[slot]);  // the slot's previous records are consumed
        if (e != hipSuccess) return hip_fail(e, "zero-copy slot wait");
        hbec::URec* rec = reinterpret_cast<hbec::URec*>(ring->pin_tiles[slot]);
        uint64_t nt = 0;
        std::vector<hbec::URec> edges;  // gf_odd: one per stripe started in this slot, after the main records
        while (si < zs.size() && nt + edges.size() + 1 < ring->tile_cap) {
            const ZcStripe& z = zs[si];
            const uint64_t span = hbec::urec_span(z.shard_len);
            if (off == 0 && hbec::odd_enabled()) edges.push_back({z.dev, 0, z.shard_len, 0});
            if (off < span) rec[nt++] = {z.dev, 0, z.shard_len, off};
            off += tile;
            if (off >= span) {
                off = 0;
                ++si;
            }
        }
        std::copy(edges.begin(), edges.end(), rec + nt);
        e = hipMemcpyAsync(ring->dev_tiles[slot], rec, (nt + edges.size()) * sizeof(hbec::URec), hipMemcpyHostToDevice,
                           ring->s_cmp);
        if (e != hipSuccess) return hip_fail(e, "zero-copy records H2D");
        const hbec::URec* d_rec = reinterpret_cast<const hbec::URec*>(ring->dev_tiles[slot]);
        int rc = hbec::launch_unaligned_passes(d_rec, nt, in_idx, out_idx, rows, 0, ring->s_cmp, zero_copy_max_blocks(),
                                               d_rec + nt, edges.size());
        if (rc) return rc;
        e = hipEventRecord(ring->ev_cmp[slot], ring->s_cmp);
        if (e != hipSuccess) return hip_fail(e, "zero-copy event");
    }
    e = hipStreamSynchronize(ring->s_cmp);
    if (e != hipSuccess) return hip_fail(e, "zero-copy drain");
    return HBEC_OK;
}

// Zero-copy with ShardHash (hbec_encode_host_md5 when every stripe is pinned):
// the stripes kernel codes each stripe in place over PCIe, exactly as
// zero_copy_run, and also writes every shard column it holds (inputs and
// outputs) to a device hash arena (StripeArgs::mirror), so nothing crosses
// PCIe twice and no CPU copy runs.  A full arena is hashed by one md5_list
// launch on its own stream while the stripes kernel fills the next ones.
// Stripe s's shard i lands at arena + its offset + i*S; its digest at
// (s * n_shards + i) * 16 of d_digest.
int zero_copy_md5_run(Ring* ring, const std::vector<ZcStripe>& zs, const std::vector<int>& in_idx,
                      const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, uint8_t* d_digest,
                      int n_shards) {
    const int K = (int)in_idx.size(), R = (int)out_idx.size();
    int rc = ring_md5_init(*ring);
    if (rc) return rc;
    const uint64_t tile = (uint64_t)hbec::stripes_tile_bytes(std::min(K, hbec::kStripeMaxK));
    ArenaCursor ac{ring, ring->s_cmp, d_digest};
    hipError_t e = hipSuccess;
    size_t si = 0;
    for (int c = 0; si < zs.size(); ++c) {
        const int slot = c % kSlots;
        e = hipEventSynchronize(ring->ev_cmp[slot]);  // the slot's previous records are consumed
        if (e != hipSuccess) return hip_fail(e, "zero-copy slot wait");
        hbec::TileRec* rec = ring->pin_tiles[slot];
        uint64_t nt = 0;
        while (si < zs.size()) {
            const ZcStripe& z = zs[si];
            const uint64_t S = z.shard_len;
            const uint64_t tiles = (S + tile - 1) / tile;
            const uint64_t bytes = ((uint64_t)n_shards * S + 255) & ~uint64_t(255);
            if (tiles > ring->tile_cap || bytes > ring->arena_cap)
                return fail(HBEC_ERR_INVALID_ARG, "stripe too large for a hash arena");
            if (nt > 0 && nt + tiles > ring->tile_cap) break;
            if (!ac.fits(bytes, (uint64_t)(K + R))) {
                if (nt > 0) break;  // launch this chunk first: the arena is hashed after its kernels
                rc = ac.flush();
                if (rc) return rc;
            }
            const uint64_t mbase = ac.base();
            for (uint64_t off = 0; off < S; off += tile) {
                hbec::TileRec& t = rec[nt++];
                t.in_addr = z.dev + off;
                t.out_addr = mbase + off;
                t.in_stride = t.out_stride = (uint32_t)S;
                t.valid = (uint32_t)std::min<uint64_t>(tile, S - off);
                t.pad_ = 0;
            }
            for (int i : in_idx) ac.add(mbase + (uint64_t)i * S, S, (uint64_t)si * (uint64_t)n_shards + (uint64_t)i);
            for (int i : out_idx) ac.add(mbase + (uint64_t)i * S, S, (uint64_t)si * (uint64_t)n_shards + (uint64_t)i);
            ac.used += bytes;
            ++si;
        }
        e = hipMemcpyAsync(ring->dev_tiles[slot], rec, nt * sizeof(hbec::TileRec), hipMemcpyHostToDevice,
                           ring->s_cmp);
        if (e != hipSuccess) return hip_fail(e, "zero-copy records H2D");
        rc = hbec::launch_stripe_passes(ring->dev_tiles[slot], nt, in_idx, out_idx, rows, 0, ring->s_cmp,
                                        zero_copy_blocks_per_cu(), true, zero_copy_max_blocks());
        if (rc) return rc;
        e = hipEventRecord(ring->ev_cmp[slot], ring->s_cmp);
        if (e != hipSuccess) return hip_fail(e, "zero-copy event");
    }
    rc = ac.finish();
    if (rc) return rc;
    e = hipStreamSynchronize(ring->s_cmp);
    if (e != hipSuccess) return hip_fail(e, "zero-copy drain");
    return HBEC_OK;
}

// Zero-copy with ShardHash for pinned stripes at any alignment / shard length
// (15 object sizes in 16: ecSplit's S = ceil(len / k)): the mirrored gf_odd
// plan kernel codes each stripe in place over PCIe, as
// zero_copy_unaligned_run, and stores every shard column it holds to the
// stripe's hash arena, where shard i sits 16-B aligned at arena + i * P
// (P = odd_mirror_pitch_host(S)); gf_odd_mirror_copy adds the guard-band
// bytes (<= 160 per shard) afterwards.  The arena is then hashed by md5_list
// exactly as in zero_copy_md5_run.
int zero_copy_unaligned_md5_run(Ring* ring, const std::vector<ZcStripe>& zs, const std::vector<int>& in_idx,
                                const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, uint8_t* d_digest,
                                int n_shards) {
    static_assert(sizeof(hbec::URec) == sizeof(hbec::TileRec), "record slots are shared");
    const int K = (int)in_idx.size(), R = (int)out_idx.size();
    int rc = ring_md5_init(*ring);
    if (rc) return rc;
    const uint64_t tile = hbec::urec_tile_for(std::min(K, hbec::kOddMaxK), true);
    ArenaCursor ac{ring, ring->s_cmp, d_digest};
    hipError_t e = hipSuccess;
    size_t si = 0;
    for (int c = 0; si < zs.size(); ++c) {
        const int slot = c % kSlots;
        e = hipEventSynchronize(ring->ev_cmp[slot]);  // the slot's previous records are consumed
        if (e != hipSuccess) return hip_fail(e, "zero-copy slot wait");
        hbec::URec* rec = reinterpret_cast<hbec::URec*>(ring->pin_tiles[slot]);
        uint64_t nt = 0;
        std::vector<hbec::URec> edges;  // one per stripe of this slot, after the main records
        while (si < zs.size()) {
            const ZcStripe& z = zs[si];
            const uint64_t S = z.shard_len;
            const uint64_t span = hbec::urec_span(S);
            const uint64_t tiles = (span + tile - 1) / tile;
            const uint64_t bytes = ((uint64_t)n_shards * hbec::odd_mirror_pitch_host(S) + 255) & ~uint64_t(255);
            if (tiles + 2 > ring->tile_cap || bytes > ring->arena_cap)
                return fail(HBEC_ERR_INVALID_ARG, "stripe too large for a hash arena");
            // a stripe of S <= 160 adds an edge record and no main record, so
            // the slot is full when main + edge records would pass tile_cap,
            // whether or not a main record exists yet
            const bool any = nt > 0 || !edges.empty();
            if (any && nt + edges.size() + tiles + 1 > ring->tile_cap) break;
            if (!ac.fits(bytes, (uint64_t)(K + R))) {
                if (any) break;  // launch this chunk first: the arena is hashed after its kernels
                rc = ac.flush();
                if (rc) return rc;
            }
            const uint64_t mbase = ac.base();  // 256-B aligned
            for (uint64_t off = 0; off < span; off += tile) rec[nt++] = {z.dev, mbase, S, off};
            edges.push_back({z.dev, mbase, S, 0});
            const uint64_t P = hbec::odd_mirror_pitch_host(S);
            for (int i : in_idx) ac.add(mbase + (uint64_t)i * P, S, (uint64_t)si * (uint64_t)n_shards + (uint64_t)i);
            for (int i : out_idx) ac.add(mbase + (uint64_t)i * P, S, (uint64_t)si * (uint64_t)n_shards + (uint64_t)i);
            ac.used += bytes;
            ++si;
        }
        std::copy(edges.begin(), edges.end(), rec + nt);
        e = hipMemcpyAsync(ring->dev_tiles[slot], rec, (nt + edges.size()) * sizeof(hbec::URec), hipMemcpyHostToDevice,
                           ring->s_cmp);
        if (e != hipSuccess) return hip_fail(e, "zero-copy records H2D");
        const hbec::URec* d_rec = reinterpret_cast<const hbec::URec*>(ring->dev_tiles[slot]);
        rc = hbec::launch_unaligned_passes(d_rec, nt, in_idx, out_idx, rows, 0, ring->s_cmp, zero_copy_max_blocks(),
                                           d_rec + nt, edges.size(), true);
        if (rc) return rc;
        e = hipEventRecord(ring->ev_cmp[slot], ring->s_cmp);
        if (e != hipSuccess) return hip_fail(e, "zero-copy event");
    }
    rc = ac.finish();
    if (rc) return rc;
    e = hipStreamSynchronize(ring->s_cmp);
    if (e != hipSuccess) return hip_fail(e, "zero-copy drain");
    return HBEC_OK;
}

std::atomic<uint64_t> g_md5_zc_calls{0}, g_md5_ring_calls{0};

bool zero_copy_md5_enabled() {
    static const bool on = hbec::tune_knob("HBEC_MD5_ZEROCOPY", 1) != 0;
    return on;
}

// Code every stripe: inputs = shards in_idx, outputs = shards out_idx with `rows`.
// With d_digest (device, n * n_shards * 16 B), also hash every input and
// output shard of every stripe while it is in the device slot: digest of
// shard i of stripe s at (s * n_shards + i) * 16.
int host_run_on(Ring* ring, const hbec_stripe* stripes, uint64_t n, const std::vector<int>& in_idx,
                const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, uint8_t* d_digest,
                int n_shards);

// A call that fails part-way may leave work queued on the ring's streams
// (slot copies, kernels writing a hash arena, hashes); the next caller of
// the ring reuses slots only after their events, but starts over at hash
// arena 0, so a failed call drains every stream before the ring goes back.
void ring_drain(Ring* r) {
    hipStream_t all[4 + Ring::kArenas] = {r->s_h2d, r->s_cmp, r->s_d2h};
    int n = 3;
    for (int a = 0; a < Ring::kArenas; ++a) all[n++] = r->s_md5[a];
    for (int i = 0; i < n; ++i)
        if (all[i]) (void)hipStreamSynchronize(all[i]);
    (void)hipGetLastError();
}

int host_run(const hbec_stripe* stripes, uint64_t n, const std::vector<int>& in_idx,
             const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, uint8_t* d_digest = nullptr,
             int n_shards = 0) {
    if (out_idx.empty() || n == 0) return HBEC_OK;
    Ring* ring = nullptr;
    int rc = ring_acquire(&ring);
    if (rc) return rc;
    struct Releaser {
        Ring* r;
        bool ok = false;
        ~Releaser() {
            if (!ok) ring_drain(r);
            ring_release(r);
        }
    } rel{ring};
    rc = host_run_on(ring, stripes, n, in_idx, out_idx, rows, d_digest, n_shards);
    rel.ok = rc == HBEC_OK;
    return rc;
}

int host_run_on(Ring* ring, const hbec_stripe* stripes, uint64_t n, const std::vector<int>& in_idx,
                const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, uint8_t* d_digest,
                int n_shards) {
    const int K = (int)in_idx.size(), R = (int)out_idx.size();
    int rc = HBEC_OK;
    // Pinned stripes are coded in place (zero-copy); the rest take the ring.
    // Hashing needs every shard on the device: when every stripe is pinned,
    // the zero-copy kernel also copies them to a device hash arena
    // (zero_copy_md5_run); otherwise the whole batch takes the ring.
    if (d_digest && zero_copy_enabled() && zero_copy_md5_enabled()) {
        int top = 0;
        for (int i : in_idx) top = std::max(top, i);
        for (int i : out_idx) top = std::max(top, i);
        std::vector<ZcStripe> zs;
        zs.reserve(n);
        // every stripe pinned: the aligned mirror kernel when all are 16-B
        // aligned with S % 16 == 0, else the mirrored gf_odd plan for all
        const bool any_align = hbec::zero_copy_any_alignment() && hbec::odd_enabled();
        bool all_aligned = true;
        for (uint64_t s = 0; s < n; ++s) {
            const uint64_t S = stripes[s].shard_len;
            if (!stripes[s].base || S == 0) break;
            const bool aligned = (reinterpret_cast<uintptr_t>(stripes[s].base) & 15u) == 0 && S % 16 == 0 &&
                                 S < (1ull << 32);
            if (!aligned && (!any_align || !hbec::pos32_shard(S))) break;
            const uint64_t d = pinned_device_addr(stripes[s].base, (uint64_t)(top + 1) * S);
            if (!d) break;
            all_aligned = all_aligned && aligned && (d & 15u) == 0;
            zs.push_back({d, S});
        }
        if (zs.size() == n && !all_aligned && !any_align) zs.clear();
        if (zs.size() == n && !all_aligned) {
            const uint64_t max_cols = (std::min(ring->in_cap / in_idx.size(), ring->out_cap / out_idx.size()) / 16) * 16;
            for (const ZcStripe& z : zs)
                if (z.shard_len > max_cols)
                    return fail(HBEC_ERR_INVALID_ARG, "hashing needs every stripe to fit one staging slot");
            g_md5_zc_calls.fetch_add(1, std::memory_order_relaxed);
            return zero_copy_unaligned_md5_run(ring, zs, in_idx, out_idx, rows, d_digest, n_shards);
        }
        if (zs.size() == n) {
            // the same stripe bound as the ring (hbec.h: one staging slot)
            const uint64_t max_cols = (std::min(ring->in_cap / in_idx.size(), ring->out_cap / out_idx.size()) / 16) * 16;
            for (const ZcStripe& z : zs)
                if (z.shard_len > max_cols)
                    return fail(HBEC_ERR_INVALID_ARG, "hashing needs every stripe to fit one staging slot");
            g_md5_zc_calls.fetch_add(1, std::memory_order_relaxed);
            return zero_copy_md5_run(ring, zs, in_idx, out_idx, rows, d_digest, n_shards);
        }
    }
    if (d_digest) g_md5_ring_calls.fetch_add(1, std::memory_order_relaxed);
    std::vector<hbec_stripe> staged;
    if (!d_digest && zero_copy_enabled()) {
        int top = 0;
        for (int i : in_idx) top = std::max(top, i);
        for (int i : out_idx) top = std::max(top, i);
        std::vector<ZcStripe> zs, zu;  // aligned (stripes kernel) / any alignment (unaligned kernel)
        for (uint64_t s = 0; s < n; ++s) {
            const uint64_t S = stripes[s].shard_len;
            if (S == 0) continue;
            const uint64_t d = stripes[s].base ? pinned_device_addr(stripes[s].base, (uint64_t)(top + 1) * S) : 0;
            const bool aligned = (reinterpret_cast<uintptr_t>(stripes[s].base) & 15u) == 0 && S % 16 == 0 &&
                                 S < (1ull << 32) && (d & 15u) == 0;
            if (d && aligned) zs.push_back({d, S});
            else if (d && hbec::zero_copy_any_alignment() && hbec::pos32_shard(S)) zu.push_back({d, S});  // gf_odd: 32-bit positions
            else staged.push_back(stripes[s]);
        }
        if (!zs.empty()) {
            rc = zero_copy_run(ring, zs, in_idx, out_idx, rows);
            if (rc) return rc;
        }
        if (!zu.empty()) {
            rc = zero_copy_unaligned_run(ring, zu, in_idx, out_idx, rows);
            if (rc) return rc;
        }
        if (staged.empty()) return HBEC_OK;
        stripes = staged.data();
        n = staged.size();
    }
    rc = ring_staging_init(*ring);
    if (rc) return rc;
    const uint64_t tile = (uint64_t)hbec::stripes_tile_bytes(std::min(K, hbec::kStripeMaxK));
    // max columns per piece so that K*lpad fits the IN slot and R*lpad the OUT slot
    const uint64_t max_cols = (std::min(ring->in_cap / K, ring->out_cap / R) / 16) * 16;
    if (max_cols < 16) return fail(HBEC_ERR_INVALID_ARG, "staging slot too small");
    if (d_digest) {
        for (uint64_t s = 0; s < n; ++s)
            if (stripes[s].shard_len > max_cols)
                return fail(HBEC_ERR_INVALID_ARG, "hashing needs every stripe to fit one staging slot");
        rc = ring_md5_init(*ring);
        if (rc) return rc;
    }
    ArenaCursor ac{ring, ring->s_cmp, d_digest};  // hash arenas (d_digest only)

    // Cut the batch into chunks of pieces that fit a slot.
    std::vector<std::vector<Piece>> chunks(1);
    uint64_t in_used = 0, out_used = 0, tiles_used = 0;
    for (uint64_t s = 0; s < n; ++s) {
        const uint64_t S = stripes[s].shard_len;
        if (S == 0) continue;
        if (!stripes[s].base) return fail(HBEC_ERR_INVALID_ARG, "stripe with null base");
        for (uint64_t col = 0; col < S; col += max_cols) {
            Piece p;
            p.stripe = s;
            p.col = col;
            p.len = std::min(max_cols, S - col);
            p.lpad = (p.len + 15) / 16 * 16;
            const uint64_t nt = (p.lpad + tile - 1) / tile;
            if (in_used + K * p.lpad > ring->in_cap || out_used + R * p.lpad > ring->out_cap ||
                tiles_used + nt > ring->tile_cap) {
                chunks.emplace_back();
                in_used = out_used = tiles_used = 0;
            }
            p.in_off = in_used;
            p.out_off = out_used;
            in_used += K * p.lpad;
            out_used += R * p.lpad;
            tiles_used += nt;
            chunks.back().push_back(p);
        }
    }
    if (chunks.back().empty()) chunks.pop_back();

    // in the slots inputs are packed 0..K-1 and outputs 0..R-1
    std::vector<int> slot_in(K), slot_out(R);
    for (int j = 0; j < K; ++j) slot_in[j] = j;
    for (int r = 0; r < R; ++r) slot_out[r] = r;

    std::vector<int64_t> slot_chunk(kSlots, -1);
    auto scatter = [&](int slot) -> int {
        const int64_t c = slot_chunk[slot];
        if (c < 0) return HBEC_OK;
        hipError_t e = hipEventSynchronize(ring->ev_done[slot]);
        if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
        const auto& pieces = chunks[c];
        ring->pool->parallel_for(pieces.size() * R, [&](size_t i) {
            const Piece& p = pieces[i / R];
            const int r = (int)(i % R);
            const hbec_stripe& st = stripes[p.stripe];
            std::memcpy(static_cast<uint8_t*>(st.base) + (uint64_t)out_idx[r] * st.shard_len + p.col,
                        ring->pin_out[slot] + p.out_off + (uint64_t)r * p.lpad, p.len);
        });
        slot_chunk[slot] = -1;
        return HBEC_OK;
    };

    for (size_t c = 0; c < chunks.size(); ++c) {
        const int slot = (int)(c % kSlots);
        rc = scatter(slot);  // the slot's previous chunk is complete; hand its output back
        if (rc) return rc;
        const auto& pieces = chunks[c];
        // gather inputs into the pinned IN slot and build the tile records
        ring->pool->parallel_for(pieces.size() * K, [&](size_t i) {
            const Piece& p = pieces[i / K];
            const int j = (int)(i % K);
            const hbec_stripe& st = stripes[p.stripe];
            uint8_t* dst = ring->pin_in[slot] + p.in_off + (uint64_t)j * p.lpad;
            std::memcpy(dst, static_cast<const uint8_t*>(st.base) + (uint64_t)in_idx[j] * st.shard_len + p.col,
                        p.len);
            if (p.lpad > p.len) std::memset(dst + p.len, 0, p.lpad - p.len);
        });
        uint64_t nt = 0, in_bytes = 0, out_bytes = 0;
        const uint64_t din = reinterpret_cast<uint64_t>(ring->dev_in[slot]);
        const uint64_t dout = reinterpret_cast<uint64_t>(ring->dev_out[slot]);
        for (const Piece& p : pieces) {
            for (uint64_t off = 0; off < p.lpad; off += tile) {
                hbec::TileRec& t = ring->pin_tiles[slot][nt++];
                t.in_addr = din + p.in_off + off;
                t.out_addr = dout + p.out_off + off;
                t.in_stride = (uint32_t)p.lpad;
                t.out_stride = (uint32_t)p.lpad;
                t.valid = (uint32_t)std::min<uint64_t>(tile, p.lpad - off);
                t.pad_ = 0;
            }
            in_bytes = std::max(in_bytes, p.in_off + K * p.lpad);
            out_bytes = std::max(out_bytes, p.out_off + R * p.lpad);
        }
        hipError_t e = hipSuccess;
        if (e == hipSuccess)
            e = hipMemcpyAsync(ring->dev_tiles[slot], ring->pin_tiles[slot], nt * sizeof(hbec::TileRec),
                               hipMemcpyHostToDevice, ring->s_h2d);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ring->dev_in[slot], ring->pin_in[slot], in_bytes, hipMemcpyHostToDevice, ring->s_h2d);
        if (e == hipSuccess) e = hipEventRecord(ring->ev_h2d[slot], ring->s_h2d);
        if (e == hipSuccess) e = hipStreamWaitEvent(ring->s_cmp, ring->ev_h2d[slot], 0);
        if (e != hipSuccess) return hip_fail(e, "host path H2D");
        rc = hbec::launch_stripe_passes(ring->dev_tiles[slot], nt, slot_in, slot_out, rows, 0, ring->s_cmp);
        if (rc) return rc;
        if (d_digest) {  // the chunk's shards -> hash arena (D2D, same stream, before the slot is released)
            if (!ac.fits(in_bytes + out_bytes, pieces.size() * (uint64_t)(K + R))) {
                rc = ac.flush();
                if (rc) return rc;
            }
            const uint64_t ain = ac.base();
            const uint64_t aout = ain + in_bytes;
            e = hipMemcpyAsync(reinterpret_cast<void*>(ain), ring->dev_in[slot], in_bytes, hipMemcpyDeviceToDevice,
                               ring->s_cmp);
            if (e == hipSuccess)
                e = hipMemcpyAsync(reinterpret_cast<void*>(aout), ring->dev_out[slot], out_bytes,
                                   hipMemcpyDeviceToDevice, ring->s_cmp);
            if (e != hipSuccess) return hip_fail(e, "hash arena copy");
            for (const Piece& p : pieces) {
                for (int j = 0; j < K; ++j)
                    ac.add(ain + p.in_off + (uint64_t)j * p.lpad, p.len, p.stripe * (uint64_t)n_shards + (uint64_t)in_idx[j]);
                for (int r = 0; r < R; ++r)
                    ac.add(aout + p.out_off + (uint64_t)r * p.lpad, p.len,
                           p.stripe * (uint64_t)n_shards + (uint64_t)out_idx[r]);
            }
            ac.used += (in_bytes + out_bytes + 255) & ~uint64_t(255);
        }
        e = hipEventRecord(ring->ev_cmp[slot], ring->s_cmp);
        if (e == hipSuccess) e = hipStreamWaitEvent(ring->s_d2h, ring->ev_cmp[slot], 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(ring->pin_out[slot], ring->dev_out[slot], out_bytes, hipMemcpyDeviceToHost,
                               ring->s_d2h);
        if (e == hipSuccess) e = hipEventRecord(ring->ev_done[slot], ring->s_d2h);
        if (e != hipSuccess) return hip_fail(e, "host path D2H");
        slot_chunk[slot] = (int64_t)c;
    }
    for (size_t i = 0; i < chunks.size() + kSlots; ++i) {  // drain in chunk order
        const int slot = (int)(i % kSlots);
        rc = scatter(slot);
        if (rc) return rc;
    }
    if (d_digest) return ac.finish();
    return HBEC_OK;
}

// One process, several GPUs (how a single object server would use a node):
// stripes are cut into contiguous runs of about equal bytes, one per device,
// and each run is coded by its own host thread on its device's ring (rings
// are per device), all at once.  Stripes are independent (ecutils.go:38-70),
// so there is no exchange between devices.
template <typename Fn>
int run_on_devices(const hbec_stripe* stripes, uint64_t n, const int* devices, int n_devices, Fn fn) {
    if (n && !stripes) return fail(HBEC_ERR_INVALID_ARG, "null argument");
    std::vector<int> devs;
    if (devices) {
        if (n_devices <= 0) return fail(HBEC_ERR_INVALID_ARG, "n_devices must be > 0");
        devs.assign(devices, devices + n_devices);
    } else {
        int count = 0;
        hipError_t e = hipGetDeviceCount(&count);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
        for (int d = 0; d < count; ++d) devs.push_back(d);
        if (n_devices > 0 && n_devices < count) devs.resize(n_devices);
    }
    if (devs.empty()) return fail(HBEC_ERR_DEVICE, "no device");
    if (n == 0) return HBEC_OK;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += stripes[i].shard_len;
    // contiguous runs of ~total / D shard bytes
    std::vector<uint64_t> cut(devs.size() + 1, n);
    cut[0] = 0;
    {
        uint64_t acc = 0;
        size_t d = 1;
        for (uint64_t i = 0; i < n && d < devs.size(); ++i) {
            acc += stripes[i].shard_len;
            while (d < devs.size() && acc * devs.size() >= total * d) cut[d++] = i + 1;
        }
    }
    std::vector<int> rcs(devs.size(), HBEC_OK);
    std::vector<std::string> errs(devs.size());
    std::vector<std::thread> th;
    for (size_t d = 0; d < devs.size(); ++d) {
        if (cut[d + 1] <= cut[d]) continue;
        th.emplace_back([&, d] {
            hipError_t e = hipSetDevice(devs[d]);
            if (e != hipSuccess) {
                rcs[d] = hip_fail(e, "hipSetDevice");
            } else {
                rcs[d] = fn(stripes + cut[d], cut[d + 1] - cut[d]);
            }
            if (rcs[d]) errs[d] = hbec_last_error();
        });
    }
    for (auto& t : th) t.join();
    for (size_t d = 0; d < devs.size(); ++d)
        if (rcs[d]) return fail(rcs[d], "device " + std::to_string(devs[d]) + ": " + errs[d]);
    return HBEC_OK;
}

}  // namespace

uint64_t hbec::host_md5_max_shard(const hbec_codec* codec) {
    const uint64_t slot = env_size("HBEC_HOST_SLOT_MB", 64) << 20;  // as ring_init
    const int k = hbec_data_shards(codec), m = hbec_parity_shards(codec);
    if (k < 1 || m < 1) return 0;
    return (std::min(slot / (uint64_t)k, slot / (uint64_t)m) / 16) * 16;
}

int hbec::host_threads() {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t share = env_size("OMP_NUM_THREADS", 16);
    const size_t want = std::min<size_t>(env_size("HBEC_HOST_THREADS", share), hw);
    return (int)std::max<size_t>(1, want);
}

extern "C" {

int hbec_host_alloc(size_t bytes, void** out) {
    return hbec::guarded("hbec_host_alloc", [&]() -> int {
        if (!out || bytes == 0) return fail(HBEC_ERR_INVALID_ARG, "null out or zero size");
        *out = nullptr;
        void* h = nullptr;
        // portable + mapped: every device of the process may code it in place
        // (coherent or non-coherent flags measured the same: 46.2-46.4 GiB/s)
        hipError_t e = hipHostMalloc(&h, bytes, hipHostMallocPortable | hipHostMallocMapped);
        if (e != hipSuccess) return hip_fail(e, "hipHostMalloc");
        void* d = nullptr;
        e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess || !d) {
            (void)hipHostFree(h);
            return hip_fail(e != hipSuccess ? e : hipErrorInvalidValue, "hipHostGetDevicePointer");
        }
        {
            std::lock_guard<std::mutex> g(g_pin_mu);
            g_pinned[reinterpret_cast<uint64_t>(h)] = PinnedRange{(uint64_t)bytes, reinterpret_cast<uint64_t>(d)};
        }
        *out = h;
        return HBEC_OK;
    });
}

void hbec_host_free(void* p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> g(g_pin_mu);
        g_pinned.erase(reinterpret_cast<uint64_t>(p));
    }
    (void)hipHostFree(p);
}

int hbec_host_device_addr(const void* p, uint64_t len, uint64_t* dev) {
    return hbec::guarded("hbec_host_device_addr", [&]() -> int {
        if (!dev) return fail(HBEC_ERR_INVALID_ARG, "null out");
        *dev = pinned_device_addr(p, len);
        return HBEC_OK;
    });
}

int hbec_encode_host(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes) {
    return hbec::guarded("hbec_encode_host", [&]() -> int {
        if (!codec || (n_stripes && !stripes)) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        const int k = hbec_data_shards(codec), m = hbec_parity_shards(codec);
        if (m == 0) return HBEC_OK;
        std::vector<uint8_t> mat((size_t)(k + m) * k);
        hbec_matrix(codec, mat.data());
        std::vector<uint8_t> rows(mat.begin() + (size_t)k * k, mat.end());
        std::vector<int> in_idx(k), out_idx(m);
        for (int j = 0; j < k; ++j) in_idx[j] = j;
        for (int r = 0; r < m; ++r) out_idx[r] = k + r;
        return host_run(stripes, n_stripes, in_idx, out_idx, rows);
    });
}

int hbec_encode_host_md5(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes, uint8_t* digests) {
    return hbec::guarded("hbec_encode_host_md5", [&]() -> int {
        if (!codec || !digests || (n_stripes && !stripes)) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        if (n_stripes == 0) return HBEC_OK;
        const int k = hbec_data_shards(codec), m = hbec_parity_shards(codec), n = k + m;
        if (m == 0) return fail(HBEC_ERR_INVALID_ARG, "encode_host_md5 needs parity shards");
        for (uint64_t s = 0; s < n_stripes; ++s)
            if (stripes[s].shard_len == 0) return fail(HBEC_ERR_SHARD_NO_DATA, "stripe with zero shard length");
        std::vector<uint8_t> mat((size_t)n * k);
        hbec_matrix(codec, mat.data());
        std::vector<uint8_t> rows(mat.begin() + (size_t)k * k, mat.end());
        std::vector<int> in_idx(k), out_idx(m);
        for (int j = 0; j < k; ++j) in_idx[j] = j;
        for (int r = 0; r < m; ++r) out_idx[r] = k + r;
        hipStream_t st = nullptr;
        int rc0 = stream_acquire(&st);
        if (rc0) return rc0;
        struct StreamBack {
            hipStream_t s;
            ~StreamBack() { stream_release(s); }
        } back{st};
        hipError_t e = hipSuccess;
        void* d_dig = nullptr;
        const size_t bytes = (size_t)n_stripes * n * 16;
        int rc = hbec::scratch_alloc(bytes, st, &d_dig);
        if (!rc) {
            e = hipStreamSynchronize(st);  // allocation visible to the ring's streams
            if (e != hipSuccess) rc = hip_fail(e, "scratch");
        }
        if (!rc) rc = host_run(stripes, n_stripes, in_idx, out_idx, rows, static_cast<uint8_t*>(d_dig), n);
        if (!rc) {
            e = hipMemcpyAsync(digests, d_dig, bytes, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) rc = hip_fail(e, "digests D2H");
        }
        hbec::scratch_free(d_dig, st);
        (void)hipStreamSynchronize(st);
        return rc;
    });
}

int hbec_host_md5_stats(uint64_t* zero_copy_calls, uint64_t* ring_calls) {
    if (zero_copy_calls) *zero_copy_calls = g_md5_zc_calls.load(std::memory_order_relaxed);
    if (ring_calls) *ring_calls = g_md5_ring_calls.load(std::memory_order_relaxed);
    return HBEC_OK;
}

int hbec_device_count(int* n) {
    return hbec::guarded("hbec_device_count", [&]() -> int {
        if (!n) return fail(HBEC_ERR_INVALID_ARG, "null out");
        *n = 0;
        hipError_t e = hipGetDeviceCount(n);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
        return HBEC_OK;
    });
}

int hbec_set_device(int device) {
    return hbec::guarded("hbec_set_device", [&]() -> int {
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
        return HBEC_OK;
    });
}

int hbec_encode_host_devices(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes, const int* devices,
                             int n_devices) {
    return hbec::guarded("hbec_encode_host_devices", [&]() -> int {
        return run_on_devices(stripes, n_stripes, devices, n_devices, [codec](const hbec_stripe* s, uint64_t n) {
            return hbec_encode_host(codec, s, n);
        });
    });
}

int hbec_reconstruct_host_devices(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes,
                                  const uint8_t* present, int data_only, const int* devices, int n_devices) {
    return hbec::guarded("hbec_reconstruct_host_devices", [&]() -> int {
        if (!present) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        return run_on_devices(stripes, n_stripes, devices, n_devices, [=](const hbec_stripe* s, uint64_t n) {
            return hbec_reconstruct_host(codec, s, n, present, data_only);
        });
    });
}

int hbec_reconstruct_host(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes,
                          const uint8_t* present, int data_only) {
    return hbec::guarded("hbec_reconstruct_host", [&]() -> int {
        if (!codec || !present || (n_stripes && !stripes)) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        const int k = hbec_data_shards(codec), m = hbec_parity_shards(codec), n = k + m;
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
        return host_run(stripes, n_stripes, surv, outs, rows);
    });
}

}  // extern "C"
