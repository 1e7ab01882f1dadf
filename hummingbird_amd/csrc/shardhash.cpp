// shardhash.cpp — ShardHash (MD5 of a shard body, objectserver/indexdb.go:746-753)
// on the GPU: one-shot batches, streaming chains fed stripe by stripe, and
// encode + hash of every shard with the two overlapped.
//
// Why the hash is not computed inside the encode kernel's output pass: the
// encode streams each object's shards in 1-4 KiB column tiles spread over
// many waves at once, while an MD5 chain must see its shard's 64-byte blocks
// strictly in order on one lane.  Instead hbec_encode_md5_batch cuts the shard
// range into column segments: the encode of segment s+1 (HBM-bound, one block
// per CU) runs on the caller's stream while the MD5 chains consume segment s
// (VALU-latency-bound, one lane per chain) on a side stream, so the hash
// mostly hides under the encode.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/hbec.h"
#include "internal.h"
#include "pool.h"

namespace hbec {

hipError_t launch_md5(const void* const* bases, const uint64_t* strides, int n_views, uint32_t chain_stride,
                      uint32_t view0, uint64_t n_obj, uint64_t len, uint64_t total, uint32_t flags, void* state,
                      uint8_t* digest, bool aligned, hipStream_t stream);
uint64_t md5_state_bytes();

namespace {

constexpr int kViewsPerLaunch = 32;
constexpr uint32_t kInit = 1u, kFinal = 2u;

// All views of one update/final step, launched 32 views at a time.
int md5_step(const hbec_view* views, int n_views, uint64_t n_obj, uint64_t len, uint64_t total, uint32_t flags,
             void* state, uint8_t* digest, hipStream_t stream) {
    const uint64_t carry = total & 63u;
    const uint64_t first = carry ? 64u - carry : 0u;  // data offset of the first whole block
    bool aligned = true;
    for (int v = 0; v < n_views; ++v) {
        const uintptr_t b = reinterpret_cast<uintptr_t>(views[v].base) + first;
        if ((b & 15u) || (views[v].obj_stride & 15u)) aligned = false;
    }
    for (int v0 = 0; v0 < n_views; v0 += kViewsPerLaunch) {
        const int nv = std::min(kViewsPerLaunch, n_views - v0);
        const void* bases[kViewsPerLaunch];
        uint64_t strides[kViewsPerLaunch];
        for (int v = 0; v < nv; ++v) {
            bases[v] = views[v0 + v].base;
            strides[v] = views[v0 + v].obj_stride;
        }
        hipError_t e = launch_md5(bases, strides, nv, (uint32_t)n_views, (uint32_t)v0, n_obj, len, total, flags,
                                  state, digest, aligned, stream);
        if (e != hipSuccess) return hip_fail(e, "md5 launch");
    }
    return HBEC_OK;
}

int check_digests(const uint8_t* d) {
    if (!d) return fail(HBEC_ERR_INVALID_ARG, "md5: null digest buffer");
    if (reinterpret_cast<uintptr_t>(d) & 3u) return fail(HBEC_ERR_INVALID_ARG, "md5: digest buffer not 4-byte aligned");
    return HBEC_OK;
}

int check_views(const hbec_view* views, int n_views, uint64_t n_obj, uint64_t len) {
    if (!views || n_views <= 0) return fail(HBEC_ERR_INVALID_ARG, "md5: need at least one view");
    if (n_obj > (1ull << 31) / 64 * 64) return fail(HBEC_ERR_INVALID_ARG, "md5: too many objects for one call");
    if (len > 0)
        for (int v = 0; v < n_views; ++v)
            if (!views[v].base) return fail(HBEC_ERR_INVALID_ARG, "md5: null view");
    return HBEC_OK;
}

// Side streams for the segment pipeline: taken per call, returned right after
// the call has queued its work (later users only queue behind it).  Created
// on first use per device and kept for the life of the process.
std::mutex g_side_mu;
std::vector<std::pair<int, hipStream_t>> g_side_free;

int side_stream_get(int dev, hipStream_t* s) {
    {
        std::lock_guard<std::mutex> g(g_side_mu);
        for (size_t i = 0; i < g_side_free.size(); ++i)
            if (g_side_free[i].first == dev) {
                *s = g_side_free[i].second;
                g_side_free.erase(g_side_free.begin() + (long)i);
                return HBEC_OK;
            }
    }
    static const bool prio = tune_knob("HBEC_MD5_SIDE_PRIO", 0) == 1;
    hipError_t e;
    if (prio) {
        int lo = 0, hi = 0;
        e = hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
    } else {
        e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    }
    if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
    return HBEC_OK;
}

void side_stream_put(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_side_mu);
    g_side_free.emplace_back(dev, s);
}

// Library-owned stream-ordered memory pool per device for the per-call chain
// state (the default pool returns memory to the driver at every sync, which
// turned each call's hipMallocAsync into a real allocation).
std::mutex g_pool_mu;
std::map<int, hipMemPool_t> g_pools;

int state_pool(int dev, hipMemPool_t* out) {
    std::lock_guard<std::mutex> g(g_pool_mu);
    auto it = g_pools.find(dev);
    if (it == g_pools.end()) {
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        hipMemPool_t pool;
        hipError_t e = hipMemPoolCreate(&pool, &props);
        if (e != hipSuccess) return hip_fail(e, "hipMemPoolCreate");
        uint64_t keep = UINT64_MAX;
        e = hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        if (e != hipSuccess) return hip_fail(e, "hipMemPoolSetAttribute");
        it = g_pools.emplace(dev, pool).first;
    }
    *out = it->second;
    return HBEC_OK;
}

// Event-ordered "b waits for everything queued on a so far".
int order_after(hipStream_t b, hipStream_t a) {
    hipEvent_t ev;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return hip_fail(e, "hipEventCreate");
    e = hipEventRecord(ev, a);
    if (e == hipSuccess) e = hipStreamWaitEvent(b, ev, 0);
    hipEventDestroy(ev);  // released once the recorded work completes
    if (e != hipSuccess) return hip_fail(e, "stream ordering");
    return HBEC_OK;
}

// md5_list records (md5.hip Md5ListRec)
struct ListRec {
    uint64_t addr, len, slot, pad;
};

// Records for n buffers, longest first (a wave lasts as long as its longest chain).
void list_records(const void* const* bufs, const uint64_t* lens, uint64_t n, std::vector<ListRec>& recs,
                  bool* aligned) {
    recs.resize(n);
    *aligned = true;
    for (uint64_t i = 0; i < n; ++i) {
        recs[i] = ListRec{reinterpret_cast<uint64_t>(bufs[i]), lens[i], i, 0};
        if (recs[i].addr & 15u) *aligned = false;
    }
    std::stable_sort(recs.begin(), recs.end(), [](const ListRec& a, const ListRec& b) { return a.len > b.len; });
}

// Pinned staging ring for hbec_md5_host: per slot a pinned buffer, a device
// buffer, pinned + device record arrays, a stream and an event.  Pooled per
// device; one call at a time per ring.
constexpr int kHashSlots = 3;
struct HashRing {
    int dev = 0;
    size_t cap = 0, rec_cap = 0;
    uint8_t* pin[kHashSlots] = {};
    uint8_t* dbuf[kHashSlots] = {};
    ListRec* pin_rec[kHashSlots] = {};
    ListRec* drec[kHashSlots] = {};
    hipStream_t stream[kHashSlots] = {};
    hipEvent_t ev[kHashSlots] = {};
    ~HashRing() {
        for (int i = 0; i < kHashSlots; ++i) {
            if (pin[i]) (void)hipHostFree(pin[i]);
            if (pin_rec[i]) (void)hipHostFree(pin_rec[i]);
            if (dbuf[i]) (void)hipFree(dbuf[i]);
            if (drec[i]) (void)hipFree(drec[i]);
            if (ev[i]) (void)hipEventDestroy(ev[i]);
            if (stream[i]) (void)hipStreamDestroy(stream[i]);
        }
    }
};

// Bounded per device like the host path's rings (HBEC_HOST_RINGS, default
// 8; each pins 192 MiB): callers beyond the bound wait for one to come back.
std::mutex g_hash_mu;
std::condition_variable g_hash_cv;
std::vector<HashRing*> g_hash_free;
std::map<int, int> g_hash_made;

int hash_ring_limit() {
    static const int v = [] {
        const int x = (int)env_knob("HBEC_HOST_RINGS", 0);
        return x > 0 ? x : 8;
    }();
    return v;
}

int hash_ring_make(int dev, HashRing** out);

int hash_ring_acquire(HashRing** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    {
        std::unique_lock<std::mutex> lk(g_hash_mu);
        for (;;) {
            for (size_t i = 0; i < g_hash_free.size(); ++i)
                if (g_hash_free[i]->dev == dev) {
                    *out = g_hash_free[i];
                    g_hash_free.erase(g_hash_free.begin() + (long)i);
                    return HBEC_OK;
                }
            if (g_hash_made[dev] < hash_ring_limit()) break;
            g_hash_cv.wait(lk);
        }
        ++g_hash_made[dev];  // reserved: made below, outside the lock
    }
    const int rc = hash_ring_make(dev, out);
    if (rc) {
        {
            std::lock_guard<std::mutex> g(g_hash_mu);
            --g_hash_made[dev];
        }
        g_hash_cv.notify_one();
    }
    return rc;
}

int hash_ring_make(int dev, HashRing** out) {
    hipError_t e = hipSuccess;
    std::unique_ptr<HashRing> r(new (std::nothrow) HashRing());
    if (!r) return fail(HBEC_ERR_NOMEM, "hash ring");
    r->dev = dev;
    const long long mb = env_knob("HBEC_HOST_SLOT_MB", 64);
    r->cap = (size_t)(mb > 0 ? mb : 64) << 20;
    r->rec_cap = 65536;
    for (int i = 0; i < kHashSlots && e == hipSuccess; ++i) {
        e = hipHostMalloc(reinterpret_cast<void**>(&r->pin[i]), r->cap, hipHostMallocDefault);
        if (e == hipSuccess)
            e = hipHostMalloc(reinterpret_cast<void**>(&r->pin_rec[i]), r->rec_cap * sizeof(ListRec),
                              hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc(&r->dbuf[i], r->cap);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&r->drec[i]), r->rec_cap * sizeof(ListRec));
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&r->stream[i], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&r->ev[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) return hip_fail(e, "hash ring");
    *out = r.release();
    return HBEC_OK;
}

void hash_ring_release(HashRing* r) {
    for (int i = 0; i < kHashSlots; ++i) (void)hipStreamSynchronize(r->stream[i]);
    {
        std::lock_guard<std::mutex> g(g_hash_mu);
        g_hash_free.push_back(r);
    }
    g_hash_cv.notify_all();
}

}  // namespace

int scratch_alloc(size_t bytes, hipStream_t stream, void** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    hipMemPool_t pool;
    int rc = state_pool(dev, &pool);
    if (rc) return rc;
    e = hipMallocFromPoolAsync(out, std::max<size_t>(bytes, 16), pool, stream);
    if (e != hipSuccess) return hip_fail(e, "hipMallocFromPoolAsync");
    return HBEC_OK;
}

void scratch_free(void* p, hipStream_t stream) {
    if (p) (void)hipFreeAsync(p, stream);
}

// Segment length for the encode/hash pipeline: ~n segments, 4 KiB multiples
// (whole MD5 blocks, whole encode tiles), none below 16 KiB.  n = 8 for
// k <= 4 and 1 (encode, then hash, one stream) above: the pipelined encode
// kernels for k >= 5 hold most of a SIMD's register file (8+3: 506 of 512),
// so co-resident MD5 waves block their launch and the overlap turns into
// serialisation (profiles/r01_md5_sweep.jsonl: 8+3 pipelined 3.4 ms vs 2.45
// sequential; 4+2 3.13 vs 3.87).  HBEC_MD5_SEGMENTS overrides n.
static const int g_md5_segments = (int)std::max(0LL, tune_knob("HBEC_MD5_SEGMENTS", 0));

static uint64_t md5_segment(uint64_t shard_len, int k) {
    const int n = g_md5_segments ? g_md5_segments : (k <= 4 ? 8 : 1);
    if (n == 1) return shard_len;
    uint64_t seg = (shard_len / (uint64_t)n + 4095) & ~uint64_t(4095);
    return std::max<uint64_t>(seg, 16384);
}

}  // namespace hbec

using namespace hbec;

struct hbec_md5 {
    int n_views = 0;
    uint64_t n_obj = 0;
    uint64_t total = 0;
    bool started = false;
    void* d_state = nullptr;
};

extern "C" {

int hbec_md5_batch(const hbec_view* views, int n_views, uint64_t n_objects, uint64_t len, uint8_t* d_digests,
                   void* hip_stream) {
    return hbec::guarded("hbec_md5_batch", [&]() -> int {
        int rc = check_views(views, n_views, n_objects, len);
        if (rc) return rc;
        rc = check_digests(d_digests);
        if (rc) return rc;
        if (n_objects == 0) return HBEC_OK;
        return md5_step(views, n_views, n_objects, len, 0, kInit | kFinal, nullptr, d_digests,
                        static_cast<hipStream_t>(hip_stream));
    });
}

int hbec_md5_list(const void* const* d_bufs, const uint64_t* lens, uint64_t n, uint8_t* d_digests,
                  void* hip_stream) {
    return hbec::guarded("hbec_md5_list", [&]() -> int {
        if (n == 0) return HBEC_OK;
        if (!d_bufs || !lens) return fail(HBEC_ERR_INVALID_ARG, "md5_list: null argument");
        int rc = check_digests(d_digests);
        if (rc) return rc;
        for (uint64_t i = 0; i < n; ++i)
            if (!d_bufs[i] && lens[i]) return fail(HBEC_ERR_INVALID_ARG, "md5_list: null buffer");
        std::vector<ListRec> recs;
        bool aligned = true;
        list_records(d_bufs, lens, n, recs, &aligned);
        hipStream_t stream = static_cast<hipStream_t>(hip_stream);
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
        hipMemPool_t pool;
        rc = state_pool(dev, &pool);
        if (rc) return rc;
        void* drec = nullptr;
        e = hipMallocFromPoolAsync(&drec, n * sizeof(ListRec), pool, stream);
        if (e != hipSuccess) return hip_fail(e, "hipMallocFromPoolAsync");
        // pageable source: staged by the runtime before the call returns
        e = hipMemcpyAsync(drec, recs.data(), n * sizeof(ListRec), hipMemcpyHostToDevice, stream);
        if (e == hipSuccess) e = launch_md5_list(drec, n, d_digests, aligned, stream);
        (void)hipFreeAsync(drec, stream);
        if (e != hipSuccess) return hip_fail(e, "md5_list");
        return HBEC_OK;
    });
}

int hbec_md5_host(const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint8_t* digests) {
    return hbec::guarded("hbec_md5_host", [&]() -> int {
        if (n == 0) return HBEC_OK;
        if (!bufs || !lens || !digests) return fail(HBEC_ERR_INVALID_ARG, "md5_host: null argument");
        for (uint64_t i = 0; i < n; ++i)
            if (!bufs[i] && lens[i]) return fail(HBEC_ERR_INVALID_ARG, "md5_host: null buffer");
        HashRing* ring = nullptr;
        int rc = hash_ring_acquire(&ring);
        if (rc) return rc;
        struct Rel {
            HashRing* r;
            ~Rel() { hash_ring_release(r); }
        } rel{ring};
        int dev = ring->dev;
        hipMemPool_t mpool;
        rc = state_pool(dev, &mpool);
        if (rc) return rc;
        uint8_t* d_dig = nullptr;
        hipError_t e = hipMallocFromPoolAsync(reinterpret_cast<void**>(&d_dig), n * 16, mpool, ring->stream[0]);
        if (e != hipSuccess) return hip_fail(e, "hipMallocFromPoolAsync");
        for (int i = 1; i < kHashSlots && e == hipSuccess; ++i) {  // every slot stream sees the allocation
            e = hipEventRecord(ring->ev[0], ring->stream[0]);
            if (e == hipSuccess) e = hipStreamWaitEvent(ring->stream[i], ring->ev[0], 0);
        }
        if (e != hipSuccess) return hip_fail(e, "md5_host ordering");
        // longest first; chunks of buffers that fit a slot (16-B aligned offsets)
        std::vector<uint64_t> order(n);
        for (uint64_t i = 0; i < n; ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return lens[a] > lens[b]; });
        std::vector<std::vector<uint64_t>> chunks;
        std::vector<uint64_t> big;  // longer than a slot: streamed through slot 0 piece by piece
        uint64_t used = 0;
        for (uint64_t i : order) {
            const uint64_t sz = (lens[i] + 15) & ~uint64_t(15);
            if (lens[i] > ring->cap) {
                big.push_back(i);
                continue;
            }
            if (chunks.empty() || used + sz > ring->cap || chunks.back().size() >= ring->rec_cap) {
                chunks.emplace_back();
                used = 0;
            }
            chunks.back().push_back(i);
            used += sz;
        }
        Pool pool(host_threads() - 1);
        for (size_t c = 0; c < chunks.size(); ++c) {
            const int s = (int)(c % kHashSlots);
            e = hipEventSynchronize(ring->ev[s]);  // slot free: its previous chunk has been hashed
            if (e != hipSuccess) return hip_fail(e, "md5_host wait");
            const auto& ch = chunks[c];
            std::vector<uint64_t> off(ch.size());
            uint64_t o = 0;
            for (size_t j = 0; j < ch.size(); ++j) {
                off[j] = o;
                o += (lens[ch[j]] + 15) & ~uint64_t(15);
            }
            pool.parallel_for(ch.size(), [&](size_t j) {
                if (lens[ch[j]]) std::memcpy(ring->pin[s] + off[j], bufs[ch[j]], lens[ch[j]]);
            });
            const uint64_t dbase = reinterpret_cast<uint64_t>(ring->dbuf[s]);
            for (size_t j = 0; j < ch.size(); ++j) ring->pin_rec[s][j] = ListRec{dbase + off[j], lens[ch[j]], ch[j], 0};
            e = hipMemcpyAsync(ring->drec[s], ring->pin_rec[s], ch.size() * sizeof(ListRec), hipMemcpyHostToDevice,
                               ring->stream[s]);
            if (e == hipSuccess && o)
                e = hipMemcpyAsync(ring->dbuf[s], ring->pin[s], o, hipMemcpyHostToDevice, ring->stream[s]);
            if (e == hipSuccess) e = launch_md5_list(ring->drec[s], ch.size(), d_dig, true, ring->stream[s]);
            if (e == hipSuccess) e = hipEventRecord(ring->ev[s], ring->stream[s]);
            if (e != hipSuccess) return hip_fail(e, "md5_host chunk");
        }
        for (int s = 0; s < kHashSlots; ++s) {
            e = hipStreamSynchronize(ring->stream[s]);
            if (e != hipSuccess) return hip_fail(e, "md5_host drain");
        }
        // buffers larger than a slot: one streaming chain each, slot-sized pieces
        for (uint64_t i : big) {
            hbec_md5* ctx = nullptr;
            rc = hbec_md5_new(1, 1, &ctx);
            if (rc) return rc;
            for (uint64_t pos = 0; pos < lens[i] && rc == HBEC_OK; pos += ring->cap) {
                const uint64_t len = std::min<uint64_t>(ring->cap, lens[i] - pos);
                pool.parallel_for(16, [&](size_t t) {
                    const uint64_t a = len * t / 16, b = len * (t + 1) / 16;
                    std::memcpy(ring->pin[0] + a, bufs[i] + pos + a, b - a);
                });
                e = hipMemcpyAsync(ring->dbuf[0], ring->pin[0], len, hipMemcpyHostToDevice, ring->stream[0]);
                if (e != hipSuccess) rc = hip_fail(e, "md5_host H2D");
                hbec_view v{ring->dbuf[0], 0};
                if (!rc) rc = hbec_md5_update(ctx, &v, len, ring->stream[0]);
                if (!rc) {
                    e = hipStreamSynchronize(ring->stream[0]);  // pinned slot reused by the next piece
                    if (e != hipSuccess) rc = hip_fail(e, "md5_host sync");
                }
            }
            if (!rc) rc = hbec_md5_final(ctx, d_dig + i * 16, ring->stream[0]);
            hbec_md5_free(ctx);  // hipFree synchronises with the queued final
            if (rc) return rc;
        }
        e = hipMemcpyAsync(digests, d_dig, n * 16, hipMemcpyDeviceToHost, ring->stream[0]);
        (void)hipFreeAsync(d_dig, ring->stream[0]);
        if (e == hipSuccess) e = hipStreamSynchronize(ring->stream[0]);
        if (e != hipSuccess) return hip_fail(e, "md5_host digests");
        return HBEC_OK;
    });
}

int hbec_md5_new(int n_views, uint64_t n_objects, hbec_md5** out) {
    return hbec::guarded("hbec_md5_new", [&]() -> int {
        if (!out || n_views <= 0 || n_objects == 0) return fail(HBEC_ERR_INVALID_ARG, "md5_new: bad arguments");
        *out = nullptr;
        hbec_md5* c = new (std::nothrow) hbec_md5();
        if (!c) return fail(HBEC_ERR_NOMEM, "md5_new");
        c->n_views = n_views;
        c->n_obj = n_objects;
        hipError_t e = hipMalloc(&c->d_state, (size_t)n_views * n_objects * md5_state_bytes());
        if (e != hipSuccess) {
            delete c;
            return e == hipErrorOutOfMemory ? fail(HBEC_ERR_NOMEM, "md5 state") : hip_fail(e, "hipMalloc");
        }
        *out = c;
        return HBEC_OK;
    });
}

void hbec_md5_free(hbec_md5* c) {
    if (!c) return;
    if (c->d_state) hipFree(c->d_state);
    delete c;
}

int hbec_md5_update(hbec_md5* c, const hbec_view* views, uint64_t len, void* hip_stream) {
    return hbec::guarded("hbec_md5_update", [&]() -> int {
        if (!c) return fail(HBEC_ERR_INVALID_ARG, "md5_update: null context");
        int rc = check_views(views, c->n_views, c->n_obj, len);
        if (rc) return rc;
        if (len == 0 && c->started) return HBEC_OK;
        rc = md5_step(views, c->n_views, c->n_obj, len, c->total, c->started ? 0u : kInit, c->d_state, nullptr,
                      static_cast<hipStream_t>(hip_stream));
        if (rc) return rc;
        c->started = true;
        c->total += len;
        return HBEC_OK;
    });
}

int hbec_md5_final(hbec_md5* c, uint8_t* d_digests, void* hip_stream) {
    return hbec::guarded("hbec_md5_final", [&]() -> int {
        if (!c) return fail(HBEC_ERR_INVALID_ARG, "md5_final: null context");
        int rc0 = check_digests(d_digests);
        if (rc0) return rc0;
        std::vector<hbec_view> none((size_t)c->n_views, hbec_view{nullptr, 0});
        int rc = md5_step(none.data(), c->n_views, c->n_obj, 0, c->total, kFinal | (c->started ? 0u : kInit),
                          c->d_state, d_digests, static_cast<hipStream_t>(hip_stream));
        if (rc) return rc;
        c->started = false;
        c->total = 0;
        return HBEC_OK;
    });
}

int hbec_encode_md5_batch(hbec_codec* codec, const hbec_view* views, uint64_t n_objects, uint64_t shard_len,
                          uint8_t* d_digests, void* hip_stream) {
    return hbec::guarded("hbec_encode_md5_batch", [&]() -> int {
        if (!codec || !views) return fail(HBEC_ERR_INVALID_ARG, "encode_md5: null argument");
        const int n = hbec_data_shards(codec) + hbec_parity_shards(codec);
        int rc = check_digests(d_digests);
        if (rc) return rc;
        if (n_objects == 0) return HBEC_OK;
        if (shard_len == 0) return fail(HBEC_ERR_SHARD_NO_DATA, "encode_md5: zero shard length");
        rc = check_views(views, n, n_objects, shard_len);
        if (rc) return rc;
        hipStream_t main = static_cast<hipStream_t>(hip_stream);
        const uint64_t seg = md5_segment(shard_len, hbec_data_shards(codec));
        if (seg >= shard_len) {  // one segment: encode, then hash every shard
            rc = hbec_encode_batch(codec, views, n_objects, shard_len, hip_stream);
            if (rc) return rc;
            return md5_step(views, n, n_objects, shard_len, 0, kInit | kFinal, nullptr, d_digests, main);
        }
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
        hipMemPool_t pool;
        rc = state_pool(dev, &pool);
        if (rc) return rc;
        void* state = nullptr;
        e = hipMallocFromPoolAsync(&state, (size_t)n * n_objects * md5_state_bytes(), pool, main);
        if (e != hipSuccess) return hip_fail(e, "hipMallocFromPoolAsync");
        hipStream_t side;
        rc = side_stream_get(dev, &side);
        if (rc) {
            hipFreeAsync(state, main);
            return rc;
        }
        std::vector<hbec_view> sv((size_t)n);
        static const uint64_t head = (uint64_t)std::max(0LL, tune_knob("HBEC_MD5_HEAD_KIB", 0)) * 1024u;
        static const int enc_grid = (int)tune_knob("HBEC_MD5_ENC_GRID", 0);
        for (uint64_t off = 0; off < shard_len && rc == HBEC_OK;) {
            const uint64_t want = (off == 0 && head > 0) ? std::min(head, seg) : seg;
            const uint64_t len = std::min(want, shard_len - off);
            for (int i = 0; i < n; ++i) sv[i] = hbec_view{static_cast<uint8_t*>(views[i].base) + off, views[i].obj_stride};
            set_thread_grid_cap(off > 0 ? enc_grid : 0);
            rc = hbec_encode_batch(codec, sv.data(), n_objects, len, hip_stream);
            set_thread_grid_cap(0);
            if (rc) break;
            rc = order_after(side, main);  // segment encoded (and, first time, state allocated)
            if (rc) break;
            const uint32_t flags = (off == 0 ? kInit : 0u) | (off + len == shard_len ? kFinal : 0u);
            rc = md5_step(sv.data(), n, n_objects, len, off, flags, state, d_digests, side);
            off += len;
        }
        const int rc2 = order_after(main, side);  // caller's stream: digests ready
        hipFreeAsync(state, main);
        side_stream_put(dev, side);
        return rc ? rc : rc2;
    });
}

}  // extern "C"
