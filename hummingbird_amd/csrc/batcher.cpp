// batcher.cpp — batched stabilization driver.
//
// In the reference every nursery object is stabilized by its own call chain
// (objectserver/nurserystabilizer.go:72-99: one object at a time per device,
// `object-nursery.concurrency` workers, a 1 ms sleep between objects), and
// ecSplit encodes each stripe with its own Encoder call (ecutils.go:59).  On
// the GPU a single 1 MiB encode is dominated by launch + PCIe latency, so this
// driver lets concurrent callers share launches: each caller submits one host
// stripe (ecSplit databuf layout) and blocks; a worker thread takes everything
// queued — up to its share of max_batch_bytes, or whatever has arrived when
// max_wait_us passes after it started waiting — codes it with one streaming
// host-path call (hostpath.cpp), and wakes the callers.
//
// Several workers (HBEC_BATCHER_WORKERS, default 2) split max_batch_bytes
// between them, so one batch's callers can wake up and queue their next
// stripes while another batch is on the GPU: the per-batch wake-up, fill and
// launch overheads overlap the other batch's transfer.
//
// Encode + ShardHash requests have workers of their own
// (HBEC_BATCHER_MD5_WORKERS, default 4).  An MD5 chain is strictly serial,
// one GPU lane per shard (md5.hip): a 256 KiB shard takes ~2.3 ms however
// small the batch, so a worker that waits for its batch's digests is
// latency-bound.  With several hashing workers, batch i's hashes run on the
// GPU while batches i+1.. are encoded and hashed: encode + hash throughput
// grows with the number of waiting callers instead of stopping at one batch
// per 2.3 ms, and plain Encode batches never queue behind a hash.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hbec.h"
#include "internal.h"

using hbec::fail;

namespace {

struct Request {
    hbec_stripe stripe;
    int op;  // 0 encode, 1 reconstruct, 2 encode + ShardHash
    uint8_t* digests = nullptr;  // op 2: (k+m) * 16 B
    std::vector<uint8_t> present;
    int data_only = 0;
    int rc = HBEC_OK;
    std::string err;
    // completion: each caller sleeps on its own condition variable, so a
    // finished batch wakes exactly its callers (not every queued one)
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
};

}  // namespace

struct hbec_batcher {
    hbec_codec* codec = nullptr;
    int device = 0;
    uint64_t max_batch_bytes = 0;
    std::chrono::microseconds max_wait{0};
    std::chrono::microseconds quiet{0};  // HBEC_BATCHER_QUIET_US: stop filling after this long with no arrival
    std::mutex mu;
    std::condition_variable cv_work;
    std::deque<Request*> queue;
    bool stop = false;
    uint64_t batch_cap = 0;  // bytes one worker takes per batch: max_batch_bytes / workers
    int md5_workers = 0;     // workers reserved for Encode + ShardHash groups
    uint64_t md5_cap = 0;    // bytes one MD5 worker takes: max_batch_bytes / md5_workers
    std::vector<std::thread> workers;
    // statistics
    uint64_t batches = 0, stripes = 0;

    // Code one homogeneous group with one host-path call; if that call fails,
    // retry each member alone so every caller gets its own result.
    int code(const std::vector<Request*>& batch, int n_shards) {
        auto one = [&](const std::vector<Request*>& g) -> int {
            std::vector<hbec_stripe> st(g.size());
            for (size_t i = 0; i < g.size(); ++i) st[i] = g[i]->stripe;
            if (g[0]->op == 0) return hbec_encode_host(codec, st.data(), st.size());
            if (g[0]->op == 2) {
                std::vector<uint8_t> dig(st.size() * (size_t)n_shards * 16);
                const int rc = hbec_encode_host_md5(codec, st.data(), st.size(), dig.data());
                if (rc == HBEC_OK)
                    for (size_t i = 0; i < g.size(); ++i)
                        std::memcpy(g[i]->digests, dig.data() + i * (size_t)n_shards * 16, (size_t)n_shards * 16);
                return rc;
            }
            return hbec_reconstruct_host(codec, st.data(), st.size(), g[0]->present.data(), g[0]->data_only);
        };
        int rc = one(batch);
        std::string err = rc ? hbec_last_error() : "";
        if (rc == HBEC_OK || batch.size() == 1) {
            for (auto* r : batch) {
                r->rc = rc;
                r->err = err;
            }
            return rc;
        }
        for (auto* r : batch) {
            r->rc = one({r});
            r->err = r->rc ? hbec_last_error() : "";
        }
        return rc;
    }

    // md5_only: this worker takes only Encode + ShardHash groups; otherwise
    // it takes any group except those (when MD5 workers exist)
    void run(bool md5_only) {
        (void)hipSetDevice(device);
        std::unique_lock<std::mutex> lk(mu);
        const int n_shards = hbec_data_shards(codec) + hbec_parity_shards(codec);
        for (;;) {
            auto mine = [&](const Request* r) { return md5_workers == 0 || (r->op == 2) == md5_only; };
            auto first_mine = [&]() -> Request* {
                for (auto* r : queue)
                    if (mine(r)) return r;
                return nullptr;
            };
            cv_work.wait(lk, [&] { return stop || first_mine() != nullptr; });
            if (stop && !first_mine()) return;
            // let the batch fill: until max bytes are queued, max_wait has
            // passed since this worker started waiting, or no request has
            // arrived for quiet (the callers that were going to come have
            // come: small stripes never fill max bytes, and waiting out
            // max_wait would dominate their round trip)
            const auto t0 = std::chrono::steady_clock::now();
            const auto deadline = t0 + max_wait;
            // MD5 groups stay smaller (max_batch_bytes / md5 workers): a group
            // is held ~2.3 ms by its hash however small it is, so the bytes
            // are better spread over more workers hashing at once
            const uint64_t cap = md5_only && md5_workers > 0 ? md5_cap : batch_cap;
            size_t seen_n = 0;
            auto last_arrival = t0;
            while (!stop) {
                uint64_t queued = 0;
                size_t n_mine = 0;
                for (auto* r : queue)
                    if (mine(r)) {
                        queued += r->stripe.shard_len * (uint64_t)n_shards;
                        ++n_mine;
                    }
                if (queued >= cap) break;
                const auto now = std::chrono::steady_clock::now();
                if (n_mine != seen_n) {
                    seen_n = n_mine;
                    last_arrival = now;
                }
                if (now >= deadline || now - last_arrival >= quiet) break;
                (void)cv_work.wait_until(lk, std::min(deadline, last_arrival + quiet));
            }
            const Request* head = first_mine();
            if (!head) continue;  // another worker took it while this one waited
            // one homogeneous group (same op and erasure pattern as the oldest
            // request), gathered from the WHOLE queue: a request of another
            // kind between them does not split the batch
            std::vector<Request*> batch;
            try {  // reserved up front: nothing below may throw once requests leave the queue
                batch.reserve(queue.size());
            } catch (...) {
                lk.unlock();
                std::this_thread::sleep_for(std::chrono::microseconds(100));  // requests stay queued; retry
                lk.lock();
                continue;
            }
            uint64_t bytes = 0;
            for (auto it = queue.begin(); it != queue.end();) {
                Request* r = *it;
                const bool same = r->op == head->op && r->present == head->present && r->data_only == head->data_only;
                const uint64_t b = r->stripe.shard_len * (uint64_t)n_shards;
                if (same && (batch.empty() || bytes + b <= cap)) {
                    batch.push_back(r);
                    bytes += b;
                    it = queue.erase(it);
                } else {
                    ++it;
                }
            }
            lk.unlock();
            // no exception may escape the worker (std::terminate): a throw before
            // the per-request results were recorded fails the whole group
            int thrown = HBEC_OK;
            try {
                (void)code(batch, n_shards);
            } catch (const std::bad_alloc&) {
                thrown = HBEC_ERR_NOMEM;
            } catch (...) {
                thrown = HBEC_ERR_DEVICE;
            }
            if (thrown != HBEC_OK)
                for (auto* r : batch) {
                    r->rc = thrown;
                    try {  // the message is best effort
                        r->err = thrown == HBEC_ERR_NOMEM ? "batcher: host allocation failed"
                                                          : "batcher: unexpected exception";
                    } catch (...) {
                    }
                }
            for (auto* r : batch) {
                // notify while holding r->m: the caller cannot see `done`, return and
                // destroy r (it lives on the caller's stack) before this scope ends
                std::lock_guard<std::mutex> g(r->m);
                r->done = true;
                r->cv.notify_one();
            }
            lk.lock();
            ++batches;
            stripes += batch.size();
        }
    }

    int submit(Request& r) {
        // per-request checks before queueing, so one caller's bad stripe
        // never fails the unrelated callers batched with it
        if (!r.stripe.base) return fail(HBEC_ERR_INVALID_ARG, "stripe with null base");
        if (r.op == 2 && r.stripe.shard_len > hbec::host_md5_max_shard(codec))
            return fail(HBEC_ERR_INVALID_ARG, "hashing needs every stripe to fit one staging slot");
        {
            std::lock_guard<std::mutex> g(mu);
            if (stop) return fail(HBEC_ERR_INVALID_ARG, "batcher stopped");
            queue.push_back(&r);
        }
        cv_work.notify_all();  // a worker filling its batch re-checks the size; an idle one starts
        std::unique_lock<std::mutex> lk(r.m);
        r.cv.wait(lk, [&] { return r.done; });
        return r.rc ? fail(r.rc, r.err) : HBEC_OK;
    }
};

extern "C" {

int hbec_batcher_new(hbec_codec* codec, uint64_t max_batch_bytes, uint32_t max_wait_us, hbec_batcher** out) {
    return hbec::guarded("hbec_batcher_new", [&]() -> int {
        if (!codec || !out) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        *out = nullptr;
        std::unique_ptr<hbec_batcher> b(new (std::nothrow) hbec_batcher());
        if (!b) return fail(HBEC_ERR_NOMEM, "batcher allocation");
        hipError_t e = hipGetDevice(&b->device);
        if (e != hipSuccess) return hbec::hip_fail(e, "hipGetDevice");
        b->codec = codec;
        b->max_batch_bytes = max_batch_bytes ? max_batch_bytes : (256ull << 20);
        b->max_wait = std::chrono::microseconds(max_wait_us);
        b->quiet = std::chrono::microseconds(std::max(1LL, hbec::tune_knob("HBEC_BATCHER_QUIET_US", 20)));
        const int n_workers = (int)std::min(8LL, std::max(1LL, hbec::env_knob("HBEC_BATCHER_WORKERS", 2)));
        b->md5_workers = (int)std::min(16LL, std::max(0LL, hbec::env_knob("HBEC_BATCHER_MD5_WORKERS", 4)));
        b->batch_cap = std::max<uint64_t>(1, b->max_batch_bytes / (uint64_t)n_workers);
        b->md5_cap = std::max<uint64_t>(1, b->max_batch_bytes / (uint64_t)std::max(1, b->md5_workers));
        hbec_batcher* raw = b.get();
        for (int w = 0; w < n_workers; ++w) b->workers.emplace_back([raw] { raw->run(false); });
        for (int w = 0; w < b->md5_workers; ++w) b->workers.emplace_back([raw] { raw->run(true); });
        *out = b.release();
        return HBEC_OK;
    });
}

void hbec_batcher_free(hbec_batcher* b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> g(b->mu);
        b->stop = true;
    }
    b->cv_work.notify_all();
    for (auto& w : b->workers) w.join();
    delete b;
}

int hbec_batcher_encode(hbec_batcher* b, const hbec_stripe* stripe) {
    return hbec::guarded("hbec_batcher_encode", [&]() -> int {
        if (!b || !stripe) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        if (stripe->shard_len == 0) return HBEC_OK;
        Request r;
        r.stripe = *stripe;
        r.op = 0;
        return b->submit(r);
    });
}

int hbec_batcher_encode_md5(hbec_batcher* b, const hbec_stripe* stripe, uint8_t* digests) {
    return hbec::guarded("hbec_batcher_encode_md5", [&]() -> int {
        if (!b || !stripe || !digests) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        if (stripe->shard_len == 0) return fail(HBEC_ERR_SHARD_NO_DATA, "stripe with zero shard length");
        Request r;
        r.stripe = *stripe;
        r.op = 2;
        r.digests = digests;
        return b->submit(r);
    });
}

int hbec_batcher_reconstruct(hbec_batcher* b, const hbec_stripe* stripe, const uint8_t* present, int data_only) {
    return hbec::guarded("hbec_batcher_reconstruct", [&]() -> int {
        if (!b || !stripe || !present) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        if (stripe->shard_len == 0) return HBEC_OK;
        const int n = hbec_data_shards(b->codec) + hbec_parity_shards(b->codec);
        Request r;
        r.stripe = *stripe;
        r.op = 1;
        r.present.assign(present, present + n);
        for (auto& v : r.present) v = v ? 1 : 0;
        r.data_only = data_only ? 1 : 0;
        return b->submit(r);
    });
}

int hbec_batcher_stats(hbec_batcher* b, uint64_t* batches, uint64_t* stripes) {
    return hbec::guarded("hbec_batcher_stats", [&]() -> int {
        if (!b) return fail(HBEC_ERR_INVALID_ARG, "null argument");
        std::lock_guard<std::mutex> g(b->mu);
        if (batches) *batches = b->batches;
        if (stripes) *stripes = b->stripes;
        return HBEC_OK;
    });
}

}  // extern "C"
