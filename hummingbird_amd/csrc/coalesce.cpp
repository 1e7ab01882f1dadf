// coalesce.cpp — group commit for the per-call Encode / Reconstruct /
// ReconstructData entry points (the plain drop-in of INTEGRATION.md §2-3).
//
// In the reference every Stabilize / degraded GET / repair goroutine calls
// klauspost on its own one-stripe databuf (objectserver/ecutils.go:59,111,168;
// nursery concurrency x devices, replicator.go:487,530, plus per-request
// goroutines).  On the GPU one 1 MiB stripe per call is bound by launch and
// PCIe latency, so concurrent calls are coalesced here, inside the library,
// with no deadline and no extra thread.  Up to HBEC_COALESCE_DIRECT
// concurrent callers each run at once through the per-call path (their
// zero-copy launches overlap on the GPU), so latency at low concurrency is
// unchanged.  Beyond that, a call that finds fewer than max_in_flight()
// groups running leads — it takes every queued call with the same (device,
// codec, op, erasure pattern) and codes them all with ONE host-path call
// (hostpath.cpp: zero-copy for pinned databufs) — while calls that arrive
// meanwhile queue and form the next group.
// If a group's batched call fails, each member is retried alone so every
// caller gets its own result.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/hbec.h"
#include "internal.h"

namespace hbec {

namespace {

struct CoReq {
    hbec_codec* codec = nullptr;
    int dev = 0;
    int op = 0;  // 0 encode, 1 reconstruct
    uint8_t* base = nullptr;
    uint64_t s = 0;
    std::vector<uint8_t> present;
    int data_only = 0;
    int rc = HBEC_OK;
    std::string err;
    bool taken = false, done = false, lead = false;
    CoReq* next = nullptr;       // group membership as an intrusive list: forming a group allocates nothing
    std::condition_variable cv;  // this caller's own wake-up: done, or asked to lead

    bool same_group(const CoReq& o) const {
        return codec == o.codec && dev == o.dev && op == o.op && data_only == o.data_only && present == o.present;
    }
};

// Groups coded at once (HBEC_COALESCE_INFLIGHT, default 2): below this many
// concurrent callers every call still runs at once, as if uncoalesced.  A
// call that is handed a slot but was already taken into another group passes
// the slot on, so at most this many groups ever run.
int max_in_flight() {
    static const int v = [] {
        const int x = (int)hbec::tune_knob("HBEC_COALESCE_INFLIGHT", 0);
        return x > 0 ? x : 2;
    }();
    return v;
}

// Below this many pinned calls inside the library at once (counting the new
// one), a call runs alone at once (HBEC_COALESCE_DIRECT, default 16): up to
// ~16 callers, independent zero-copy launches overlap on the GPU and beat
// grouping (1 MiB: 35 vs 25-29 GiB/s at 16 callers); from ~64 callers,
// grouping wins (38-42 vs 35 GiB/s) (profiles/r02_coalesce_direct.jsonl).
int direct_limit() {
    static const int v = (int)std::max(0LL, hbec::tune_knob("HBEC_COALESCE_DIRECT", 16));
    return v;
}

struct Coalescer {
    std::mutex mu;
    int inside = 0;  // pinned calls between entry and return
    std::deque<CoReq*> q;
    int leaders = 0;  // calls holding a lead slot: coding a group, or woken to form one
    uint64_t groups = 0, calls = 0;
};

Coalescer g_co;

uint64_t group_cap_bytes() {
    static const uint64_t cap = [] {
        const long long v = hbec::tune_knob("HBEC_COALESCE_MB", 0);
        return (uint64_t)(v > 0 ? v : 256) << 20;
    }();
    return cap;
}

// Code one group (list from `head`, n members).  Direct per-call path for a
// group of one; else one batched host-path call, falling back to per-member
// calls if that fails.
void run_group(CoReq* head, size_t n, const DirectFns& fn) {
    auto single = [&](CoReq* r) {
        r->rc = r->op == 0 ? fn.encode(r->codec, r->base, r->s)
                           : fn.reconstruct(r->codec, r->base, r->s, r->present.data(), r->data_only);
        r->err = r->rc ? hbec_last_error() : "";
    };
    if (n == 1) {
        single(head);
        return;
    }
    std::vector<hbec_stripe> st;
    st.reserve(n);
    for (CoReq* x = head; x; x = x->next) st.push_back(hbec_stripe{x->base, x->s});
    const CoReq& h = *head;
    const int rc = h.op == 0 ? hbec_encode_host(h.codec, st.data(), st.size())
                             : hbec_reconstruct_host(h.codec, st.data(), st.size(), h.present.data(), h.data_only);
    for (CoReq* x = head; x; x = x->next) {
        if (rc == HBEC_OK)
            x->rc = HBEC_OK;
        else
            single(x);
    }
}

// A whole group failed by exception: every member gets the code (the message
// is best effort — assigning it may itself fail to allocate).
void fail_group(CoReq* head, int code, const char* msg) noexcept {
    for (CoReq* x = head; x; x = x->next) {
        x->rc = code;
        try {
            x->err = msg;
        } catch (...) {
        }
    }
}

}  // namespace

bool coalesce_enabled() {
    static const bool on = hbec::env_knob("HBEC_COALESCE", 1) != 0;
    return on;
}

int coalesced_call(hbec_codec* codec, int op, uint8_t* base, uint64_t s, const uint8_t* present, int n_shards,
                   int data_only, const DirectFns& fn) {
    CoReq r;
    r.codec = codec;
    r.op = op;
    r.base = base;
    r.s = s;
    r.data_only = data_only ? 1 : 0;
    if (op == 1) {
        r.present.assign(present, present + n_shards);
        for (auto& v : r.present) v = v ? 1 : 0;
    }
    hipError_t e = hipGetDevice(&r.dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    // Only stripes the GPU can code in place (pinned, device-mapped; 16-B
    // aligned, or any alignment through the unaligned kernel) are grouped: a
    // group of those is ONE zero-copy launch (per alignment class) with no
    // CPU copy.  Pageable stripes take the per-call path, whose bounce-buffer
    // copies then run in parallel on the callers' own threads — 64 concurrent
    // callers reach 30 GiB/s that way vs 9 GiB/s funnelled through one
    // leader's staging ring (profiles/r02_percall.jsonl).
    const bool aligned = (reinterpret_cast<uintptr_t>(base) & 15u) == 0 && s % 16 == 0;
    const bool pinned = (aligned || zero_copy_any_alignment()) && pinned_device_addr(base, s * (uint64_t)n_shards) != 0;
    if (!pinned) return op == 0 ? fn.encode(codec, base, s) : fn.reconstruct(codec, base, s, present, data_only);
    const uint64_t cap = group_cap_bytes();
    std::unique_lock<std::mutex> lk(g_co.mu);
    if (++g_co.inside <= direct_limit()) {  // few callers: run alone, now (a group of one)
        ++g_co.groups;
        ++g_co.calls;
        lk.unlock();
        int rc = HBEC_OK;
        try {
            rc = op == 0 ? fn.encode(codec, base, s) : fn.reconstruct(codec, base, s, present, data_only);
        } catch (...) {
            lk.lock();
            --g_co.inside;
            throw;  // guarded() at the entry point maps it
        }
        lk.lock();
        --g_co.inside;
        return rc;
    }
    struct Leave {  // leaves the count on every way out of the queued path
        std::unique_lock<std::mutex>& lk;
        ~Leave() {
            if (!lk.owns_lock()) lk.lock();
            --g_co.inside;
        }
    } leave{lk};
    g_co.q.push_back(&r);
    // Every wake-up is addressed: a finished group wakes its own members, and
    // hands its lead slot to the oldest queued call.  (One shared condition
    // variable woke all ~128 waiters per group and ran 4 KiB stripes at
    // 42 k calls/s.)
    auto pass_slot = [&] {
        for (CoReq* x : g_co.q)  // every queued call is untaken
            if (!x->lead) {
                x->lead = true;
                x->cv.notify_one();
                return;
            }
        --g_co.leaders;
    };
    if (g_co.leaders < max_in_flight()) {
        ++g_co.leaders;
        r.lead = true;
    }
    for (;;) {
        r.cv.wait(lk, [&] { return r.done || r.lead; });
        if (r.lead) {
            r.lead = false;
            if (r.taken) {  // another leader's group took this call first
                pass_slot();
            } else {
                // lead: this call plus every queued call of the same group, up
                // to cap bytes (nothing below allocates while members are marked)
                CoReq* head = nullptr;
                CoReq** tail = &head;
                size_t members = 0;
                uint64_t bytes = 0;
                for (CoReq* x : g_co.q) {
                    if (!(x == &r || x->same_group(r))) continue;
                    const uint64_t b = x->s * (uint64_t)n_shards;
                    if (x != &r && bytes + b > cap) continue;
                    x->taken = true;
                    x->next = nullptr;
                    *tail = x;
                    tail = &x->next;
                    ++members;
                    bytes += b;
                }
                g_co.q.erase(std::remove_if(g_co.q.begin(), g_co.q.end(), [](CoReq* x) { return x->taken; }),
                             g_co.q.end());
                ++g_co.groups;
                g_co.calls += members;
                lk.unlock();
                // no exception may leave the group half-done: the other
                // members would wait forever
                try {
                    run_group(head, members, fn);
                } catch (const std::bad_alloc&) {
                    fail_group(head, HBEC_ERR_NOMEM, "coalesced call: host allocation failed");
                } catch (...) {
                    fail_group(head, HBEC_ERR_DEVICE, "coalesced call: unexpected exception");
                }
                lk.lock();
                for (CoReq* x = head; x;) {
                    CoReq* nx = x->next;  // read before `done`: a woken member may return at once
                    x->done = true;
                    if (x != &r) x->cv.notify_one();
                    x = nx;
                }
                pass_slot();
            }
        }
        if (r.done) break;
    }
    return r.rc ? fail(r.rc, r.err) : HBEC_OK;
}

void coalesce_stats(uint64_t* groups, uint64_t* calls) {
    std::lock_guard<std::mutex> g(g_co.mu);
    if (groups) *groups = g_co.groups;
    if (calls) *calls = g_co.calls;
}

}  // namespace hbec
