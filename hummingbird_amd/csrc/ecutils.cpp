// ecutils.cpp — the stripe loops of objectserver/ecutils.go over C io callbacks,
// with every GF step on the GPU, pipelined: stripe i+1 is read while stripe i
// is on the GPU (pinned two-slot ring, see Ring below).
//
//   hbec_ec_shard_length  <- ecShardLength   ecutils.go:14-24
//   hbec_ec_split         <- ecSplit         ecutils.go:26-72
//   hbec_ec_reconstruct   <- ecReconstruct   ecutils.go:74-132
//   hbec_ec_glue          <- ecGlue          ecutils.go:134-186
//   hbec_parse_ec_scheme  <- parseECScheme   ecobj.go:82-98
//   hbec_range_chunk_align<- rangeChunkAlign ecobj.go:814-824
//
// Byte semantics follow the Go line by line (zero-pad to a multiple of k,
// contiguous split, per-stripe shard size ceil(remaining/k) capped at chunk,
// truncation of the last stripe on glue).  Reference quirk kept: ecReconstruct
// never marks a body failed, so a body whose read fails is retried on the
// next stripe (ecutils.go:103-107).
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hbec.h"
#include "internal.h"

using hbec::fail;

namespace {

enum ReadStatus { READ_OK = 0, READ_EOF = 1, READ_UNEXPECTED_EOF = 2, READ_ERR = 3 };

// io.ReadFull: fill buf completely.  EOF only when nothing was read.
ReadStatus read_full(hbec_read_fn rd, void* ctx, uint8_t* buf, size_t n, size_t* got) {
    size_t have = 0;
    while (have < n) {
        int64_t r = rd(ctx, buf + have, n - have);
        if (r < 0) {
            *got = have;
            return READ_ERR;
        }
        if (r == 0) break;
        have += (size_t)r;
    }
    *got = have;
    if (have == n) return READ_OK;
    return have == 0 ? READ_EOF : READ_UNEXPECTED_EOF;
}

struct CodecHolder {
    hbec_codec* c = nullptr;
    ~CodecHolder() { hbec_free(c); }
};

// ecReconstruct / ecGlue per-stripe shard size (ecutils.go:86-92, :144-150)
int64_t stripe_shard_size(int k, int chunk, int64_t remaining) {
    int64_t s = chunk;
    if (remaining < (int64_t)chunk * k) {
        s = remaining / k;
        if (remaining % k != 0) ++s;
    }
    return s;
}


// ---------------------------------------------------------------------------
// Two-slot stripe ring: pinned host stripe buffers (the Go loops' databuf),
// device stripe buffers, one stream, one event per slot.  Pooled per device
// (the stripe loops run once per object; pinned allocation is expensive).
// The loops below read stripe i+1 from the callbacks while stripe i's H2D,
// kernel and D2H run, then write stripe i: GPU time hides under the I/O.
// Callers see the Go loop's write sequence; the one visible difference is
// that stripe i+1 is read before stripe i is written.
// ---------------------------------------------------------------------------
struct Ring {
    int dev = 0;
    size_t host_bytes = 0, dev_bytes = 0;
    hipStream_t stream = nullptr;
    uint8_t* host[2] = {nullptr, nullptr};
    uint8_t* dbuf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
};

std::mutex g_ring_mu;
std::vector<Ring*> g_rings;
constexpr size_t kMaxPooledRings = 8;

void ring_destroy(Ring* r) {
    for (int i = 0; i < 2; ++i) {
        if (r->host[i]) (void)hipHostFree(r->host[i]);
        if (r->dbuf[i]) (void)hipFree(r->dbuf[i]);
        if (r->ev[i]) (void)hipEventDestroy(r->ev[i]);
    }
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
}

int ring_acquire(size_t host_bytes, size_t dev_bytes, Ring** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hbec::hip_fail(e, "hipGetDevice");
    {
        std::lock_guard<std::mutex> g(g_ring_mu);
        for (size_t i = 0; i < g_rings.size(); ++i) {
            Ring* r = g_rings[i];
            if (r->dev == dev && r->host_bytes >= host_bytes && r->dev_bytes >= dev_bytes) {
                g_rings.erase(g_rings.begin() + (long)i);
                *out = r;
                return HBEC_OK;
            }
        }
    }
    std::unique_ptr<Ring> r(new (std::nothrow) Ring());
    if (!r) return fail(HBEC_ERR_NOMEM, "stripe ring");
    r->dev = dev;
    r->host_bytes = std::max<size_t>(host_bytes, 1);
    r->dev_bytes = std::max<size_t>(dev_bytes, 16);
    e = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
        e = hipHostMalloc(reinterpret_cast<void**>(&r->host[i]), r->host_bytes, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc(&r->dbuf[i], r->dev_bytes);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&r->ev[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        ring_destroy(r.release());
        return e == hipErrorOutOfMemory ? fail(HBEC_ERR_NOMEM, "stripe ring") : hbec::hip_fail(e, "stripe ring");
    }
    *out = r.release();
    return HBEC_OK;
}

void ring_release(Ring* r) {
    std::lock_guard<std::mutex> g(g_ring_mu);
    if (g_rings.size() >= kMaxPooledRings) {
        ring_destroy(g_rings.front());
        g_rings.erase(g_rings.begin());
    }
    g_rings.push_back(r);
}

struct RingHolder {
    Ring* r = nullptr;
    ~RingHolder() {
        if (r) {
            (void)hipStreamSynchronize(r->stream);  // nothing of ours still in flight
            ring_release(r);
        }
    }
};

uint64_t round16(uint64_t v) { return (v + 15) & ~uint64_t(15); }

// Device slot layout for a stripe of n shards of s bytes: shard i at i * pad,
// pad = s when 16-aligned (one contiguous copy each way), else round16(s)
// (per-shard copies; the vector kernels then run over pad bytes, whose tail
// is never copied back).
struct SlotLayout {
    uint64_t s = 0, pad = 0;
    bool contiguous() const { return pad == s; }
};

SlotLayout layout_for(uint64_t s) { return SlotLayout{s, (s % 16) == 0 ? s : round16(s)}; }

// H2D of shards [lo, hi) of a host stripe (shard i at host + i*s) into device
// slot b's layout.
hipError_t upload(const Ring& r, int b, const uint8_t* host, const SlotLayout& L, int lo, int hi) {
    if (hi <= lo) return hipSuccess;
    if (L.contiguous())
        return hipMemcpyAsync(r.dbuf[b] + (size_t)lo * L.s, host + (size_t)lo * L.s, (size_t)(hi - lo) * L.s,
                              hipMemcpyHostToDevice, r.stream);
    for (int i = lo; i < hi; ++i) {
        hipError_t e = hipMemcpyAsync(r.dbuf[b] + (size_t)i * L.pad, host + (size_t)i * L.s, L.s,
                                      hipMemcpyHostToDevice, r.stream);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t download(const Ring& r, int b, uint8_t* host, const SlotLayout& L, int i) {
    return hipMemcpyAsync(host + (size_t)i * L.s, r.dbuf[b] + (size_t)i * L.pad, L.s, hipMemcpyDeviceToHost,
                          r.stream);
}

// Host stripe buffers for the loops: pageable (Go's databuf) until the first
// stripe that needs the GPU acquires the ring, pinned ring buffers after that.
// So a healthy ecGlue never touches the GPU, and read errors come first, as
// in Go, even on a host without one.
struct HostBufs {
    size_t bytes = 0;
    std::vector<uint8_t> pageable[2];
    uint8_t* get(const Ring* r, int b) {
        if (r) return r->host[b];
        if (pageable[b].size() < bytes) pageable[b].resize(bytes);
        return pageable[b].data();
    }
};

void device_views(const Ring& r, int b, const SlotLayout& L, int n, std::vector<hbec_view>& v) {
    v.resize((size_t)n);
    for (int i = 0; i < n; ++i) v[i] = hbec_view{r.dbuf[b] + (size_t)i * L.pad, 0};
}

// Queue a reconstruct of one stripe in slot b: survivors up, rebuilt shards
// down.  present[i] = 1 for shards read.  Returns the shard indices written.
int queue_reconstruct(hbec_codec* c, const Ring& r, int b, uint8_t* host, const SlotLayout& L,
                      const std::vector<uint8_t>& present, int data_only, std::vector<int>& outputs) {
    const int k = hbec_data_shards(c), n = k + hbec_parity_shards(c);
    std::vector<int> surv((size_t)k), outs((size_t)n);
    std::vector<uint8_t> rows((size_t)n * k);
    int n_out = 0;
    int rc = hbec_decode_rows(c, present.data(), data_only, surv.data(), outs.data(), &n_out, rows.data());
    if (rc) return rc;
    outputs.assign(outs.begin(), outs.begin() + n_out);
    if (n_out == 0) return HBEC_OK;
    hipError_t e = hipSuccess;
    if (L.contiguous()) {
        e = upload(r, b, host, L, surv.front(), surv.back() + 1);  // one copy over the survivors' span
    } else {
        for (int j = 0; j < k && e == hipSuccess; ++j) e = upload(r, b, host, L, surv[j], surv[j] + 1);
    }
    if (e != hipSuccess) return hbec::hip_fail(e, "stripe upload");
    std::vector<hbec_view> v;
    device_views(r, b, L, n, v);
    rc = hbec_reconstruct_batch(c, v.data(), present.data(), 1, L.pad, data_only, r.stream);
    if (rc) return rc;
    for (int o : outputs) {
        e = download(r, b, host, L, o);
        if (e != hipSuccess) return hbec::hip_fail(e, "stripe download");
    }
    e = hipEventRecord(r.ev[b], r.stream);
    if (e != hipSuccess) return hbec::hip_fail(e, "hipEventRecord");
    return HBEC_OK;
}

int wait_slot(const Ring& r, int b) {
    hipError_t e = hipEventSynchronize(r.ev[b]);
    if (e != hipSuccess) return hbec::hip_fail(e, "stripe wait");
    return HBEC_OK;
}

}  // namespace

extern "C" {

int64_t hbec_ec_shard_length(int64_t length, int64_t data_shards) {
    if (length < 0) return 0;
    if (data_shards <= 0) return 0;
    const int64_t shards = data_shards;
    int64_t s = length / shards;
    if (length % shards > 0) s += 1;
    return s;
}

// ecSplit (ecutils.go:26-72).
int hbec_ec_split(int k, int m, hbec_read_fn read, void* fp, int chunk_size, int64_t content_length,
                  hbec_write_fn write, void* const* writers) {
    return hbec::guarded("hbec_ec_split", [&]() -> int {
        CodecHolder enc;
        int rc = hbec_new(k, m, &enc.c);
        if (rc) return rc;
        if (!read || chunk_size < 0) return fail(HBEC_ERR_INVALID_ARG, "ecSplit: bad arguments");
        const int n = k + m;
        std::vector<char> failed(n, 0);
        struct Pending {
            bool live = false;
            uint8_t* host = nullptr;
            uint64_t s = 0;
        } pend[2];
        RingHolder ring;
        HostBufs bufs;
        bufs.bytes = (size_t)n * (size_t)chunk_size;  // databuf := make([]byte, (k+m)*chunkSize)  (ecutils.go:32)
        auto ensure_ring = [&]() -> int {
            if (ring.r) return HBEC_OK;
            return ring_acquire(bufs.bytes, (size_t)n * round16((uint64_t)chunk_size), &ring.r);
        };
        // write one finished stripe (ecutils.go:62-69): a failing writer is dropped
        auto flush = [&](int b) -> int {
            if (!pend[b].live) return HBEC_OK;
            pend[b].live = false;
            int r2 = wait_slot(*ring.r, b);
            if (r2) return r2;
            const uint64_t s = pend[b].s;
            for (int i = 0; i < n; ++i)
                if (writers && writers[i] && !failed[i])
                    if (!write || write(writers[i], pend[b].host + (size_t)i * s, s) != 0) failed[i] = 1;
            return HBEC_OK;
        };
        int64_t total = 0;
        int b = 0;
        std::vector<hbec_view> v;
        while (total < content_length) {
            uint8_t* databuf = bufs.get(ring.r, b);
            int64_t expected = (int64_t)k * chunk_size;
            if (content_length - total < expected) expected = content_length - total;
            size_t got = 0;
            ReadStatus st = read_full(read, fp, databuf, (size_t)expected, &got);
            if (st == READ_ERR || st == READ_UNEXPECTED_EOF || got == 0) {
                const int r2 = flush(b ^ 1);  // the Go loop wrote the previous stripe before this read
                if (r2) return r2;
                if (st == READ_ERR) return fail(HBEC_ERR_IO, "ecSplit: read failed");
                return fail(HBEC_ERR_UNEXPECTED_EOF, "ecSplit: unexpected EOF");
            }
            total += (int64_t)got;
            while (got % (size_t)k != 0) databuf[got++] = 0;  // zero pad (ecutils.go:51-54)
            rc = ensure_ring();
            if (rc) return rc;
            const SlotLayout L = layout_for(got / (size_t)k);
            hipError_t e = upload(*ring.r, b, databuf, L, 0, k);
            if (e != hipSuccess) return hbec::hip_fail(e, "ecSplit upload");
            device_views(*ring.r, b, L, n, v);
            rc = hbec_encode_batch(enc.c, v.data(), 1, L.pad, ring.r->stream);
            if (rc) return rc;
            if (L.contiguous()) {
                e = hipMemcpyAsync(databuf + (size_t)k * L.s, ring.r->dbuf[b] + (size_t)k * L.s, (size_t)m * L.s,
                                   hipMemcpyDeviceToHost, ring.r->stream);
            } else {
                for (int r = 0; r < m && e == hipSuccess; ++r) e = download(*ring.r, b, databuf, L, k + r);
            }
            if (e == hipSuccess) e = hipEventRecord(ring.r->ev[b], ring.r->stream);
            if (e != hipSuccess) return hbec::hip_fail(e, "ecSplit download");
            pend[b] = Pending{true, databuf, L.s};
            rc = flush(b ^ 1);  // previous stripe: write it while this one is on the GPU
            if (rc) return rc;
            b ^= 1;
        }
        return flush(b ^ 1);
    });
}

// ecReconstruct (ecutils.go:74-132).
int hbec_ec_reconstruct(int k, int m, hbec_read_fn read, void* const* bodies, int chunk_size,
                        int64_t content_length, hbec_write_fn write, void* const* dsts, const int* dst_chunk_num,
                        int n_dsts) {
    return hbec::guarded("hbec_ec_reconstruct", [&]() -> int {
        CodecHolder enc;
        int rc = hbec_new(k, m, &enc.c);
        if (rc) return rc;
        const int n = k + m;
        if (!bodies || chunk_size < 0 || n_dsts < 0 || (n_dsts > 0 && (!dsts || !dst_chunk_num || !write)))
            return fail(HBEC_ERR_INVALID_ARG, "ecReconstruct: bad arguments");
        for (int i = 0; i < n_dsts; ++i)
            if (dst_chunk_num[i] < 0 || dst_chunk_num[i] >= n)
                return fail(HBEC_ERR_INVALID_ARG, "ecReconstruct: chunk number out of range");
        struct Pending {
            bool live = false, gpu = false;
            uint8_t* host = nullptr;
            uint64_t s = 0;
        } pend[2];
        RingHolder ring;
        HostBufs bufs;
        bufs.bytes = (size_t)n * (size_t)chunk_size;
        auto flush = [&](int b) -> int {
            if (!pend[b].live) return HBEC_OK;
            pend[b].live = false;
            if (pend[b].gpu) {
                int r2 = wait_slot(*ring.r, b);
                if (r2) return r2;
            }
            const uint64_t s = pend[b].s;
            for (int i = 0; i < n_dsts; ++i)  // ecutils.go:115-120
                if (write(dsts[i], pend[b].host + (size_t)dst_chunk_num[i] * s, s) != 0)
                    return fail(HBEC_ERR_IO, "ecReconstruct: write failed");
            return HBEC_OK;
        };
        std::vector<uint8_t> present((size_t)n);
        std::vector<int> outputs;
        int64_t total = 0;
        int b = 0;
        while (total < content_length) {
            const int64_t exp = stripe_shard_size(k, chunk_size, content_length - total);
            if (exp <= 0) return fail(HBEC_ERR_INVALID_ARG, "ecReconstruct: chunk size is zero");
            uint8_t* databuf = bufs.get(ring.r, b);
            int n_present = 0;
            for (int i = 0; i < n; ++i) {  // a failed read is missing for this stripe only (ecutils.go:103-109)
                present[i] = 0;
                if (bodies[i]) {
                    size_t got = 0;
                    if (read && read_full(read, bodies[i], databuf + (size_t)i * exp, (size_t)exp, &got) == READ_OK)
                        present[i] = 1;
                }
                n_present += present[i];
            }
            const SlotLayout L = layout_for((uint64_t)exp);
            bool gpu = false;
            if (n_present < n) {  // Reconstruct (ecutils.go:111) is a no-op when nothing is missing
                // klauspost's checkShards runs before the count: a stripe with
                // no shard at all is ErrShardNoData, not ErrTooFewShards
                if (n_present == 0) rc = fail(HBEC_ERR_SHARD_NO_DATA, "no shard data");
                if (!rc && !ring.r) rc = ring_acquire(bufs.bytes, (size_t)n * round16((uint64_t)chunk_size), &ring.r);
                if (!rc) rc = queue_reconstruct(enc.c, *ring.r, b, databuf, L, present, 0, outputs);
                if (rc) {
                    const int r2 = flush(b ^ 1);
                    return r2 ? r2 : rc;
                }
                gpu = !outputs.empty();
            }
            pend[b] = Pending{true, gpu, databuf, L.s};
            for (int i = 0; i < k; ++i) {  // every data shard now has exp bytes
                int64_t dl = exp;
                if (content_length - total < dl) dl = content_length - total;
                total += dl;
            }
            rc = flush(b ^ 1);
            if (rc) return rc;
            b ^= 1;
        }
        return flush(b ^ 1);
    });
}

// ecGlue (ecutils.go:134-186): healthy stripes never touch the GPU.
int hbec_ec_glue(int k, int m, hbec_read_fn read, void* const* bodies, int chunk_size, int64_t content_length,
                 hbec_write_fn write, void* const* dsts, int n_dsts) {
    return hbec::guarded("hbec_ec_glue", [&]() -> int {
        CodecHolder enc;
        int rc = hbec_new(k, m, &enc.c);
        if (rc) return rc;
        const int n = k + m;
        if (!bodies || chunk_size < 0 || n_dsts < 0 || (n_dsts > 0 && !dsts))
            return fail(HBEC_ERR_INVALID_ARG, "ecGlue: bad arguments");
        std::vector<void*> live(dsts, dsts + n_dsts);
        std::vector<char> failed(n, 0);
        struct Pending {
            bool live = false, gpu = false;
            uint8_t* host = nullptr;
            uint64_t s = 0;
            int64_t remaining = 0;  // object bytes left when this stripe was read
        } pend[2];
        RingHolder ring;
        HostBufs bufs;
        bufs.bytes = (size_t)n * (size_t)chunk_size;
        auto flush = [&](int b) -> int {
            if (!pend[b].live) return HBEC_OK;
            pend[b].live = false;
            if (pend[b].gpu) {
                int r2 = wait_slot(*ring.r, b);
                if (r2) return r2;
            }
            const uint64_t s = pend[b].s;
            int64_t remaining = pend[b].remaining;
            for (int i = 0; i < k; ++i) {  // data shards, the last truncated (ecutils.go:171-183)
                size_t len = (size_t)s;
                if (remaining < (int64_t)len) len = (size_t)remaining;
                for (int j = 0; j < n_dsts; ++j)
                    if (live[j] && (!write || write(live[j], pend[b].host + (size_t)i * s, len) != 0)) live[j] = nullptr;
                remaining -= (int64_t)len;
            }
            return HBEC_OK;
        };
        std::vector<uint8_t> present((size_t)n);
        std::vector<int> outputs;
        int64_t written = 0;
        int b = 0;
        while (written < content_length) {
            const int64_t exp = stripe_shard_size(k, chunk_size, content_length - written);
            if (exp <= 0) return fail(HBEC_ERR_INVALID_ARG, "ecGlue: chunk size is zero");
            uint8_t* databuf = bufs.get(ring.r, b);
            bool data_missing = false;
            int n_present = 0;
            for (int i = 0; i < n; ++i) {  // a failed body stays failed (ecutils.go:152-163)
                present[i] = 0;
                if (bodies[i] && !failed[i]) {
                    size_t got = 0;
                    if (read && read_full(read, bodies[i], databuf + (size_t)i * exp, (size_t)exp, &got) == READ_OK)
                        present[i] = 1;
                    else
                        failed[i] = 1;
                }
                if (i < k && !present[i]) data_missing = true;
                n_present += present[i];
            }
            const SlotLayout L = layout_for((uint64_t)exp);
            bool gpu = false;
            if (data_missing) {  // ReconstructData (ecutils.go:168)
                if (n_present == 0) rc = fail(HBEC_ERR_SHARD_NO_DATA, "no shard data");  // checkShards first
                if (!rc && !ring.r) rc = ring_acquire(bufs.bytes, (size_t)n * round16((uint64_t)chunk_size), &ring.r);
                if (!rc) rc = queue_reconstruct(enc.c, *ring.r, b, databuf, L, present, 1, outputs);
                if (rc) {
                    const int r2 = flush(b ^ 1);
                    return r2 ? r2 : rc;
                }
                gpu = !outputs.empty();
            }
            pend[b].live = true;
            pend[b].gpu = gpu;
            pend[b].host = databuf;
            pend[b].s = L.s;
            pend[b].remaining = content_length - written;
            for (int i = 0; i < k; ++i) {
                int64_t len = exp;
                if (content_length - written < len) len = content_length - written;
                written += len;
            }
            rc = flush(b ^ 1);
            if (rc) return rc;
            b ^= 1;
        }
        return flush(b ^ 1);
    });
}

namespace {
// rangeBytesWriter (ecobj.go:826-850): passes on the bytes after the first
// start_offset, up to `length` of them, and reports every write as whole.
struct RangeWriter {
    hbec_write_fn write;
    void* ctx;
    int64_t start_offset, length;
};

int range_write(void* c, const uint8_t* buf, size_t n) {
    RangeWriter& r = *static_cast<RangeWriter*>(c);
    if (r.start_offset > (int64_t)n) {
        r.start_offset -= (int64_t)n;
        return 0;
    }
    if (r.length <= 0) return 0;
    buf += r.start_offset;
    n -= (size_t)r.start_offset;
    r.start_offset = 0;
    if ((int64_t)n > r.length) n = (size_t)r.length;
    r.length -= (int64_t)n;
    return n ? r.write(r.ctx, buf, n) : 0;
}
}  // namespace

int hbec_ec_glue_range(int k, int m, hbec_read_fn read, void* const* bodies, int chunk_size, int64_t content_length,
                       int64_t start, int64_t end, hbec_write_fn write, void* const* dsts, int n_dsts) {
    return hbec::guarded("hbec_ec_glue_range", [&]() -> int {
        if (k <= 0 || chunk_size <= 0 || n_dsts < 0 || (n_dsts > 0 && !dsts))
            return fail(HBEC_ERR_INVALID_ARG, "ecGlue range: bad arguments");
        if (start < 0 || end < start || end > content_length)
            return fail(HBEC_ERR_INVALID_ARG, "ecGlue range: need 0 <= start <= end <= content length");
        if (start == end) return HBEC_OK;
        // object bytes of the covered stripes: [obj0, obj1)
        const int64_t stripe = (int64_t)k * chunk_size;
        const int64_t obj0 = start / stripe * stripe;
        const int64_t obj1 = std::min<int64_t>(content_length, (end + stripe - 1) / stripe * stripe);
        std::vector<RangeWriter> rw((size_t)n_dsts);
        std::vector<void*> ctx((size_t)n_dsts, nullptr);
        for (int j = 0; j < n_dsts; ++j) {
            rw[j] = RangeWriter{write, dsts[j], start - obj0, end - start};
            if (dsts[j]) ctx[j] = &rw[j];  // nil stays nil
        }
        return hbec_ec_glue(k, m, read, bodies, chunk_size, obj1 - obj0, write ? range_write : nullptr,
                            ctx.data(), n_dsts);
    });
}

// ecObject.CopyRange's decode exactly as the reference computes it
// (ecobj.go:238-265): glue rangeChunkAlign's shard-byte span (shardEnd capped
// at the object's content length) as if it were the content length, and pass
// the glue through a rangeBytesWriter that starts at start % chunk_size.
int hbec_ec_copy_range(int k, int m, hbec_read_fn read, void* const* bodies, int chunk_size, int64_t content_length,
                       int64_t start, int64_t end, hbec_write_fn write, void* const* dsts, int n_dsts) {
    return hbec::guarded("hbec_ec_copy_range", [&]() -> int {
        if (k <= 0 || chunk_size <= 0 || n_dsts < 0 || (n_dsts > 0 && !dsts))
            return fail(HBEC_ERR_INVALID_ARG, "CopyRange: bad arguments");
        // Go's rangeBytesWriter would panic on b[negative:] (ecobj.go:826-850);
        // here a negative start or an inverted range is refused before any read
        if (start < 0 || end < start) return fail(HBEC_ERR_INVALID_ARG, "CopyRange: need 0 <= start <= end");
        int64_t shard_start = 0, shard_end = 0;
        hbec_range_chunk_align(start, end, chunk_size, k, &shard_start, &shard_end);
        if (shard_end > content_length) shard_end = content_length;
        std::vector<RangeWriter> rw((size_t)n_dsts);
        std::vector<void*> ctx((size_t)n_dsts, nullptr);
        for (int j = 0; j < n_dsts; ++j) {
            // Go's % truncates toward zero, as C++'s does
            rw[j] = RangeWriter{write, dsts[j], start % (int64_t)chunk_size, end - start};
            if (dsts[j]) ctx[j] = &rw[j];
        }
        if (shard_end - shard_start <= 0) return HBEC_OK;  // ecGlue's loop does not run
        return hbec_ec_glue(k, m, read, bodies, chunk_size, shard_end - shard_start, write ? range_write : nullptr,
                            ctx.data(), n_dsts);
    });
}

int hbec_parse_ec_scheme(const char* scheme, char* algo, size_t algo_cap, int64_t* data_shards,
                         int64_t* parity_shards, int64_t* chunk_size) {
    return hbec::guarded("hbec_parse_ec_scheme", [&]() -> int {
        if (!scheme) return fail(HBEC_ERR_INVALID_ARG, "scheme is NULL");
        std::vector<std::string> sec;
        std::string cur;
        for (const char* p = scheme; *p; ++p) {
            if (*p == '/') {
                sec.push_back(cur);
                cur.clear();
            } else {
                cur.push_back(*p);
            }
        }
        sec.push_back(cur);
        if (sec.size() != 4) return fail(HBEC_ERR_SCHEME, std::to_string(sec.size()) + " scheme sections");
        // strconv.Atoi: optional sign then one or more ASCII digits, into Go's
        // int (64-bit on the reference's amd64 build), ErrRange beyond it
        auto atoi_go = [](const std::string& s, int64_t* out) {
            size_t i = 0;
            if (!s.empty() && (s[0] == '+' || s[0] == '-')) i = 1;
            if (i >= s.size()) return false;
            for (size_t j = i; j < s.size(); ++j)
                if (s[j] < '0' || s[j] > '9') return false;
            errno = 0;
            long long v = std::strtoll(s.c_str(), nullptr, 10);
            if (errno == ERANGE) return false;
            *out = (int64_t)v;
            return true;
        };
        int64_t k = 0, m = 0, c = 0;
        if (!atoi_go(sec[1], &k)) return fail(HBEC_ERR_SCHEME, "Invalid data shard count");
        if (!atoi_go(sec[2], &m)) return fail(HBEC_ERR_SCHEME, "Invalid parity shard count");
        if (!atoi_go(sec[3], &c)) return fail(HBEC_ERR_SCHEME, "Invalid chunk size");
        if (algo) {
            if (algo_cap < sec[0].size() + 1) return fail(HBEC_ERR_INVALID_ARG, "algo buffer too small");
            std::memcpy(algo, sec[0].c_str(), sec[0].size() + 1);
        }
        if (data_shards) *data_shards = k;
        if (parity_shards) *parity_shards = m;
        if (chunk_size) *chunk_size = c;
        return HBEC_OK;
    });
}

void hbec_range_chunk_align(int64_t start, int64_t end, int64_t chunk_size, int data_shards, int64_t* out_start,
                            int64_t* out_end) {
    const int64_t stripe = chunk_size * (int64_t)data_shards;
    if (stripe == 0) {
        if (out_start) *out_start = 0;
        if (out_end) *out_end = 0;
        return;
    }
    const int64_t start_chunk = start / stripe;
    const int64_t end_chunk = end / stripe;
    start = start_chunk * chunk_size;
    if (end % stripe == 0)
        end = end_chunk * chunk_size;
    else
        end = (end_chunk + 1) * chunk_size;
    if (out_start) *out_start = start;
    if (out_end) *out_end = end;
}

}  // extern "C"
