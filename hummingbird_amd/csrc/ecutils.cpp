// ecutils.cpp — the stripe loops of objectserver/ecutils.go over C io callbacks,
// with every GF step on the GPU codec (hbec_encode / hbec_reconstruct).
//
//   hbec_ec_shard_length  <- ecShardLength   ecutils.go:14-24
//   hbec_ec_split         <- ecSplit         ecutils.go:26-72
//   hbec_ec_split_md5     <- ecSplit + the receivers' ShardHash (indexdb.go:746-753)
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
#include <climits>
#include <cstdlib>
#include <cstring>
#include <memory>
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

// Device side of ecSplit with hashing: one stripe buffer (k+m shards) plus the
// digests, a private stream, and the per-shard MD5 chains.
struct DeviceStripe {
    hipStream_t stream = nullptr;
    uint8_t* buf = nullptr;
    hbec_md5* md5 = nullptr;
    ~DeviceStripe() {
        hbec_md5_free(md5);
        if (buf) hipFree(buf);
        if (stream) hipStreamDestroy(stream);
    }
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

}  // namespace

extern "C" {

int64_t hbec_ec_shard_length(int64_t length, int data_shards) {
    if (length < 0) return 0;
    if (data_shards <= 0) return 0;
    const int64_t shards = data_shards;
    int64_t s = length / shards;
    if (length % shards > 0) s += 1;
    return s;
}

static int ec_split(int k, int m, hbec_read_fn read, void* fp, int chunk_size, int64_t content_length,
                    hbec_write_fn write, void* const* writers, uint8_t* shard_md5) {
    CodecHolder enc;
    int rc = hbec_new(k, m, &enc.c);
    if (rc) return rc;
    if (!read || chunk_size < 0) return fail(HBEC_ERR_INVALID_ARG, "ecSplit: bad arguments");
    const int n = k + m;
    // databuf := make([]byte, (k+m)*chunkSize)   (ecutils.go:32)
    std::vector<uint8_t> databuf((size_t)n * (size_t)chunk_size);
    std::vector<uint8_t*> shards(n);
    std::vector<size_t> lens(n);
    std::vector<char> failed(n, 0);
    std::vector<hbec_view> views(n);
    DeviceStripe dev;
    if (shard_md5) {
        hipError_t e = hipStreamCreateWithFlags(&dev.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMalloc(&dev.buf, 16u * (size_t)n + databuf.size());  // digests, then stripe
        if (e != hipSuccess) return hbec::hip_fail(e, "ecSplit device buffers");
        rc = hbec_md5_new(n, 1, &dev.md5);
        if (rc) return rc;
    }
    int64_t total = 0;
    while (total < content_length) {
        int64_t expected = (int64_t)k * chunk_size;
        if (content_length - total < expected) expected = content_length - total;
        size_t got = 0;
        ReadStatus st = read_full(read, fp, databuf.data(), (size_t)expected, &got);
        if (st == READ_ERR) return fail(HBEC_ERR_IO, "ecSplit: read failed");
        if (st == READ_UNEXPECTED_EOF) return fail(HBEC_ERR_UNEXPECTED_EOF, "ecSplit: unexpected EOF");
        if (got == 0) return fail(HBEC_ERR_UNEXPECTED_EOF, "ecSplit: unexpected EOF");
        total += (int64_t)got;
        while (got % (size_t)k != 0) databuf[got++] = 0;  // zero pad (ecutils.go:51-54)
        const size_t s = got / (size_t)k;
        for (int i = 0; i < n; ++i) {
            shards[i] = databuf.data() + (size_t)i * s;
            lens[i] = s;
        }
        if (!shard_md5) {
            rc = hbec_encode(enc.c, shards.data(), lens.data(), n);
            if (rc) return rc;
        } else {  // stripe to the GPU, encode and hash there, parity back
            uint8_t* d_stripe = dev.buf + 16u * (size_t)n;
            for (int i = 0; i < n; ++i) views[i] = hbec_view{d_stripe + (size_t)i * s, 0};
            hipError_t e = hipMemcpyAsync(d_stripe, databuf.data(), (size_t)k * s, hipMemcpyHostToDevice, dev.stream);
            if (e != hipSuccess) return hbec::hip_fail(e, "ecSplit H2D");
            rc = hbec_encode_batch(enc.c, views.data(), 1, s, dev.stream);
            if (!rc) rc = hbec_md5_update(dev.md5, views.data(), s, dev.stream);
            if (rc) return rc;
            e = hipMemcpyAsync(shards[k], d_stripe + (size_t)k * s, (size_t)m * s, hipMemcpyDeviceToHost, dev.stream);
            if (e == hipSuccess) e = hipStreamSynchronize(dev.stream);
            if (e != hipSuccess) return hbec::hip_fail(e, "ecSplit D2H");
        }
        for (int i = 0; i < n; ++i) {
            if (writers && writers[i] && !failed[i]) {
                if (!write || write(writers[i], shards[i], s) != 0) failed[i] = 1;
            }
        }
    }
    if (shard_md5) {
        uint8_t* d_dig = dev.buf;
        rc = hbec_md5_final(dev.md5, d_dig, dev.stream);
        if (rc) return rc;
        hipError_t e = hipMemcpyAsync(shard_md5, d_dig, 16u * (size_t)n, hipMemcpyDeviceToHost, dev.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(dev.stream);
        if (e != hipSuccess) return hbec::hip_fail(e, "ecSplit digests");
    }
    return HBEC_OK;
}

int hbec_ec_split(int k, int m, hbec_read_fn read, void* fp, int chunk_size, int64_t content_length,
                  hbec_write_fn write, void* const* writers) {
    return ec_split(k, m, read, fp, chunk_size, content_length, write, writers, nullptr);
}

int hbec_ec_split_md5(int k, int m, hbec_read_fn read, void* fp, int chunk_size, int64_t content_length,
                      hbec_write_fn write, void* const* writers, uint8_t* shard_md5) {
    if (!shard_md5) return fail(HBEC_ERR_INVALID_ARG, "ecSplit: null digest buffer");
    return ec_split(k, m, read, fp, chunk_size, content_length, write, writers, shard_md5);
}

int hbec_ec_reconstruct(int k, int m, hbec_read_fn read, void* const* bodies, int chunk_size,
                        int64_t content_length, hbec_write_fn write, void* const* dsts, const int* dst_chunk_num,
                        int n_dsts) {
    CodecHolder enc;
    int rc = hbec_new(k, m, &enc.c);
    if (rc) return rc;
    const int n = k + m;
    if (!bodies || chunk_size < 0 || n_dsts < 0 || (n_dsts > 0 && (!dsts || !dst_chunk_num || !write)))
        return fail(HBEC_ERR_INVALID_ARG, "ecReconstruct: bad arguments");
    for (int i = 0; i < n_dsts; ++i)
        if (dst_chunk_num[i] < 0 || dst_chunk_num[i] >= n)
            return fail(HBEC_ERR_INVALID_ARG, "ecReconstruct: chunk number out of range");
    std::vector<uint8_t> databuf((size_t)n * (size_t)chunk_size);
    std::vector<uint8_t*> data(n);
    std::vector<size_t> lens(n);
    int64_t total = 0;
    while (total < content_length) {
        const int64_t exp = stripe_shard_size(k, chunk_size, content_length - total);
        if (exp <= 0) return fail(HBEC_ERR_INVALID_ARG, "ecReconstruct: chunk size is zero");
        for (int i = 0; i < n; ++i) {
            data[i] = databuf.data() + (size_t)i * (size_t)exp;
            lens[i] = bodies[i] ? (size_t)exp : 0;
        }
        for (int i = 0; i < n; ++i) {
            if (bodies[i]) {
                size_t got = 0;
                if (!read || read_full(read, bodies[i], data[i], (size_t)exp, &got) != READ_OK) lens[i] = 0;
            }
        }
        rc = hbec_reconstruct(enc.c, data.data(), lens.data(), n, 0);
        if (rc) return rc;
        for (int i = 0; i < n_dsts; ++i) {
            const int c = dst_chunk_num[i];
            if (write(dsts[i], data[c], lens[c]) != 0) return fail(HBEC_ERR_IO, "ecReconstruct: write failed");
        }
        for (int i = 0; i < k; ++i) {
            int64_t dl = (int64_t)lens[i];
            if (content_length - total < dl) dl = content_length - total;
            total += dl;
        }
    }
    return HBEC_OK;
}

int hbec_ec_glue(int k, int m, hbec_read_fn read, void* const* bodies, int chunk_size, int64_t content_length,
                 hbec_write_fn write, void* const* dsts, int n_dsts) {
    CodecHolder enc;
    int rc = hbec_new(k, m, &enc.c);
    if (rc) return rc;
    const int n = k + m;
    if (!bodies || chunk_size < 0 || n_dsts < 0 || (n_dsts > 0 && !dsts))
        return fail(HBEC_ERR_INVALID_ARG, "ecGlue: bad arguments");
    std::vector<void*> live(dsts, dsts + n_dsts);
    std::vector<uint8_t> databuf((size_t)n * (size_t)chunk_size);
    std::vector<uint8_t*> data(n);
    std::vector<size_t> lens(n);
    std::vector<char> failed(n, 0);
    int64_t written = 0;
    while (written < content_length) {
        const int64_t exp = stripe_shard_size(k, chunk_size, content_length - written);
        if (exp <= 0) return fail(HBEC_ERR_INVALID_ARG, "ecGlue: chunk size is zero");
        for (int i = 0; i < n; ++i) {
            data[i] = databuf.data() + (size_t)i * (size_t)exp;
            lens[i] = (bodies[i] && !failed[i]) ? (size_t)exp : 0;
        }
        for (int i = 0; i < n; ++i) {
            if (bodies[i] && !failed[i]) {
                size_t got = 0;
                if (!read || read_full(read, bodies[i], data[i], (size_t)exp, &got) != READ_OK) {
                    lens[i] = 0;
                    failed[i] = 1;
                }
            }
        }
        rc = hbec_reconstruct(enc.c, data.data(), lens.data(), n, 1);
        if (rc) return rc;
        for (int i = 0; i < k; ++i) {
            size_t len = lens[i];
            if (content_length - written < (int64_t)len) len = (size_t)(content_length - written);
            for (int j = 0; j < n_dsts; ++j) {
                if (live[j]) {
                    if (!write || write(live[j], data[i], len) != 0) live[j] = nullptr;
                }
            }
            written += (int64_t)len;
        }
    }
    return HBEC_OK;
}

int hbec_parse_ec_scheme(const char* scheme, char* algo, size_t algo_cap, int* data_shards, int* parity_shards,
                         int* chunk_size) {
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
    // strconv.Atoi: optional sign then one or more ASCII digits
    auto atoi_go = [](const std::string& s, int* out) {
        size_t i = 0;
        if (!s.empty() && (s[0] == '+' || s[0] == '-')) i = 1;
        if (i >= s.size()) return false;
        for (size_t j = i; j < s.size(); ++j)
            if (s[j] < '0' || s[j] > '9') return false;
        errno = 0;
        long long v = std::strtoll(s.c_str(), nullptr, 10);
        if (errno == ERANGE || v < INT_MIN || v > INT_MAX) return false;
        *out = (int)v;
        return true;
    };
    int k = 0, m = 0, c = 0;
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
