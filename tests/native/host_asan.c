/* Host-side sanitizer driver (ASan/UBSan on the CPU path).
 *
 * Linked against an AddressSanitizer + UBSan build of libhbec's HOST code
 * (device code is not instrumented: -fsanitize sits behind -Xarch_host, see
 * hummingbird_amd/build.py build_asan).  Exercises the host-memory machinery
 * where an overrun would hide: the staging ring's column pieces and chunking,
 * the zero-copy registry, the multi-device split, the batcher's queue, the
 * per-call staging, and the ecutils stripe loops over callbacks.  Correctness
 * is checked by round trips (encode -> erase -> reconstruct == original) and
 * Verify, so no oracle is linked.
 *
 *   host_asan        host-only entry points (no GPU needed)
 *   host_asan gpu    plus the host paths above on the GPU
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hbec.h"

#define CHECK(cond, code)                                                                   \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            fprintf(stderr, "FAIL %d at line %d: %s\n", code, __LINE__, hbec_last_error()); \
            return code;                                                                    \
        }                                                                                   \
    } while (0)

static uint64_t g_rng = 0x48424543u;
static uint8_t rnd8(void) {
    g_rng = g_rng * 6364136223846793005ull + 1442695040888963407ull;
    return (uint8_t)(g_rng >> 56);
}

static int cpu_part(void) {
    hbec_codec* c = NULL;
    CHECK(hbec_new(8, 3, &c) == HBEC_OK, 1);
    uint8_t m[11 * 8];
    CHECK(hbec_matrix(c, m) == HBEC_OK, 2);
    uint8_t present[11] = {0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1};
    int surv[8], outs[11], nout = 0;
    uint8_t rows[11 * 8];
    CHECK(hbec_decode_rows(c, present, 0, surv, outs, &nout, rows) == HBEC_OK && nout == 3, 3);
    /* validation paths must not touch memory they were not given */
    uint8_t* shards[11] = {0};
    size_t lens[11] = {0};
    CHECK(hbec_encode(c, shards, lens, 11) == HBEC_ERR_SHARD_NO_DATA, 4);
    CHECK(hbec_encode(c, shards, lens, 5) == HBEC_ERR_TOO_FEW_SHARDS, 5);
    hbec_free(c);
    char algo[4];
    int64_t k, p, chunk;
    const int rc = hbec_parse_ec_scheme("reedsolomon/4/2/1048576", algo, sizeof algo, &k, &p, &chunk);
    CHECK(rc != HBEC_OK || strlen(algo) < sizeof algo, 6); /* short buffer: rejected or truncated */
    CHECK(hbec_parse_ec_scheme("reedsolomon/4/2/x", algo, sizeof algo, &k, &p, &chunk) == HBEC_ERR_SCHEME, 7);
    int64_t s, e;
    hbec_range_chunk_align(61, 80, 10, 2, &s, &e);
    CHECK(s == 30 && e == 40, 8);
    CHECK(hbec_ec_shard_length(1007, 10) == 101, 9);
    printf("host_asan cpu ok\n");
    return 0;
}

/* ---- GPU part ---------------------------------------------------------- */

static uint8_t* make_stripe(int k, int m, uint64_t s, void* mem) {
    uint8_t* b = mem ? (uint8_t*)mem : (uint8_t*)malloc((size_t)(k + m) * s);
    for (uint64_t i = 0; i < (uint64_t)k * s; ++i) b[i] = rnd8();
    memset(b + (size_t)k * s, 0, (size_t)m * s);
    return b;
}

/* encode, keep a copy, erase shard 0 and the first parity shard, reconstruct, compare */
static int stripes_roundtrip(hbec_codec* c, int k, int m, hbec_stripe* st, uint64_t n, const int* devices,
                             int n_devices) {
    const int n_sh = k + m;
    int rc = devices ? hbec_encode_host_devices(c, st, n, devices, n_devices) : hbec_encode_host(c, st, n);
    CHECK(rc == HBEC_OK, 20);
    uint8_t** keep = (uint8_t**)calloc(n, sizeof(uint8_t*));
    for (uint64_t i = 0; i < n; ++i) {
        const size_t bytes = (size_t)n_sh * st[i].shard_len;
        uint8_t* shp[32];
        size_t lens[32];
        int ok = 0;
        for (int j = 0; j < n_sh; ++j) {
            shp[j] = (uint8_t*)st[i].base + (size_t)j * st[i].shard_len;
            lens[j] = st[i].shard_len;
        }
        CHECK(hbec_verify(c, shp, lens, n_sh, &ok) == HBEC_OK && ok == 1, 21);
        keep[i] = (uint8_t*)malloc(bytes);
        memcpy(keep[i], st[i].base, bytes);
        memset(st[i].base, 0x5A, st[i].shard_len);
        memset((uint8_t*)st[i].base + (size_t)k * st[i].shard_len, 0xA5, st[i].shard_len);
    }
    uint8_t present[32];
    for (int j = 0; j < n_sh; ++j) present[j] = (j == 0 || j == k) ? 0 : 1;
    rc = devices ? hbec_reconstruct_host_devices(c, st, n, present, 0, devices, n_devices)
                 : hbec_reconstruct_host(c, st, n, present, 0);
    CHECK(rc == HBEC_OK, 22);
    for (uint64_t i = 0; i < n; ++i) {
        CHECK(memcmp(keep[i], st[i].base, (size_t)n_sh * st[i].shard_len) == 0, 23);
        free(keep[i]);
    }
    free(keep);
    return 0;
}

struct BatcherJob {
    hbec_batcher* b;
    hbec_stripe st;
    int k, m, rc;
};

static void* batcher_worker(void* arg) {
    struct BatcherJob* j = (struct BatcherJob*)arg;
    uint8_t dig[32 * 16];
    j->rc = hbec_batcher_encode(j->b, &j->st);
    if (!j->rc) j->rc = hbec_batcher_encode_md5(j->b, &j->st, dig);
    uint8_t present[32];
    for (int i = 0; i < j->k + j->m; ++i) present[i] = i == 1 ? 0 : 1;
    if (!j->rc) {
        memset((uint8_t*)j->st.base + j->st.shard_len, 0, j->st.shard_len);
        j->rc = hbec_batcher_reconstruct(j->b, &j->st, present, 0);
    }
    return NULL;
}

/* per-call databuf entries from many threads: pinned stripes take the
 * coalescer, pageable ones the per-call concurrency gate */
struct PercallJob {
    hbec_codec* c;
    uint8_t* base;
    uint64_t s;
    int k, m, rc;
};

static void* percall_worker(void* arg) {
    struct PercallJob* j = (struct PercallJob*)arg;
    for (int it = 0; it < 4 && !j->rc; ++it) {
        j->rc = hbec_encode_databuf(j->c, j->base, j->s);
        if (j->rc) break;
        uint8_t present[32];
        for (int i = 0; i < j->k + j->m; ++i) present[i] = i == 0 ? 0 : 1;
        memset(j->base, 0, j->s);
        j->rc = hbec_reconstruct_databuf(j->c, j->base, j->s, present, 1);
        int ok = 0;
        if (!j->rc) j->rc = hbec_verify_databuf(j->c, j->base, j->s, &ok);
        if (!j->rc && !ok) j->rc = -100;
    }
    return NULL;
}

/* in-memory io for the ecutils loops */
struct Mem {
    uint8_t* p;
    size_t len, cap, pos;
};
static int64_t mem_read(void* ctx, uint8_t* buf, size_t n) {
    struct Mem* m = (struct Mem*)ctx;
    size_t left = m->len - m->pos, take = n < left ? n : left;
    if (take > 7) take = take / 2 + 1; /* short reads, like a socket */
    memcpy(buf, m->p + m->pos, take);
    m->pos += take;
    return (int64_t)take;
}
static int mem_write(void* ctx, const uint8_t* buf, size_t n) {
    struct Mem* m = (struct Mem*)ctx;
    if (m->len + n > m->cap) {
        m->cap = (m->len + n) * 2;
        m->p = (uint8_t*)realloc(m->p, m->cap);
    }
    memcpy(m->p + m->len, buf, n);
    m->len += n;
    return 0;
}

static int ecutils_part(void) {
    const int k = 4, m = 2, chunk = 1000;
    const int64_t len = 10007; /* 3 stripes, the last one padded */
    struct Mem obj = {(uint8_t*)malloc(len), (size_t)len, (size_t)len, 0};
    for (int64_t i = 0; i < len; ++i) obj.p[i] = rnd8();
    struct Mem sh[6];
    void* w[6];
    for (int i = 0; i < 6; ++i) {
        sh[i] = (struct Mem){NULL, 0, 0, 0};
        w[i] = &sh[i];
    }
    CHECK(hbec_ec_split(k, m, mem_read, &obj, chunk, len, mem_write, w) == HBEC_OK, 40);
    const int64_t slen = hbec_ec_shard_length(len, k);
    for (int i = 0; i < 6; ++i) CHECK((int64_t)sh[i].len == slen, 41);
    /* glue with shards 0 and 4 missing */
    struct Mem out = {NULL, 0, 0, 0};
    void* dst[1] = {&out};
    void* bodies[6];
    for (int i = 0; i < 6; ++i) {
        sh[i].pos = 0;
        bodies[i] = (i == 0 || i == 4) ? NULL : &sh[i];
    }
    CHECK(hbec_ec_glue(k, m, mem_read, bodies, chunk, len, mem_write, dst, 1) == HBEC_OK, 42);
    CHECK(out.len == (size_t)len && memcmp(out.p, obj.p, (size_t)len) == 0, 43);
    /* rebuild shard 0 from the others */
    struct Mem r0 = {NULL, 0, 0, 0};
    void* rd[1] = {&r0};
    int which[1] = {0};
    for (int i = 0; i < 6; ++i) sh[i].pos = 0;
    CHECK(hbec_ec_reconstruct(k, m, mem_read, bodies, chunk, len, mem_write, rd, which, 1) == HBEC_OK, 44);
    CHECK(r0.len == sh[0].len && memcmp(r0.p, sh[0].p, r0.len) == 0, 45);
    free(obj.p);
    free(out.p);
    free(r0.p);
    for (int i = 0; i < 6; ++i) free(sh[i].p);
    return 0;
}

static int gpu_part(void) {
    int nd = 0;
    CHECK(hbec_device_count(&nd) == HBEC_OK && nd >= 1, 10);
    hbec_codec* c = NULL;
    CHECK(hbec_new(4, 2, &c) == HBEC_OK, 11);
    const int k = 4, m = 2;
    /* 1. staging ring: mixed sizes incl. odd lengths and a stripe wider than a 64 MiB slot */
    const uint64_t sizes[] = {1 << 18, 1 << 18, 1 << 18, 1024, 251, 2, 786434, 17 << 20, 1 << 18};
    const int ns = (int)(sizeof sizes / sizeof sizes[0]);
    hbec_stripe st[16];
    for (int i = 0; i < ns; ++i) st[i] = (hbec_stripe){make_stripe(k, m, sizes[i], NULL), sizes[i]};
    int rc = stripes_roundtrip(c, k, m, st, ns, NULL, 0);
    if (rc) return rc;
    /* 2. the same through three host threads (multi-device split, all on device 0) */
    int devs[3] = {0, 0, 0};
    rc = stripes_roundtrip(c, k, m, st, ns, devs, 3);
    if (rc) return rc;
    for (int i = 0; i < ns; ++i) free(st[i].base);
    /* 3. zero-copy: stripes inside one hbec_host_alloc buffer, plus one pageable */
    void* pin = NULL;
    const uint64_t zs[] = {1 << 18, 1 << 18, 4096, 1 << 18};
    size_t total = 0;
    for (int i = 0; i < 4; ++i) total += (size_t)(k + m) * zs[i];
    CHECK(hbec_host_alloc(total, &pin) == HBEC_OK, 12);
    size_t off = 0;
    for (int i = 0; i < 4; ++i) {
        st[i] = (hbec_stripe){make_stripe(k, m, zs[i], (uint8_t*)pin + off), zs[i]};
        off += (size_t)(k + m) * zs[i];
        uint64_t dev = 0;
        CHECK(hbec_host_device_addr(st[i].base, (k + m) * zs[i], &dev) == HBEC_OK && dev != 0, 13);
    }
    st[4] = (hbec_stripe){make_stripe(k, m, 1 << 16, NULL), 1 << 16};
    rc = stripes_roundtrip(c, k, m, st, 5, NULL, 0);
    if (rc) return rc;
    free(st[4].base);
    /* 4. per-call Encode / ReconstructData on pinned shards (zero-copy) and on malloc'd shards */
    for (int pass = 0; pass < 2; ++pass) {
        const size_t s = 1 << 16;
        uint8_t* base = pass == 0 ? (uint8_t*)pin : (uint8_t*)malloc((k + m) * s);
        uint8_t* shp[6];
        size_t lens[6];
        for (int j = 0; j < 6; ++j) {
            shp[j] = base + j * s;
            lens[j] = s;
        }
        CHECK(hbec_encode(c, shp, lens, 6) == HBEC_OK, 14);
        int ok = 0;
        CHECK(hbec_verify(c, shp, lens, 6, &ok) == HBEC_OK && ok, 15);
        memset(shp[2], 0, s);
        lens[2] = 0;
        CHECK(hbec_reconstruct(c, shp, lens, 6, 1) == HBEC_OK && lens[2] == s, 16);
        CHECK(hbec_verify(c, shp, lens, 6, &ok) == HBEC_OK && ok, 17);
        if (pass == 1) free(base);
    }
    hbec_host_free(pin);
    /* 5. encode + ShardHash of host stripes */
    for (int i = 0; i < 3; ++i) st[i] = (hbec_stripe){make_stripe(k, m, 4096u << i, NULL), 4096u << i};
    uint8_t dig[3 * 6 * 16];
    CHECK(hbec_encode_host_md5(c, st, 3, dig) == HBEC_OK, 18);
    for (int i = 0; i < 3; ++i) free(st[i].base);
    /* 6. batcher with concurrent callers */
    hbec_batcher* b = NULL;
    CHECK(hbec_batcher_new(c, 8 << 20, 200, &b) == HBEC_OK, 19);
    pthread_t th[12];
    struct BatcherJob jobs[12];
    for (int i = 0; i < 12; ++i) {
        const uint64_t s = (i % 3 == 0) ? 1 << 18 : 4096 + 16 * i;
        jobs[i] = (struct BatcherJob){b, {make_stripe(k, m, s, NULL), s}, k, m, 0};
        pthread_create(&th[i], NULL, batcher_worker, &jobs[i]);
    }
    for (int i = 0; i < 12; ++i) {
        pthread_join(th[i], NULL);
        CHECK(jobs[i].rc == HBEC_OK, 30);
        uint8_t* shp[6];
        size_t lens[6];
        int ok = 0;
        for (int j = 0; j < 6; ++j) {
            shp[j] = (uint8_t*)jobs[i].st.base + j * jobs[i].st.shard_len;
            lens[j] = jobs[i].st.shard_len;
        }
        CHECK(hbec_verify(c, shp, lens, 6, &ok) == HBEC_OK && ok, 31);
        free(jobs[i].st.base);
    }
    hbec_batcher_free(b);
    /* 7. 24 concurrent per-call callers, half on one pinned pool, half pageable */
    {
        enum { NT = 24 };
        const uint64_t s = 4096;
        void* pool = NULL;
        CHECK(hbec_host_alloc((size_t)(NT / 2) * (k + m) * s, &pool) == HBEC_OK, 32);
        pthread_t pt[NT];
        struct PercallJob pj[NT];
        for (int i = 0; i < NT; ++i) {
            uint8_t* mem = i % 2 == 0 ? (uint8_t*)pool + (size_t)(i / 2) * (k + m) * s : NULL;
            pj[i] = (struct PercallJob){c, make_stripe(k, m, s, mem), s, k, m, 0};
            pthread_create(&pt[i], NULL, percall_worker, &pj[i]);
        }
        for (int i = 0; i < NT; ++i) {
            pthread_join(pt[i], NULL);
            CHECK(pj[i].rc == HBEC_OK, 33);
            if (i % 2) free(pj[i].base);
        }
        hbec_host_free(pool);
    }
    hbec_free(c);
    rc = ecutils_part();
    if (rc) return rc;
    printf("host_asan gpu ok\n");
    return 0;
}

int main(int argc, char** argv) {
    const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    int rc = cpu_part();
    if (rc || !gpu) return rc;
    return gpu_part();
}
