/* Stripe-loop throughput through the C ABI (what a cgo caller of
 * hbec_ec_split / _reconstruct / _glue sees), memory-backed readers and
 * writers (memcpy), one object of OBJ_MIB MiB, chunk 1 MiB.
 *
 *   gcc -O2 -std=c11 -Iinclude scripts/bench_ecutils.c -Lhummingbird_amd -lhbec \
 *       -Wl,-rpath,$PWD/hummingbird_amd -o /tmp/bench_ecutils && /tmp/bench_ecutils 4 2 256
 *
 * Prints one JSON object per loop: object-data GiB/s (object bytes / wall).
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hbec.h"

typedef struct {
    const uint8_t* p;
    size_t len, pos;
} Reader;

typedef struct {
    uint8_t* p;
    size_t cap, pos;
} Writer;

static int64_t rd(void* ctx, uint8_t* buf, size_t n) {
    Reader* r = (Reader*)ctx;
    size_t left = r->len - r->pos;
    if (left == 0) return 0;
    if (n > left) n = left;
    memcpy(buf, r->p + r->pos, n);
    r->pos += n;
    return (int64_t)n;
}

static int wr(void* ctx, const uint8_t* buf, size_t n) {
    Writer* w = (Writer*)ctx;
    if (w->pos + n > w->cap) return 1;
    memcpy(w->p + w->pos, buf, n);
    w->pos += n;
    return 0;
}

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void report(const char* loop, int k, int m, double obj_bytes, double best) {
    printf("{\"loop\": \"%s\", \"k\": %d, \"m\": %d, \"object_MiB\": %.0f, \"seconds\": %.4f, "
           "\"object_data_GiB_s\": %.2f}\n",
           loop, k, m, obj_bytes / 1048576.0, best, obj_bytes / best / 1073741824.0);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 4, m = argc > 2 ? atoi(argv[2]) : 2;
    const size_t obj_mib = argc > 3 ? (size_t)atoll(argv[3]) : 256;
    const int chunk = 1 << 20, n = k + m, reps = 3;
    const size_t len = obj_mib << 20;
    const size_t shard = (size_t)hbec_ec_shard_length((int64_t)len, k);
    uint8_t* obj = malloc(len);
    uint64_t seed = 0x48424543ull;
    for (size_t i = 0; i + 8 <= len; i += 8) {
        uint64_t v = splitmix(&seed);
        memcpy(obj + i, &v, 8);
    }
    uint8_t* files[64];
    Writer ws[64];
    void* wctx[64];
    for (int i = 0; i < n; ++i) {
        files[i] = malloc(shard);
        ws[i] = (Writer){files[i], shard, 0};
        wctx[i] = &ws[i];
    }
    double best = 1e30;
    int rc = 0;
    for (int r = 0; r < reps; ++r) {
        Reader in = {obj, len, 0};
        for (int i = 0; i < n; ++i) ws[i].pos = 0;
        double t0 = now();
        rc |= hbec_ec_split(k, m, rd, &in, chunk, (int64_t)len, wr, wctx);
        double t = now() - t0;
        if (t < best) best = t;
    }
    if (rc) { fprintf(stderr, "ec_split: %s\n", hbec_last_error()); return 1; }
    report("ec_split", k, m, (double)len, best);

    /* ecGlue healthy (no GPU work) and with data shards 0..m-1 lost */
    uint8_t* out = malloc(len);
    Writer ow = {out, len, 0};
    void* octx[1] = {&ow};
    Reader br[64];
    void* bctx[64];
    for (int lost = 0; lost <= 1; ++lost) {
        best = 1e30;
        for (int r = 0; r < reps; ++r) {
            for (int i = 0; i < n; ++i) {
                br[i] = (Reader){files[i], shard, 0};
                bctx[i] = (lost && i < m) ? NULL : &br[i];
            }
            ow.pos = 0;
            double t0 = now();
            rc |= hbec_ec_glue(k, m, rd, bctx, chunk, (int64_t)len, wr, octx, 1);
            double t = now() - t0;
            if (t < best) best = t;
        }
        if (rc || memcmp(out, obj, len) != 0) { fprintf(stderr, "ec_glue failed %s\n", hbec_last_error()); return 1; }
        report(lost ? "ec_glue_degraded" : "ec_glue_healthy", k, m, (double)len, best);
    }
    /* ecReconstruct of shards 0..m-1 */
    uint8_t* rebuilt[64];
    Writer rw[64];
    void* rctx[64];
    int nums[64];
    for (int i = 0; i < m; ++i) {
        rebuilt[i] = malloc(shard);
        rw[i] = (Writer){rebuilt[i], shard, 0};
        rctx[i] = &rw[i];
        nums[i] = i;
    }
    best = 1e30;
    for (int r = 0; r < reps; ++r) {
        for (int i = 0; i < n; ++i) {
            br[i] = (Reader){files[i], shard, 0};
            bctx[i] = i < m ? NULL : &br[i];
        }
        for (int i = 0; i < m; ++i) rw[i].pos = 0;
        double t0 = now();
        rc |= hbec_ec_reconstruct(k, m, rd, bctx, chunk, (int64_t)len, wr, rctx, nums, m);
        double t = now() - t0;
        if (t < best) best = t;
    }
    for (int i = 0; i < m && !rc; ++i)
        if (memcmp(rebuilt[i], files[i], shard) != 0) rc = 1;
    if (rc) { fprintf(stderr, "ec_reconstruct failed %s\n", hbec_last_error()); return 1; }
    report("ec_reconstruct", k, m, (double)len, best);
    return 0;
}
