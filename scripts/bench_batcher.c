/* Batched stabilization driver (hbec_batcher_*) under many concurrent native
 * callers, the way concurrent Stabilize goroutines would reach it through
 * cgo: T pthreads, each encoding P 1 MiB 4+2 stripes (ecSplit databuf
 * layout, one call per stripe), from pinned (hbec_host_alloc, zero-copy) or
 * pageable (malloc) memory.  No interpreter in the loop.
 *
 *   gcc -O2 -std=c11 -pthread -Iinclude scripts/bench_batcher.c -Lhummingbird_amd -lhbec \
 *       -Wl,-rpath,$PWD/hummingbird_amd -o /tmp/bench_batcher
 *   /tmp/bench_batcher THREADS PER_THREAD PINNED MAX_BATCH_MB MAX_WAIT_US [MODE]
 *
 * MODE 0 (default): hbec_batcher_encode (the explicit batching driver);
 * MODE 2: hbec_batcher_encode_md5 (Encode + ShardHash of every shard);
 * MODE 1: plain per-call hbec_encode_databuf (the 3-line shim swap of
 *         INTEGRATION.md), coalesced inside the library (HBEC_COALESCE=0 in
 *         the environment measures it uncoalesced).
 *
 * Prints one JSON line: object-data GiB/s, us per object, batches; checks
 * every stripe's parity afterwards with hbec_verify.
 */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hbec.h"

enum { K = 4, M = 2 };
static size_t S = 1 << 18;  /* shard bytes: object bytes / K (argv[7], default 1 MiB objects) */

typedef struct {
    hbec_codec* codec;
    int mode;
    hbec_batcher* bat;
    uint8_t* pool;
    int first, count;
    int rc;
} Job;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void* caller(void* arg) {
    Job* j = (Job*)arg;
    for (int i = j->first; i < j->first + j->count && !j->rc; ++i) {
        uint8_t* base = j->pool + (size_t)i * (K + M) * S;
        if (j->mode == 1) {
            j->rc = hbec_encode_databuf(j->codec, base, S);
        } else if (j->mode == 2) {
            hbec_stripe st = {base, S};
            uint8_t dig[(K + M) * 16];  /* digests not checked here: tests compare them with hashlib */
            j->rc = hbec_batcher_encode_md5(j->bat, &st, dig);
        } else {
            hbec_stripe st = {base, S};
            j->rc = hbec_batcher_encode(j->bat, &st);
        }
    }
    return NULL;
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 64;
    const int per = argc > 2 ? atoi(argv[2]) : 32;
    const int pinned = argc > 3 ? atoi(argv[3]) : 1;
    const uint64_t max_mb = argc > 4 ? (uint64_t)atoll(argv[4]) : 96;
    const uint32_t wait_us = argc > 5 ? (uint32_t)atoi(argv[5]) : 300;
    const int mode = argc > 6 ? atoi(argv[6]) : 0;
    if (argc > 7) S = (size_t)atoll(argv[7]) / K;
    if (S == 0 || S % 16) return 2;
    if (threads < 1 || threads > 1024 || per < 1) return 2;
    const size_t n = (size_t)threads * per, stripe = (size_t)(K + M) * S;
    uint8_t* pool = NULL;
    if (pinned) {
        if (hbec_host_alloc(n * stripe, (void**)&pool)) { fprintf(stderr, "%s\n", hbec_last_error()); return 1; }
    } else {
        pool = malloc(n * stripe);
        if (!pool) return 1;
    }
    uint64_t seed = 0x48424543ull;
    for (size_t o = 0; o < n; ++o)
        for (size_t b = 0; b < (size_t)K * S; b += 8) {
            uint64_t z = (seed += 0x9E3779B97F4A7C15ull);
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            memcpy(pool + o * stripe + b, &z, 8);
        }
    hbec_codec* codec = NULL;
    hbec_batcher* bat = NULL;
    if (hbec_new(K, M, &codec) || hbec_batcher_new(codec, max_mb << 20, wait_us, &bat)) {
        fprintf(stderr, "%s\n", hbec_last_error());
        return 1;
    }
    pthread_t* th = malloc(sizeof(pthread_t) * threads);
    Job* jobs = calloc(threads, sizeof(Job));
    /* warm-up: a few stripes per caller, all at once, so every worker has made
     * its ring before the clock starts (a long-running server's steady state) */
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (Job){codec, mode, bat, pool, t * per, per < 4 ? per : 4, 0};
        pthread_create(&th[t], NULL, caller, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    uint64_t b0 = 0, s0 = 0;
    if (mode == 1) hbec_coalesce_stats(&b0, &s0);
    else hbec_batcher_stats(bat, &b0, &s0);
    const double t0 = now();
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (Job){codec, mode, bat, pool, t * per, per, 0};
        pthread_create(&th[t], NULL, caller, &jobs[t]);
    }
    int rc = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        rc |= jobs[t].rc;
    }
    const double secs = now() - t0;
    uint64_t b1 = 0, s1 = 0;
    if (mode == 1) hbec_coalesce_stats(&b1, &s1);
    else hbec_batcher_stats(bat, &b1, &s1);
    hbec_batcher_free(bat);
    if (rc) { fprintf(stderr, "batcher: %s\n", hbec_last_error()); return 1; }
    int bad = 0;
    for (size_t o = 0; o < n && !bad; ++o) {
        uint8_t* sh[K + M];
        size_t lens[K + M];
        for (int i = 0; i < K + M; ++i) {
            sh[i] = pool + o * stripe + (size_t)i * S;
            lens[i] = S;
        }
        int ok = 0;
        if (hbec_verify(codec, sh, lens, K + M, &ok) || !ok) bad = 1;
    }
    const char* co = getenv("HBEC_COALESCE");
    printf("{\"measure\": \"%s_native_callers_Encode_%zuB_%s\", \"threads\": %d, \"objects\": %zu, "
           "\"max_batch_MiB\": %llu, \"max_wait_us\": %u, \"seconds\": %.4f, \"object_data_GiB_s\": %.2f, "
           "\"us_per_object\": %.2f, \"objects_per_s\": %.0f, \"batches\": %llu, \"parity_ok\": %s}\n",
           mode == 1 ? (co && co[0] == '0' ? "percall_databuf_uncoalesced" : "percall_databuf_coalesced")
                     : (mode == 2 ? "batcher_md5" : "batcher"),
           (size_t)K * S, pinned ? "pinned" : "pageable", threads, n, (unsigned long long)max_mb, wait_us, secs,
           n * (double)K * S / secs / (double)(1 << 30), secs / n * 1e6, n / secs, (unsigned long long)(b1 - b0),
           bad ? "false" : "true");
    hbec_free(codec);
    if (pinned) hbec_host_free(pool);
    else free(pool);
    return bad;
}
