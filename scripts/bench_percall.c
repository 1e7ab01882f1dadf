/* Per-call latency of the plain drop-in (one
 * hbec_encode_databuf / hbec_reconstruct_databuf per 1 MiB 4+2 stripe) at the
 * reference's own concurrency: the nursery stabilizer runs
 * object-nursery.concurrency = 2 objects at a time per device
 * (replicator.go:487,530), so T = 1, 2, 4, 8 threads, each calling in a loop.
 *
 *   gcc -O2 -std=c11 -pthread -Iinclude scripts/bench_percall.c -Lhummingbird_amd -lhbec \
 *       -Wl,-rpath,$PWD/hummingbird_amd -o /tmp/bench_percall
 *   /tmp/bench_percall THREADS CALLS_PER_THREAD PINNED OP   (OP 0 encode, 1 reconstruct {0,1})
 *
 * Prints one JSON line: median / p90 us per call, object-data GiB/s. */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hbec.h"

enum { K = 4, M = 2, S = 1 << 18 };

typedef struct {
    hbec_codec* codec;
    uint8_t* buf;
    int calls, op, rc;
    double* lat;
} Job;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void* caller(void* arg) {
    Job* j = (Job*)arg;
    static const uint8_t present[K + M] = {0, 0, 1, 1, 1, 1};
    for (int i = 0; i < j->calls && !j->rc; ++i) {
        const double t0 = now();
        j->rc = j->op == 0 ? hbec_encode_databuf(j->codec, j->buf, S)
                           : hbec_reconstruct_databuf(j->codec, j->buf, S, present, 0);
        j->lat[i] = now() - t0;
    }
    return NULL;
}

static int cmp(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 1;
    const int calls = argc > 2 ? atoi(argv[2]) : 200;
    const int pinned = argc > 3 ? atoi(argv[3]) : 0;
    const int op = argc > 4 ? atoi(argv[4]) : 0;
    if (threads < 1 || threads > 256 || calls < 1) return 2;
    const size_t stripe = (size_t)(K + M) * S;
    hbec_codec* codec = NULL;
    if (hbec_new(K, M, &codec)) return 1;
    pthread_t th[256];
    Job jobs[256];
    double* lat = calloc((size_t)threads * calls, sizeof(double));
    for (int t = 0; t < threads; ++t) {
        uint8_t* b = NULL;
        if (pinned) {
            if (hbec_host_alloc(stripe, (void**)&b)) { fprintf(stderr, "%s\n", hbec_last_error()); return 1; }
        } else if (!(b = malloc(stripe))) {
            return 1;
        }
        for (size_t i = 0; i < stripe; ++i) b[i] = (uint8_t)(i * 131 + t);
        jobs[t] = (Job){codec, b, 8, 0, 0, lat + (size_t)t * calls};
        if (op == 1 && hbec_encode_databuf(codec, b, S)) return 1;  /* a codeword to rebuild */
    }
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, caller, &jobs[t]);  /* warm-up */
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    for (int t = 0; t < threads; ++t) {
        jobs[t].calls = calls;
        jobs[t].op = op;
    }
    const double t0 = now();
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, caller, &jobs[t]);
    int rc = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        rc |= jobs[t].rc;
    }
    const double secs = now() - t0;
    if (rc) { fprintf(stderr, "call failed: %s\n", hbec_last_error()); return 1; }
    int ok = 1;
    for (int t = 0; t < threads && ok; ++t) {
        int v = 0;
        if (hbec_verify_databuf(codec, jobs[t].buf, S, &v) || !v) ok = 0;
    }
    const size_t n = (size_t)threads * calls;
    qsort(lat, n, sizeof(double), cmp);
    printf("{\"measure\": \"percall_%s_1MiB_%s\", \"threads\": %d, \"calls\": %zu, \"p50_us\": %.1f, "
           "\"p90_us\": %.1f, \"object_data_GiB_s\": %.2f, \"parity_ok\": %s}\n",
           op ? "Reconstruct01" : "Encode", pinned ? "pinned" : "pageable", threads, n, lat[n / 2] * 1e6,
           lat[n * 9 / 10] * 1e6, n * (double)K * S / secs / (double)(1 << 30), ok ? "true" : "false");
    return ok ? 0 : 1;
}
