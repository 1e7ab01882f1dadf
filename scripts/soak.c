/* Concurrency soak of every host-facing entry point at once (the way a busy
 * object server reaches the library: Stabilize, degraded GETs, repairs and
 * the auditor on arbitrary OS threads).  T threads run for SECONDS, each
 * cycling over its own stripes and picking an operation per iteration:
 *
 *   0  hbec_encode_databuf (pinned: coalescer; pageable: per-call gate)
 *   1  hbec_reconstruct_databuf of 1-2 erased shards, data-only or full
 *   2  hbec_batcher_encode
 *   3  hbec_batcher_encode_md5 (digest of shard 0 checked against a CPU MD5
 *      of the same bytes is left to the tests; here: call succeeds)
 *   4  hbec_batcher_reconstruct
 *   5  hbec_encode_host of a small batch of the thread's stripes
 *   6  hbec_verify_databuf
 *
 * After every write operation the stripe is verified (hbec_verify_databuf)
 * and every rebuilt shard compared with a saved copy, so a wrong byte, a
 * lost wake-up (hang: the run is under `timeout`) or a crash ends the run.
 * Sizes mix 4 KiB and 1 MiB objects with odd-sized ones (S % 16 != 0:
 * shards at odd offsets, the unaligned kernels), 4+2.  Prints one JSON line.
 *
 *   gcc -O2 -std=c11 -pthread -Iinclude scripts/soak.c -Lhummingbird_amd -lhbec \
 *       -Wl,-rpath,$PWD/hummingbird_amd -o gpurun_out/soak
 *   timeout -k 10 180 gpurun_out/soak THREADS SECONDS
 *
 * Stall report: when no operation completes for STALL_S seconds, every task
 * of the process (the soak threads, the library's pool and batcher workers
 * and the HIP runtime's threads) prints its stack (SIGUSR1 handler,
 * backtrace_symbols_fd; resolve libhbec.so+offset with addr2line) once. */
#define _GNU_SOURCE
#include <dirent.h>
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <stdatomic.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hbec.h"

enum { K = 4, M = 2, N = K + M, PER = 6 };

static hbec_codec* g_codec;
static hbec_batcher* g_bat;
static double g_stop;

typedef struct {
    int id, pinned;
    uint8_t* base[PER];
    uint8_t* keep[PER];
    size_t s[PER];
    uint64_t ops[7], rng;
    int rc, where;
    volatile int cur;  /* operation in progress (-1: none), for the stall report */
} Job;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static uint64_t next(uint64_t* x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static atomic_flag g_dump_lock = ATOMIC_FLAG_INIT;

static void dump_handler(int sig) {
    (void)sig;
    void* fr[64];
    while (atomic_flag_test_and_set(&g_dump_lock)) {
    }
    char hdr[64];
    const int n = snprintf(hdr, sizeof hdr, "--- task %ld\n", (long)syscall(SYS_gettid));
    if (write(2, hdr, (size_t)n) < 0) {
    }
    const int d = backtrace(fr, 64);
    backtrace_symbols_fd(fr, d, 2);
    atomic_flag_clear(&g_dump_lock);
}

/* signal every task of the process in turn (each prints its own stack) */
static void dump_all_tasks(void) {
    DIR* dir = opendir("/proc/self/task");
    if (!dir) return;
    const pid_t pid = getpid();
    struct dirent* e;
    while ((e = readdir(dir)) != NULL) {
        const long tid = atol(e->d_name);
        if (tid <= 0) continue;
        syscall(SYS_tgkill, pid, tid, SIGUSR1);
        struct timespec ts = {0, 20 * 1000 * 1000};
        nanosleep(&ts, NULL);
    }
    closedir(dir);
}

static int check(Job* j, int i) {
    int ok = 0;
    if (hbec_verify_databuf(g_codec, j->base[i], j->s[i], &ok) || !ok) return -1001;
    if (memcmp(j->base[i], j->keep[i], N * j->s[i])) return -1002;
    return 0;
}

static void* run(void* arg) {
    Job* j = (Job*)arg;
    while (now() < g_stop && !j->rc) {
        const int i = (int)(next(&j->rng) % PER), op = (int)(next(&j->rng) % 7);
        uint8_t* b = j->base[i];
        const size_t s = j->s[i];
        int rc = 0;
        j->cur = op;
        switch (op) {
            case 0:
                memset(b + K * s, 0x33, M * s);
                rc = hbec_encode_databuf(g_codec, b, s);
                break;
            case 1: {
                uint8_t present[N];
                for (int t = 0; t < N; ++t) present[t] = 1;
                const int e0 = (int)(next(&j->rng) % N), e1 = (int)(next(&j->rng) % N);
                present[e0] = present[e1] = 0;
                const int data_only = (int)(next(&j->rng) & 1);
                for (int t = 0; t < N; ++t)
                    if (!present[t] && (t < K || !data_only)) memset(b + t * s, 0x77, s);
                rc = hbec_reconstruct_databuf(g_codec, b, s, present, data_only);
                if (!rc && data_only)  /* parity shards stay as they were erased: restore them */
                    for (int t = K; t < N; ++t)
                        if (!present[t]) memcpy(b + t * s, j->keep[i] + t * s, s);
                break;
            }
            case 2: {
                hbec_stripe st = {b, s};
                memset(b + K * s, 0x55, M * s);
                rc = hbec_batcher_encode(g_bat, &st);
                break;
            }
            case 3: {
                hbec_stripe st = {b, s};
                uint8_t dig[N * 16];
                if (s <= (1u << 20)) rc = hbec_batcher_encode_md5(g_bat, &st, dig);
                break;
            }
            case 4: {
                hbec_stripe st = {b, s};
                uint8_t present[N] = {1, 0, 1, 1, 0, 1};
                memset(b + 1 * s, 0x99, s);
                memset(b + 4 * s, 0x99, s);
                rc = hbec_batcher_reconstruct(g_bat, &st, present, 0);
                break;
            }
            case 5: {
                hbec_stripe st[PER];
                for (int t = 0; t < PER; ++t) {
                    st[t] = (hbec_stripe){j->base[t], j->s[t]};
                    memset(j->base[t] + K * j->s[t], 0x11, M * j->s[t]);
                }
                rc = hbec_encode_host(g_codec, st, PER);
                for (int t = 0; t < PER && !rc; ++t) rc = check(j, t);
                break;
            }
            case 6: {
                int ok = 0;
                rc = hbec_verify_databuf(g_codec, b, s, &ok);
                if (!rc && !ok) rc = -1003;
                break;
            }
        }
        j->cur = 10 + op;  /* the check after op */
        if (!rc && op != 5 && op != 6) rc = check(j, i);
        j->cur = -1;
        if (rc) {
            j->rc = rc;
            j->where = op;
        }
        ++j->ops[op];
    }
    return NULL;
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 32;
    const double secs = argc > 2 ? atof(argv[2]) : 60.0;
    if (threads < 1 || threads > 256) return 2;
    if (hbec_new(K, M, &g_codec) || hbec_batcher_new(g_codec, 64u << 20, 200, &g_bat)) {
        fprintf(stderr, "%s\n", hbec_last_error());
        return 1;
    }
    Job* jobs = calloc(threads, sizeof(Job));
    pthread_t* th = malloc(sizeof(pthread_t) * threads);
    uint64_t seed = 0x48424543ull;
    for (int t = 0; t < threads; ++t) {
        Job* j = &jobs[t];
        j->id = t;
        j->cur = -1;
        j->pinned = t % 2 == 0;
        j->rng = seed + (uint64_t)t * 7919u;
        for (int i = 0; i < PER; ++i) {
            static const size_t sizes[PER] = {1u << 18, 1024u, 262141u, 1027u, 1024u, 333u};
            j->s[i] = sizes[i];  /* 1 MiB, 4 KiB and odd-sized objects */
            const size_t bytes = N * j->s[i];
            if (j->pinned) {
                if (hbec_host_alloc(bytes, (void**)&j->base[i])) {
                    fprintf(stderr, "%s\n", hbec_last_error());
                    return 1;
                }
            } else {
                j->base[i] = malloc(bytes);
            }
            j->keep[i] = malloc(bytes);
            for (size_t o = 0; o < K * j->s[i]; o += 8) {
                const uint64_t z = next(&seed);
                memcpy(j->base[i] + o, &z, 8);
            }
            if (hbec_encode_databuf(g_codec, j->base[i], j->s[i])) {
                fprintf(stderr, "%s\n", hbec_last_error());
                return 1;
            }
            memcpy(j->keep[i], j->base[i], bytes);
        }
    }
    {
        void* fr[4];
        backtrace(fr, 4); /* load the unwinder before any signal */
        struct sigaction sa;
        memset(&sa, 0, sizeof sa);
        sa.sa_handler = dump_handler;
        sa.sa_flags = SA_RESTART;
        sigaction(SIGUSR1, &sa, NULL);
    }
    const double stall_s = getenv("SOAK_STALL_S") ? atof(getenv("SOAK_STALL_S")) : 20.0;
    double last_progress = now();
    uint64_t last_ops = 0;
    int dumped = 0;
    const double t0 = now();
    g_stop = t0 + secs;
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, run, &jobs[t]);
    /* progress every 10 s on stderr (long runs must not look hung) */
    while (now() < g_stop) {
        struct timespec ts = {10, 0};
        const double left = g_stop - now();
        if (left < 10.0) ts = (struct timespec){(time_t)left, (long)((left - (time_t)left) * 1e9)};
        nanosleep(&ts, NULL);
        uint64_t sofar = 0;
        int bad = 0;
        for (int t = 0; t < threads; ++t) {
            for (int o = 0; o < 7; ++o) sofar += jobs[t].ops[o];
            bad |= jobs[t].rc != 0;
        }
        int hist[20] = {0};
        for (int t = 0; t < threads; ++t) {
            const int c = jobs[t].cur;
            hist[c < 0 ? 19 : c]++;
        }
        uint64_t g = 0, c = 0, b = 0, bs = 0;
        hbec_coalesce_stats(&g, &c);
        hbec_batcher_stats(g_bat, &b, &bs);
        fprintf(stderr, "soak: %.0f s, %llu ops%s; in op 0-6: %d %d %d %d %d %d %d; in check after 0-4: %d %d %d %d %d; "
                "coalesce %llu/%llu, batches %llu/%llu\n", now() - t0, (unsigned long long)sofar, bad ? ", FAILED" : "",
                hist[0], hist[1], hist[2], hist[3], hist[4], hist[5], hist[6], hist[10], hist[11], hist[12], hist[13],
                hist[14], (unsigned long long)g, (unsigned long long)c, (unsigned long long)b, (unsigned long long)bs);
        fflush(stderr);
        if (sofar != last_ops) {
            last_ops = sofar;
            last_progress = now();
        } else if (!dumped && now() - last_progress >= stall_s) {
            fprintf(stderr, "soak: no operation completed for %.0f s: stacks of every task follow\n", now() - last_progress);
            fflush(stderr);
            dump_all_tasks();
            dumped = 1;
        }
        if (bad) break;
    }
    int rc = 0, where = -1, who = -1;
    uint64_t ops[7] = {0}, total = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc && !rc) {
            rc = jobs[t].rc;
            where = jobs[t].where;
            who = t;
        }
        for (int o = 0; o < 7; ++o) ops[o] += jobs[t].ops[o];
    }
    for (int o = 0; o < 7; ++o) total += ops[o];
    uint64_t groups = 0, calls = 0, batches = 0, stripes = 0;
    hbec_coalesce_stats(&groups, &calls);
    hbec_batcher_stats(g_bat, &batches, &stripes);
    hbec_batcher_free(g_bat);
    printf("{\"measure\": \"soak\", \"threads\": %d, \"seconds\": %.1f, \"ops\": %llu, \"per_op\": [%llu, %llu, %llu, "
           "%llu, %llu, %llu, %llu], \"coalesce_groups\": %llu, \"coalesce_calls\": %llu, \"batches\": %llu, "
           "\"batched_stripes\": %llu, \"rc\": %d, \"failed_op\": %d, \"failed_thread\": %d}\n",
           threads, now() - t0, (unsigned long long)total, (unsigned long long)ops[0], (unsigned long long)ops[1],
           (unsigned long long)ops[2], (unsigned long long)ops[3], (unsigned long long)ops[4],
           (unsigned long long)ops[5], (unsigned long long)ops[6], (unsigned long long)groups,
           (unsigned long long)calls, (unsigned long long)batches, (unsigned long long)stripes, rc, where, who);
    if (rc) fprintf(stderr, "soak failed: thread %d op %d rc %d: %s\n", who, where, rc, hbec_last_error());
    hbec_free(g_codec);
    return rc ? 1 : 0;
}
