/*
 * gf_oracle.c — CPU oracle for the Hummingbird EC hot path.
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker / reported CPU baseline.  The
 * product library (libhbec.so) never links or calls this file.
 *
 * It is a C restatement of the codec that objectserver/ecutils.go:27,59,77,
 * 111,135,168 obtains from github.com/klauspost/reedsolomon (un-vendored,
 * unpinned, ~v1.6-v1.9 by the Go 1.10.2 toolchain era of .travis.yml:7-8):
 *
 *   - GF(2^8) poly 0x11D, generator 2                (klauspost galois.go)
 *   - matrix = Vandermonde(k+m,k) x inv(top k x k)   (matrix.go buildMatrix)
 *   - encode: parity_r = XOR_j M[k+r][j]*data_j      (reedsolomon.go Encode)
 *   - reconstruct: first k present shards, inv(sub)  (reedsolomon.go reconstruct)
 *
 * Two arithmetic implementations of the same slice multiply:
 *   ORC_SCALAR — log/exp table per byte (the literal field definition);
 *   ORC_AVX2   — low/high nibble 16-entry tables with VPSHUFB, the scheme of
 *                klauspost's galMulAVX2 / galMulAVX2Xor (galois_amd64.s).
 * Both are checked against the upstream KATs (tests/golden/kats.json) by
 * tests/test_oracle.py.  ORC_AVX2 over all host cores is the "port" CPU
 * baseline reported by bench.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#define ORC_SCALAR 0
#define ORC_AVX2 1

static uint8_t g_exp[510];
static uint8_t g_log[256];
static uint8_t g_mul[256][256];
static uint8_t g_mul_lo[256][16]; /* c * i       (klauspost mulTableLow)  */
static uint8_t g_mul_hi[256][16]; /* c * (i<<4)  (klauspost mulTableHigh) */
static int g_init = 0;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void orc_init_tables(void) {
    int x = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (uint8_t)x;
        g_exp[i + 255] = (uint8_t)x;
        g_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            g_mul[a][b] = (a == 0 || b == 0) ? 0 : g_exp[g_log[a] + g_log[b]];
    for (int c = 0; c < 256; c++)
        for (int i = 0; i < 16; i++) {
            g_mul_lo[c][i] = g_mul[c][i];
            g_mul_hi[c][i] = g_mul[c][i << 4];
        }
    g_init = 1;
}

static void ensure_init(void) { pthread_once(&g_once, orc_init_tables); }

uint8_t orc_gal_mul(uint8_t a, uint8_t b) {
    ensure_init();
    /* literal log/exp definition, not the product table */
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

uint8_t orc_gal_exp(uint8_t a, int n) {
    ensure_init();
    if (n == 0) return 1;
    if (a == 0) return 0;
    return g_exp[(g_log[a] * n) % 255];
}

static uint8_t gal_div(uint8_t a, uint8_t b) {
    if (a == 0) return 0;
    int d = (int)g_log[a] - (int)g_log[b];
    if (d < 0) d += 255;
    return g_exp[d];
}

/* Gauss-Jordan over GF(2^8) (matrix.go gaussianElimination). 0 ok, -1 singular. */
int orc_invert(int n, const uint8_t *in, uint8_t *out) {
    ensure_init();
    int w = 2 * n;
    uint8_t *a = (uint8_t *)calloc((size_t)n * w, 1);
    if (!a) return -2;
    for (int r = 0; r < n; r++) {
        memcpy(a + r * w, in + r * n, n);
        a[r * w + n + r] = 1;
    }
    for (int r = 0; r < n; r++) {
        if (a[r * w + r] == 0) {
            for (int b = r + 1; b < n; b++) {
                if (a[b * w + r] != 0) {
                    for (int c = 0; c < w; c++) {
                        uint8_t t = a[r * w + c];
                        a[r * w + c] = a[b * w + c];
                        a[b * w + c] = t;
                    }
                    break;
                }
            }
        }
        if (a[r * w + r] == 0) { free(a); return -1; }
        if (a[r * w + r] != 1) {
            uint8_t s = gal_div(1, a[r * w + r]);
            for (int c = 0; c < w; c++) a[r * w + c] = g_mul[s][a[r * w + c]];
        }
        for (int b = r + 1; b < n; b++) {
            uint8_t s = a[b * w + r];
            if (s) for (int c = 0; c < w; c++) a[b * w + c] ^= g_mul[s][a[r * w + c]];
        }
    }
    for (int d = 0; d < n; d++)
        for (int ab = 0; ab < d; ab++) {
            uint8_t s = a[ab * w + d];
            if (s) for (int c = 0; c < w; c++) a[ab * w + c] ^= g_mul[s][a[d * w + c]];
        }
    for (int r = 0; r < n; r++) memcpy(out + r * n, a + r * w + n, n);
    free(a);
    return 0;
}

/* matrix.go buildMatrix: (k+m) x k systematic matrix, row-major. */
int orc_build_matrix(int k, int m, uint8_t *out) {
    ensure_init();
    int total = k + m;
    if (k <= 0 || m < 0) return -1;
    if (total > 256) return -2;
    uint8_t *vm = (uint8_t *)malloc((size_t)total * k);
    uint8_t *inv = (uint8_t *)malloc((size_t)k * k);
    for (int r = 0; r < total; r++)
        for (int c = 0; c < k; c++) vm[r * k + c] = orc_gal_exp((uint8_t)r, c);
    int rc = orc_invert(k, vm, inv);
    if (rc == 0) {
        for (int r = 0; r < total; r++)
            for (int c = 0; c < k; c++) {
                uint8_t v = 0;
                for (int i = 0; i < k; i++) v ^= g_mul[vm[r * k + i]][inv[i * k + c]];
                out[r * k + c] = v;
            }
    }
    free(vm);
    free(inv);
    return rc;
}

/* ---------------- slice multiply kernels ---------------- */
static void mul_slice_scalar(uint8_t c, const uint8_t *in, uint8_t *out, size_t n, int xor_) {
    if (c == 0) {
        if (!xor_) memset(out, 0, n);
        return;
    }
    uint8_t lc = g_log[c];
    for (size_t i = 0; i < n; i++) {
        uint8_t v = in[i] ? g_exp[lc + g_log[in[i]]] : 0;
        out[i] = xor_ ? (uint8_t)(out[i] ^ v) : v;
    }
}

#if defined(__x86_64__)
__attribute__((target("avx2")))
static void mul_slice_avx2(uint8_t c, const uint8_t *in, uint8_t *out, size_t n, int xor_) {
    const __m128i lo128 = _mm_loadu_si128((const __m128i *)g_mul_lo[c]);
    const __m128i hi128 = _mm_loadu_si128((const __m128i *)g_mul_hi[c]);
    const __m256i tlo = _mm256_broadcastsi128_si256(lo128);
    const __m256i thi = _mm256_broadcastsi128_si256(hi128);
    const __m256i mask = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(in + i));
        __m256i l = _mm256_and_si256(x, mask);
        __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
        __m256i r = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
        if (xor_) r = _mm256_xor_si256(r, _mm256_loadu_si256((const __m256i *)(out + i)));
        _mm256_storeu_si256((__m256i *)(out + i), r);
    }
    for (; i < n; i++) {
        uint8_t v = (uint8_t)(g_mul_lo[c][in[i] & 15] ^ g_mul_hi[c][in[i] >> 4]);
        out[i] = xor_ ? (uint8_t)(out[i] ^ v) : v;
    }
}
#endif

static int have_avx2(void) {
#if defined(__x86_64__)
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2");
#else
    return 0;
#endif
}

int orc_have_avx2(void) { return have_avx2(); }

/* out[r] = XOR_j coeffs[r*k + j] * in[j] — klauspost codeSomeShards, with the
 * byte range split into 32 KiB blocks so every output block stays in L1 while
 * the k inputs stream past (what klauspost's per-goroutine split achieves). */
void orc_apply(int rows, int k, const uint8_t *coeffs, const uint8_t *const *in,
               uint8_t *const *out, size_t len, int impl) {
    ensure_init();
    if (impl == ORC_AVX2 && !have_avx2()) impl = ORC_SCALAR;
    const size_t blk = 32 * 1024;
    for (size_t s = 0; s < len; s += blk) {
        size_t n = len - s < blk ? len - s : blk;
        for (int j = 0; j < k; j++)
            for (int r = 0; r < rows; r++) {
                uint8_t c = coeffs[r * k + j];
#if defined(__x86_64__)
                if (impl == ORC_AVX2)
                    mul_slice_avx2(c, in[j] + s, out[r] + s, n, j > 0);
                else
#endif
                    mul_slice_scalar(c, in[j] + s, out[r] + s, n, j > 0);
            }
    }
}

/* Encode in place: shards[0..k) data, shards[k..k+m) parity, all len bytes. */
int orc_encode(int k, int m, uint8_t *const *shards, size_t len, int impl) {
    uint8_t *mat = (uint8_t *)malloc((size_t)(k + m) * k);
    int rc = orc_build_matrix(k, m, mat);
    if (rc == 0 && m > 0) orc_apply(m, k, mat + k * k, (const uint8_t *const *)shards, shards + k, len, impl);
    free(mat);
    return rc;
}

/* ---------------- synthetic inputs ---------------- */
static inline uint64_t splitmix_next(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_splitmix_fill(uint64_t seed, uint8_t *out, size_t n) {
    uint64_t s = seed;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v = splitmix_next(&s);
        memcpy(out + i, &v, 8); /* little-endian host */
    }
    if (i < n) {
        uint64_t v = splitmix_next(&s);
        memcpy(out + i, &v, n - i);
    }
}

/* object i of a batch: seed ^ (i * golden) */
void orc_fill_objects(uint64_t base_seed, uint64_t first, size_t count, size_t obj_len,
                      size_t obj_stride, uint8_t *out) {
    for (size_t i = 0; i < count; i++)
        orc_splitmix_fill(base_seed ^ ((first + i) * 0x9E3779B97F4A7C15ull), out + i * obj_stride, obj_len);
}

/* ---------------- threaded batch encode (CPU baseline) ---------------- */
typedef struct {
    int k, m, impl;
    const uint8_t *mat;
    const uint8_t *objs;
    size_t obj_len, shard_len;
    uint8_t *parity; /* n * m * shard_len */
    size_t begin, end;
} orc_job;

static void *orc_worker(void *arg) {
    orc_job *j = (orc_job *)arg;
    const uint8_t *in[256];
    uint8_t *out[256];
    for (size_t o = j->begin; o < j->end; o++) {
        for (int d = 0; d < j->k; d++) in[d] = j->objs + o * j->obj_len + (size_t)d * j->shard_len;
        for (int p = 0; p < j->m; p++) out[p] = j->parity + (o * j->m + p) * j->shard_len;
        orc_apply(j->m, j->k, j->mat + j->k * j->k, in, out, j->shard_len, j->impl);
    }
    return NULL;
}

/* Encodes n objects of obj_len bytes laid out back to back (obj_len must be a
 * multiple of k: one stripe per object, the BASELINE configs).  Returns the
 * wall seconds, or a negative value on error. */
double orc_encode_batch(int k, int m, const uint8_t *objs, size_t n, size_t obj_len, uint8_t *parity,
                        int threads, int impl) {
    ensure_init();
    if (k <= 0 || m <= 0 || obj_len % (size_t)k) return -1.0;
    uint8_t mat[256 * 256];
    if (orc_build_matrix(k, m, mat) != 0) return -2.0;
    if (threads < 1) threads = 1;
    if ((size_t)threads > n) threads = (int)(n ? n : 1);
    pthread_t *tid = (pthread_t *)calloc(threads, sizeof(pthread_t));
    orc_job *jobs = (orc_job *)calloc(threads, sizeof(orc_job));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (orc_job){k, m, impl, mat, objs, obj_len, obj_len / k, parity,
                            n * t / threads, n * (t + 1) / threads};
        pthread_create(&tid[t], NULL, orc_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(tid);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ecSplit-style single object, timed (config 1): per call matrix build and a
 * (k+m)*chunk buffer allocation, as objectserver/ecutils.go:27-35 does. */
double orc_ecsplit_once(int k, int m, const uint8_t *obj, size_t len, size_t chunk, int impl, int with_setup) {
    ensure_init();
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint8_t mat[256 * 256];
    static uint8_t smat[256 * 256];
    static int sk = -1, sm = -1;
    uint8_t *buf;
    const uint8_t *mp;
    if (with_setup) {
        orc_build_matrix(k, m, mat);
        mp = mat;
        buf = (uint8_t *)malloc((size_t)(k + m) * chunk);
        memset(buf, 0, (size_t)(k + m) * chunk);
    } else {
        if (sk != k || sm != m) { orc_build_matrix(k, m, smat); sk = k; sm = m; }
        mp = smat;
        buf = (uint8_t *)malloc((size_t)(k + m) * chunk);
    }
    size_t done = 0;
    while (done < len) {
        size_t want = (size_t)k * chunk;
        if (len - done < want) want = len - done;
        memcpy(buf, obj + done, want);
        done += want;
        size_t rd = want;
        while (rd % (size_t)k) buf[rd++] = 0;
        size_t s = rd / k;
        const uint8_t *in[256];
        uint8_t *out[256];
        for (int i = 0; i < k; i++) in[i] = buf + i * s;
        for (int i = 0; i < m; i++) out[i] = buf + (k + i) * s;
        orc_apply(m, k, mp + k * k, in, out, s, impl);
    }
    free(buf);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---------------- threaded batch reconstruct (CPU baseline) ----------------
 * Rebuilds `rows` missing shards of n objects from k survivor shards with the
 * given decode rows (the caller computes them as Encoder.Reconstruct does).
 * Survivor j of object o is at in_base[j] + o*in_stride[j]; output r at
 * out_base[r] + o*out_stride[r]. */
typedef struct {
    int rows, k, impl;
    const uint8_t *coeffs;
    const uint8_t *const *in_base;
    const size_t *in_stride;
    uint8_t *const *out_base;
    const size_t *out_stride;
    size_t len, begin, end;
} orc_rjob;

static void *orc_rworker(void *arg) {
    orc_rjob *j = (orc_rjob *)arg;
    const uint8_t *in[256];
    uint8_t *out[256];
    for (size_t o = j->begin; o < j->end; o++) {
        for (int d = 0; d < j->k; d++) in[d] = j->in_base[d] + o * j->in_stride[d];
        for (int r = 0; r < j->rows; r++) out[r] = j->out_base[r] + o * j->out_stride[r];
        orc_apply(j->rows, j->k, j->coeffs, in, out, j->len, j->impl);
    }
    return NULL;
}

double orc_apply_batch(int rows, int k, const uint8_t *coeffs, const uint8_t *const *in_base,
                       const size_t *in_stride, uint8_t *const *out_base, const size_t *out_stride, size_t n,
                       size_t len, int threads, int impl) {
    ensure_init();
    if (threads < 1) threads = 1;
    if ((size_t)threads > n) threads = (int)(n ? n : 1);
    pthread_t *tid = (pthread_t *)calloc(threads, sizeof(pthread_t));
    orc_rjob *jobs = (orc_rjob *)calloc(threads, sizeof(orc_rjob));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (orc_rjob){rows, k, impl, coeffs, in_base, in_stride, out_base, out_stride, len,
                             n * t / threads, n * (t + 1) / threads};
        pthread_create(&tid[t], NULL, orc_rworker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(tid);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
