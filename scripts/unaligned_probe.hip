// unaligned_probe.hip — tuning aid, not product.  Does gfx950 stream 16-B
// global loads / stores at byte-granular (not 16-B aligned) addresses at the
// aligned rate?  ecSplit's shards sit at base + i*S with S = ceil(len/k)
// (objectserver/ecutils.go:14-35), so 15 object sizes in 16 put them at odd
// offsets.  Kernels:
//   copy  : 1 GiB, dst[i] = src[i] at (src_off, dst_off) byte offsets;
//   xor42 : n databufs of 6 shards (shard j at o*6S + j*S), out[r] = XOR_j in[j]
//           ^ r over the four inputs into shards 4, 5; pipelined like the
//           product's gf_apply_vec_pipe2 (next tile's loads in flight, one
//           block barrier per tile, 1 block of 4 waves per CU);
//           the tail column of each shard is clamped to [S-16, S).
// Prints one JSON line per case: ms, GB/s, % of 8 TB/s, and a byte check.
//   hipcc --offload-arch=gfx950 -O3 scripts/unaligned_probe.hip -o /tmp/uprobe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) const u32x4_u gu_c;
typedef __attribute__((address_space(1))) u32x4_u gu;

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(3);                                                          \
        }                                                                     \
    } while (0)

__device__ __forceinline__ u32x4 ldu(uint64_t a) { return __builtin_nontemporal_load(reinterpret_cast<gu_c*>(a)); }
__device__ __forceinline__ void stu(uint64_t a, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<gu*>(a)); }

__global__ __launch_bounds__(256) void fill(uint8_t* p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * 256) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        reinterpret_cast<uint64_t*>(p)[i] = z ^ (z >> 31);
    }
}

// grid-stride copy, U blocks of 16 B per lane per iteration
template <int U>
__global__ __launch_bounds__(256) void copy_k(uint64_t src, uint64_t dst, uint64_t n16) {
    const uint64_t chunk = (uint64_t)U * 256;
    for (uint64_t b = (uint64_t)blockIdx.x * chunk; b < n16; b += (uint64_t)gridDim.x * chunk) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ldu(src + (b + u * 256 + threadIdx.x) * 16);
#pragma unroll
        for (int u = 0; u < U; ++u) stu(dst + (b + u * 256 + threadIdx.x) * 16, v[u]);
    }
}

struct Tile {
    uint64_t in[4], out[2];  // shard bases
    uint64_t off;            // tile's first shard position
    uint64_t last;           // S - 16: last full column (the clamp)
    uint64_t live;           // S, or 0 for a past-the-end stand-in tile
};

__device__ __forceinline__ void coords(Tile& t, uint64_t base, uint64_t S, uint32_t tpo, uint32_t i, uint32_t n) {
    const uint32_t ii = i < n ? i : n - 1;
    const uint32_t o = ii / tpo;
    const uint64_t off = (uint64_t)(ii - o * tpo) * 1024u;
    const uint64_t ob = base + (uint64_t)o * 6u * S;
#pragma unroll
    for (int j = 0; j < 4; ++j) t.in[j] = ob + (uint64_t)j * S;
#pragma unroll
    for (int r = 0; r < 2; ++r) t.out[r] = ob + (uint64_t)(4 + r) * S;
    t.off = off;
    t.last = S - 16u;
    t.live = i < n ? S : 0u;
}

// lane column = min(off + lane*16, S - 16): the shard's last lane codes [S-16, S)
__device__ __forceinline__ void tload(u32x4 (&x)[4], const Tile& t, uint32_t lane) {
    uint64_t c = t.off + lane * 16u;
    c = c < t.last ? c : t.last;
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = ldu(t.in[j] + c);
}

__device__ __forceinline__ void tstore(const u32x4 (&x)[4], const Tile& t, uint32_t lane) {
    uint64_t c = t.off + lane * 16u;
    const bool st = c < t.live;
    c = c < t.last ? c : t.last;
    u32x4 a = x[0] ^ x[1] ^ x[2] ^ x[3];
    if (st) {
        stu(t.out[0] + c, a);
        a.x ^= 1u;
        stu(t.out[1] + c, a);
    }
}

template <int SLEEP>
__global__ __launch_bounds__(256, 1) void xor42(uint64_t base, uint64_t S, uint32_t tpo, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nb = gridDim.x;
    const uint32_t blk = (nb % 8u == 0u) ? (blockIdx.x % 8u) * (nb / 8u) + blockIdx.x / 8u : blockIdx.x;
    const uint32_t nw = nb * 4;
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(blk * 4);
    const uint32_t dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w0 >= n) return;
    Tile cur, nxt;
    coords(cur, base, S, tpo, w0 + dw, n);
    u32x4 x[4];
    tload(x, cur, lane);
    coords(nxt, base, S, tpo, w0 + dw + nw, n);
    for (uint32_t b0 = w0 + nw; b0 < n; b0 += nw) {
        u32x4 y[4];
        tload(y, nxt, lane);
        if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
        __builtin_amdgcn_s_barrier();
        Tile after;
        coords(after, base, S, tpo, b0 + dw + nw, n);
        tstore(x, cur, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = y[j];
        cur = nxt;
        nxt = after;
    }
    tstore(x, cur, lane);
}

static float time_ms(std::vector<float>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const uint64_t GiB = 1ull << 30;
    int dev_cus = 0;
    CK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *a, *b;
    CK(hipMalloc(&a, GiB + 4096));
    CK(hipMalloc(&b, 7 * GiB));
    hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, a, GiB + 4096);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 15;
    // ---- copy ----
    const int offs[][2] = {{0, 0}, {4, 0}, {0, 4}, {1, 0}, {0, 1}, {3, 7}, {8, 8}, {15, 1}};
    for (int round = 0; round < 2; ++round)
        for (auto& o : offs) {
            const uint64_t n16 = GiB / 16 - 256 * 4;
            std::vector<float> ts;
            for (int r = 0; r < reps + 2; ++r) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(copy_k<4>, dim3(dev_cus * 8), dim3(256), 0, 0, (uint64_t)a + o[0], (uint64_t)b + o[1], n16);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) ts.push_back(ms);
            }
            // check a 1 MiB window at the start and at the end
            bool ok = true;
            std::vector<uint8_t> hs(1 << 20), hd(1 << 20);
            const uint64_t len = n16 * 16;
            for (uint64_t at : {(uint64_t)0, len - (1 << 20)}) {
                CK(hipMemcpy(hs.data(), a + o[0] + at, 1 << 20, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hd.data(), b + o[1] + at, 1 << 20, hipMemcpyDeviceToHost));
                ok = ok && memcmp(hs.data(), hd.data(), 1 << 20) == 0;
            }
            const float ms = time_ms(ts);
            const double gbs = 2.0 * len / (ms * 1e-3) / 1e9;
            printf("{\"case\": \"copy\", \"round\": %d, \"src_off\": %d, \"dst_off\": %d, \"ms\": %.4f, \"GB_s\": %.1f, "
                   "\"frac\": %.4f, \"ok\": %s}\n",
                   round, o[0], o[1], ms, gbs, gbs / 8000.0, ok ? "true" : "false");
            fflush(stdout);
        }
    // ---- xor 4 -> 2 over databufs ----
    const uint64_t Ss[] = {262144, 262143, 262145, 262140, 250001};
    const uint32_t nobj = 4096;
    for (int round = 0; round < 2; ++round)
        for (uint64_t S : Ss)
            for (int boff : {0, 3}) {
                const uint32_t tpo = (uint32_t)((S + 1023) / 1024);
                const uint32_t n = nobj * tpo;
                const uint64_t base = (uint64_t)b + boff;
                hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, b, (uint64_t)nobj * 6 * S + 64);
                std::vector<float> ts;
                for (int r = 0; r < reps + 3; ++r) {
                    CK(hipEventRecord(e0, 0));
                    hipLaunchKernelGGL(xor42<8>, dim3(dev_cus), dim3(256), 0, 0, base, S, tpo, n);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (r >= 3) ts.push_back(ms);
                }
                // check objects 0 and nobj-1
                bool ok = true;
                std::vector<uint8_t> h(6 * S);
                for (uint32_t o : {0u, nobj - 1u}) {
                    CK(hipMemcpy(h.data(), (void*)(base + (uint64_t)o * 6 * S), 6 * S, hipMemcpyDeviceToHost));
                    for (uint64_t p = 0; p < S && ok; ++p) {
                        ok = h[4 * S + p] == (uint8_t)(h[p] ^ h[S + p] ^ h[2 * S + p] ^ h[3 * S + p]);
                    }
                }
                const float ms = time_ms(ts);
                const double nbytes = (double)nobj * 6 * S;
                const double gbs = nbytes / (ms * 1e-3) / 1e9;
                printf("{\"case\": \"xor42 databuf\", \"round\": %d, \"S\": %llu, \"base_off\": %d, \"ms\": %.4f, "
                       "\"GB_s\": %.1f, \"frac\": %.4f, \"ok\": %s}\n",
                       round, (unsigned long long)S, boff, ms, gbs, gbs / 8000.0, ok ? "true" : "false");
                fflush(stdout);
            }
    return 0;
}
