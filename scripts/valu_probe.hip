// valu_probe.hip — issue cost of the bit-plane field multiply against the
// v_perm table multiply, in registers only (no memory in the loop): one wave
// per SIMD, s_memtime around ITERS rounds; prints cycles per round.  The
// static VALU count per round comes from the ISA (--save-temps).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I hummingbird_amd/csrc scripts/valu_probe.hip -o /tmp/valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "odd_impl.h"

using namespace hbec;

constexpr int ITERS = 256;

template <int XS, int K, int R>
__global__ __launch_bounds__(256, 1) void probe_bp(uint32_t* out, uint64_t* cyc) {
    u32x4 x0[K], x1[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        x0[j] = u32x4{threadIdx.x * 7u + j, threadIdx.x ^ (j * 13u), threadIdx.x + 99u * j, j * 0x01010101u};
        x1[j] = x0[j] ^ u32x4{0x5A5A5A5Au, 3u, 5u, 7u};
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
        u32x4 a0[R], a1[R];
        bp_dot2<XS, K, R>(a0, a1, x0, x1);
#pragma unroll
        for (int j = 0; j < K; ++j) {  // every input changes every round (nothing hoisted)
            x0[j] ^= a0[j % R];
            x1[j] ^= a1[j % R];
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) v ^= x0[j][0] ^ x0[j][1] ^ x1[j][2] ^ x1[j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K, int R>
__global__ __launch_bounds__(256, 1) void probe_perm(uint32_t* out, uint64_t* cyc, PassArgs a) {
    u32x4 x0[K], x1[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        x0[j] = u32x4{threadIdx.x * 7u + j, threadIdx.x ^ (j * 13u), threadIdx.x + 99u * j, j * 0x01010101u};
        x1[j] = x0[j] ^ u32x4{0x5A5A5A5Au, 3u, 5u, 7u};
    }
    const Tables<K, R, 1> tb = load_tables<K, R, 1>(a.tab);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
        u32x4 a0[R], a1[R];
#pragma unroll
        for (int r = 0; r < R; ++r) a0[r] = a1[r] = u32x4{0, 0, 0, 0};
        gf_dot<K, R, 1>(a0, x0, a.tab, tb);
        gf_dot<K, R, 1>(a1, x1, a.tab, tb);
#pragma unroll
        for (int j = 0; j < K; ++j) {  // every input changes every round (nothing hoisted)
            x0[j] ^= a0[j % R];
            x1[j] ^= a1[j % R];
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) v ^= x0[j][0] ^ x0[j][1] ^ x1[j][2] ^ x1[j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// transposes only (8 K + 8 R dwords per round)
template <int K, int R>
__global__ __launch_bounds__(256, 1) void probe_tr(uint32_t* out, uint64_t* cyc) {
    uint32_t d[K + R][8];
#pragma unroll
    for (int j = 0; j < K + R; ++j)
#pragma unroll
        for (int b = 0; b < 8; ++b) d[j][b] = threadIdx.x * (j + 3u) + b * 0x01010101u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int j = 0; j < K + R; ++j) {
            bp_transpose8(d[j]);
            d[j][0] ^= d[(j + 1) % (K + R)][7];
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < K + R; ++j)
#pragma unroll
        for (int b = 0; b < 8; ++b) v ^= d[j][b];
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static double median_cyc(uint64_t* h, int n) {
    std::sort(h, h + n);
    return (double)h[n / 2] / ITERS;
}

int main() {
    uint32_t* out;
    uint64_t* cyc;
    const int blocks = 256;
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&cyc, blocks * 8);
    uint64_t h[blocks];
    PassArgs a;
    memset(&a, 0, sizeof(a));
    for (int r = 0; r < kMaxR; ++r)
        for (int j = 0; j < kMaxK; ++j)
            for (int q = 0; q < 5; ++q) a.tab[r][j][q] = 0x01020304u * (r + 1) + j * 0x11111111u + q;
    auto run = [&](const char* name, auto launch) {
        for (int rep = 0; rep < 3; ++rep) launch();
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("{\"probe\": \"%s\", \"cycles_per_round\": %.1f}\n", name, median_cyc(h, blocks));
    };
    run("bp 8+3", [&] { probe_bp<2, 8, 3><<<blocks, 256>>>(out, cyc); });
    run("perm 8+3 (2 columns)", [&] { probe_perm<8, 3><<<blocks, 256>>>(out, cyc, a); });
    run("transposes 8+3", [&] { probe_tr<8, 3><<<blocks, 256>>>(out, cyc); });
    run("bp 10+4", [&] { probe_bp<5, 10, 4><<<blocks, 256>>>(out, cyc); });
    run("perm 10+4 (2 columns)", [&] { probe_perm<10, 4><<<blocks, 256>>>(out, cyc, a); });
    run("transposes 10+4", [&] { probe_tr<10, 4><<<blocks, 256>>>(out, cyc); });
    run("bp 4+2", [&] { probe_bp<9, 4, 2><<<blocks, 256>>>(out, cyc); });
    run("perm 4+2 (2 columns)", [&] { probe_perm<4, 2><<<blocks, 256>>>(out, cyc, a); });
    return 0;
}
