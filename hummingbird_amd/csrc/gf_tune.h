// gf_tune.h — tuning-only device code, compiled into the kernels only when a
// tuning build defines HBEC_GF_LDS (scripts/tune.py; profiles/r01_tune_lds.jsonl).
// The product multiply (gf_device.h) keeps every table in registers.
#pragma once
#include "gf_device.h"

namespace hbec {

// ---- Tuning only: field multiply through LDS tables (HBEC_GF_LDS) ----
// The default multiply above keeps every table in registers (v_perm_b32).
// These variants exist to measure the classic alternatives on the same
// kernel (profiles/r01_tune_lds.jsonl):
//   1: one 256-B product table c*x per coefficient (K*R*256 B of LDS), one
//      ds_read_u8 per byte per output row;
//   2: log / antilog tables (c*x = exp[log c + log x]), log[0] and log 0 =
//      511 and exp[>= 510] = 0 so zero needs no branch; one ds_read_u16 per
//      input byte plus one ds_read_u8 per byte per output row.
#ifndef HBEC_GF_LDS
#define HBEC_GF_LDS 0
#endif

__host__ __device__ constexpr int gf_lds_bytes(int k, int r) {
    return HBEC_GF_LDS == 1 ? k * r * 256 : (HBEC_GF_LDS == 2 ? 512 + 1024 : 16);
}

template <int K, int R>
struct LdsGf {
    const uint8_t* lt;
    uint32_t logc[R][K];
};

// All threads of the block build the tables, then one barrier: call before
// any wave of the block can leave the kernel.
template <int K, int R>
__device__ LdsGf<K, R> gf_lds_init(uint8_t* lt, const TabArray& tab) {
    LdsGf<K, R> g;
    g.lt = lt;
#if HBEC_GF_LDS == 1
    for (uint32_t i = threadIdx.x; i < (uint32_t)(K * R * 256); i += blockDim.x) {
        const uint32_t rj = i >> 8, x = i & 255u, r = rj / K, j = rj % K;
        const uint32_t* t = tab[r][j];
        lt[i] = (uint8_t)(perm(t[1], t[0], x & 7u) ^ perm(t[3], t[2], (x >> 3) & 7u) ^ perm(t[4], t[4], x >> 6));
    }
    __syncthreads();
#elif HBEC_GF_LDS == 2
    uint16_t* lg = reinterpret_cast<uint16_t*>(lt);
    uint8_t* ex = lt + 512;
    for (uint32_t i = threadIdx.x; i < 1024u; i += blockDim.x) {
        uint32_t p = 0;
        if (i < 510u) {
            p = 1;
            for (uint32_t e = i % 255u; e; --e) p = (p << 1) ^ ((p & 0x80u) ? 0x11Du : 0u);
            if (i < 255u) lg[p] = (uint16_t)i;
        }
        ex[i] = (uint8_t)p;
    }
    if (threadIdx.x == 0) lg[0] = 511;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t c = (tab[r][j][0] >> 8) & 0xFFu;  // c * 1: byte 1 of the low field table
            g.logc[r][j] = c ? __builtin_amdgcn_readfirstlane((uint32_t)lg[c]) : 511u;
        }
#endif
    return g;
}

template <int K, int R>
__device__ __forceinline__ void gf_dot_lds(u32x4 (&acc)[R], const u32x4 (&x)[K], const LdsGf<K, R>& g) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint32_t w = x[j][e];
#if HBEC_GF_LDS == 2
            const uint16_t* lg = reinterpret_cast<const uint16_t*>(g.lt);
            const uint8_t* ex = g.lt + 512;
            const uint32_t l0 = lg[w & 255u], l1 = lg[(w >> 8) & 255u], l2 = lg[(w >> 16) & 255u], l3 = lg[w >> 24];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t lc = g.logc[r][j];
                acc[r][e] ^= (uint32_t)ex[l0 + lc] | ((uint32_t)ex[l1 + lc] << 8) | ((uint32_t)ex[l2 + lc] << 16) |
                             ((uint32_t)ex[l3 + lc] << 24);
            }
#else
            const uint32_t b0 = w & 255u, b1 = (w >> 8) & 255u, b2 = (w >> 16) & 255u, b3 = w >> 24;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint8_t* t = g.lt + (r * K + j) * 256;
                acc[r][e] ^= (uint32_t)t[b0] | ((uint32_t)t[b1] << 8) | ((uint32_t)t[b2] << 16) | ((uint32_t)t[b3] << 24);
            }
#endif
        }
    }
}

}  // namespace hbec
