// gf_device.h — device-side GF(2^8) building blocks shared by the gfx950
// kernels (kernels.hip, stripes.hip): 16-B streaming loads/stores, the
// v_perm_b32 field multiply (3-bit/3-bit/2-bit split of each byte) and the
// v_bitop3 XOR3 folding.  See kernels.hip for the scheme.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"
#include "tuning.h"

namespace hbec {

// Workgroups are dispatched round-robin over MI355X's 8 XCDs (block b runs on
// XCD b % 8).  Renumber them so the blocks resident on one XCD take adjacent
// tiles of every grid-stride front (one contiguous run per XCD and L2).
// 8+3: +1.4-1.8 %, 4+2: +0.3-0.5 % vs. the raw block id (profiles/r01_tune_xcd.jsonl).
__device__ __forceinline__ uint32_t xcd_block() {
    const uint32_t nb = gridDim.x;
    return (nb % 8u == 0u) ? (blockIdx.x % 8u) * (nb / 8u) + blockIdx.x / 8u : blockIdx.x;
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    // v_perm_b32: byte i of result = byte sel.u8[i] of the 64-bit {hi, lo}
    // (selector 0-3 -> lo, 4-7 -> hi).
    return __builtin_amdgcn_perm(hi, lo, sel);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Shard streams are touched once: non-temporal loads and stores (plain ones
// lost 2-3 %, profiles/r01_tune_*.jsonl).
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// Global-address-space (addrspace 1) views for addresses built from integers
// (tile records): without them hipcc emits flat_* ops, which complete out of
// order and force vmcnt(0)/lgkmcnt(0) waits.
typedef __attribute__((address_space(1))) const u32x4 gu32x4_c;
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ u32x4 ld16_addr(uint64_t addr) {
    return __builtin_nontemporal_load(reinterpret_cast<gu32x4_c*>(addr));
}

// plain (temporal) load: lines another wave reads next stay in L2
__device__ __forceinline__ u32x4 ld16_addr_t(uint64_t addr) { return *reinterpret_cast<gu32x4_c*>(addr); }

__device__ __forceinline__ void st16_addr(uint64_t addr, u32x4 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<gu32x4*>(addr));
}

// Lane l receives lane l+1's value (DPP wave_shl:1, a VALU move; lane 63
// gets 0).  Replaces ds_bpermute, which goes through the LDS pipe.
__device__ __forceinline__ uint32_t lane_next(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}

__device__ __forceinline__ u32x4 lane_next4(const u32x4& v) {
    return u32x4{lane_next(v[0]), lane_next(v[1]), lane_next(v[2]), lane_next(v[3])};
}

// Bytes [d, d + 16) of the 32 bytes lo:hi, d wave-uniform in [0, 16): the
// 5 source dwords are selected by d's bits 3 and 2 (v_cndmask on a uniform
// condition), then v_alignbyte_b32(a, b, s) = ({a, b} >> 8s)[31:0] shifts.
__device__ __forceinline__ u32x4 realign16(const u32x4& lo, const u32x4& hi, uint32_t d) {
    const uint32_t sh = d & 3u;
    const bool b2 = (d & 8u) != 0, b1 = (d & 4u) != 0;
    const uint32_t t0 = b2 ? lo[2] : lo[0], t1 = b2 ? lo[3] : lo[1], t2 = b2 ? hi[0] : lo[2];
    const uint32_t t3 = b2 ? hi[1] : lo[3], t4 = b2 ? hi[2] : hi[0], t5 = b2 ? hi[3] : hi[1];
    const uint32_t s0 = b1 ? t1 : t0, s1 = b1 ? t2 : t1, s2 = b1 ? t3 : t2, s3 = b1 ? t4 : t3, s4 = b1 ? t5 : t4;
    return u32x4{__builtin_amdgcn_alignbyte(s1, s0, sh), __builtin_amdgcn_alignbyte(s2, s1, sh),
                 __builtin_amdgcn_alignbyte(s3, s2, sh), __builtin_amdgcn_alignbyte(s4, s3, sh)};
}

struct Sel {
    uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel selectors(uint32_t x) {
    Sel s;
    s.s0 = x & 0x07070707u;
    s.s1 = (x >> 3) & 0x07070707u;
    s.s2 = (x >> 6) & 0x03030303u;
    return s;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

__device__ __forceinline__ uint32_t gf_mul_sel(const Sel& s, uint32_t t0, uint32_t t1, uint32_t t2,
                                               uint32_t t3, uint32_t t4) {
    return perm(t1, t0, s.s0) ^ perm(t3, t2, s.s1) ^ perm(t4, t4, s.s2);
}

// Coefficient tables of one pass.  v_perm_b32 may read only one SGPR (GFX9
// constant-bus limit), so the low halves t[0] and t[2] are copied to VGPRs
// once per kernel instead of by a v_mov before every perm; from K*R =
// HBEC_ALLVGPR_MIN (tuning.h) the high words too (SGPR spills otherwise).

// VMIN: K*R at or above which the high words live in VGPRs too (kernels
// with many scalar live values pass 1: all five words in VGPRs)
template <int K, int R, int VMIN = HBEC_ALLVGPR_MIN>
struct Tables {
    static constexpr bool kAllV = K * R >= VMIN;
    uint32_t lo0[R][K];
    uint32_t lo2[R][K];
    uint32_t hi[kAllV ? R : 1][kAllV ? K : 1][3];
};

__device__ __forceinline__ uint32_t to_vgpr(uint32_t x) {
    uint32_t r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}

typedef uint32_t TabArray[kMaxR][kMaxK][5];

template <int K, int R, int VMIN = HBEC_ALLVGPR_MIN>
__device__ __forceinline__ Tables<K, R, VMIN> load_tables(const TabArray& tab) {
    Tables<K, R, VMIN> t;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j) {
            t.lo0[r][j] = to_vgpr(tab[r][j][0]);
            t.lo2[r][j] = to_vgpr(tab[r][j][2]);
            if constexpr (Tables<K, R, VMIN>::kAllV) {
                t.hi[r][j][0] = to_vgpr(tab[r][j][1]);
                t.hi[r][j][1] = to_vgpr(tab[r][j][3]);
                t.hi[r][j][2] = to_vgpr(tab[r][j][4]);
            }
        }
    return t;
}

// acc[r] ^= XOR_j C[r][j] * x[j] for one 16-B column of K inputs.  The 3K
// perm terms per (row, dword) are folded by v_bitop3 XOR3s; a pending odd
// term is carried so every XOR3 retires two terms.
template <int K, int R, int VMIN = HBEC_ALLVGPR_MIN>
__device__ __forceinline__ void gf_dot(u32x4 (&acc)[R], const u32x4 (&x)[K], const TabArray& tab,
                                       const Tables<K, R, VMIN>& tb) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        uint32_t pend[R];
        bool has = false;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const Sel sx = selectors(x[j][e]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                uint32_t h1, h3, h4;
                if constexpr (Tables<K, R, VMIN>::kAllV) {
                    h1 = tb.hi[r][j][0];
                    h3 = tb.hi[r][j][1];
                    h4 = tb.hi[r][j][2];
                } else {
                    h1 = tab[r][j][1];
                    h3 = tab[r][j][3];
                    h4 = tab[r][j][4];
                }
                const uint32_t p0 = perm(h1, tb.lo0[r][j], sx.s0);
                const uint32_t p1 = perm(h3, tb.lo2[r][j], sx.s1);
                const uint32_t p2 = perm(h4, h4, sx.s2);
                if (!has) {
                    acc[r][e] = xor3(acc[r][e], p0, p1);
                    pend[r] = p2;
                } else {
                    acc[r][e] = xor3(acc[r][e], pend[r], p0);
                    acc[r][e] = xor3(acc[r][e], p1, p2);
                }
            }
            has = !has;
        }
        if (has) {
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][e] ^= pend[r];
        }
    }
}

// ---- Packed coordinates (gf_apply_packed, gf_verify_packed) ----
// Element e (16 B) of the concatenated shard columns of all objects is byte
// (e % spo)*16 of object e / spo (spo = shard_len / 16).  Lanes past n_elems
// are clamped to the last element: they load live bytes and store / flag
// nothing.
template <int U>
struct PackedCoord {
    uint32_t obj[U];  // per lane
    uint32_t off[U];  // per lane: byte offset inside the shard
};

template <int U>
__device__ __forceinline__ void packed_coords(PackedCoord<U>& c, uint32_t t, uint32_t lane, uint32_t n_elems,
                                              uint32_t spo, double inv) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint32_t e = (t * (uint32_t)U + (uint32_t)u) * 64u + lane;
        e = e < n_elems ? e : n_elems - 1u;  // clamped lanes load live bytes, store nothing
        uint32_t q = (uint32_t)((double)e * inv);  // e < 2^31: exact up to one step, fixed below
        int32_t r = (int32_t)(e - q * spo);
        if (r < 0) {
            q -= 1u;
            r += (int32_t)spo;
        } else if (r >= (int32_t)spo) {
            q += 1u;
            r -= (int32_t)spo;
        }
        c.obj[u] = q;
        c.off[u] = (uint32_t)r * 16u;
    }
}

}  // namespace hbec
