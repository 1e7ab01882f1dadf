// odd.hip — GF(2^8) apply / accumulate / verify over shards at ANY byte
// offset and of ANY length: the shape most real objects take.  ecSplit sets
// S = ceil(len / k) (objectserver/ecutils.go:14-24), a multiple of 16 for one
// object size in 16, and its databuf puts shard i at i*S (ecutils.go:31-35),
// so an arbitrary object's k+m shards start at k+m different byte offsets mod
// 16.  The aligned kernels (kernels.hip) cannot take them.
//
// What the hardware prefers (scripts/unaligned_probe.hip, profiles/r03_unaligned_probe.jsonl):
// 16-B loads and stores at byte-misaligned addresses stream at 52-55 % of
// 8 TB/s for the 4+2 pattern against 70 % aligned, and misaligned STORES cost
// most (a copy loses 11-14 % with misaligned stores, 4-9 % with misaligned
// loads).  So every access here is a 16-B-aligned block, and the shift to a
// common byte frame happens in registers:
//
//  * Frame.  Column i of an object covers shard positions [c_i, c_i + 16),
//    c_i = c0 + 16 i, with c0 = -32 + (-out0 mod 16): output 0's stores are
//    then aligned as they are.  One wave window = 64 consecutive columns; it
//    STORES 62 blocks (the last two lanes only feed their neighbours), and
//    windows step 62 columns = 992 B.
//  * Inputs.  Lane i loads the aligned block of input j holding position c_i
//    (buffer loads: the descriptor's range makes blocks outside the shard read
//    as zero, no clamping), takes lane i+1's block by a DPP lane shift
//    (v_mov_b32_dpp wave_shl:1, no LDS) and shifts its column out of the 32
//    bytes (v_cndmask dword select + v_alignbyte, d_j = (in_j + c0) mod 16
//    wave-uniform).
//  * Outputs.  Output r's aligned blocks sit at positions c_i + delta_r,
//    delta_r = (-(out_r + c0)) mod 16: lane i stores bytes [delta_r, delta_r
//    + 16) of its column and lane i+1's (the same DPP shift), a 16-B-aligned
//    store.  Blocks that straddle the shard's head or tail are stored bytewise
//    (only the first and last window of a shard do that); every output byte
//    has exactly one owner lane, so accumulate passes (k > 8: out ^= ...) read
//    the old block and write it back race-free.
//  * Verify.  The stored parity is loaded and shifted like an input and
//    compared column by column with the recomputed one (bytes outside [0, S)
//    masked); nothing is written but one flag per object.
//
// Schedule: the one of gf_apply_vec_pipe2 — compile-time K <= 8 with the
// coefficient tables hoisted once, one 4-wave block per CU, the next tile's
// loads in flight while the current tile computes and stores, one block
// barrier per tile with a block-uniform trip count (past-the-end waves load a
// stand-in tile and store nothing), XCD-grouped block order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "gf_device.h"
#include "kernels.h"

namespace hbec {

constexpr uint32_t kOddStore = 62;            // blocks stored per 64-lane window
constexpr uint32_t kOddWin = kOddStore * 16;  // shard bytes per window (992)

#ifndef HBEC_ODD_SLEEP
#define HBEC_ODD_SLEEP 0  // x 64 cycles after the next tile's loads
#endif
#ifndef HBEC_ODD_BARRIER
#define HBEC_ODD_BARRIER 1
#endif
#ifndef HBEC_ODD_VMIN
#define HBEC_ODD_VMIN 1  // K*R from which all table words live in VGPRs (1: always)
#endif
#ifndef HBEC_ODD_LB
#define HBEC_ODD_LB 1  // launch_bounds min blocks per CU (register budget)
#endif
#ifndef HBEC_ODD_U_SMALL
#define HBEC_ODD_U_SMALL 0  // windows per wave tile for K <= 4 (0: 4 / K)
#endif
// How a column is shifted into the frame: 1 = through LDS (the block is
// written at lane*16 and read back at lane*16 + d: one ds_write_b128 and one
// unaligned ds_read_b128); 0 = in registers (DPP lane shift, v_cndmask dword
// select, v_alignbyte: ~19 VALU per column).
#ifndef HBEC_ODD_REALIGN
#define HBEC_ODD_REALIGN 1
#endif

enum : int { kOddApply = 0, kOddAcc = 1, kOddVerify = 2 };

// windows per wave tile of the strided kernel: ~4 loads per lane in flight
// for K <= 4 (as gf_apply_vec_pipe2's 1 KiB x 4 / K), one window above
__host__ __device__ constexpr int odd_u(int k) {
    return k <= 4 ? (HBEC_ODD_U_SMALL > 0 ? HBEC_ODD_U_SMALL : (4 / k)) : 1;
}
constexpr int kOddPlanU = 1;  // plans: one window per record

// One tile, wave-uniform.  Positions are 32-bit: the host sends shards of
// 2^31 bytes or more to the round-2 kernels.
template <int K, int R>
struct OddTile {
    uint64_t in[K];   // input shard bases (any alignment)
    uint64_t out[R];  // output (or stored parity) shard bases
    int32_t S;
    int32_t c;        // shard position of the tile's first column (>= -32)
    uint32_t live;    // 0: past-the-end stand-in (loaded, never stored)
    uint32_t obj;     // flag index (verify)
};

__device__ __forceinline__ int32_t odd_c0(uint64_t out0) { return (int32_t)((16u - ((uint32_t)out0 & 15u)) & 15u) - 32; }

// Buffer view of one shard: its 16-B blocks from base & ~15 on; a column's
// block offset may be negative (wraps to huge) or past the end: both read
// as zero, so loads need no clamping.
struct OddSrc {
    __amdgpu_buffer_rsrc_t rs;
    uint64_t base;  // base & ~15 (global-load variant)
    int32_t nb;     // blocks holding shard bytes (global-load variant)
    int32_t g;      // block of the tile's first column
};

__device__ __forceinline__ OddSrc odd_src(uint64_t base, int32_t S, int32_t c) {
    const int32_t l = (int32_t)((uint32_t)base & 15u);
    OddSrc o;
    o.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base & ~(uint64_t)15), (short)0,
                                             (int)((uint32_t)(l + S + 15) & ~15u), 0x00020000);
    o.g = (l + c) >> 4;  // arithmetic: floor for c < 0
    o.base = base & ~(uint64_t)15;
    o.nb = (l + S + 15) >> 4;
    return o;
}

#ifndef HBEC_ODD_GLOBAL
#define HBEC_ODD_GLOBAL 0  // 1: global loads at a clamped block index instead of buffer loads
#endif

__device__ __forceinline__ u32x4 odd_ld(const OddSrc& o, int32_t col) {
    if constexpr (HBEC_ODD_GLOBAL) {
        // blocks outside [0, nb) hold no shard byte: clamp to one that exists
        const int32_t b = __builtin_amdgcn_readfirstlane(o.nb) - 1;
        int32_t i = col + o.g;
        i = i < 0 ? 0 : (i > b ? b : i);
        return ld16_addr(o.base + (uint64_t)(uint32_t)(i * 16));
    } else {
        return __builtin_amdgcn_raw_buffer_load_b128(o.rs, (uint32_t)((col + o.g) * 16), 0, 2 /* nt */);
    }
}

__device__ __forceinline__ uint32_t odd_d(uint64_t base, int32_t c) { return ((uint32_t)base + (uint32_t)c) & 15u; }

typedef __attribute__((address_space(1))) uint8_t gu8_t;

// bytes [lo, hi) of the block v to p (byte stores; head / tail blocks only)
__device__ __forceinline__ void odd_store_part(uint64_t p, const u32x4& v, int32_t lo, int32_t hi) {
    gu8_t* d = reinterpret_cast<gu8_t*>(p);
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (b >= lo && b < hi) d[b] = (uint8_t)(v[b >> 2] >> (8 * (b & 3)));
}

// ---- tile sources ----
// A source names tile t compactly (id(): a few scalars, carried one and two
// tiles ahead) and expands it to shard bases where they are used (at()), so
// the pipeline does not hold three tiles of K + R 64-bit bases in SGPRs.
// Strided batch (PassArgs): tile t = (object t / tpo, tile t % tpo).
struct OddIdS {
    uint32_t obj, ti, live;
};

template <int K, int R, int U>
struct OddStrided {
    using Id = OddIdS;
    const PassArgs& a;
    __device__ __forceinline__ Id id(uint32_t t, uint32_t n) const {
        const uint32_t tt = t < n ? t : n - 1u;
        const uint32_t tpo = a.tiles_per_obj;
        const uint32_t obj = tt / tpo;
        return Id{obj, tt - obj * tpo, t < n ? 1u : 0u};
    }
    __device__ __forceinline__ void at(OddTile<K, R>& b, const Id& i) const {
#pragma unroll
        for (int j = 0; j < K; ++j) b.in[j] = reinterpret_cast<uint64_t>(a.in[j]) + (uint64_t)i.obj * a.in_stride[j];
#pragma unroll
        for (int r = 0; r < R; ++r) b.out[r] = reinterpret_cast<uint64_t>(a.out[r]) + (uint64_t)i.obj * a.out_stride[r];
        b.S = (int32_t)a.shard_len;
        b.c = odd_c0(b.out[0]) + (int32_t)(i.ti * (uint32_t)(U * kOddWin));
        b.live = i.live;
        b.obj = i.obj;
    }
};

// Plan records (URec): input j of the record's stripe at (bit j of in_sel ?
// b : a) + in_idx[j] * S; rec.p0 = the record's first window * 992.
struct OddIdP {
    URec rec;
    uint32_t live;
};

template <int K, int R>
struct OddPlan {
    using Id = OddIdP;
    const UPlanArgs& p;
    const URec* __restrict__ recs;
    __device__ __forceinline__ Id id(uint32_t t, uint32_t n) const { return Id{recs[t < n ? t : n - 1u], t < n ? 1u : 0u}; }
    __device__ __forceinline__ void at(OddTile<K, R>& b, const Id& i) const {
        const uint64_t S = i.rec.shard_len;
#pragma unroll
        for (int j = 0; j < K; ++j) b.in[j] = (((p.in_sel >> j) & 1u) ? i.rec.b : i.rec.a) + (uint64_t)p.in_idx[j] * S;
#pragma unroll
        for (int r = 0; r < R; ++r)
            b.out[r] = (((p.out_sel >> r) & 1u) ? i.rec.b : i.rec.a) + (uint64_t)p.out_idx[r] * S;
        b.S = (int32_t)S;
        b.c = odd_c0(b.out[0]) + (int32_t)i.rec.p0;
        b.live = i.live;
        b.obj = 0;
    }
};

// ---- shifting a column into the frame ----
// LDS staging: per wave, one 1 KiB + 32 B slot per shard that is shifted.
constexpr uint32_t kOddSlot = 1024 + 32;

template <int NS>
struct OddLds {
    uint8_t* base;  // this wave's NS slots
};

// block v of lane l -> bytes [d, d + 16) of (v of lane l ++ v of lane l+1)
template <int NS>
__device__ __forceinline__ void odd_put(const OddLds<NS>& L, int slot, uint32_t lane, const u32x4& v) {
    *reinterpret_cast<u32x4*>(L.base + slot * kOddSlot + lane * 16u) = v;
}
typedef u32x4 u32x4_u1 __attribute__((aligned(1)));
template <int NS>
__device__ __forceinline__ u32x4 odd_get(const OddLds<NS>& L, int slot, uint32_t lane, uint32_t d) {
    return *reinterpret_cast<const u32x4_u1*>(L.base + slot * kOddSlot + lane * 16u + d);
}

// ---- one tile ----
template <int K, int R, int U, int MODE>
struct OddRegs {
    static constexpr int NL = K + (MODE == kOddVerify ? R : 0);  // shards loaded per column
    u32x4 x[U][NL];
};

template <int K, int R, int U, int MODE>
__device__ __forceinline__ void odd_load(OddRegs<K, R, U, MODE>& X, const OddTile<K, R>& b, uint32_t lane) {
    OddSrc src[OddRegs<K, R, U, MODE>::NL];
#pragma unroll
    for (int j = 0; j < K; ++j) src[j] = odd_src(b.in[j], b.S, b.c);
    if constexpr (MODE == kOddVerify) {
#pragma unroll
        for (int r = 0; r < R; ++r) src[K + r] = odd_src(b.out[r], b.S, b.c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < OddRegs<K, R, U, MODE>::NL; ++j)
            X.x[u][j] = odd_ld(src[j], (int32_t)(u * kOddStore + lane));
}

// LDS slots per wave: K inputs (+ R stored parity for verify, + R outputs)
template <int K, int R, int MODE>
__host__ __device__ constexpr int odd_slots() { return K + R; }

template <int K, int R, int U, int MODE>
__device__ __forceinline__ void odd_finish(const OddRegs<K, R, U, MODE>& X, const OddTile<K, R>& b,
                                           const TabArray& tab, const Tables<K, R, HBEC_ODD_VMIN>& tb, uint32_t lane,
                                           uint32_t* flags, const OddLds<odd_slots<K, R, MODE>()>& L) {
    uint32_t d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) d[j] = __builtin_amdgcn_readfirstlane(odd_d(b.in[j], b.c));
    const int32_t S = b.S;
    bool bad = false;
    OddSrc old[MODE == kOddAcc ? R : 1];
    uint32_t dl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        dl[r] = __builtin_amdgcn_readfirstlane((16u - odd_d(b.out[r], b.c)) & 15u);
        if constexpr (MODE == kOddAcc) old[r] = odd_src(b.out[r], S, b.c + (int32_t)dl[r]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int32_t w0 = b.c + (int32_t)(u * kOddWin);  // window's first column
        const int32_t cpos = w0 + 16 * (int32_t)lane;
        // window-uniform: every block this window stores (or compares) lies inside [0, S)
        const bool interior = w0 >= 0 && w0 + (int32_t)kOddWin + 16 <= S;
        u32x4 x[K];
        if constexpr (HBEC_ODD_REALIGN == 1) {
#pragma unroll
            for (int j = 0; j < K; ++j) odd_put(L, j, lane, X.x[u][j]);
            if constexpr (MODE == kOddVerify) {
#pragma unroll
                for (int r = 0; r < R; ++r) odd_put(L, K + r, lane, X.x[u][K + r]);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = odd_get(L, j, lane, d[j]);
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = realign16(X.x[u][j], lane_next4(X.x[u][j]), d[j]);
        }
        u32x4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
        gf_dot<K, R, HBEC_ODD_VMIN>(acc, x, tab, tb);
        if constexpr (MODE == kOddVerify) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t dp = __builtin_amdgcn_readfirstlane(odd_d(b.out[r], b.c));
                u32x4 st;
                if constexpr (HBEC_ODD_REALIGN == 1)
                    st = odd_get(L, K + r, lane, dp);
                else
                    st = realign16(X.x[u][K + r], lane_next4(X.x[u][K + r]), dp);
                const u32x4 df = st ^ acc[r];
                if (interior) {
                    bad |= lane < kOddStore && (df[0] | df[1] | df[2] | df[3]) != 0u;
                } else if (lane < kOddStore) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        // bytes of dword e at positions cpos + 4e .. + 3 that lie in [0, S)
                        uint32_t m = 0;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int32_t pos = cpos + 4 * e + q;
                            m |= (pos >= 0 && pos < S) ? (0xFFu << (8 * q)) : 0u;
                        }
                        bad |= (df[e] & m) != 0u;
                    }
                }
            }
        } else {
            u32x4 blk[R];
            if constexpr (HBEC_ODD_REALIGN == 1) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (dl[r] != 0u) odd_put(L, K + r, lane, acc[r]);  // wave-uniform (r = 0 never)
#pragma unroll
                for (int r = 0; r < R; ++r) blk[r] = dl[r] == 0u ? acc[r] : odd_get(L, K + r, lane, dl[r]);
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (dl[r] == 0u)  // wave-uniform: output r is in the frame (always r = 0)
                        blk[r] = acc[r];
                    else
                        blk[r] = realign16(acc[r], lane_next4(acc[r]), dl[r]);
                }
            }
            if constexpr (MODE == kOddAcc) {
#pragma unroll
                for (int r = 0; r < R; ++r) blk[r] ^= odd_ld(old[r], (int32_t)(u * kOddStore + lane));
            }
            if (b.live != 0u) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int32_t q = cpos + (int32_t)dl[r];  // block start: out[r] + q is 16-B aligned
                    const uint64_t p = b.out[r] + (uint64_t)(int64_t)q;
                    if (interior) {
                        if (lane < kOddStore) st16_addr(p, blk[r]);
                    } else if (lane < kOddStore && q < S && q + 16 > 0) {
                        if (q >= 0 && q + 16 <= S)
                            st16_addr(p, blk[r]);
                        else
                            odd_store_part(p, blk[r], q < 0 ? -q : 0, q + 16 > S ? S - q : 16);
                    }
                }
            }
        }
    }
    if constexpr (MODE == kOddVerify) {
        if (b.live != 0u && __any(bad)) {
            if (lane == 0u) atomicOr(flags + b.obj, 1u);
        }
    }
}

template <int K, int R, int U, int MODE, class Src>
__device__ __forceinline__ void odd_body(const Src& src, uint32_t n, const TabArray& tab, uint32_t* flags) {
    constexpr uint32_t WPB = kPipeBlockThreads / 64;
    constexpr int NS = odd_slots<K, R, MODE>();
    __shared__ __attribute__((aligned(16))) uint8_t lds[HBEC_ODD_REALIGN == 1 ? WPB * NS * kOddSlot : 16];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * WPB;
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(xcd_block() * WPB);  // the block's first wave
    const uint32_t dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave0 >= n) return;  // whole blocks only: the loop below has block barriers
    const OddLds<NS> L{lds + (HBEC_ODD_REALIGN == 1 ? dw * NS * kOddSlot : 0)};
    const Tables<K, R, HBEC_ODD_VMIN> tb = load_tables<K, R, HBEC_ODD_VMIN>(tab);
    typename Src::Id cur = src.id(wave0 + dw, n);
    OddRegs<K, R, U, MODE> X;
    {
        OddTile<K, R> b;
        src.at(b, cur);
        odd_load<K, R, U, MODE>(X, b, lane);
    }
    typename Src::Id nxt = src.id(wave0 + dw + nw, n);
    for (uint32_t b0 = wave0 + nw; b0 < n; b0 += nw) {  // block-uniform trip count
        OddRegs<K, R, U, MODE> Y;
        {
            OddTile<K, R> b;
            src.at(b, nxt);
            odd_load<K, R, U, MODE>(Y, b, lane);
        }
        if (HBEC_ODD_SLEEP > 0) __builtin_amdgcn_s_sleep(HBEC_ODD_SLEEP);
        if (HBEC_ODD_BARRIER) __builtin_amdgcn_s_barrier();
        const typename Src::Id after = src.id(b0 + dw + nw, n);
        {
            OddTile<K, R> b;
            src.at(b, cur);
            odd_finish<K, R, U, MODE>(X, b, tab, tb, lane, flags, L);
        }
        X = Y;
        cur = nxt;
        nxt = after;
    }
    OddTile<K, R> b;
    src.at(b, cur);
    odd_finish<K, R, U, MODE>(X, b, tab, tb, lane, flags, L);
}

template <int K, int R, int MODE>
__global__ __launch_bounds__(kPipeBlockThreads, HBEC_ODD_LB) void gf_odd(PassArgs a, uint32_t* flags) {
    constexpr int U = odd_u(K);
    odd_body<K, R, U, MODE>(OddStrided<K, R, U>{a}, a.n_tiles, a.tab, flags);
}

template <int K, int R, int MODE>
__global__ __launch_bounds__(kPipeBlockThreads, HBEC_ODD_LB) void gf_odd_plan(UPlanArgs p, const URec* __restrict__ recs) {
    odd_body<K, R, kOddPlanU, MODE>(OddPlan<K, R>{p, recs}, p.n_recs, p.tab, nullptr);
}

// ---------------------------------------------------------------------------
// launch table
// ---------------------------------------------------------------------------
template <int K, int MODE>
static const void* odd_for_r(int r, bool plan) {
    switch (r) {
        case 1: return plan ? (const void*)&gf_odd_plan<K, 1, MODE> : (const void*)&gf_odd<K, 1, MODE>;
        case 2: return plan ? (const void*)&gf_odd_plan<K, 2, MODE> : (const void*)&gf_odd<K, 2, MODE>;
        case 3: return plan ? (const void*)&gf_odd_plan<K, 3, MODE> : (const void*)&gf_odd<K, 3, MODE>;
        case 4: return plan ? (const void*)&gf_odd_plan<K, 4, MODE> : (const void*)&gf_odd<K, 4, MODE>;
    }
    return nullptr;
}

template <int MODE>
static const void* odd_kernel_(int k, int r, bool plan) {
    switch (k) {
        case 1: return odd_for_r<1, MODE>(r, plan);
        case 2: return odd_for_r<2, MODE>(r, plan);
        case 3: return odd_for_r<3, MODE>(r, plan);
        case 4: return odd_for_r<4, MODE>(r, plan);
        case 5: return odd_for_r<5, MODE>(r, plan);
        case 6: return odd_for_r<6, MODE>(r, plan);
        case 7: return odd_for_r<7, MODE>(r, plan);
        case 8: return odd_for_r<8, MODE>(r, plan);
    }
    return nullptr;
}

static const void* odd_kernel(int k, int r, int mode, bool plan) {
    if (plan && mode == kOddVerify) return nullptr;
    switch (mode) {
        case kOddApply: return odd_kernel_<kOddApply>(k, r, plan);
        case kOddAcc: return odd_kernel_<kOddAcc>(k, r, plan);
        case kOddVerify: return odd_kernel_<kOddVerify>(k, r, plan);
    }
    return nullptr;
}

#ifndef HBEC_ODD_DEFAULT
#define HBEC_ODD_DEFAULT 0  // until gf_odd beats the round-2 kernels on every odd shape
#endif
bool odd_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("HBEC_ODD");
        return e ? e[0] != '0' : HBEC_ODD_DEFAULT != 0;
    }();
    return on;
}

#ifndef HBEC_ODD_BPC_DEFAULT
#define HBEC_ODD_BPC_DEFAULT 1
#endif
int odd_blocks_per_cu() {
    static const int v = [] {
        const char* e = std::getenv("HBEC_ODD_BPC");
        const int x = e ? std::atoi(e) : 0;
        return x > 0 ? x : HBEC_ODD_BPC_DEFAULT;
    }();
    return v;
}

uint64_t urec_tile() { return odd_enabled() ? (uint64_t)kOddPlanU * kOddWin : (uint64_t)unaligned_tile_bytes(); }
uint64_t urec_span(uint64_t shard_len) { return odd_enabled() ? shard_len + 32u : shard_len; }

uint32_t odd_tile_bytes(int k) { return (uint32_t)odd_u(k) * kOddWin; }
uint32_t odd_plan_tile_bytes() { return (uint32_t)kOddPlanU * kOddWin; }

// Tiles per shard: enough windows for every output block of the shard, from
// the frame's first column (c0 >= -32) to position S.
uint32_t odd_tiles_per_obj(int k, uint64_t shard_len) {
    const uint64_t span = shard_len + 32u;
    const uint64_t tile = odd_tile_bytes(k);
    return (uint32_t)((span + tile - 1) / tile);
}

bool odd_supported(int k, int r) { return k >= 1 && k <= kOddMaxK && r >= 1 && r <= kMaxR; }

hipError_t launch_odd(int k, int r, int mode, const PassArgs& a, uint32_t* flags, int grid, hipStream_t stream) {
    const void* fn = odd_kernel(k, r, mode, false);
    if (!fn) return hipErrorInvalidValue;
    void* args[] = {const_cast<PassArgs*>(&a), &flags};
    return hipLaunchKernel(fn, dim3(grid), dim3(kPipeBlockThreads), args, 0, stream);
}

hipError_t launch_odd_plan(int k, int r, int mode, const UPlanArgs& p, int grid, hipStream_t stream) {
    const void* fn = odd_kernel(k, r, mode, true);
    if (!fn) return hipErrorInvalidValue;
    const URec* recs = p.recs;
    void* args[] = {const_cast<UPlanArgs*>(&p), &recs};
    return hipLaunchKernel(fn, dim3(grid), dim3(kPipeBlockThreads), args, 0, stream);
}

}  // namespace hbec
