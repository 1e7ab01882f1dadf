// odd.hip — GF(2^8) apply / accumulate / verify over shards at ANY byte
// offset and of ANY length: the shape most real objects take.  ecSplit sets
// S = ceil(len / k) (objectserver/ecutils.go:14-24), a multiple of 16 for one
// object size in 16, and its databuf puts shard i at i*S (ecutils.go:31-35),
// so an arbitrary object's k+m shards start at k+m different byte offsets mod
// 16.  The aligned kernels (kernels.hip) cannot take them.
//
// What the hardware prefers (scripts/unaligned_probe.hip, profiles/r03_unaligned_probe.jsonl):
// 16-B loads and stores at byte-misaligned addresses stream at 52-55 % of
// 8 TB/s for the 4+2 pattern against 70 % aligned; a copy loses 4.5 % with
// dword-aligned (not 16-B-aligned) loads, 9 % with byte-misaligned loads and
// 11-14 % with misaligned stores.  So:
//
//  * Frame.  Column i of an object covers shard positions [c_i, c_i + 16),
//    c_i = c0 + 16 i, with c0 = -32 + (-out0 mod 16): output 0's blocks are
//    16-B aligned as they are.  One wave window = 64 consecutive columns; it
//    STORES 62 blocks (the last two lanes only feed their neighbours), and
//    windows step 62 columns = 992 B.
//  * Inputs are loaded as dword-aligned 16-B blocks (the block holding the
//    column's first byte, rounded down to a dword): the column is then bytes
//    [sh, sh + 16) of the lane's block and lane l+1's first dword, one DPP
//    lane shift (v_mov_b32_dpp wave_shl:1) and four v_alignbyte_b32 with the
//    wave-uniform shift sh_j = (in_j + c0) mod 4.
//  * Outputs are stored as 16-B-aligned blocks only: output r's blocks sit at
//    positions c_i + delta_r, delta_r = (-(out_r + c0)) mod 16, so lane i
//    stores bytes [delta_r, delta_r + 16) of its column and lane i+1's (DPP
//    shifts, a v_cndmask dword select and v_alignbyte; output 0 needs none).
//  * Guard band.  The main kernel stores (compares) only blocks that lie in
//    [G, S - G), G = 48 B: every column such a block needs is then read
//    whole from inside the shard, so no load needs a clamp that matters and
//    no store a byte mask, and every output byte has one owner lane (the
//    accumulate passes of k > 8 read the old block and write it back
//    race-free).  The < 64 head and < 64 tail bytes of each output shard (all
//    of a shard of S <= 160 B) are coded byte by byte by gf_odd_edges, a
//    second, tiny launch.
//  * Verify: the stored parity is loaded and shifted like an input and
//    compared column by column; nothing is written but one flag per object.
//
// Schedule: the one of gf_apply_vec_pipe2 — compile-time K <= 8 with the
// coefficient tables hoisted once, 4-wave blocks, the next tile's loads in
// flight while the current tile computes and stores, one block barrier per
// tile with a block-uniform trip count (past-the-end waves load a stand-in
// tile and store nothing), XCD-grouped block order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "gf_device.h"
#include "kernels.h"

namespace hbec {

constexpr uint32_t kOddStore = 62;            // blocks stored per 64-lane window
constexpr uint32_t kOddWin = kOddStore * 16;  // shard bytes per window (992)
constexpr int32_t kOddGuard = 48;             // bytes at each end left to gf_odd_edges
constexpr int32_t kOddEdgeSlots = 160;        // edge bytes handled per (shard, output): 80 head + 80 tail
// the main kernel runs on shards longer than this (shorter ones: gf_odd_edges only)
constexpr uint64_t kOddMinMain = (uint64_t)kOddEdgeSlots;

#ifndef HBEC_ODD_SLEEP
#define HBEC_ODD_SLEEP 0  // x 64 cycles after the next tile's loads
#endif
#ifndef HBEC_ODD_BARRIER
#define HBEC_ODD_BARRIER 1  // apply: one block barrier per tile
#endif
#ifndef HBEC_ODD_VBARRIER
#define HBEC_ODD_VBARRIER 0  // verify: none (8+3 57 -> 66 %, 6+3 63 -> 70 %, profiles/r03_tune_odd3.jsonl)
#endif
#ifndef HBEC_ODD_VMIN
#define HBEC_ODD_VMIN 1  // K*R from which all table words live in VGPRs (1: always)
#endif
#ifndef HBEC_ODD_LB
#define HBEC_ODD_LB 1  // launch_bounds min blocks per CU (register budget)
#endif
#ifndef HBEC_ODD_U_SMALL
#define HBEC_ODD_U_SMALL 2  // windows per wave tile for K <= 4 (0: 4 / K); 2: 4+2 62.5 -> 65 % (r03_tune_odd3)
#endif
#ifndef HBEC_ODD_U_VERIFY
#define HBEC_ODD_U_VERIFY 0  // windows per wave tile of verify for K <= 4 (0: as apply)
#endif
#ifndef HBEC_ODD_ALOAD
#define HBEC_ODD_ALOAD 0  // 1: 16-B-aligned input loads, shifted by realign16 (0: dword-aligned loads, 1 DPP)
#endif
#ifndef HBEC_ODD_EDGE_PLAIN
#define HBEC_ODD_EDGE_PLAIN 0  // 1: blocks in a 128-B line shared with the next / previous window: plain (L2) stores
#endif
#ifndef HBEC_ODD_NT_ST
#define HBEC_ODD_NT_ST 1  // 0: plain stores for every output block
#endif
#ifndef HBEC_ODD_PLAN_U
#define HBEC_ODD_PLAN_U 1  // windows per plan record
#endif

enum : int { kOddApply = 0, kOddAcc = 1, kOddVerify = 2 };

// windows per wave tile of the strided kernel: ~4 loads per lane in flight
// for K <= 4 (as gf_apply_vec_pipe2's 1 KiB x 4 / K), one window above
__host__ __device__ constexpr int odd_u(int k, int mode = kOddApply) {
    return (mode == kOddVerify && HBEC_ODD_U_VERIFY > 0 && k <= 4)
               ? HBEC_ODD_U_VERIFY
               : (k <= 4 ? (HBEC_ODD_U_SMALL > 0 ? HBEC_ODD_U_SMALL : (4 / k)) : 1);
}
constexpr int kOddPlanU = HBEC_ODD_PLAN_U;  // plans: windows per record

// One tile, wave-uniform.  Positions are 32-bit: the host sends shards of
// 2^31 bytes or more to the round-2 kernels.
template <int K, int R>
struct OddTile {
    uint64_t in[K];   // input shard bases (any alignment)
    uint64_t out[R];  // output (or stored parity) shard bases
    int32_t S;
    int32_t c;        // shard position of the tile's first column
    uint32_t live;    // 0: past-the-end stand-in (loaded, never stored)
    uint32_t obj;     // flag index (verify)
    // mirrored plans (zero-copy encode + ShardHash): each shard's 16-B-aligned
    // slot in the device hash arena, shard position p at slot + p
    uint64_t m_in[K];
    uint64_t m_out[R];
};

// hash-arena pitch of a mirrored stripe: shard i at arena + i * P (16-B aligned)
__host__ __device__ __forceinline__ uint64_t odd_mirror_pitch(uint64_t S) { return (S + 31u) & ~(uint64_t)15; }

__device__ __forceinline__ int32_t odd_c0(uint64_t out0) { return (int32_t)((16u - ((uint32_t)out0 & 15u)) & 15u) - 32; }

// One shard's dword-aligned 16-B blocks for one tile: lane column col's block
// starts off + 16 col bytes after base4, clamped into the shard's dwords
// (the clamp only ever moves columns the guard band keeps from being stored).
struct OddIn {
    uint64_t base4;  // base & ~3
    int32_t off;     // block start of the tile's first column, from base4
    int32_t lim;     // last block start inside the shard's dwords
    uint32_t sh;     // the column's first byte within the block (0..3)
};

constexpr uint32_t kOddLdAlign = HBEC_ODD_ALOAD ? 16u : 4u;  // input block alignment

__device__ __forceinline__ OddIn odd_in(uint64_t base, int32_t S, int32_t c) {
    constexpr uint32_t A = kOddLdAlign;
    const int32_t l4 = (int32_t)((uint32_t)base & (A - 1u));
    const int32_t t = l4 + c;
    OddIn o;
    o.base4 = base & ~(uint64_t)(A - 1u);
    o.sh = (uint32_t)t & (A - 1u);
    o.off = t - (int32_t)o.sh;
    o.lim = ((l4 + S + (int32_t)A - 1) & ~((int32_t)A - 1)) - 16;
    return o;
}

__device__ __forceinline__ u32x4 odd_ld(const OddIn& o, int32_t col) {
    int32_t v = o.off + 16 * col;
    v = v < 0 ? 0 : (v > o.lim ? o.lim : v);
    return ld16_addr(o.base4 + (uint64_t)(uint32_t)v);
}

// bytes [sh, sh + 16) of the lane's block and lane l+1's first dword (or,
// with 16-B-aligned loads, lane l+1's block)
__device__ __forceinline__ u32x4 odd_shift_in(const u32x4& v, uint32_t sh) {
    if constexpr (HBEC_ODD_ALOAD) return realign16(v, lane_next4(v), sh);
    const uint32_t n0 = lane_next(v[0]);
    return u32x4{__builtin_amdgcn_alignbyte(v[1], v[0], sh), __builtin_amdgcn_alignbyte(v[2], v[1], sh),
                 __builtin_amdgcn_alignbyte(v[3], v[2], sh), __builtin_amdgcn_alignbyte(n0, v[3], sh)};
}

typedef __attribute__((address_space(1))) uint8_t gu8_t;

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

template <int K, int R, bool MIR = false>
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
        if constexpr (MIR) {
            // rec.b = the stripe's arena (inputs and outputs are all at rec.a)
            const uint64_t P = odd_mirror_pitch(S);
#pragma unroll
            for (int j = 0; j < K; ++j) b.m_in[j] = i.rec.b + (uint64_t)p.in_idx[j] * P;
#pragma unroll
            for (int r = 0; r < R; ++r) b.m_out[r] = i.rec.b + (uint64_t)p.out_idx[r] * P;
        }
    }
};

// ---- one tile ----
template <int K, int R, int U, int MODE>
struct OddRegs {
    // shards loaded per column: verify loads the stored parity columns, the
    // accumulate mode the old output blocks (with the inputs, one tile ahead)
    static constexpr int NL = K + (MODE == kOddVerify || MODE == kOddAcc ? R : 0);
    u32x4 x[U][NL];
};

template <int K, int R, int U, int MODE>
__device__ __forceinline__ void odd_load(OddRegs<K, R, U, MODE>& X, const OddTile<K, R>& b, uint32_t lane) {
    constexpr int NL = OddRegs<K, R, U, MODE>::NL;
    OddIn src[NL];
#pragma unroll
    for (int j = 0; j < K; ++j) src[j] = odd_in(b.in[j], b.S, b.c);
    if constexpr (MODE == kOddVerify) {
#pragma unroll
        for (int r = 0; r < R; ++r) src[K + r] = odd_in(b.out[r], b.S, b.c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < (MODE == kOddAcc ? K : NL); ++j) X.x[u][j] = odd_ld(src[j], (int32_t)(u * kOddStore + lane));
    if constexpr (MODE == kOddAcc) {
        // the old output block each lane will rewrite: output r's aligned block
        // at q = column + dl_r; lanes that store nothing read one inside the band
        const int32_t hi = b.S - kOddGuard - 16;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t dl = __builtin_amdgcn_readfirstlane((16u - (((uint32_t)b.out[r] + (uint32_t)b.c) & 15u)) & 15u);
            const int32_t e = (int32_t)(((uint32_t)b.c + dl) & 15u);  // q = e mod 16
            const int32_t qmin = kOddGuard + e, qmax = hi - ((hi - e) & 15);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int32_t q = b.c + (int32_t)(u * kOddWin) + 16 * (int32_t)lane + (int32_t)dl;
                const int32_t qc = q < qmin ? qmin : (q > qmax ? qmax : q);
                X.x[u][K + r] = ld16_addr(b.out[r] + (uint64_t)(int64_t)qc);
            }
        }
    }
}

// output block store: non-temporal, or (HBEC_ODD_EDGE_PLAIN) plain for blocks
// whose 128-B line the neighbouring window writes too, so L2 merges the halves
__device__ __forceinline__ void odd_st(uint64_t addr, const u32x4& v, uint64_t win0, bool mine) {
    if constexpr (HBEC_ODD_EDGE_PLAIN) {
        const bool edge = (addr & ~(uint64_t)127) < win0 || (addr | 127u) >= win0 + kOddWin;
        if (mine && edge) *reinterpret_cast<gu32x4*>(addr) = v;
        if (mine && !edge) st16_addr(addr, v);
    } else if constexpr (HBEC_ODD_NT_ST) {
        if (mine) st16_addr(addr, v);
    } else {
        if (mine) *reinterpret_cast<gu32x4*>(addr) = v;
    }
}

template <int K, int R, int U, int MODE, bool MIR = false>
__device__ __forceinline__ void odd_finish(const OddRegs<K, R, U, MODE>& X, const OddTile<K, R>& b,
                                           const TabArray& tab, const Tables<K, R, HBEC_ODD_VMIN>& tb, uint32_t lane,
                                           uint32_t* flags, uint32_t mir = 0) {
    constexpr int NL = OddRegs<K, R, U, MODE>::NL;
    uint32_t sh[K + (MODE == kOddVerify ? R : 0)];
#pragma unroll
    for (int j = 0; j < K; ++j) sh[j] = __builtin_amdgcn_readfirstlane(((uint32_t)b.in[j] + (uint32_t)b.c) & (kOddLdAlign - 1u));
    if constexpr (MODE == kOddVerify) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            sh[K + r] = __builtin_amdgcn_readfirstlane(((uint32_t)b.out[r] + (uint32_t)b.c) & (kOddLdAlign - 1u));
    }
    const int32_t S = b.S;
    const int32_t hi = S - kOddGuard - 16;  // last block start the main kernel stores / compares
    bool bad = false;
    uint32_t dl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) dl[r] = __builtin_amdgcn_readfirstlane((16u - (((uint32_t)b.out[r] + (uint32_t)b.c) & 15u)) & 15u);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int32_t cpos = b.c + (int32_t)(u * kOddWin) + 16 * (int32_t)lane;  // this lane's column
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = odd_shift_in(X.x[u][j], sh[j]);
        u32x4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
        gf_dot<K, R, HBEC_ODD_VMIN>(acc, x, tab, tb);
        if constexpr (MIR && MODE != kOddVerify) {
            // mirror: every arena slot is 16-B aligned, so column i's arena
            // block starts at qm = cpos + dm, dm = -c mod 16; same guard band
            // (the head and tail bytes are copied by gf_odd_mirror_copy)
            const uint32_t dm = __builtin_amdgcn_readfirstlane((0u - (uint32_t)b.c) & 15u);
            const int32_t qm = cpos + (int32_t)dm;
            const bool mm = b.live != 0u && lane < kOddStore && qm >= kOddGuard && qm <= hi;
            if (mir & 1u) {
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const u32x4 v = realign16(x[j], lane_next4(x[j]), dm);
                    if (mm) st16_addr(b.m_in[j] + (uint64_t)(int64_t)qm, v);
                }
            }
            if (MODE == kOddApply && (mir & 2u)) {  // outputs are final only in a single input pass
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const u32x4 v = realign16(acc[r], lane_next4(acc[r]), dm);
                    if (mm) st16_addr(b.m_out[r] + (uint64_t)(int64_t)qm, v);
                }
            }
        }
        if constexpr (MODE == kOddVerify) {
            // frame columns = output 0's blocks: compare those inside the guard band
            const bool mine = b.live != 0u && lane < kOddStore && cpos >= kOddGuard && cpos <= hi;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const u32x4 df = odd_shift_in(X.x[u][K + r], sh[K + r]) ^ acc[r];
                bad |= mine && (df[0] | df[1] | df[2] | df[3]) != 0u;
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                u32x4 blk = acc[r];
                if (dl[r] != 0u) blk = realign16(acc[r], lane_next4(acc[r]), dl[r]);  // wave-uniform (never r = 0)
                const int32_t q = cpos + (int32_t)dl[r];  // block start: out[r] + q is 16-B aligned
                const bool mine = b.live != 0u && lane < kOddStore && q >= kOddGuard && q <= hi;
                if constexpr (MODE == kOddAcc) blk ^= X.x[u][K + r];  // the old block (odd_load)
                const uint64_t win0 = b.out[r] + (uint64_t)(int64_t)(b.c + (int32_t)(u * kOddWin) + (int32_t)dl[r]);
                odd_st(b.out[r] + (uint64_t)(int64_t)q, blk, win0, mine);
            }
        }
    }
    if constexpr (MODE == kOddVerify) {
        if (__any(bad)) {
            if (lane == 0u) atomicOr(flags + b.obj, 1u);
        }
    }
}

template <int K, int R, int U, int MODE, class Src, bool MIR = false>
__device__ __forceinline__ void odd_body(const Src& src, uint32_t n, const TabArray& tab, uint32_t* flags,
                                         uint32_t mir = 0) {
    constexpr uint32_t WPB = kPipeBlockThreads / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * WPB;
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(xcd_block() * WPB);  // the block's first wave
    const uint32_t dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave0 >= n) return;  // whole blocks only: the loop below has block barriers
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
        if (MODE == kOddVerify ? HBEC_ODD_VBARRIER : HBEC_ODD_BARRIER) __builtin_amdgcn_s_barrier();
        const typename Src::Id after = src.id(b0 + dw + nw, n);
        {
            OddTile<K, R> b;
            src.at(b, cur);
            odd_finish<K, R, U, MODE, MIR>(X, b, tab, tb, lane, flags, mir);
        }
        X = Y;
        cur = nxt;
        nxt = after;
    }
    OddTile<K, R> b;
    src.at(b, cur);
    odd_finish<K, R, U, MODE, MIR>(X, b, tab, tb, lane, flags, mir);
}

template <int K, int R, int MODE>
__global__ __launch_bounds__(kPipeBlockThreads, HBEC_ODD_LB) void gf_odd(PassArgs a, uint32_t* flags) {
    constexpr int U = odd_u(K, MODE);
    odd_body<K, R, U, MODE>(OddStrided<K, R, U>{a}, a.n_tiles, a.tab, flags);
}

template <int K, int R, int MODE, bool MIR = false>
__global__ __launch_bounds__(kPipeBlockThreads, HBEC_ODD_LB) void gf_odd_plan(UPlanArgs p, const URec* __restrict__ recs) {
    odd_body<K, R, kOddPlanU, MODE, OddPlan<K, R, MIR>, MIR>(OddPlan<K, R, MIR>{p, recs}, p.n_recs, p.tab, nullptr,
                                                            p.mirror);
}

// Mirror copies (zero-copy encode + ShardHash): for every edge record (one per
// stripe, rec.a = stripe, rec.b = its arena) and shard idx[t], copy shard
// bytes from the stripe to the arena slot: the guard-band head and tail the
// main kernel leaves (positions [0, 80) and [S - 80, S): full == 0), or the
// whole shard (full == 1: outputs of a k > kOddMaxK accumulate, final only
// after the last pass).  One block per (record, shard), bytes by thread.
__global__ __launch_bounds__(kBlockThreads) void gf_odd_mirror_copy(const URec* __restrict__ erecs, uint32_t n_erecs,
                                                                    MirrorCopyArgs a) {
    const uint32_t e = blockIdx.x / a.n_idx, t = blockIdx.x % a.n_idx;
    if (e >= n_erecs) return;
    const URec rec = erecs[e];
    const uint64_t S = rec.shard_len, P = odd_mirror_pitch(S);
    const gu8_t* src = reinterpret_cast<const gu8_t*>(rec.a + (uint64_t)a.idx[t] * S);
    gu8_t* dst = reinterpret_cast<gu8_t*>(rec.b + (uint64_t)a.idx[t] * P);
    if (a.full) {
        for (uint64_t q = threadIdx.x; q < S; q += blockDim.x) dst[q] = src[q];
        return;
    }
    for (uint32_t slot = threadIdx.x; slot < (uint32_t)kOddEdgeSlots; slot += blockDim.x) {
        const uint64_t half = kOddEdgeSlots / 2;
        uint64_t q;
        if (S <= (uint64_t)kOddEdgeSlots) {
            if (slot >= S) continue;
            q = slot;
        } else {
            q = slot < half ? slot : S - kOddEdgeSlots + slot;
        }
        dst[q] = src[q];
    }
}

// ---------------------------------------------------------------------------
// gf_odd_edges: the bytes the main kernel leaves to the guard band, coded one
// byte per thread: for output r of a shard of S bytes, positions [0, qmin_r)
// and [qmax_r + 16, S), qmin_r / qmax_r the first / last 16-B-aligned block
// of output r inside [G, S - G) (all of [0, S) when S <= kOddMinMain).  In
// verify mode the compared columns are output 0's blocks for every r.  K <= 16
// inputs, R <= 4 outputs per launch (one pass of apply_views).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool odd_edge_pos(int32_t S, uint64_t out_frame, int32_t slot, int32_t* pos) {
    if (S <= kOddEdgeSlots) {
        *pos = slot;
        return slot < S;
    }
    const int32_t e = (int32_t)((16u - ((uint32_t)out_frame & 15u)) & 15u);  // aligned block positions = e mod 16
    const int32_t qmin = kOddGuard + e;
    const int32_t top = S - kOddGuard - 16;
    const int32_t qmax = top - ((top - e) & 15);
    if (slot < kOddEdgeSlots / 2) {
        *pos = slot;
        return slot < qmin;
    }
    *pos = S - kOddEdgeSlots + slot;
    return *pos >= qmax + 16;
}

__device__ __forceinline__ uint32_t odd_edge_byte(const TabArray& tab, int r, int K, const uint64_t* in, int32_t p) {
    uint32_t v = 0;
    for (int j = 0; j < K; ++j) {
        const uint32_t x = *reinterpret_cast<const gu8_t*>(in[j] + (uint64_t)p);
        const uint32_t* t = tab[r][j];
        v ^= gf_mul_sel(selectors(x), t[0], t[1], t[2], t[3], t[4]);
    }
    return v & 0xFFu;
}

template <int MODE>
__global__ __launch_bounds__(kBlockThreads) void gf_odd_edges(PassArgs a, int K, int R, uint32_t* flags) {
    const uint64_t per_obj = (uint64_t)R * kOddEdgeSlots;
    const uint64_t total = a.n_obj * per_obj;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t obj = v / per_obj;
        const uint32_t rs = (uint32_t)(v - obj * per_obj);
        const int r = (int)(rs / kOddEdgeSlots);
        const int32_t slot = (int32_t)(rs - (uint32_t)r * kOddEdgeSlots);
        uint64_t in[kMaxK];
        for (int j = 0; j < K; ++j) in[j] = reinterpret_cast<uint64_t>(a.in[j]) + obj * a.in_stride[j];
        const uint64_t out = reinterpret_cast<uint64_t>(a.out[r]) + obj * a.out_stride[r];
        const uint64_t frame = MODE == kOddVerify ? reinterpret_cast<uint64_t>(a.out[0]) + obj * a.out_stride[0] : out;
        int32_t p;
        if (!odd_edge_pos((int32_t)a.shard_len, frame, slot, &p)) continue;
        uint32_t val = odd_edge_byte(a.tab, r, K, in, p);
        gu8_t* d = reinterpret_cast<gu8_t*>(out + (uint64_t)p);
        if (MODE == kOddVerify) {
            if (val != *d) atomicOr(flags + obj, 1u);
        } else {
            if (MODE == kOddAcc) val ^= *d;
            *d = (uint8_t)val;
        }
    }
}

// plans: one edge record per stripe / object (URec, p0 unused)
template <int MODE>
__global__ __launch_bounds__(kBlockThreads) void gf_odd_edges_plan(UPlanArgs p, const URec* __restrict__ erecs,
                                                                  uint32_t n_erecs, int K, int R) {
    const uint64_t per = (uint64_t)R * kOddEdgeSlots;
    const uint64_t total = (uint64_t)n_erecs * per;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = v / per;
        const uint32_t rs = (uint32_t)(v - e * per);
        const int r = (int)(rs / kOddEdgeSlots);
        const int32_t slot = (int32_t)(rs - (uint32_t)r * kOddEdgeSlots);
        const URec rec = erecs[e];
        const uint64_t S = rec.shard_len;
        uint64_t in[kMaxK];
        for (int j = 0; j < K; ++j) in[j] = (((p.in_sel >> j) & 1u) ? rec.b : rec.a) + (uint64_t)p.in_idx[j] * S;
        const uint64_t out = (((p.out_sel >> r) & 1u) ? rec.b : rec.a) + (uint64_t)p.out_idx[r] * S;
        int32_t q;
        if (!odd_edge_pos((int32_t)S, out, slot, &q)) continue;
        uint32_t val = odd_edge_byte(p.tab, r, K, in, q);
        gu8_t* d = reinterpret_cast<gu8_t*>(out + (uint64_t)q);
        if (MODE == kOddAcc) val ^= *d;
        *d = (uint8_t)val;
    }
}

// ---------------------------------------------------------------------------
// launch table
// ---------------------------------------------------------------------------
template <int K, int R, int MODE>
static const void* odd_pick(bool plan, bool mirror) {
    if (!plan) return (const void*)&gf_odd<K, R, MODE>;
    if constexpr (MODE != kOddVerify) {
        if (mirror) return (const void*)&gf_odd_plan<K, R, MODE, true>;
    }
    return (const void*)&gf_odd_plan<K, R, MODE>;
}

template <int K, int MODE>
static const void* odd_for_r(int r, bool plan, bool mirror) {
    switch (r) {
        case 1: return odd_pick<K, 1, MODE>(plan, mirror);
        case 2: return odd_pick<K, 2, MODE>(plan, mirror);
        case 3: return odd_pick<K, 3, MODE>(plan, mirror);
        case 4: return odd_pick<K, 4, MODE>(plan, mirror);
    }
    return nullptr;
}

template <int MODE>
static const void* odd_kernel_(int k, int r, bool plan, bool mirror) {
    switch (k) {
        case 1: return odd_for_r<1, MODE>(r, plan, mirror);
        case 2: return odd_for_r<2, MODE>(r, plan, mirror);
        case 3: return odd_for_r<3, MODE>(r, plan, mirror);
        case 4: return odd_for_r<4, MODE>(r, plan, mirror);
        case 5: return odd_for_r<5, MODE>(r, plan, mirror);
        case 6: return odd_for_r<6, MODE>(r, plan, mirror);
        case 7: return odd_for_r<7, MODE>(r, plan, mirror);
        case 8: return odd_for_r<8, MODE>(r, plan, mirror);
#if HBEC_ODD_MAXK > 8
        case 9: return odd_for_r<9, MODE>(r, plan, mirror);
        case 10: return odd_for_r<10, MODE>(r, plan, mirror);
        case 11: return odd_for_r<11, MODE>(r, plan, mirror);
        case 12: return odd_for_r<12, MODE>(r, plan, mirror);
#endif
#if HBEC_ODD_MAXK > 12
        case 13: return odd_for_r<13, MODE>(r, plan, mirror);
        case 14: return odd_for_r<14, MODE>(r, plan, mirror);
        case 15: return odd_for_r<15, MODE>(r, plan, mirror);
        case 16: return odd_for_r<16, MODE>(r, plan, mirror);
#endif
    }
    return nullptr;
}

static const void* odd_kernel(int k, int r, int mode, bool plan, bool mirror = false) {
    if (plan && mode == kOddVerify) return nullptr;
    switch (mode) {
        case kOddApply: return odd_kernel_<kOddApply>(k, r, plan, mirror);
        case kOddAcc: return odd_kernel_<kOddAcc>(k, r, plan, mirror);
        case kOddVerify: return odd_kernel_<kOddVerify>(k, r, plan, false);
    }
    return nullptr;
}

#ifndef HBEC_ODD_DEFAULT
#define HBEC_ODD_DEFAULT 1
#endif
bool odd_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("HBEC_ODD");
        return e ? e[0] != '0' : HBEC_ODD_DEFAULT != 0;
    }();
    return on;
}

#ifndef HBEC_ODD_BPC_APPLY
#define HBEC_ODD_BPC_APPLY 1
#endif
#ifndef HBEC_ODD_BPC_VERIFY
#define HBEC_ODD_BPC_VERIFY 2  // read-only: 4+2 68.5 -> 81 % with 2 blocks per CU (r03_tune_odd3)
#endif
int odd_blocks_per_cu(int mode) {
    static const int v = [] {
        const char* e = std::getenv("HBEC_ODD_BPC");
        return e ? std::atoi(e) : 0;
    }();
    return v > 0 ? v : (mode == kOddVerify ? HBEC_ODD_BPC_VERIFY : HBEC_ODD_BPC_APPLY);
}

uint64_t urec_tile() { return odd_enabled() ? (uint64_t)kOddPlanU * kOddWin : (uint64_t)unaligned_tile_bytes(); }
uint64_t urec_span(uint64_t shard_len) {
    if (!odd_enabled()) return shard_len;
    return shard_len > kOddMinMain ? shard_len + 32u : 0u;
}

uint32_t odd_tile_bytes(int k) { return (uint32_t)odd_u(k) * kOddWin; }
uint64_t odd_min_main() { return kOddMinMain; }
uint32_t odd_plan_tile_bytes() { return (uint32_t)kOddPlanU * kOddWin; }

// Tiles per shard: enough windows for every output block of the shard, from
// the frame's first column (c0 >= -32) to position S.
uint32_t odd_tiles_per_obj(int k, int mode, uint64_t shard_len) {
    const uint64_t span = shard_len + 32u;
    const uint64_t tile = (uint64_t)odd_u(k, mode) * kOddWin;
    return (uint32_t)((span + tile - 1) / tile);
}

bool odd_supported(int k, int r) { return k >= 1 && k <= kOddMaxK && r >= 1 && r <= kMaxR; }

hipError_t launch_odd(int k, int r, int mode, const PassArgs& a, uint32_t* flags, int grid, hipStream_t stream) {
    const void* fn = odd_kernel(k, r, mode, false);
    if (!fn) return hipErrorInvalidValue;
    void* args[] = {const_cast<PassArgs*>(&a), &flags};
    return hipLaunchKernel(fn, dim3(grid), dim3(kPipeBlockThreads), args, 0, stream);
}

hipError_t launch_odd_edges(int k, int r, int mode, const PassArgs& a, uint32_t* flags, hipStream_t stream) {
    if (k < 1 || k > kMaxK || r < 1 || r > kMaxR || a.n_obj == 0) return a.n_obj == 0 ? hipSuccess : hipErrorInvalidValue;
    const uint64_t total = a.n_obj * (uint64_t)r * kOddEdgeSlots;
    const int grid = (int)std::min<uint64_t>((total + kBlockThreads - 1) / kBlockThreads, 4096);
    const void* fn = mode == kOddVerify ? (const void*)&gf_odd_edges<kOddVerify>
                                        : (mode == kOddAcc ? (const void*)&gf_odd_edges<kOddAcc> : (const void*)&gf_odd_edges<kOddApply>);
    void* args[] = {const_cast<PassArgs*>(&a), &k, &r, &flags};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

hipError_t launch_odd_edges_plan(int k, int r, int mode, const UPlanArgs& p, const URec* erecs, uint32_t n_erecs,
                                 hipStream_t stream) {
    if (n_erecs == 0) return hipSuccess;
    if (k < 1 || k > kMaxK || r < 1 || r > kMaxR || mode == kOddVerify) return hipErrorInvalidValue;
    const uint64_t total = (uint64_t)n_erecs * (uint64_t)r * kOddEdgeSlots;
    const int grid = (int)std::min<uint64_t>((total + kBlockThreads - 1) / kBlockThreads, 4096);
    const void* fn = mode == kOddAcc ? (const void*)&gf_odd_edges_plan<kOddAcc> : (const void*)&gf_odd_edges_plan<kOddApply>;
    void* args[] = {const_cast<UPlanArgs*>(&p), &erecs, &n_erecs, &k, &r};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

hipError_t launch_odd_plan(int k, int r, int mode, const UPlanArgs& p, int grid, hipStream_t stream) {
    const void* fn = odd_kernel(k, r, mode, true, p.mirror != 0);
    if (!fn) return hipErrorInvalidValue;
    const URec* recs = p.recs;
    void* args[] = {const_cast<UPlanArgs*>(&p), &recs};
    return hipLaunchKernel(fn, dim3(grid), dim3(kPipeBlockThreads), args, 0, stream);
}

hipError_t launch_odd_mirror_copy(const URec* erecs, uint32_t n_erecs, const MirrorCopyArgs& a, hipStream_t stream) {
    if (n_erecs == 0 || a.n_idx == 0) return hipSuccess;
    if (a.n_idx > kMirrorMaxIdx) return hipErrorInvalidValue;
    const uint64_t blocks = (uint64_t)n_erecs * a.n_idx;
    if (blocks >= (1ull << 31)) return hipErrorInvalidValue;
    MirrorCopyArgs c = a;
    void* args[] = {&erecs, &n_erecs, &c};
    return hipLaunchKernel((const void*)&gf_odd_mirror_copy, dim3((unsigned)blocks), dim3(kBlockThreads), args, 0, stream);
}

uint64_t odd_mirror_pitch_host(uint64_t shard_len) { return odd_mirror_pitch(shard_len); }

}  // namespace hbec
