// odd_impl.h — the gf_odd kernel templates (see odd.hip for the design),
// shared by the translation units that instantiate them: odd.hip (K <= 4,
// launchers, edge and mirror kernels), odd_k58.hip (K 5..8), odd_k912.hip
// (K 9..12).  Every kernel instance lives in exactly
// one translation unit, and the units compile in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "gf_device.h"
#include "kernels.h"
#include "xor_sched.h"

namespace hbec {

constexpr uint32_t kOddStore = 62;            // blocks stored per 64-lane window
constexpr uint32_t kOddWin = kOddStore * 16;  // shard bytes per window (992)
enum : int { kOddApply = 0, kOddAcc = 1, kOddVerify = 2 };
// Verify stores nothing, so no output is realigned and lane 62's column is
// compared too: 63 columns per window (1.6 % of the loads re-read, not 3.2 %)
template <int MODE>
__host__ __device__ constexpr uint32_t odd_store() { return MODE == kOddVerify ? 63u : kOddStore; }
template <int MODE>
__host__ __device__ constexpr uint32_t odd_win() { return odd_store<MODE>() * 16u; }
// Carry (strided apply with 2 windows per wave tile, Verify below; odd 4+2 65 -> 70 %,
// r03_tune_carry): the
// windows are contiguous (columns 0..63 and 64..127 of the tile); window 0
// gets its lane 63's missing next column from window 1's lane 0 (a readlane
// + DPP with that value as the out-of-range fill) and stores 64 blocks,
// window 1 stores 62: 126 of 128 loaded columns instead of 124.
// Verify tiles of U >= 2 windows are chained the same way: window u < U-1
// compares all 64 of its columns (lane 63 borrows window u+1's first dword),
// the last 63, so a tile of 64 U loaded blocks compares 64 U - 1 and the
// 64-B lines a tile touches are its own (4+2 Verify with 4 chained windows:
// 1.060 -> 1.024 x its bytes, 80.1 -> 81.3 %; 63-column windows re-read a
// line at every window boundary; profiles/r04_ab_odd.jsonl batch V).
template <int U, int MODE>
__host__ __device__ constexpr bool odd_carry() { return MODE == kOddVerify ? U >= 2 : U == 2; }
// first column of window u within a tile, and shard bytes per tile
template <int U, int MODE, bool CARRY>
__host__ __device__ constexpr uint32_t odd_wcol(int u) { return CARRY ? 64u * (uint32_t)u : odd_store<MODE>() * (uint32_t)u; }
template <int U, int MODE, bool CARRY>
__host__ __device__ constexpr uint32_t odd_tile_span() {
    return CARRY ? (MODE == kOddVerify ? (64u * U - 1u) * 16u : (64u + kOddStore) * 16u) : U * odd_win<MODE>();
}
constexpr int32_t kOddGuard = 48;             // bytes at each end left to gf_odd_edges
constexpr int32_t kOddEdgeSlots = 160;        // edge bytes handled per (shard, output): 80 head + 80 tail
constexpr int32_t kOddEdgeSlotsLong = 128;    // the same for S > kOddMinMain: 64 head + 64 tail
// gf_odd_edges: a thread per (object, output, slot) below this many objects
// (latency-bound launches), per (object, slot) for every output above
constexpr uint64_t kOddEdgeSplitObjs = 1024;
// the main kernel runs on shards longer than this (shorter ones: gf_odd_edges only)
constexpr uint64_t kOddMinMain = (uint64_t)kOddEdgeSlots;

// all coefficient-table words in VGPRs (gf_device.h Tables: v_perm reads one SGPR)
constexpr int kOddVMin = 1;

// windows per wave tile of the strided kernel: ~4 loads per lane in flight
// for K <= 4 (as gf_apply_vec_pipe2's 1 KiB x 4 / K), one window above
__host__ __device__ constexpr int odd_u(int k, int mode = kOddApply) {
    return (mode == kOddVerify && k <= 4) ? HBEC_ODD_U_VERIFY : (k <= 4 ? HBEC_ODD_U_SMALL : (k <= 8 ? HBEC_ODD_U_MID : 1));
}
constexpr int kOddPlanU = HBEC_ODD_PLAN_U;  // plans: windows per record (tuning.h)

// Record kernels (gf_odd_rec), apply / accumulate with 2 windows per wave
// tile (K <= 4, plans): the carry of gf_odd, window 0 stores 64 blocks,
// window 1 62.  (A chained Verify of the same kind, 64 U - 1 columns per
// tile, read less but ran slower than gf_odd's 63-column windows at 4+2:
// 74.5 vs 76.6 %, profiles/r04_ab_odd.jsonl batch F; Verify records are used
// from K R >= 24, one window per tile.)
__host__ __device__ constexpr bool odd_rec_carry(int u, int mode) { return mode != kOddVerify && u >= 2; }
// Strided batches code from object records (gf_odd_rec) when they carry at
// least 18 products per column (6+3, 7+3, 8+3, 10+4, 12+4 encode), and for
// K > 8 from 24 (3-4 outputs, and 12 x 2: tuning.h); gf_odd below: the per-tile base arithmetic
// the records remove only showed where the field arithmetic already filled
// the issue slots (round-4 A/B, profiles/r04_ab_odd.jsonl: 6+3 encode 62.9 ->
// 66.9 %, 7+3 55.2 -> 60.5 %, 8+3 59.3 -> 64.5 %, 12+4 51.2 -> 57.3 %; for
// gf_odd: 4+2 encode 70.5 vs 67.6 %, 6+2 68.4 vs 67.4 %, 8+2 66.2 vs 65.0 %,
// 10+2 65.8 vs 60.6 %, the last against the LDS-table record kernel).
__host__ __device__ constexpr bool odd_use_rec(int k, int r) {
    return k * r >= HBEC_ODD_REC_MINKR && (k <= 8 || k * r >= HBEC_ODD_REC_BIGK_MINKR);
}
// shard bytes per wave tile of the record kernel
__host__ __device__ constexpr uint32_t odd_rec_span(int u, int mode) {
    return odd_rec_carry(u, mode) ? (64u * (uint32_t)(u - 1) + kOddStore) * 16u
                                  : (uint32_t)u * (mode == kOddVerify ? 63u : kOddStore) * 16u;
}

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

// Frame offset: column 0 of a shard sits at position kOddFrame + (-out0 mod 16)
// in [32, 48), so the first block any output stores (position >= kOddGuard)
// is covered by column 0 or 1 and no column lies before the shard; a shard's
// tiles then only have to reach the last stored block (<= S - 64):
// odd_frame_tiles (round 6: one tile fewer per shard for about 1 size in
// 16 at S = 4 KiB; the old frame started 32 B before the shard and its tiles
// ran to S + 32).
constexpr int32_t kOddFrame = 32;
__device__ __forceinline__ int32_t odd_c0(uint64_t out0) { return (int32_t)((16u - ((uint32_t)out0 & 15u)) & 15u) + kOddFrame; }

// One shard's dword-aligned 16-B blocks for one tile: lane column col's block
// starts off + 16 col bytes after base4, clamped into the shard's dwords
// (the clamp only ever moves columns the guard band keeps from being stored).
struct OddIn {
    uint64_t base4;  // base & ~3
    int32_t off;     // block start of the tile's first column, from base4
    int32_t lim;     // last block start inside the shard's dwords
    uint32_t sh;     // the column's first byte within the block (0..3)
};

__device__ __forceinline__ OddIn odd_in(uint64_t base, int32_t S, int32_t c) {
    const int32_t l4 = (int32_t)((uint32_t)base & 3u);
    const int32_t t = l4 + c;
    OddIn o;
    o.base4 = base & ~(uint64_t)3u;
    o.sh = (uint32_t)t & 3u;
    o.off = t - (int32_t)o.sh;
    o.lim = ((l4 + S + 3) & ~3) - 16;
    return o;
}

// (Plain, L2-retained loads for Verify — the neighbouring wave's tile reads
// the shared boundary column later — cut odd Verify traffic to <= 1.02 x
// but ran 3-6 points slower: profiles/r05_ab_plans_verify.jsonl batch r5_ab9.)
__device__ __forceinline__ u32x4 odd_ld(const OddIn& o, int32_t col) {
    int32_t v = o.off + 16 * col;
    v = v < 0 ? 0 : (v > o.lim ? o.lim : v);
    return ld16_addr(o.base4 + (uint64_t)(uint32_t)v);
}

// bytes [sh, sh + 16) of the lane's block and lane l+1's first dword
__device__ __forceinline__ u32x4 odd_shift_in(const u32x4& v, uint32_t sh) {
    const uint32_t n0 = lane_next(v[0]);
    return u32x4{__builtin_amdgcn_alignbyte(v[1], v[0], sh), __builtin_amdgcn_alignbyte(v[2], v[1], sh),
                 __builtin_amdgcn_alignbyte(v[3], v[2], sh), __builtin_amdgcn_alignbyte(n0, v[3], sh)};
}

// the same with lane 63's missing neighbour supplied (carry: the first dword
// / block of the next window, wave-uniform): DPP wave_shl:1 without bound
// control keeps `fill` in lane 63
__device__ __forceinline__ uint32_t lane_next_fill(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x130, 0xF, 0xF, false);
}

__device__ __forceinline__ u32x4 lane_next4_fill(const u32x4& v, const u32x4& fill) {
    return u32x4{lane_next_fill(v[0], fill[0]), lane_next_fill(v[1], fill[1]), lane_next_fill(v[2], fill[2]),
                 lane_next_fill(v[3], fill[3])};
}

// Lane l gets v0's lane l+1, lane 63 gets v1's lane 0 (the carry of two
// contiguous windows): DPP wave_rol:1 of v1 as the out-of-range fill of a
// wave_shl:1 of v0.  Two VALU moves; replaces a v_readlane whose SGPR result
// the next DPP move waits for (an issue stall per dword at one wave per SIMD).
__device__ __forceinline__ uint32_t lane_next_carry(uint32_t v0, uint32_t v1) {
    const int rot = __builtin_amdgcn_update_dpp(0, (int)v1, 0x134, 0xF, 0xF, false);  // wave_rol:1
    return (uint32_t)__builtin_amdgcn_update_dpp(rot, (int)v0, 0x130, 0xF, 0xF, false);
}

__device__ __forceinline__ u32x4 lane_next4_carry(const u32x4& v0, const u32x4& v1) {
    return u32x4{lane_next_carry(v0[0], v1[0]), lane_next_carry(v0[1], v1[1]), lane_next_carry(v0[2], v1[2]),
                 lane_next_carry(v0[3], v1[3])};
}

// odd_shift_in of window 0 with window 1 (v1) supplying lane 63's neighbour
__device__ __forceinline__ u32x4 odd_shift_in_carry(const u32x4& v, uint32_t sh, const u32x4& v1) {
    const uint32_t n0 = lane_next_carry(v[0], v1[0]);
    return u32x4{__builtin_amdgcn_alignbyte(v[1], v[0], sh), __builtin_amdgcn_alignbyte(v[2], v[1], sh),
                 __builtin_amdgcn_alignbyte(v[3], v[2], sh), __builtin_amdgcn_alignbyte(n0, v[3], sh)};
}

__device__ __forceinline__ u32x4 lane0(const u32x4& v) {
    return u32x4{(uint32_t)__builtin_amdgcn_readlane((int)v[0], 0), (uint32_t)__builtin_amdgcn_readlane((int)v[1], 0),
                 (uint32_t)__builtin_amdgcn_readlane((int)v[2], 0), (uint32_t)__builtin_amdgcn_readlane((int)v[3], 0)};
}

__device__ __forceinline__ u32x4 odd_shift_in_fill(const u32x4& v, uint32_t sh, const u32x4& next0) {
    const uint32_t n0 = lane_next_fill(v[0], next0[0]);
    return u32x4{__builtin_amdgcn_alignbyte(v[1], v[0], sh), __builtin_amdgcn_alignbyte(v[2], v[1], sh),
                 __builtin_amdgcn_alignbyte(v[3], v[2], sh), __builtin_amdgcn_alignbyte(n0, v[3], sh)};
}

typedef __attribute__((address_space(1))) uint8_t gu8_t;

// ---- guard-band bytes inside the main kernels (HBEC_ODD_EDGE_FUSE) ----
// A strided apply pass of shards longer than one tile codes each shard's
// head [0, 64) and tail [S - 64, S) in the tile that starts / ends the shard:
// lane l takes position l (head) or S - 64 + l (tail), loads the K input
// bytes with that tile's loads (so they come from the lines the tile reads,
// and the next tile's loads stay in flight behind them), multiplies them
// with the tile and stores the output bytes of the guard band next to the
// tile's 16-B blocks (the L2 merges them into the same lines).  Every tile
// issues the K byte loads, the other tiles from their own first column, so
// the number of loads in flight is the same on every path (a
// load under a branch made the compiler wait for the NEXT tile's loads at
// every finish).  Edge flags (wave-uniform): 1 first tile, 2 last tile;
// the host fuses only when every shard has >= 2 tiles (never both).
// The edge bytes are loaded as their aligned dwords and extracted in the
// finish (odd_edge_byte): a byte load's value reached the loop's back edge as
// a masked copy (v_and 0xff) that waited for every load in flight, the next
// tile's included (8+3 records 60 -> 43 %).
typedef __attribute__((address_space(1))) const uint32_t gu32_c;
__device__ __forceinline__ uint32_t ld_dw(uint64_t addr) { return *reinterpret_cast<gu32_c*>(addr & ~(uint64_t)3); }
__device__ __forceinline__ uint32_t odd_edge_byte(uint32_t dw, uint32_t addr_lo) { return dw >> (8u * (addr_lo & 3u)); }
__device__ __forceinline__ void st_u8(uint64_t addr, uint32_t v) { *reinterpret_cast<gu8_t*>(addr) = (uint8_t)v; }

// lane offset of an edge tile's byte (0 on the others)
__device__ __forceinline__ uint32_t odd_edge_off(uint32_t flags, uint32_t S, uint32_t lane) {
    return flags == 0u ? 0u : ((flags & 1u) ? lane : S - 64u + lane);
}

// the output bytes of an edge word: output r at shard base o; the main
// kernel stores positions [h, t) of output r
__device__ __forceinline__ void odd_edge_store(uint64_t o, uint32_t v, uint32_t flags, uint32_t S, uint32_t lane,
                                               uint32_t h, uint32_t t, bool live) {
    const uint32_t p = odd_edge_off(flags, S, lane);
    if (live && ((flags & 1u) ? p < h : p >= t)) st_u8(o + p, v);
}

// acc[r] = XOR_j C[r][j] * x[j] for one dword per input (register tables)
template <int K, int R, int VMIN>
__device__ __forceinline__ void gf_dot1(uint32_t (&acc)[R], const uint32_t (&x)[K], const TabArray& tab,
                                        const Tables<K, R, VMIN>& tb) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0u;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const Sel sx = selectors(x[j]);
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
            acc[r] = xor3(acc[r], perm(h1, tb.lo0[r][j], sx.s0), perm(h3, tb.lo2[r][j], sx.s1)) ^ perm(h4, h4, sx.s2);
        }
    }
}

// coefficient tables in LDS (record kernels, K >= HBEC_ODD_LDS_MINK): words per input, 16-B padded
__host__ __device__ constexpr uint32_t odd_lt_stride(int r) { return (uint32_t)((r * 5 + 3) & ~3); }

// Pinned outputs: every output column is
// materialised right after the field multiply (an empty asm that reads and
// writes it).  Without it the compiler sinks each output row's products into
// that row's store branch, r outer and j inner, keeping every input's
// selectors live across the stores (8+3 275 VGPRs, 10+4 392; pinned 201 and
// 267).  Measured per shape (profiles/r03_tune_pin.jsonl) and kept where it
// pays: Verify 5 <= K <= 8 (2 blocks per CU then hold 2 waves per SIMD: 8+3
// 67.7 -> 71.4 %), and plain apply passes with K <= 10 and K * R >= 36 (10+4
// encode) together with launch bounds for 2 blocks per CU and a grid of 2
// blocks per CU (odd_two_blocks): 10+4 encode 50.0 -> 53.9 %, plans 42.5 ->
// 50.9 %.  Apply with fewer products (8+3, 6+3, reconstructs) lost 4-8 %
// pinned, and 12+4 spills.
__host__ __device__ constexpr bool odd_two_blocks(int k, int r, int mode, bool mir) {
    return !mir && mode == kOddApply && k <= 10 && k * r >= 36;
}
// gf_odd strided apply codes the guard band in the main kernel
// (HBEC_ODD_EDGE_FUSE) for K <= 4, R <= 3; above (and 2..4 x 4), the extra edge words made the
// allocator copy the whole next tile at the loop's back edge (a vmcnt(0)
// per tile in gf_odd<8,2,0>; the 2-block pinned 9+4 / 10+4 spilled)
__host__ __device__ constexpr bool odd_strided_edge(int k, int r, int mode) {
    return (HBEC_ODD_EDGE_FUSE & 1) != 0 && mode == kOddApply && k <= 4 && r <= 3 && !odd_two_blocks(k, r, mode, false);
}
template <int K, int R, int MODE, bool MIR>
__host__ __device__ constexpr bool odd_pin_on() {
    return !MIR && ((MODE == kOddVerify && K >= 5 && K <= 8) || odd_two_blocks(K, R, MODE, MIR));
}
template <int K, int R, int MODE, bool MIR>
__device__ __forceinline__ void odd_pin(u32x4 (&acc)[R]) {
    if constexpr (odd_pin_on<K, R, MODE, MIR>()) {
#pragma unroll
        for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc[r]));
    }
}

template <int K, int R, int MODE, bool MIR = false>
__host__ __device__ constexpr int odd_lb() { return odd_two_blocks(K, R, MODE, MIR) ? 2 : 1; }

// ---- tile sources ----
// A source names tile t compactly (id(): a few scalars, carried one and two
// tiles ahead) and expands it to shard bases where they are used (at()), so
// the pipeline does not hold three tiles of K + R 64-bit bases in SGPRs.
// Strided batch (PassArgs): tile t = (object t / tpo, tile t % tpo).
struct OddIdS {
    uint32_t obj, ti, live;
};

template <int K, int R, int U, int MODE>
struct OddStrided {
    using Id = OddIdS;
    static constexpr bool kCarry = odd_carry<U, MODE>();
    // apply passes code the guard band in the shard's first / last tile
    static constexpr bool kEdge = odd_strided_edge(K, R, MODE);
    const PassArgs& a;
    __device__ __forceinline__ uint32_t edge(const Id& i) const {
        return (a.fuse & 1u) != 0u && i.live != 0u
                   ? (i.ti == 0u ? 1u : (i.ti + 1u == a.tiles_per_obj ? 2u : 0u)) : 0u;
    }
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
        b.c = odd_c0(b.out[0]) + (int32_t)(i.ti * odd_tile_span<U, MODE, kCarry>());
        b.live = i.live;
        b.obj = i.obj;
    }
};

// Plan records (URec): input j of the record's stripe at (bit j of in_sel ?
// b : a) + in_idx[j] * S; rec.p0 = the record's first window * 992.
struct OddIdP {
    // the record's fields as scalars: holding the URec itself let the compiler
    // index {a, b} by the in_sel bit and put the ids in LDS (r3 ISA check)
    uint64_t a, b;
    uint32_t S, p0;  // S < 2^31 on this path (larger shards take the brecs kernel)
    uint32_t live;
    uint32_t sub;  // wave tile within the record (SUB > 1)
};

// A record covers kOddPlanU windows; kernels with fewer windows per wave tile
// (U = odd_plan_u(K)) take each record as SUB = kOddPlanU / U wave tiles.
template <int K>
__host__ __device__ constexpr int odd_plan_u(int) {
    return K <= 4 ? kOddPlanU : 1;  // K > 4: 2 windows of K inputs spill (10+4 object plan 42 -> 31 %, r3b7)
}

template <int K, int R, bool MIR = false, bool CARRY = false>
struct OddPlan {
    using Id = OddIdP;
    static constexpr bool kEdge = false;  // plans: gf_odd_edges_plan
    __device__ __forceinline__ uint32_t edge(const Id&) const { return 0u; }
    // CARRY: the records hold one carried 2-window tile each (2016 B,
    // urec_tile_for); otherwise 2 x 992 B windows
    static constexpr bool kCarry = CARRY;
    static_assert(!CARRY || (!MIR && odd_plan_u<K>(0) == 2), "carried plan records: K <= 4, not mirrored");
    static constexpr uint32_t SUB = (uint32_t)(kOddPlanU / odd_plan_u<K>(0));
    const UPlanArgs& p;
    const URec* __restrict__ recs;
    __device__ __forceinline__ Id id(uint32_t t, uint32_t n) const {
        const uint32_t tt = t < n ? t : n - 1u;
        const URec& r = recs[tt / SUB];
        return Id{r.a, r.b, (uint32_t)r.shard_len, (uint32_t)r.p0, t < n ? 1u : 0u, tt % SUB};
    }
    __device__ __forceinline__ void at(OddTile<K, R>& b, const Id& i) const {
        const uint64_t S = i.S;
        const uint64_t d = i.b - i.a;  // base = a + (sel bit ? b - a : 0), no select between fields
#pragma unroll
        for (int j = 0; j < K; ++j)
            b.in[j] = i.a + (d & (0ull - (uint64_t)((p.in_sel >> j) & 1u))) + (uint64_t)p.in_idx[j] * S;
#pragma unroll
        for (int r = 0; r < R; ++r)
            b.out[r] = i.a + (d & (0ull - (uint64_t)((p.out_sel >> r) & 1u))) + (uint64_t)p.out_idx[r] * S;
        b.S = (int32_t)S;
        b.c = odd_c0(b.out[0]) + (int32_t)i.p0 + (int32_t)(i.sub * (uint32_t)odd_plan_u<K>(0) * kOddWin);
        b.live = i.live;
        b.obj = 0;
        if constexpr (MIR) {
            // rec.b = the stripe's arena (inputs and outputs are all at rec.a)
            const uint64_t P = odd_mirror_pitch(S);
#pragma unroll
            for (int j = 0; j < K; ++j) b.m_in[j] = i.b + (uint64_t)p.in_idx[j] * P;
#pragma unroll
            for (int r = 0; r < R; ++r) b.m_out[r] = i.b + (uint64_t)p.out_idx[r] * P;
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

template <int K, int R, int U, int MODE, bool CARRY = false>
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
        for (int j = 0; j < (MODE == kOddAcc ? K : NL); ++j)
            X.x[u][j] = odd_ld(src[j], (int32_t)(odd_wcol<U, MODE, CARRY>(u) + lane));
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
                const int32_t q = b.c + (int32_t)(16u * odd_wcol<U, MODE, CARRY>(u)) + 16 * (int32_t)lane + (int32_t)dl;
                const int32_t qc = q < qmin ? qmin : (q > qmax ? qmax : q);
                X.x[u][K + r] = ld16_addr(b.out[r] + (uint64_t)(int64_t)qc);
            }
        }
    }
}

// output block store (non-temporal).  Measured and rejected (r03_tune_odd4):
// plain stores for blocks whose 128-B line the neighbouring window also
// writes (-1.5..-9 %), plain stores everywhere (-1..-12 %).
__device__ __forceinline__ void odd_st(uint64_t addr, const u32x4& v, bool mine) {
    if (mine) st16_addr(addr, v);
}

// gf_odd's fused guard band of one tile (edge: its flags, wave-uniform): the
// bands of gf_odd_edges, from the edge words e[] loaded with the tile
template <int K, int R>
__device__ __forceinline__ void odd_edges(const uint32_t (&e)[K], const OddTile<K, R>& b, const TabArray& tab,
                                          const Tables<K, R, kOddVMin>& tb, uint32_t lane, uint32_t edge) {
    {
        uint32_t acc[R], x[K];
        const uint32_t p = odd_edge_off(edge, (uint32_t)b.S, lane);
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = odd_edge_byte(e[j], (uint32_t)b.in[j] + p);
        gf_dot1<K, R, kOddVMin>(acc, x, tab, tb);
        const uint32_t S = (uint32_t)b.S, top = S - (uint32_t)kOddGuard - 16u;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t e = (16u - ((uint32_t)b.out[r] & 15u)) & 15u;  // output r's aligned positions = e mod 16
            const uint32_t qmax = top - ((top - e) & 15u);
            odd_edge_store(b.out[r], acc[r], edge, S, lane, (uint32_t)kOddGuard + e, qmax + 16u, true);
        }
    }
}

template <int K, int R, int U, int MODE, bool MIR = false, bool CARRY = false>
__device__ __forceinline__ void odd_finish(const OddRegs<K, R, U, MODE>& X, const OddTile<K, R>& b,
                                           const TabArray& tab, const Tables<K, R, kOddVMin>& tb, uint32_t lane,
                                           uint32_t* flags, uint32_t mir = 0) {
    uint32_t sh[K + (MODE == kOddVerify ? R : 0)];
#pragma unroll
    for (int j = 0; j < K; ++j) sh[j] = __builtin_amdgcn_readfirstlane(((uint32_t)b.in[j] + (uint32_t)b.c) & 3u);
    if constexpr (MODE == kOddVerify) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            sh[K + r] = __builtin_amdgcn_readfirstlane(((uint32_t)b.out[r] + (uint32_t)b.c) & 3u);
    }
    const int32_t S = b.S;
    const int32_t hi = S - kOddGuard - 16;  // last block start the main kernel stores / compares
    bool bad = false;
    uint32_t dl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) dl[r] = __builtin_amdgcn_readfirstlane((16u - (((uint32_t)b.out[r] + (uint32_t)b.c) & 15u)) & 15u);
    if constexpr (CARRY && MODE == kOddVerify) {
        // chained windows: window u < U-1 compares all 64 columns (lane 63
        // borrows window u+1's first dword), the last window 63
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t cpos = b.c + 16 * 64 * u + 16 * (int32_t)lane;
            u32x4 x[K];
#pragma unroll
            for (int j = 0; j < K; ++j)
                x[j] = u + 1 < U ? odd_shift_in_carry(X.x[u][j], sh[j], X.x[u + 1 < U ? u + 1 : u][j])
                                 : odd_shift_in(X.x[u][j], sh[j]);
            u32x4 acc[R];
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
            gf_dot<K, R, kOddVMin>(acc, x, tab, tb);
            odd_pin<K, R, MODE, MIR>(acc);
            const bool mine = b.live != 0u && (u + 1 < U || lane < 63u) && cpos >= kOddGuard && cpos <= hi;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const u32x4 st = u + 1 < U ? odd_shift_in_carry(X.x[u][K + r], sh[K + r], X.x[u + 1 < U ? u + 1 : u][K + r])
                                           : odd_shift_in(X.x[u][K + r], sh[K + r]);
                const u32x4 df = st ^ acc[r];
                bad |= mine && (df[0] | df[1] | df[2] | df[3]) != 0u;
            }
        }
        if (__any(bad)) {
            if (lane == 0u) atomicOr(flags + b.obj, 1u);
        }
        return;
    } else if constexpr (CARRY) {
        static_assert(U == 2 && MODE != kOddVerify && !MIR, "carry: strided apply / accumulate, 2 windows");
        // window 1 first: its lane 0 feeds window 0's lane 63
        u32x4 x1[K], x0[K], acc1[R], acc0[R];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            x1[j] = odd_shift_in(X.x[1][j], sh[j]);
            x0[j] = odd_shift_in_carry(X.x[0][j], sh[j], X.x[1][j]);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) acc1[r] = acc0[r] = u32x4{0, 0, 0, 0};
        gf_dot<K, R, kOddVMin>(acc1, x1, tab, tb);
        gf_dot<K, R, kOddVMin>(acc0, x0, tab, tb);
        odd_pin<K, R, MODE, MIR>(acc1);
        odd_pin<K, R, MODE, MIR>(acc0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            u32x4 b0 = acc0[r], b1 = acc1[r];
            if (dl[r] != 0u) {  // wave-uniform (never r = 0)
                b0 = realign16(acc0[r], lane_next4_carry(acc0[r], acc1[r]), dl[r]);
                b1 = realign16(acc1[r], lane_next4(acc1[r]), dl[r]);
            }
            const int32_t q0 = b.c + 16 * (int32_t)lane + (int32_t)dl[r];
            const int32_t q1 = q0 + 1024;
            const bool m0 = b.live != 0u && q0 >= kOddGuard && q0 <= hi;                      // all 64 lanes
            const bool m1 = b.live != 0u && lane < kOddStore && q1 >= kOddGuard && q1 <= hi;  // 62
            if constexpr (MODE == kOddAcc) {
                b0 ^= X.x[0][K + r];
                b1 ^= X.x[1][K + r];
            }
            odd_st(b.out[r] + (uint64_t)(int64_t)q0, b0, m0);
            odd_st(b.out[r] + (uint64_t)(int64_t)q1, b1, m1);
        }
        return;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int32_t cpos = b.c + (int32_t)(u * odd_win<MODE>()) + 16 * (int32_t)lane;  // this lane's column
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = odd_shift_in(X.x[u][j], sh[j]);
        u32x4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
        gf_dot<K, R, kOddVMin>(acc, x, tab, tb);
        odd_pin<K, R, MODE, MIR>(acc);
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
            const bool mine = b.live != 0u && lane < odd_store<MODE>() && cpos >= kOddGuard && cpos <= hi;
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
                odd_st(b.out[r] + (uint64_t)(int64_t)q, blk, mine);
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
    const Tables<K, R, kOddVMin> tb = load_tables<K, R, kOddVMin>(tab);
    // Fused guard band: a tile's K edge words are loaded right before its
    // columns and coded after the previous tile's finish, in the same loop
    // step, so they never cross the loop's back edge (a loop-carried copy
    // waited for the next tile's loads: 8+3 60 -> 43 %).  Only edge tiles
    // issue them (HBEC_ODD_EDGE_COND): issued before the tile's column loads,
    // a skipped branch leaves the count the previous tile's columns are
    // waited with unchanged (LLVM keeps the shortest distance of the two
    // paths), and the extra load instructions of every other tile cost
    // 2-4 points (r06_ab_fuse.jsonl).
    auto edge_load = [&](uint32_t (&e)[K], const OddTile<K, R>& b, const typename Src::Id& i) {
        if constexpr (Src::kEdge) {
            const uint32_t fl = src.edge(i), eo = odd_edge_off(fl, (uint32_t)b.S, lane);
            if (HBEC_ODD_EDGE_COND == 0 || fl != 0u) {
#pragma unroll
                for (int j = 0; j < K; ++j) e[j] = ld_dw(b.in[j] + (fl != 0u ? (uint64_t)eo : (uint64_t)(uint32_t)b.c));
            }
        }
    };
    auto edge_code = [&](const uint32_t (&e)[K], const typename Src::Id& i) {
        if constexpr (Src::kEdge) {
            const uint32_t fl = src.edge(i);
            if (fl != 0u) {
                OddTile<K, R> b;
                src.at(b, i);
                odd_edges<K, R>(e, b, tab, tb, lane, fl);
            }
        }
    };
    typename Src::Id cur = src.id(wave0 + dw, n);
    OddRegs<K, R, U, MODE> X;
    // the edge words are carried through the loop unchanged by non-edge
    // tiles (an undefined value on that path was materialised as zeros,
    // each write waiting for the loads in flight: vmcnt(0) per tile)
    uint32_t e[K] = {};
    {
        OddTile<K, R> b;
        src.at(b, cur);
        edge_load(e, b, cur);
        odd_load<K, R, U, MODE, Src::kCarry>(X, b, lane);
        edge_code(e, cur);
    }
    typename Src::Id nxt = src.id(wave0 + dw + nw, n);
    for (uint32_t b0 = wave0 + nw; b0 < n; b0 += nw) {  // block-uniform trip count
        OddRegs<K, R, U, MODE> Y;
        {
            OddTile<K, R> b;
            src.at(b, nxt);
            edge_load(e, b, nxt);
            odd_load<K, R, U, MODE, Src::kCarry>(Y, b, lane);
        }
        // one block barrier per tile for apply; none for Verify (8+3 57 -> 66 %,
        // 6+3 63 -> 70 %, profiles/r03_tune_odd3.jsonl)
        if constexpr (MODE != kOddVerify) __builtin_amdgcn_s_barrier();
        const typename Src::Id after = src.id(b0 + dw + nw, n);
        {
            OddTile<K, R> b;
            src.at(b, cur);
            odd_finish<K, R, U, MODE, MIR, Src::kCarry>(X, b, tab, tb, lane, flags, mir);
        }
        edge_code(e, nxt);
        X = Y;
        cur = nxt;
        nxt = after;
    }
    OddTile<K, R> b;
    src.at(b, cur);
    odd_finish<K, R, U, MODE, MIR, Src::kCarry>(X, b, tab, tb, lane, flags, mir);
}

template <int K, int R, int MODE>
__global__ __launch_bounds__(kPipeBlockThreads, (odd_lb<K, R, MODE>())) void gf_odd(PassArgs a, uint32_t* flags) {
    constexpr int U = odd_u(K, MODE);
    odd_body<K, R, U, MODE>(OddStrided<K, R, U, MODE>{a}, a.n_tiles, a.tab, flags);
}

// ---------------------------------------------------------------------------
// Object records (strided batches).  Everything gf_odd's loads and finish need
// of an object's shards is fixed per object: the column frame, each loaded
// shard's dword-aligned block base and byte shift, each output's aligned block
// grid and guard band.  gf_odd_objrec (odd.hip) writes it once per object; the
// tile loop (gf_odd_rec) reads it with scalar loads issued a tile or two ahead
// and adds only the tile position.  The per-tile arithmetic this replaces
// (64-bit object bases of K + R shards and their alignment: ~250 SALU per tile
// at 8+3, profiles/r04_sq_odd.json) issued in the same slots as the field
// arithmetic at one wave per SIMD.
//
// Frame: columns at shard positions c0 + V, c0 = (-out0) mod 16 (output 0's
// 16-B grid), V = ti * span + 16 * column >= 0.
// Record (OddRec::RW words, 32-B multiples):
//   F part (finish), words [0, FW): [0] shifts (2 bits per loaded shard),
//     [1] realigns (4 bits per output), [2], [3] verify band (lo, width on V);
//     then per output r (apply / accumulate): Q lo, Q hi, lo, width.
//   L part (loads), words [FW, FW + LW): per loaded shard s (inputs, then
//     verify's stored parity): B lo, B hi, lim; accumulate passes then per
//     output: Q lo, Q hi, lo, lo + width (the old blocks are loaded too).
// Loaded shard s: the dword-aligned block holding column V's first byte is at
// B + min_u32(V, lim) (B = base + c0 rounded down to a dword, lim = S - 16 - t0
// keeps every block inside the shard; the clamp only moves columns the guard
// band keeps from any store).  Output r: block at Q + V, stored when
// (V - lo) <= width (unsigned).
// ---------------------------------------------------------------------------
template <int U, int MODE, bool CARRY>
__host__ __device__ constexpr uint32_t odd_rec_wcol(int u) { return CARRY ? 64u * (uint32_t)u : odd_store<MODE>() * (uint32_t)u; }

// Record kernels with K >= HBEC_ODD_LDS_MINK read the coefficient tables from
// LDS, one input at a time, instead of holding all 5 K R words in VGPRs
// (12+4: 240 words; the register-resident kernel spilled 134 SGPRs and ran
// at 40 % of 8 TB/s).
__host__ __device__ constexpr bool odd_rec_lds(int k) { return k >= HBEC_ODD_LDS_MINK; }
// record kernels (strided and plan tile lists) that code the guard band
// (HBEC_ODD_EDGE_FUSE bit 2; off: 8+3 / 10+4 records lost 3-4.5 points
// with it, the 8+3 / 4+2 plans 3, r06_ab_fuse.jsonl): apply, register tables or bit-plane (the LDS-table kernels, K >= 9, spilled
// 15-211 VGPRs with it and keep the gf_odd_edges launch)
// (Three tile-list instances spilled a pending scalar-load register into a
// VGPR lane with it — 4 x 4 tables, bit-plane 6+4 and 12+2 — and
// isa_check.py refused the library: they keep the gf_odd_edges_plan launch.)
__host__ __device__ constexpr bool odd_rec_edge(int k, int r, int mode, int xs, bool list) {
    return (HBEC_ODD_EDGE_FUSE & 2) != 0 && mode == kOddApply && (xs >= 0 || !odd_rec_lds(k)) &&
           !(list && ((xs < 0 && k == 4 && r == 4) || (xs >= 0 && ((k == 6 && r == 4) || (k == 12 && r == 2)))));
}
// record kernels run 2 waves per SIMD with LDS tables; the register-table
// ones at 1 (8+3 encode at 2 waves per SIMD, 256 VGPRs with 40 B of spill:
// 66.8 -> 59.3 %, profiles/r04_ab_odd.jsonl batch I)
__host__ __device__ constexpr bool odd_rec_two_blocks(int k, int, int) { return odd_rec_lds(k); }

// acc[r] ^= XOR_j C[r][j] x[j], input j's R tables (5 words each) at LDS byte
// address lt + 4 j odd_lt_stride(R), read by broadcast ds_read_b128 the
// compiler schedules and waits for (lgkmcnt(N), a few inputs ahead).  The
// base goes through an empty asm once per window, so the reads cannot be
// hoisted out of the tile loop into VGPRs (where the tables came from: 12+4
// held 240 table words and spilled).  The 3 K products per output dword are
// folded as in gf_dot.  (Reads issued by asm with a wait per input were
// 0.5-2 % slower: r04_ab_odd.jsonl batch J.)
template <int K, int R>
__device__ __forceinline__ void gf_dot_lds(u32x4 (&acc)[R], const u32x4 (&x)[K], uint32_t lt) {
    constexpr int TQ = (int)odd_lt_stride(R) / 4;
    uint32_t pend[4][R];
    typedef __attribute__((address_space(3))) const u32x4 lds_q;
    uint32_t z = lt;
    asm volatile("" : "+v"(z));  // opaque per window: the reads stay in the tile loop
    lds_q* tp = reinterpret_cast<lds_q*>(static_cast<uintptr_t>(z));
#pragma unroll
    for (int j = 0; j < K; ++j) {
        u32x4 t[TQ];
#pragma unroll
        for (int q = 0; q < TQ; ++q) t[q] = tp[j * TQ + q];
        const bool has = (j & 1) != 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const Sel sx = selectors(x[j][e]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t p0 = perm(t[(5 * r + 1) / 4][(5 * r + 1) % 4], t[(5 * r) / 4][(5 * r) % 4], sx.s0);
                const uint32_t p1 = perm(t[(5 * r + 3) / 4][(5 * r + 3) % 4], t[(5 * r + 2) / 4][(5 * r + 2) % 4], sx.s1);
                const uint32_t h4 = t[(5 * r + 4) / 4][(5 * r + 4) % 4];
                const uint32_t p2 = perm(h4, h4, sx.s2);
                if (!has) {
                    acc[r][e] = xor3(acc[r][e], p0, p1);
                    pend[e][r] = p2;
                } else {
                    acc[r][e] = xor3(acc[r][e], pend[e][r], p0);
                    acc[r][e] = xor3(acc[r][e], p1, p2);
                }
            }
        }
    }
    if constexpr ((K & 1) != 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][e] ^= pend[e][r];
    }
}

// gf_dot1 with the tables in LDS (gf_dot_lds layout): edge words of the
// LDS-table and bit-plane record kernels
template <int K, int R>
__device__ __forceinline__ void gf_dot_lds1(uint32_t (&acc)[R], const uint32_t (&x)[K], uint32_t lt) {
    constexpr int TQ = (int)odd_lt_stride(R) / 4;
    typedef __attribute__((address_space(3))) const u32x4 lds_q;
    uint32_t z = lt;
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0u;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        // one input's tables at a time: the address of input j depends on the
        // products of input j - 1 (an empty asm), so the reads are neither
        // hoisted out of the tile loop nor batched while both tiles' columns
        // are live (the bit-plane 8+3 kernel held 76 more VGPRs otherwise)
        asm volatile("" : "+v"(z) : "v"(acc[0]));
        lds_q* tp = reinterpret_cast<lds_q*>(static_cast<uintptr_t>(z));
        u32x4 t[TQ];
#pragma unroll
        for (int q = 0; q < TQ; ++q) t[q] = tp[j * TQ + q];
        const Sel sx = selectors(x[j]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t p0 = perm(t[(5 * r + 1) / 4][(5 * r + 1) % 4], t[(5 * r) / 4][(5 * r) % 4], sx.s0);
            const uint32_t p1 = perm(t[(5 * r + 3) / 4][(5 * r + 3) % 4], t[(5 * r + 2) / 4][(5 * r + 2) % 4], sx.s1);
            const uint32_t h4 = t[(5 * r + 4) / 4][(5 * r + 4) % 4];
            acc[r] = xor3(acc[r], p0, p1) ^ perm(h4, h4, sx.s2);
        }
    }
}

// ---------------------------------------------------------------------------
// Bit-plane field multiply for fixed coefficient matrices (the encode parity
// rows, xor_sched.h).  A lane's two 16-B columns of an input (the carried
// 2-window tile) are 8 dwords; an in-register 8 x 8 bit transpose within each
// byte lane turns them into 8 planes (plane b, bit 8 L + d = bit b of byte L
// of dword d), so multiplying every byte by a constant is a fixed XOR of
// planes, and the whole (8R x 8K) bit matrix of a pass is the straight-line
// network XorNet<XS>.  The same transpose (an involution) turns the 8R output
// planes back into bytes.  Per 32 bytes of every input: 48 K + 48 R transpose
// instructions plus the network (10+4: 672 + 272) against 8 K (5 + 4.5 R) for
// the v_perm tables (10+4: 1840), and no coefficient tables in registers or LDS.
// ---------------------------------------------------------------------------
// a <-> b delta swap of one transpose stage: a's bits (m << s) take b's bits
// m, b's bits m take a's bits (m << s) (two shifts, two v_bitop3 selects)
__device__ __forceinline__ void bp_swap(uint32_t& a, uint32_t& b, uint32_t s, uint32_t m) {
    const uint32_t hi = m << s;
    const uint32_t na = (a & ~hi) | ((b << s) & hi);
    const uint32_t nb = (b & ~m) | ((a >> s) & m);
    a = na;
    b = nb;
}

// 8 x 8 bit transpose within every byte lane of d[0..7]: bit b of byte L of
// d[w] <-> bit w of byte L of d[b]
__device__ __forceinline__ void bp_transpose8(uint32_t (&d)[8]) {
#pragma unroll
    for (int w = 0; w < 4; ++w) bp_swap(d[w], d[w + 4], 4u, 0x0F0F0F0Fu);
#pragma unroll
    for (int w = 0; w < 8; w += 4) {
        bp_swap(d[w], d[w + 2], 2u, 0x33333333u);
        bp_swap(d[w + 1], d[w + 3], 2u, 0x33333333u);
    }
#pragma unroll
    for (int w = 0; w < 8; w += 2) bp_swap(d[w], d[w + 1], 1u, 0x55555555u);
}

// acc0 / acc1 = C x0 / C x1 (two columns per lane, fresh accumulators)
template <int XS, int K, int R>
__device__ __forceinline__ void bp_dot2(u32x4 (&acc0)[R], u32x4 (&acc1)[R], const u32x4 (&x0)[K],
                                        const u32x4 (&x1)[K]) {
    static_assert(XorNet<XS>::K == K && XorNet<XS>::R == R, "schedule shape");
    uint32_t p[8 * K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        uint32_t d[8] = {x0[j][0], x0[j][1], x0[j][2], x0[j][3], x1[j][0], x1[j][1], x1[j][2], x1[j][3]};
        bp_transpose8(d);
#pragma unroll
        for (int b = 0; b < 8; ++b) p[8 * j + b] = d[b];
    }
    uint32_t o[8 * R];
    XorNet<XS>::run(p, o);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint32_t d[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) d[b] = o[8 * r + b];
        bp_transpose8(d);
        acc0[r] = u32x4{d[0], d[1], d[2], d[3]};
        acc1[r] = u32x4{d[4], d[5], d[6], d[7]};
    }
}

template <int K, int R, int MODE>
struct OddRec {
    static constexpr int NL = K + (MODE == kOddVerify ? R : 0);
    static constexpr int NO = MODE == kOddVerify ? 0 : R;
    static constexpr int FW = (4 + 4 * NO + 7) & ~7;
    // accumulate passes also load the old output blocks: Q lo, Q hi, lo, hi per output
    static constexpr int LA = MODE == kOddAcc ? 4 * R : 0;
    static constexpr int LW = (3 * NL + LA + 7) & ~7;
    static constexpr int RW = FW + LW;
};

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// Scalar loads issued by hand: the compiler re-issues loads of read-only
// memory right before their use (to save SGPRs), which exposed their latency
// once per tile.  odd_sload only issues; odd_swait (lgkmcnt(0), then an empty
// asm per vector) orders every use after the data has landed.
template <int N>
__device__ __forceinline__ void odd_sload(u32x8 (&v)[N], const uint32_t* p) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("s_load_dwordx8 %0, %1, %2" : "=s"(v[i]) : "s"(p), "n"(32 * i));
}
// odd_sload_now: the loads and their wait in ONE asm statement, for the
// shapes whose SGPR pressure makes the compiler spill or copy record
// registers (odd_rec_prefetch false): a copy placed between a split load and
// its wait would read registers the load has not filled yet.
template <int N>
__device__ __forceinline__ void odd_sload_now(u32x8 (&v)[N], const uint32_t* p) {
    // chunks of <= 4 loads, each with its wait (one asm statement per chunk)
#pragma unroll
    for (int i = 0; i < N; i += 4) {
        const uint32_t* q = p + 8 * i;
        if (N - i == 1) {
            asm volatile("s_load_dwordx8 %0, %1, 0\n s_waitcnt lgkmcnt(0)" : "=&s"(v[i]) : "s"(q) : "memory");
        } else if (N - i == 2) {
            asm volatile("s_load_dwordx8 %0, %2, 0\n s_load_dwordx8 %1, %2, 32\n s_waitcnt lgkmcnt(0)"
                         : "=&s"(v[i]), "=&s"(v[i + 1]) : "s"(q) : "memory");
        } else if (N - i == 3) {
            asm volatile("s_load_dwordx8 %0, %3, 0\n s_load_dwordx8 %1, %3, 32\n s_load_dwordx8 %2, %3, 64\n"
                         " s_waitcnt lgkmcnt(0)"
                         : "=&s"(v[i]), "=&s"(v[i + 1]), "=&s"(v[i + 2]) : "s"(q) : "memory");
        } else {
            asm volatile("s_load_dwordx8 %0, %4, 0\n s_load_dwordx8 %1, %4, 32\n s_load_dwordx8 %2, %4, 64\n"
                         " s_load_dwordx8 %3, %4, 96\n s_waitcnt lgkmcnt(0)"
                         : "=&s"(v[i]), "=&s"(v[i + 1]), "=&s"(v[i + 2]), "=&s"(v[i + 3]) : "s"(q) : "memory");
        }
    }
}

// Split loads (issued a tile ahead, waited after the next tile's arithmetic)
// only where the compiler keeps the record registers untouched in between:
// apply with K R <= 24 and Verify, register-resident tables.  The CPU test
// tests/test_kernel_resources.py::test_record_loads_unread_before_wait reads
// every shipped instance's code for such a read.
template <int K, int R, int MODE>
__host__ __device__ constexpr bool odd_rec_prefetch() {
    return !odd_rec_lds(K) && (MODE == kOddVerify || (MODE == kOddApply && K * R <= 24));
}
template <bool PF, int N>
__device__ __forceinline__ void odd_rec_sload(u32x8 (&v)[N], const uint32_t* p) {
    if constexpr (PF) {
        odd_sload(v, p);
    } else {
        odd_sload_now(v, p);
    }
}

// plan tile-list entries {record, tile}: 2-dword scalar loads, issued with
// the record loads (split where those are split) and waited with them
// (4-dword entries {record, tile, S, edge flags}: plan.cpp build_tile_lists)
typedef uint32_t u32x2s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void odd_sload_now2(u32x2s& v, const uint32_t* p) {
    asm volatile("s_load_dwordx4 %0, %1, 0\n s_waitcnt lgkmcnt(0)" : "=&s"(v) : "s"(p) : "memory");
}
template <bool PF>
__device__ __forceinline__ void odd_rec_sload2(u32x2s& v, const uint32_t* p) {
    if constexpr (PF) {
        asm volatile("s_load_dwordx4 %0, %1, 0" : "=s"(v) : "s"(p));
    } else {
        odd_sload_now2(v, p);
    }
}
__device__ __forceinline__ void odd_swait_pin2(u32x2s& v) { asm volatile("" : "+s"(v)); }

template <int N>
__device__ __forceinline__ void odd_swait_pin(u32x8 (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+s"(v[i]));
}
__device__ __forceinline__ void odd_swait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int N>
__device__ __forceinline__ uint32_t odd_w(const u32x8 (&v)[N], int i) { return v[i / 8][i % 8]; }

template <int K, int R, int MODE>
struct OddRT {  // the finish's scalars of one tile
    u32x8 f[OddRec<K, R, MODE>::FW / 8];
    uint32_t v0;  // ti * span
    uint32_t obj, live;
    // fused guard band: bits 30-31 the edge flags (1 first tile of its shard,
    // 2 last), bits 0-29 the shard length (the host fuses only S < 2^30)
    uint32_t edge;
};
__device__ __forceinline__ uint32_t odd_eflags(uint32_t e) { return e >> 30; }
__device__ __forceinline__ uint32_t odd_elen(uint32_t e) { return e & 0x3FFFFFFFu; }

template <int K, int R, int U, int MODE, bool CARRY, bool IMAJ = true, bool TEMP = false>
__device__ __forceinline__ void odd_rec_load(OddRegs<K, R, U, MODE>& X, const u32x8 (&l)[OddRec<K, R, MODE>::LW / 8],
                                             uint32_t v0, uint32_t lane) {
    using RC = OddRec<K, R, MODE>;
    // IMAJ (input-major): a shard's windows back to back, so the column a
    // tile shares with the next one (its last window's lanes 62-63, the next
    // tile's window 0) is requested by the two waves at the same point of
    // their load sequences (odd 8+3 bit-plane reads 1.052 -> 1.015 x its
    // bytes, 64.6 -> 65.6 %; profiles/r05_ab_bitplane.jsonl)
#pragma unroll
    for (int jj = 0; jj < RC::NL * U; ++jj) {
        const int j = IMAJ ? jj / U : jj % RC::NL;
        const int u = IMAJ ? jj % U : jj / RC::NL;
        const uint32_t v = v0 + 16u * odd_rec_wcol<U, MODE, CARRY>(u) + 16u * lane;
        const uint64_t b = (uint64_t)odd_w(l, 3 * j) | ((uint64_t)odd_w(l, 3 * j + 1) << 32);
        const uint64_t ad = b + __builtin_elementwise_min(v, odd_w(l, 3 * j + 2));
        X.x[u][j] = TEMP ? ld16_addr_t(ad) : ld16_addr(ad);
    }
    if constexpr (MODE == kOddAcc) {
        // the old output block each lane will rewrite, clamped into the band
        // (lanes that store nothing read one inside it)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            constexpr int o = 3 * RC::NL;
            const uint64_t q = (uint64_t)odd_w(l, o + 4 * r) | ((uint64_t)odd_w(l, o + 1 + 4 * r) << 32);
            const uint32_t lo = odd_w(l, o + 2 + 4 * r), hi = odd_w(l, o + 3 + 4 * r);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t v = v0 + 16u * odd_rec_wcol<U, MODE, CARRY>(u) + 16u * lane;
                X.x[u][K + r] = ld16_addr(q + __builtin_elementwise_min(__builtin_elementwise_max(v, lo), hi));
            }
        }
    }
}

// outputs pinned after the multiply: the gf_odd choice, and always with LDS
// tables (unpinned, 12+4 spilled 218 VGPRs at 2 blocks per CU)
template <int K, int R, int MODE>
__device__ __forceinline__ void odd_rec_pin(u32x4 (&acc)[R]) {
    if constexpr (odd_pin_on<K, R, MODE, false>() || odd_rec_lds(K)) {
#pragma unroll
        for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc[r]));
    }
}

template <int K, int R, int U, int MODE, bool CARRY, int XS = -1, class TB = Tables<K, R, kOddVMin>>
__device__ __forceinline__ void odd_rec_finish(const OddRegs<K, R, U, MODE>& X, const OddRT<K, R, MODE>& t,
                                               const TabArray& tab, const TB& tb,
                                               uint32_t lane, uint32_t* flags, uint32_t lt) {
    constexpr int NL = OddRec<K, R, MODE>::NL;
    const uint32_t shp = odd_w(t.f, 0), dlp = odd_w(t.f, 1);
    // v_alignbyte reads bits [1:0] of its shift: the packed shifts need no mask
    uint32_t sh[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) sh[j] = shp >> (2 * j);
    uint32_t dl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) dl[r] = (dlp >> (4 * r)) & 15u;
    auto st_mask = [&](int r, uint32_t v, uint32_t lanes) {
        return t.live != 0u && lane < lanes && (v - odd_w(t.f, 6 + 4 * r)) <= odd_w(t.f, 7 + 4 * r);
    };
    auto q_addr = [&](int r, uint32_t v) {
        return ((uint64_t)odd_w(t.f, 4 + 4 * r) | ((uint64_t)odd_w(t.f, 5 + 4 * r) << 32)) + v;
    };
    if constexpr (CARRY) {
        // U contiguous windows (2, or an even count for the bit-plane
        // kernels): window u < U - 1 takes its lane 63's missing next column
        // from window u + 1 and stores all 64 blocks, the last window 62
        static_assert(MODE != kOddVerify && (U == 2 || (XS >= 0 && U % 2 == 0)), "apply carry windows");
        u32x4 xw[U][K], acc[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j)
                xw[u][j] = u + 1 < U ? odd_shift_in_carry(X.x[u][j], sh[j], X.x[u + 1 < U ? u + 1 : u][j])
                                     : odd_shift_in(X.x[u][j], sh[j]);
        if constexpr (XS >= 0) {
#pragma unroll
            for (int u = 0; u < U; u += 2) bp_dot2<XS, K, R>(acc[u], acc[u + 1], xw[u], xw[u + 1]);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) acc[1][r] = acc[0][r] = u32x4{0, 0, 0, 0};
            gf_dot<K, R, kOddVMin>(acc[1], xw[1], tab, tb);
            gf_dot<K, R, kOddVMin>(acc[0], xw[0], tab, tb);
            odd_rec_pin<K, R, MODE>(acc[1]);
            odd_rec_pin<K, R, MODE>(acc[0]);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                u32x4 bk = acc[u][r];
                if (dl[r] != 0u)  // wave-uniform (never r = 0)
                    bk = realign16(acc[u][r], u + 1 < U ? lane_next4_carry(acc[u][r], acc[u + 1 < U ? u + 1 : u][r])
                                                        : lane_next4(acc[u][r]), dl[r]);
                if constexpr (MODE == kOddAcc) bk ^= X.x[u][K + r];
                const uint32_t v = t.v0 + 16u * lane + 1024u * (uint32_t)u;
                odd_st(q_addr(r, v), bk, st_mask(r, v, u + 1 < U ? 64u : kOddStore));
            }
        }
        return;
    } else if constexpr (XS >= 0 && MODE == kOddVerify) {
        // chained bit-plane Verify (VCHAIN in gf_odd_rec)
        static_assert(U % 2 == 0, "bit-plane column pairs");
        u32x4 xw[U][K], acc[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j)
                xw[u][j] = u + 1 < U ? odd_shift_in_carry(X.x[u][j], sh[j], X.x[u + 1 < U ? u + 1 : u][j])
                                     : odd_shift_in(X.x[u][j], sh[j]);
#pragma unroll
        for (int u = 0; u < U; u += 2) bp_dot2<XS, K, R>(acc[u], acc[u + 1], xw[u], xw[u + 1]);
        bool bad = false;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = t.v0 + 16u * (64u * (uint32_t)u + lane);
            const bool mine = t.live != 0u && (u + 1 < U || lane < 63u) && (v - odd_w(t.f, 2)) <= odd_w(t.f, 3);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const u32x4 st = u + 1 < U ? odd_shift_in_carry(X.x[u][K + r], sh[K + r], X.x[u + 1 < U ? u + 1 : u][K + r])
                                           : odd_shift_in(X.x[u][K + r], sh[K + r]);
                const u32x4 df = st ^ acc[u][r];
                bad |= mine && (df[0] | df[1] | df[2] | df[3]) != 0u;
            }
        }
        if (__any(bad)) {
            if (lane == 0u) atomicOr(flags + t.obj, 1u);
        }
    } else {
        bool bad = false;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t v = t.v0 + 16u * odd_rec_wcol<U, MODE, CARRY>(u) + 16u * lane;  // this lane's column
            u32x4 x[K];
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = odd_shift_in(X.x[u][j], sh[j]);
            u32x4 acc[R];
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
            if constexpr (odd_rec_lds(K)) {
                gf_dot_lds<K, R>(acc, x, lt);
            } else {
                gf_dot<K, R, kOddVMin>(acc, x, tab, tb);
            }
            odd_rec_pin<K, R, MODE>(acc);
            if constexpr (MODE == kOddVerify) {
                const bool mine = t.live != 0u && lane < odd_store<MODE>() && (v - odd_w(t.f, 2)) <= odd_w(t.f, 3);
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
                    if constexpr (MODE == kOddAcc) blk ^= X.x[u][K + r];
                    odd_st(q_addr(r, v), blk, st_mask(r, v, kOddStore));
                }
            }
        }
        if constexpr (MODE == kOddVerify) {
            if (__any(bad)) {
                if (lane == 0u) atomicOr(flags + t.obj, 1u);
            }
        }
    }  // !CARRY
}

// the fused guard band of an edge tile (gf_odd_rec EDGE)
template <int K, int R, int MODE, int XS, class TB>
__device__ __forceinline__ void odd_rec_edges(const uint32_t (&e)[K], const OddRT<K, R, MODE>& t,
                                              const TabArray& tab, const TB& tb, uint32_t lane, uint32_t lt) {
    {
        if (t.edge != 0u) {  // wave-uniform: the tile starts or ends its shard
            const uint32_t fl = odd_eflags(t.edge), S = odd_elen(t.edge);
            const uint32_t w1 = odd_w(t.f, 1), c = w1 >> 16;  // frame start C (record word 1, bits 16..)
            // input j's byte at position p: its base mod 4 is (t0 - C) mod 4, t0 mod 4 the packed shift
            const uint32_t shp = odd_w(t.f, 0), p = odd_edge_off(fl, S, lane);
            uint32_t acc[R], x[K];
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = odd_edge_byte(e[j], (shp >> (2 * j)) - c + p);
            if constexpr (XS >= 0 || odd_rec_lds(K)) {
                gf_dot_lds1<K, R>(acc, x, lt);
            } else {
                gf_dot1<K, R, kOddVMin>(acc, x, tab, tb);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t d = (w1 >> (4 * r)) & 15u;
                const uint64_t q = (uint64_t)odd_w(t.f, 4 + 4 * r) | ((uint64_t)odd_w(t.f, 5 + 4 * r) << 32);
                const uint32_t h = c + d + odd_w(t.f, 6 + 4 * r), e = h + odd_w(t.f, 7 + 4 * r) + 16u;
                odd_edge_store(q - (uint64_t)(c + d), acc[r], fl, S, lane, h, e, true);
            }
        }
    }
}

// A wave's tiles t0, t0 + nw, ...: (object, tile in object), stepped by
// (qq, rr) = divmod(nw, tpo).  Stand-in tiles past the end (obj >= n_obj)
// load the last tile and store nothing.
struct OddPos {
    uint32_t obj, ti;
    uint32_t se;  // plans (LIST): the stripe's S | edge flags << 30; bit 29: edge bytes only (no main stores)
};

// LDS-table record kernels fit 2 blocks per CU (2 waves per SIMD); the
// bit-plane kernels (XS >= 0) HBEC_ODD_BP_BPC (tuning.h)
// bit-plane Verify: 2 blocks per CU (2 waves per SIMD, the read-only
// kernels' occupancy) where K R <= 27 fits them in 256 VGPRs
__host__ __device__ constexpr int odd_bp_bpc(int k, int r, int mode) {
    return mode == kOddVerify && k * r <= 27 ? HBEC_ODD_BPC_VERIFY : HBEC_ODD_BP_BPC;
}
template <int K, int R, int MODE, int XS = -1>
__host__ __device__ constexpr int odd_rec_lb() {
    return XS >= 0 ? odd_bp_bpc(K, R, MODE) : (odd_rec_two_blocks(K, R, MODE) ? 2 : odd_lb<K, R, MODE>());
}
// Bit-plane record kernels: the carried 2-window tile (both columns of a
// lane form one 32-byte plane group), apply only
__host__ __device__ constexpr int odd_bp_u() { return HBEC_ODD_BP_U; }
// waves per block (one block per CU): 3 from K R >= 48 (12+4 encode 58.3 ->
// 62.9 %, 10+4 lost 2-3 points at 3; r05_ab_bitplane.jsonl)
__host__ __device__ constexpr int odd_bp_wpb(int k, int r) {
    return k * r >= HBEC_ODD_BP_WPB3_MINKR ? 3 : HBEC_ODD_BP_WPB;
}
// split record loads only without SGPR spills (K R <= 24, as odd_rec_prefetch:
// 8+4 / 10+4 / 12+4 spill 1-21 SGPRs into VGPR lanes)
template <int K, int R, int MODE>
__host__ __device__ constexpr bool odd_bp_prefetch() { return HBEC_ODD_BP_PF != 0 && K * R <= 24; }

// LIST (plans): tile t codes tile list[t].ti of record list[t].rec (one
// 8-byte entry per tile, plan.cpp build_tile_lists), so stripes of any mix
// of lengths share one launch with no idle tiles; the strided batches derive
// (object, tile) from t by division.  A tile's entry is loaded one step
// before its record loads need it, together with the previous record loads
// (no extra wait; the build-time check covers these split loads too).
template <int K, int R, int MODE, int XS = -1, bool LIST = false>
__global__ __launch_bounds__(kPipeBlockThreads, (odd_rec_lb<K, R, MODE, XS>())) void gf_odd_rec(PassArgs a, uint32_t* flags,
                                                                                            const uint32_t* __restrict__ recs) {
    using RC = OddRec<K, R, MODE>;
    constexpr bool BP = XS >= 0;
    static_assert(!BP || MODE != kOddAcc, "bit-plane records: apply and Verify");
    constexpr bool PF = BP ? odd_bp_prefetch<K, R, MODE>() : odd_rec_prefetch<K, R, MODE>();
    constexpr int U = BP ? odd_bp_u() : odd_u(K, MODE);
    constexpr bool CARRY = odd_rec_carry(U, MODE);
    // bit-plane Verify: U chained windows (window u < U - 1 compares all 64
    // columns, lane 63 borrowing window u + 1's first dword; the last 63), so
    // a tile reads only its own 64-B lines but the one it shares with the next
    constexpr bool VCHAIN = BP && MODE == kOddVerify;
    constexpr bool LDS = !BP && odd_rec_lds(K);
    // input-major loads, except the 3-wave bit-plane blocks (12+4: 61.8 % window-major vs 59.2 %)
    constexpr bool IMAJ = !(BP && odd_bp_wpb(K, R) == 3);
    // input loads with the temporal hint (HBEC_ODD_TEMP): the window-major
    // strided apply keeps the lines its neighbour tiles share in L2
    constexpr bool TEMP = MODE == kOddVerify ? (HBEC_ODD_TEMP & 1) != 0
                                             : MODE == kOddApply && ((HBEC_ODD_TEMP & 2) != 0 ||
                                                                     ((HBEC_ODD_TEMP & 4) != 0 && !IMAJ && !LIST));
    // apply: the guard-band bytes in the shard's first / last tile
    // (HBEC_ODD_EDGE_FUSE; plans: the tile list's entry flags)
    constexpr bool EDGE = odd_rec_edge(K, R, MODE, XS, LIST);
    constexpr uint32_t SPAN = VCHAIN ? (64u * U - 1u) * 16u : odd_rec_span(U, MODE);
    constexpr uint32_t WPB = BP ? (uint32_t)odd_bp_wpb(K, R) : kPipeBlockThreads / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * WPB;
    const uint32_t n = a.n_tiles, tpo = a.tiles_per_obj, n_obj = (uint32_t)a.n_obj;
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(xcd_block() * WPB);
    const uint32_t dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave0 >= n) return;  // whole blocks only: the loop below has block barriers
    // LDS tables: the LDS-table kernels, and the bit-plane kernels' edge words
    constexpr bool LDST = LDS || (EDGE && BP);
    __shared__ __attribute__((aligned(16))) uint32_t ltab[LDST ? K * odd_lt_stride(R) : 4];
    if constexpr (LDST) {
        // whole blocks reach this point (the early return above is per block)
        const uint32_t ts = odd_lt_stride(R);
        for (uint32_t i = threadIdx.x; i < (uint32_t)K * ts; i += blockDim.x) {
            const uint32_t j = i / ts, w = i - j * ts;
            ltab[i] = w < (uint32_t)(R * 5) ? a.tab[w / 5][j][w % 5] : 0u;
        }
        __syncthreads();
    }
    const uint32_t lt = (uint32_t)reinterpret_cast<uintptr_t>(&ltab[0]);  // LDS offset (low half of the flat address)
    using TB = std::conditional_t<BP, Tables<1, 1, kOddVMin>, Tables<K, R, kOddVMin>>;
    TB tb{};
    if constexpr (!BP) tb = load_tables<K, R, kOddVMin>(a.tab);
    const uint32_t qq = LIST ? 0u : nw / tpo, rr = LIST ? 0u : nw - qq * tpo;
    // LIST: p = {record, tile} of the tile the record loads are for, pe the
    // entry of the tile after it (a scalar load issued with those record
    // loads and waited with them); tq = p's tile index
    uint32_t tq = wave0 + dw;
    u32x2s pe{0u, 0u};
    auto lentry = [&](uint32_t t) { return a.list + kOddListWords * (t < n ? t : n - 1u); };
    auto step = [&](OddPos p) {
        if constexpr (LIST) {
            tq += nw;
            return OddPos{pe[0], pe[1], pe[2]};
        } else {
            p.ti += rr;
            p.obj += qq;
            if (p.ti >= tpo) {
                p.ti -= tpo;
                p.obj += 1u;
            }
            return p;
        }
    };
    auto rec = [&](const OddPos& p) {
        return recs + (size_t)__builtin_amdgcn_readfirstlane(LIST || p.obj < n_obj ? p.obj : n_obj - 1u) * RC::RW;
    };
    auto v0 = [&](const OddPos& p) { return (LIST || p.obj < n_obj ? p.ti : tpo - 1u) * SPAN; };
    // Each step issues the next tile's loads (P, L = its load record,
    // waited), fetches the tile after it's load record into L and P's finish
    // record, codes the current tile, then copies the next tile's registers
    // over the current ones.
    OddPos p;
    if constexpr (LIST) {
        odd_sload_now2(pe, lentry(tq));
        p = OddPos{pe[0], pe[1], pe[2]};
        odd_sload_now2(pe, lentry(tq + nw));
    } else {
        const uint32_t t = wave0 + dw;
        p.obj = t / tpo;
        p.ti = t - p.obj * tpo;
        p.se = 0u;
    }
    u32x8 L[RC::LW / 8];
    OddRT<K, R, MODE> tx, ty;
    OddRegs<K, R, U, MODE> X, Y;
    // strided: every shard has >= 2 tiles when the host fuses; plans: the
    // entry's flags (a one-tile stripe has two entries, head and tail, the
    // second with bit 2: its main stores are the first entry's)
    const bool fuse = (a.fuse & 1u) != 0u;
    auto fill = [&](OddRT<K, R, MODE>& tt, const OddPos& q) {
        tt.v0 = v0(q);
        tt.obj = q.obj;
        if constexpr (LIST) {
            const bool in = tq < n;
            tt.live = in && (q.se & (1u << 29)) == 0u ? 1u : 0u;
            tt.edge = EDGE && fuse && in ? (q.se & ~(1u << 29)) : 0u;
        } else {
            tt.live = q.obj < n_obj ? 1u : 0u;
            const uint32_t fl = q.ti == 0u ? 1u : (q.ti + 1u == tpo ? 2u : 0u);
            tt.edge = EDGE && fuse && tt.live && fl ? (fl << 30) | (uint32_t)a.shard_len : 0u;
        }
    };
    // EDGE: the shard base of loaded shard j is B_j + lim_j + 16 - (S & ~3)
    // (record: B = base + C rounded down to a dword, lim = S - 16 - (C +
    // (base & 3) rounded down) with base & 3 in its low 2 bits)
    // Fused guard band: a tile's K edge words are loaded right before its
    // columns and coded at the end of the same step (its finish record has
    // arrived by then), after the previous tile's finish: they never cross
    // the loop's back edge (a loop-carried copy waited for the next tile's
    // loads: 8+3 60 -> 43 %)
    auto edge_load = [&](uint32_t (&e)[K], const OddRT<K, R, MODE>& tz) {
        if constexpr (EDGE) {
            const uint32_t fl = odd_eflags(tz.edge), S = odd_elen(tz.edge), s4 = S & ~3u;
            const uint32_t eo = odd_edge_off(fl, S, lane);
            if (HBEC_ODD_EDGE_COND != 0 && fl == 0u) return;  // edge tiles only (as odd_body)
#pragma unroll
            for (int j = 0; j < K; ++j) {
                // other tiles: the byte at the tile's first column of shard j
                // (a line the tile's own loads fetch; one line for every wave
                // of the launch made an L2 hot spot: -10 to -15 points)
                const uint64_t bj = (uint64_t)odd_w(L, 3 * j) | ((uint64_t)odd_w(L, 3 * j + 1) << 32);
                const uint32_t lim = odd_w(L, 3 * j + 2);
                const uint64_t off = fl != 0u ? (uint64_t)(int64_t)(int32_t)(lim + 16u - s4 + eo)
                                                   : (uint64_t)(tz.v0 < lim ? tz.v0 : lim);
                e[j] = ld_dw(bj + off);
            }
        }
    };
    odd_rec_sload<PF>(L, rec(p) + RC::FW);
    odd_swait();
    odd_swait_pin(L);
    fill(tx, p);
    // the edge words are carried through the loop unchanged by non-edge
    // tiles (an undefined value on that path was materialised as zeros,
    // each write waiting for the loads in flight: vmcnt(0) per tile)
    uint32_t ex[K] = {};
    edge_load(ex, tx);
    odd_rec_load<K, R, U, MODE, CARRY || VCHAIN, IMAJ, TEMP>(X, L, tx.v0, lane);
    odd_rec_sload<PF>(tx.f, rec(p));
    p = step(p);
    odd_rec_sload<PF>(L, rec(p) + RC::FW);
    if constexpr (LIST) odd_rec_sload2<PF>(pe, lentry(tq + nw));
    odd_swait();
    odd_swait_pin(L);
    odd_swait_pin(tx.f);
    if constexpr (LIST) odd_swait_pin2(pe);
    if constexpr (EDGE) odd_rec_edges<K, R, MODE, XS>(ex, tx, a.tab, tb, lane, lt);
    auto half = [&](OddRegs<K, R, U, MODE>& Z, OddRT<K, R, MODE>& tz, const OddRegs<K, R, U, MODE>& W,
                    const OddRT<K, R, MODE>& tw) {
        fill(tz, p);
        uint32_t (&ez)[K] = ex;
        edge_load(ez, tz);
        odd_rec_load<K, R, U, MODE, CARRY || VCHAIN, IMAJ, TEMP>(Z, L, tz.v0, lane);
        odd_rec_sload<PF>(tz.f, rec(p));
        p = step(p);
        odd_rec_sload<PF>(L, rec(p) + RC::FW);
        if constexpr (LIST) odd_rec_sload2<PF>(pe, lentry(tq + nw));
        // (s_sleep pacing after these loads: no effect on the bit-plane kernels, r05_ab_bitplane.jsonl r5_ab4)
        // bit-plane Verify at 2 waves per SIMD: a block barrier per tile keeps
        // the waves sharing tile-boundary lines together (8+3 77.2 -> 78.4 %,
        // reads 1.054 -> 1.026 x); at one wave per SIMD it costs 10 points
        if constexpr (MODE != kOddVerify || (VCHAIN && HBEC_ODD_BP_VBARRIER && odd_bp_bpc(K, R, MODE) >= 2))
            __builtin_amdgcn_s_barrier();
        odd_rec_finish<K, R, U, MODE, CARRY, XS>(W, tw, a.tab, tb, lane, flags, lt);
        odd_swait();
        odd_swait_pin(L);
        odd_swait_pin(tz.f);
        if constexpr (LIST) odd_swait_pin2(pe);
        if constexpr (EDGE) odd_rec_edges<K, R, MODE, XS>(ez, tz, a.tab, tb, lane, lt);
    };
    for (uint32_t b0 = wave0 + nw; b0 < n; b0 += nw) {  // block-uniform trip count
        half(Y, ty, X, tx);
        X = Y;
        tx = ty;
    }
    odd_rec_finish<K, R, U, MODE, CARRY, XS>(X, tx, a.tab, tb, lane, flags, lt);
}

template <int K, int R, int MODE, bool MIR = false, bool CARRY = false>
__global__ __launch_bounds__(kPipeBlockThreads, (odd_lb<K, R, MODE, MIR>())) void gf_odd_plan(UPlanArgs p, const URec* __restrict__ recs) {
    using Src = OddPlan<K, R, MIR, CARRY>;
    odd_body<K, R, odd_plan_u<K>(0), MODE, Src, MIR>(Src{p, recs}, p.n_recs * Src::SUB, p.tab, nullptr, p.mirror);
}

// ---------------------------------------------------------------------------
// launch table: kernel of (K, r, mode, plan?, mirrored?)
// ---------------------------------------------------------------------------
// variant: plans, the carried-record kernel; strided, the object-record
// kernel (gf_odd_rec) instead of gf_odd
template <int K, int R, int MODE>
static const void* odd_pick(bool plan, bool mirror, bool variant, bool list = false) {
    const bool carry = variant;
    if (!plan) {
        if constexpr (MODE != kOddVerify) {  // plans never verify
            if (list) return (const void*)&gf_odd_rec<K, R, MODE, -1, true>;
        }
        if (list) return nullptr;
        return variant ? (const void*)&gf_odd_rec<K, R, MODE> : (const void*)&gf_odd<K, R, MODE>;
    }
    if constexpr (MODE != kOddVerify) {  // plans never verify
        if (mirror) return (const void*)&gf_odd_plan<K, R, MODE, true>;
        if constexpr (odd_plan_u<K>(0) == 2) {
            if (carry) return (const void*)&gf_odd_plan<K, R, MODE, false, true>;
        }
        return (const void*)&gf_odd_plan<K, R, MODE>;
    }
    return nullptr;
}

template <int K, int MODE>
static const void* odd_for_r(int r, bool plan, bool mirror, bool carry, bool list) {
    switch (r) {
        case 1: return odd_pick<K, 1, MODE>(plan, mirror, carry, list);
        case 2: return odd_pick<K, 2, MODE>(plan, mirror, carry, list);
        case 3: return odd_pick<K, 3, MODE>(plan, mirror, carry, list);
        case 4: return odd_pick<K, 4, MODE>(plan, mirror, carry, list);
    }
    return nullptr;
}

template <int K>
static const void* odd_kernel_k(int r, int mode, bool plan, bool mirror, bool carry, bool list) {
    switch (mode) {
        case kOddApply: return odd_for_r<K, kOddApply>(r, plan, mirror, carry, list);
        case kOddAcc: return odd_for_r<K, kOddAcc>(r, plan, mirror, carry, list);
        case kOddVerify: return (plan || list) ? nullptr : odd_for_r<K, kOddVerify>(r, false, false, carry, false);
    }
    return nullptr;
}

template <int K0, int K1>
static const void* odd_kernel_range(int k, int r, int mode, bool plan, bool mirror, bool carry = false,
                                    bool list = false) {
    if constexpr (K0 > K1) {
        return nullptr;
    } else {
        if (k == K0) return odd_kernel_k<K0>(r, mode, plan, mirror, carry, list);
        return odd_kernel_range<K0 + 1, K1>(k, r, mode, plan, mirror, carry, list);
    }
}

// bit-plane record kernel of kXorShapes[xs] (odd_bp.hip), mode 0; list: the
// plan tile-list instance
const void* odd_kernel_bp(int xs, int mode, bool list);

// the other translation units' ranges
const void* odd_kernel_k58(int k, int r, int mode, bool plan, bool mirror, bool variant, bool list);
const void* odd_kernel_k912(int k, int r, int mode, bool plan, bool mirror, bool variant, bool list);

}  // namespace hbec
