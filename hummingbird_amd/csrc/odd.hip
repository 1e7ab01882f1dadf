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
//
// This unit: K <= 4 kernels, the edge / mirror-copy kernels and the host
// launchers; the templates are in odd_impl.h.
#include <atomic>

#include "internal.h"
#include "odd_impl.h"

namespace hbec {

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
// SLOTS per shard: kOddEdgeSlots (shards of any length; all of a shard of
// S <= kOddMinMain), or kOddEdgeSlotsLong for S > kOddMinMain: the head
// [0, qmin) and tail [qmax + 16, S) lie in [0, 64) and [S - 64, S)
// (qmin <= G + 15, qmax >= S - G - 31), so each 64-lane wave then codes
// exactly one end of one shard
template <int SLOTS = kOddEdgeSlots>
__device__ __forceinline__ bool odd_edge_pos(int32_t S, uint64_t out_frame, int32_t slot, int32_t* pos) {
    if (SLOTS == kOddEdgeSlots && S <= kOddEdgeSlots) {
        *pos = slot;
        return slot < S;
    }
    const int32_t e = (int32_t)((16u - ((uint32_t)out_frame & 15u)) & 15u);  // aligned block positions = e mod 16
    const int32_t qmin = kOddGuard + e;
    const int32_t top = S - kOddGuard - 16;
    const int32_t qmax = top - ((top - e) & 15);
    if (slot < SLOTS / 2) {
        *pos = slot;
        return slot < qmin;
    }
    *pos = S - SLOTS + slot;
    return *pos >= qmax + 16;
}

// One edge position p of every output of a pass: the K input bytes are
// loaded once and their selectors shared by the R outputs (the table words
// tab[r][j] are wave-uniform: scalar loads); output r is coded, stored or
// compared only where position p is in r's guard band (odd_edge_pos on r's
// frame).  MODE: apply, accumulate (out ^= ...), verify (flag the object).
template <int MODE, int SLOTS = kOddEdgeSlots>
__device__ __forceinline__ void odd_edge_all(const TabArray& tab, int K, int r0, int R, const uint64_t* in,
                                             const uint64_t* out, uint64_t vframe, int32_t S, int32_t slot,
                                             uint32_t* flag) {
    bool act[kMaxR] = {false, false, false, false};
    int32_t pos[kMaxR];
    bool any = false;
    for (int r = r0; r < R; ++r) {
        act[r] = odd_edge_pos<SLOTS>(S, MODE == kOddVerify ? vframe : out[r], slot, &pos[r]);
        any |= act[r];
    }
    if (!any) return;
    // every active output's position is the same byte of the shard: the
    // guard band differs per output only in where it ends
    int32_t p = 0;
    for (int r = r0; r < R; ++r)
        if (act[r]) p = pos[r];
    uint32_t v[kMaxR] = {0u, 0u, 0u, 0u};
    for (int j = 0; j < K; ++j) {
        const Sel s = selectors(*reinterpret_cast<const gu8_t*>(in[j] + (uint64_t)p));
        for (int r = r0; r < R; ++r) {
            const uint32_t* t = tab[r][j];
            v[r] ^= gf_mul_sel(s, t[0], t[1], t[2], t[3], t[4]);
        }
    }
    for (int r = r0; r < R; ++r) {
        if (!act[r]) continue;
        gu8_t* d = reinterpret_cast<gu8_t*>(out[r] + (uint64_t)p);
        uint32_t val = v[r] & 0xFFu;
        if (MODE == kOddVerify) {
            if (val != *d) atomicOr(flag, 1u);
        } else {
            if (MODE == kOddAcc) val ^= *d;
            *d = (uint8_t)val;
        }
    }
}

// one thread per (object, edge slot) for all R outputs, or (split: calls of
// few objects, where latency and not lines bound the kernel) per (object,
// output, slot); 32-bit index math below 2^32 threads (< 6 M objects)
template <int MODE, bool SPLIT, int SLOTS>
__global__ __launch_bounds__(kBlockThreads) void gf_odd_edges(PassArgs a, int K, int R, uint32_t* flags) {
    const uint32_t groups = SPLIT ? (uint32_t)R : 1u;  // (a constant divisor when not split)
    const uint64_t per = (uint64_t)groups * SLOTS;
    const uint64_t total = a.n_obj * per;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += step) {
        uint64_t obj;
        uint32_t rs;
        if (total < (1ull << 32)) {
            const uint32_t o = (uint32_t)v / (uint32_t)per;
            obj = o;
            rs = (uint32_t)v - o * (uint32_t)per;
        } else {
            obj = v / per;
            rs = (uint32_t)(v - obj * per);
        }
        const uint32_t g = rs / (uint32_t)SLOTS;
        const int32_t slot = (int32_t)(rs - g * (uint32_t)SLOTS);
        uint64_t in[kMaxK], out[kMaxR];
        for (int j = 0; j < K; ++j) in[j] = reinterpret_cast<uint64_t>(a.in[j]) + obj * a.in_stride[j];
        for (int r = 0; r < R; ++r) out[r] = reinterpret_cast<uint64_t>(a.out[r]) + obj * a.out_stride[r];
        odd_edge_all<MODE, SLOTS>(a.tab, K, SPLIT ? (int)g : 0, SPLIT ? (int)g + 1 : R, in, out, out[0],
                           (int32_t)a.shard_len, slot, flags + obj);
    }
}

// plans: one edge record per stripe / object (URec, p0 unused)
template <int MODE, bool SPLIT, int SLOTS>
__global__ __launch_bounds__(kBlockThreads) void gf_odd_edges_plan(UPlanArgs p, const URec* __restrict__ erecs,
                                                                  uint32_t n_erecs, int K, int R) {
    const uint64_t per = (uint64_t)(SPLIT ? R : 1) * SLOTS;
    const uint64_t total = (uint64_t)n_erecs * per;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t e = (uint32_t)(v / per);
        const uint32_t rs = (uint32_t)(v - (uint64_t)e * per);
        const uint32_t g = rs / (uint32_t)SLOTS;
        const int32_t slot = (int32_t)(rs - g * (uint32_t)SLOTS);
        const URec rec = erecs[e];
        const uint64_t S = rec.shard_len;
        uint64_t in[kMaxK], out[kMaxR];
        for (int j = 0; j < K; ++j) in[j] = (((p.in_sel >> j) & 1u) ? rec.b : rec.a) + (uint64_t)p.in_idx[j] * S;
        for (int r = 0; r < R; ++r) out[r] = (((p.out_sel >> r) & 1u) ? rec.b : rec.a) + (uint64_t)p.out_idx[r] * S;
        odd_edge_all<MODE, SLOTS>(p.tab, K, SPLIT ? (int)g : 0, SPLIT ? (int)g + 1 : R, in, out, out[0], (int32_t)S,
                                  slot, nullptr);
    }
}

// ---------------------------------------------------------------------------
// gf_odd_objrec / gf_odd_planrec: the object records gf_odd_rec reads (layout:
// OddRec, odd_impl.h), one thread per object of a strided pass or per stripe
// of a plan.  mode 2 (verify) records the stored parity as loaded shards
// K..K+R-1 and the compared band.  A shard of S <= kOddMinMain (plans only)
// gets empty bands: its tiles store nothing.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t ceil16(int32_t x) { return (x + 15) & ~15; }
__device__ __forceinline__ int32_t floor16(int32_t x) { return x & ~15; }

// in_b(s) / out_b(r): the byte address of loaded shard s / output r
template <class InB, class OutB>
__device__ __forceinline__ void odd_rec_write(int K, int R, int mode, int32_t S, InB in_b, OutB out_b, uint32_t* f,
                                              uint32_t* l) {
    // frame: output 0's 16-B grid, first column at c0 in [kOddFrame, kOddFrame + 16)
    const int32_t c0 = (int32_t)((0u - (uint32_t)out_b(0)) & 15u) + kOddFrame;
    const int32_t hi = S - kOddGuard - 16;  // last block start stored / compared
    const bool main = S > kOddMinMain;
    const int NL = K + (mode == kOddVerify ? R : 0), NO = mode == kOddVerify ? 0 : R;
    uint32_t shp = 0, dlp = 0;
    for (int s = 0; s < NL; ++s) {
        const uint64_t b = s < K ? in_b(s) : out_b(s - K);
        const int32_t t0 = (int32_t)(b & 3u) + c0;  // column 0's first byte, from the shard's dword base
        const uint64_t base = (b & ~(uint64_t)3) + (uint64_t)(t0 & ~3);
        l[3 * s] = (uint32_t)base;
        l[3 * s + 1] = (uint32_t)(base >> 32);
        // blocks end inside the shard's dwords; the low 2 bits (S mod 4 in the
        // exact limit: the clamp moves by < 4 B, below every stored column)
        // carry base mod 4 for the fused guard band (gf_odd_rec EDGE)
        l[3 * s + 2] = main ? (((uint32_t)(S - 16 - (t0 & ~3)) & ~3u) | (uint32_t)(b & 3u)) : 0u;
        shp |= ((uint32_t)t0 & 3u) << (2 * s);
    }
    for (int r = 0; r < NO; ++r) {
        const uint64_t o = out_b(r);
        const uint32_t dl = (0u - ((uint32_t)o + (uint32_t)c0)) & 15u;
        const uint64_t q = o + (uint64_t)(c0 + (int32_t)dl);  // 16-B aligned
        int32_t lo = ceil16(kOddGuard - c0 - (int32_t)dl), top = floor16(hi - c0 - (int32_t)dl);
        if (!main) lo = -16, top = -32;  // (V - lo) <= width holds for no V < 2^31
        const uint32_t width = (uint32_t)(top >= lo ? top - lo : 0);
        f[4 + 4 * r] = (uint32_t)q;
        f[5 + 4 * r] = (uint32_t)(q >> 32);
        f[6 + 4 * r] = (uint32_t)lo;
        f[7 + 4 * r] = width;
        if (mode == kOddAcc) {  // the old blocks, loaded with the inputs
            l[3 * NL + 4 * r] = (uint32_t)q;
            l[3 * NL + 4 * r + 1] = (uint32_t)(q >> 32);
            l[3 * NL + 4 * r + 2] = main ? (uint32_t)lo : 0u;
            l[3 * NL + 4 * r + 3] = main ? (uint32_t)lo + width : 0u;
        }
        dlp |= dl << (4 * r);
    }
    int32_t vlo = ceil16(kOddGuard - c0), vtop = floor16(hi - c0);
    if (!main) vlo = -16, vtop = -32;
    f[0] = shp;
    f[1] = dlp | ((uint32_t)c0 << 16);  // frame start C for the fused guard band
    f[2] = (uint32_t)vlo;
    f[3] = (uint32_t)(vtop >= vlo ? vtop - vlo : 0);
}

__global__ __launch_bounds__(kBlockThreads) void gf_odd_objrec(PassArgs a, int K, int R, int mode, uint32_t fw,
                                                              uint32_t rw, uint32_t* __restrict__ recs) {
    const uint64_t obj = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (obj >= a.n_obj) return;
    uint32_t* f = recs + obj * rw;
    odd_rec_write(
        K, R, mode, (int32_t)a.shard_len,
        [&](int s) { return reinterpret_cast<uint64_t>(a.in[s]) + obj * a.in_stride[s]; },
        [&](int r) { return reinterpret_cast<uint64_t>(a.out[r]) + obj * a.out_stride[r]; }, f, f + fw);
}

// plans: one record per stripe / object record (URec: a = stripe or data
// arena, b = parity arena, shard i of a base at i * S)
__global__ __launch_bounds__(kBlockThreads) void gf_odd_planrec(UPlanArgs p, const URec* __restrict__ orecs,
                                                               uint32_t n, int K, int R, int mode, uint32_t fw,
                                                               uint32_t rw, uint32_t* __restrict__ recs) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const URec rec = orecs[e];
    const uint64_t S = rec.shard_len;
    uint32_t* f = recs + (uint64_t)e * rw;
    odd_rec_write(
        K, R, mode, (int32_t)S,
        [&](int s) { return (((p.in_sel >> s) & 1u) ? rec.b : rec.a) + (uint64_t)p.in_idx[s] * S; },
        [&](int r) { return (((p.out_sel >> r) & 1u) ? rec.b : rec.a) + (uint64_t)p.out_idx[r] * S; }, f, f + fw);
}

static uint32_t odd_rec_fw(int r, int mode) { return (uint32_t)((4 + 4 * (mode == kOddVerify ? 0 : r) + 7) & ~7); }

uint32_t odd_waves_per_block(int xs) {
    return xs >= 0 && xs < kXorShapeCount ? (uint32_t)odd_bp_wpb(kXorShapes[xs].k, kXorShapes[xs].R)
                                          : kPipeBlockThreads / 64;
}

uint32_t odd_rec_words(int k, int r, int mode) {
    const int nl = k + (mode == kOddVerify ? r : 0), la = mode == kOddAcc ? 4 * r : 0;
    return odd_rec_fw(r, mode) + (uint32_t)((3 * nl + la + 7) & ~7);
}

bool odd_uses_records(int k, int r) { return odd_use_rec(k, r); }

hipError_t launch_odd_objrec(int k, int r, int mode, const PassArgs& a, uint32_t* recs, hipStream_t stream) {
    if (a.n_obj == 0) return hipSuccess;
    if (k < 1 || k > kOddMaxK || r < 1 || r > kMaxR || !pos32_shard(a.shard_len) || a.shard_len <= kOddMinMain)
        return hipErrorInvalidValue;
    const uint64_t grid = (a.n_obj + kBlockThreads - 1) / kBlockThreads;
    if (grid >= (1ull << 31)) return hipErrorInvalidValue;
    uint32_t fw = odd_rec_fw(r, mode), rw = odd_rec_words(k, r, mode);
    void* args[] = {const_cast<PassArgs*>(&a), &k, &r, &mode, &fw, &rw, &recs};
    return hipLaunchKernel((const void*)&gf_odd_objrec, dim3((unsigned)grid), dim3(kBlockThreads), args, 0, stream);
}

hipError_t launch_odd_planrec(int k, int r, int mode, const UPlanArgs& p, const URec* orecs, uint32_t n,
                              uint32_t* recs, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (k < 1 || k > kOddMaxK || r < 1 || r > kMaxR || mode == kOddVerify) return hipErrorInvalidValue;
    const uint32_t grid = (n + kBlockThreads - 1) / kBlockThreads;
    uint32_t fw = odd_rec_fw(r, mode), rw = odd_rec_words(k, r, mode);
    void* args[] = {const_cast<UPlanArgs*>(&p), &orecs, &n, &k, &r, &mode, &fw, &rw, &recs};
    return hipLaunchKernel((const void*)&gf_odd_planrec, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

// variant: odd_pick's (plans: carried records; strided: object records);
// list: the record kernel over a plan's tile list
static const void* odd_kernel(int k, int r, int mode, bool plan, bool mirror, bool variant, bool list = false) {
    if (k <= 4) return odd_kernel_range<1, 4>(k, r, mode, plan, mirror, variant, list);
    if (k <= 8) return odd_kernel_k58(k, r, mode, plan, mirror, variant, list);
    return odd_kernel_k912(k, r, mode, plan, mirror, variant, list);
}

bool odd_enabled() {
    static const bool on = tune_knob("HBEC_ODD", 1) != 0;
    return on;
}

int odd_blocks_per_cu(int mode, int k, int r, bool mirror, bool records, int xs) {
    static const int v = (int)tune_knob("HBEC_ODD_BPC", 0);
    if (v > 0) return v;
    if (xs >= 0) return odd_bp_bpc(k, r, mode);  // launch bounds sized for it (odd_rec_lb)
    if (mode == kOddVerify) return HBEC_ODD_BPC_VERIFY;
    if (records && odd_rec_two_blocks(k, r, mode)) return 2;  // launch bounds sized for it (odd_rec_lb)
    return odd_two_blocks(k, r, mode, mirror) ? 2 : HBEC_ODD_BPC_APPLY;  // launch bounds sized for it (odd_lb)
}

uint64_t urec_tile() { return odd_enabled() ? (uint64_t)kOddPlanU * kOddWin : (uint64_t)unaligned_tile_bytes(); }
// Record tile of a plan / zero-copy batch coded with k inputs per pass (the
// gf_odd_plan instance that reads the records): K <= 4 plain kernels take a
// record as one carried 2-window tile (2016 B), the others as 2 x 992 B
// windows (mirrored, or K > 4 one window per wave tile).
uint64_t urec_tile_for(int k, bool mirror) {
    if (!odd_enabled()) return (uint64_t)unaligned_tile_bytes();
    if (!mirror && k <= 4 && kOddPlanU == 2) return (uint64_t)(64 + kOddStore) * 16u;
    return (uint64_t)kOddPlanU * kOddWin;
}
uint64_t urec_span(uint64_t shard_len) {
    if (!odd_enabled()) return shard_len;
    return shard_len > kOddMinMain ? shard_len + 32u : 0u;
}

uint32_t odd_tile_bytes(int k) { return odd_u(k) == 2 ? (64u + kOddStore) * 16u : (uint32_t)odd_u(k) * kOddWin; }
uint64_t odd_min_main() { return kOddMinMain; }
uint32_t odd_plan_tile_bytes() { return (uint32_t)kOddPlanU * kOddWin; }

// The record kernels' tile spans (plan tile lists, odd_frame_tiles).
void odd_plan_spans(uint32_t (&spans)[kOddSpans]) {
    // table record kernels: 5 <= K <= 12 one 992-B window per tile, K <= 4 the
    // carried 2-window tile; bit-plane kernels HBEC_ODD_BP_U carried windows
    static_assert(odd_rec_span(2, kOddApply) == odd_rec_span(HBEC_ODD_BP_U, kOddApply), "two tile spans");
    spans[0] = odd_rec_span(1, kOddApply);
    spans[1] = odd_rec_span(2, kOddApply);
}

uint32_t odd_rec_tile_span(int k, int mode, int xs) {
    if (xs >= 0 && mode == kOddVerify) return (64u * odd_bp_u() - 1u) * 16u;  // chained windows (VCHAIN)
    return xs >= 0 ? odd_rec_span(odd_bp_u(), mode) : odd_rec_span(odd_u(k, mode), mode);
}

// Tiles per shard of S > kOddMinMain bytes: every block stored (compared)
// lies at V <= S - 64 - kOddFrame in the frame (column V at position
// kOddFrame + (-out0 mod 16) + V), and a tile stores `tile` bytes of V.
uint64_t odd_frame_tiles(uint64_t shard_len, uint64_t tile) {
    const uint64_t last = shard_len - (uint64_t)(kOddGuard + 16 + kOddFrame);  // S > kOddMinMain: positive
    return last / tile + 1u;
}

uint32_t odd_tiles_per_obj(int k, int mode, uint64_t shard_len, bool records, int xs) {
    const uint64_t tile = xs >= 0 ? (uint64_t)odd_rec_tile_span(k, mode, xs)
                          : records ? (uint64_t)odd_rec_span(odd_u(k, mode), mode)
                          : mode == kOddVerify ? (odd_u(k, mode) >= 2 ? (uint64_t)(64u * odd_u(k, mode) - 1u) * 16u
                                                                      : (uint64_t)odd_win<kOddVerify>())
                                               : (odd_u(k, mode) == 2 ? (uint64_t)(64 + kOddStore) * 16u
                                                                                         : (uint64_t)odd_u(k, mode) * kOddWin);
    return (uint32_t)odd_frame_tiles(shard_len, tile);
}

bool odd_supported(int k, int r) { return k >= 1 && k <= kOddMaxK && r >= 1 && r <= kMaxR; }

bool odd_edge_fuse(int k, int r, int mode, bool records, int xs, bool list, uint64_t max_s) {
    static const bool on = tune_knob("HBEC_ODD_EDGE_FUSE", 1) != 0;  // tuning builds: 0 = the separate edge launch
    static const uint64_t lim = (uint64_t)tune_knob("HBEC_ODD_EDGE_MAX_S", HBEC_ODD_EDGE_MAX_S);
    return on && max_s <= lim && (records ? odd_rec_edge(k, r, mode, xs, list) : odd_strided_edge(k, r, mode));
}

int odd_bp_schedule(int k, int r, int mode, const uint32_t (*tab)[kMaxK][5], bool plan) {
    // tuning builds: HBEC_ODD_BP = 0 none, 1 the measured choice (XorShape
    // strided / plan), 2 every compiled schedule
    static const int on = (int)tune_knob("HBEC_ODD_BP", 1);
    if (!on || mode == kOddAcc || k > kOddMaxK || r > kMaxR) return -1;
    for (int i = 0; i < kXorShapeCount; ++i) {
        const XorShape& x = kXorShapes[i];
        const bool use = mode == kOddVerify ? (!plan && x.verify) : (plan ? x.plan : x.strided);
        if (x.k != k || x.R != r || (on == 1 && !use)) continue;
        bool eq = true;
        for (int q = 0; q < r && eq; ++q)
            for (int j = 0; j < k && eq; ++j) eq = ((tab[q][j][0] >> 8) & 0xFFu) == x.coef[q][j];  // t[0] byte 1 = c * 1
        if (eq) return i;
    }
    return -1;
}

std::atomic<uint64_t> g_odd_launches[3];  // bit-plane, record, strided (hbec_odd_path_stats)
std::atomic<uint64_t> g_odd_edge_launches[2];  // guard-band launches, main launches coding them (hbec_odd_edge_stats)

hipError_t launch_odd(int k, int r, int mode, const PassArgs& a, uint32_t* flags, const uint32_t* recs, int grid,
                      hipStream_t stream, int xs) {
    if (!pos32_shard(a.shard_len)) return hipErrorInvalidValue;  // 32-bit shard positions
    g_odd_launches[xs >= 0 ? 0 : (recs ? 1 : 2)].fetch_add(1, std::memory_order_relaxed);
    if (a.fuse) g_odd_edge_launches[1].fetch_add(1, std::memory_order_relaxed);
    if (xs >= 0) {
        if (!recs || mode == kOddAcc || xs >= kXorShapeCount || kXorShapes[xs].k != k || kXorShapes[xs].R != r)
            return hipErrorInvalidValue;
        const void* fn = odd_kernel_bp(xs, mode, a.list != nullptr);
        if (!fn) return hipErrorInvalidValue;
        void* args[] = {const_cast<PassArgs*>(&a), &flags, &recs};
        return hipLaunchKernel(fn, dim3(grid), dim3(64 * odd_waves_per_block(xs)), args, 0, stream);
    }
    if (a.list && !recs) return hipErrorInvalidValue;
    const void* fn = odd_kernel(k, r, mode, false, false, recs != nullptr, a.list != nullptr);
    if (!fn) return hipErrorInvalidValue;
    void* args[] = {const_cast<PassArgs*>(&a), &flags, &recs};
    return hipLaunchKernel(fn, dim3(grid), dim3(kPipeBlockThreads), args, 0, stream);
}

hipError_t launch_odd_edges(int k, int r, int mode, const PassArgs& a, uint32_t* flags, hipStream_t stream) {
    if (k < 1 || k > kMaxK || r < 1 || r > kMaxR || a.n_obj == 0) return a.n_obj == 0 ? hipSuccess : hipErrorInvalidValue;
    if (!pos32_shard(a.shard_len)) return hipErrorInvalidValue;
    // few objects: a thread per output too (shorter per-thread chains); many:
    // the K input bytes once for every output (fewer line touches: 16384 short
    // 8+3 objects 59.6 -> 52.4 us, r05_edges_*_kernel_stats.csv)
    const bool split = a.n_obj < kOddEdgeSplitObjs;
    const bool lng = a.shard_len > kOddMinMain;  // 64 + 64 slots: one shard end per wave
    const uint64_t total = a.n_obj * (uint64_t)(split ? r : 1) * (uint64_t)(lng ? kOddEdgeSlotsLong : kOddEdgeSlots);
    const int grid = (int)std::min<uint64_t>((total + kBlockThreads - 1) / kBlockThreads, 4096);
    const void* fns[3][2][2] = {
        {{(const void*)&gf_odd_edges<kOddApply, false, kOddEdgeSlots>, (const void*)&gf_odd_edges<kOddApply, false, kOddEdgeSlotsLong>},
         {(const void*)&gf_odd_edges<kOddApply, true, kOddEdgeSlots>, (const void*)&gf_odd_edges<kOddApply, true, kOddEdgeSlotsLong>}},
        {{(const void*)&gf_odd_edges<kOddAcc, false, kOddEdgeSlots>, (const void*)&gf_odd_edges<kOddAcc, false, kOddEdgeSlotsLong>},
         {(const void*)&gf_odd_edges<kOddAcc, true, kOddEdgeSlots>, (const void*)&gf_odd_edges<kOddAcc, true, kOddEdgeSlotsLong>}},
        {{(const void*)&gf_odd_edges<kOddVerify, false, kOddEdgeSlots>, (const void*)&gf_odd_edges<kOddVerify, false, kOddEdgeSlotsLong>},
         {(const void*)&gf_odd_edges<kOddVerify, true, kOddEdgeSlots>, (const void*)&gf_odd_edges<kOddVerify, true, kOddEdgeSlotsLong>}}};
    const void* fn = fns[mode][split ? 1 : 0][lng ? 1 : 0];
    g_odd_edge_launches[0].fetch_add(1, std::memory_order_relaxed);
    void* args[] = {const_cast<PassArgs*>(&a), &k, &r, &flags};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

hipError_t launch_odd_edges_plan(int k, int r, int mode, const UPlanArgs& p, const URec* erecs, uint32_t n_erecs,
                                 hipStream_t stream, bool lng) {
    if (n_erecs == 0) return hipSuccess;
    if (k < 1 || k > kMaxK || r < 1 || r > kMaxR || mode == kOddVerify) return hipErrorInvalidValue;
    const bool split = n_erecs < kOddEdgeSplitObjs;
    const uint64_t total = (uint64_t)n_erecs * (uint64_t)(split ? r : 1) * (uint64_t)(lng ? kOddEdgeSlotsLong : kOddEdgeSlots);
    const int grid = (int)std::min<uint64_t>((total + kBlockThreads - 1) / kBlockThreads, 4096);
    const void* fns[2][2][2] = {
        {{(const void*)&gf_odd_edges_plan<kOddApply, false, kOddEdgeSlots>, (const void*)&gf_odd_edges_plan<kOddApply, false, kOddEdgeSlotsLong>},
         {(const void*)&gf_odd_edges_plan<kOddApply, true, kOddEdgeSlots>, (const void*)&gf_odd_edges_plan<kOddApply, true, kOddEdgeSlotsLong>}},
        {{(const void*)&gf_odd_edges_plan<kOddAcc, false, kOddEdgeSlots>, (const void*)&gf_odd_edges_plan<kOddAcc, false, kOddEdgeSlotsLong>},
         {(const void*)&gf_odd_edges_plan<kOddAcc, true, kOddEdgeSlots>, (const void*)&gf_odd_edges_plan<kOddAcc, true, kOddEdgeSlotsLong>}}};
    const void* fn = fns[mode == kOddAcc ? 1 : 0][split ? 1 : 0][lng ? 1 : 0];
    g_odd_edge_launches[0].fetch_add(1, std::memory_order_relaxed);
    void* args[] = {const_cast<UPlanArgs*>(&p), &erecs, &n_erecs, &k, &r};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

hipError_t launch_odd_plan(int k, int r, int mode, const UPlanArgs& p, int grid, hipStream_t stream) {
    g_odd_launches[2].fetch_add(1, std::memory_order_relaxed);
    const void* fn = odd_kernel(k, r, mode, true, p.mirror != 0, p.carry != 0);
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

extern "C" int hbec_odd_path_stats(uint64_t* bitplane, uint64_t* records, uint64_t* strided) {
    if (bitplane) *bitplane = hbec::g_odd_launches[0].load();
    if (records) *records = hbec::g_odd_launches[1].load();
    if (strided) *strided = hbec::g_odd_launches[2].load();
    return 0;
}

extern "C" int hbec_odd_edge_stats(uint64_t* edge_launches, uint64_t* fused_launches) {
    if (edge_launches) *edge_launches = hbec::g_odd_edge_launches[0].load();
    if (fused_launches) *fused_launches = hbec::g_odd_edge_launches[1].load();
    return 0;
}
