// kernels.hip — gfx950 (CDNA4) GF(2^8) shard kernels for the Hummingbird EC path.
//
// One kernel body serves both hot operations of objectserver/ecutils.go:
//   * Encode       (ecSplit      -> Encoder.Encode,      ecutils.go:59)
//       out[r] = XOR_j M[k+r][j] * data[j]
//   * Reconstruct  (ecReconstruct-> Encoder.Reconstruct, ecutils.go:111;
//                   ecGlue       -> ReconstructData,     ecutils.go:168)
//       out[e] = XOR_j D[e][j] * survivor[j]   (D = decode rows built on host)
//
// Field multiply without tables in memory: a byte x is split into bit fields
// x[2:0], x[5:3], x[7:6]; c*x = c*x[2:0] ^ c*(x[5:3]<<3) ^ c*(x[7:6]<<6)
// (GF multiply is linear over XOR).  Each field indexes an 8-entry (or
// 4-entry) byte table held in two (one) registers, and v_perm_b32 performs
// that lookup for all 4 bytes of a dword at once.  So one coefficient costs 3
// v_perm_b32 per input dword plus XORs, and the selector extraction (5 VALU
// ops) is shared by every output row.  No LDS, no MFMA: the kernel is an HBM
// stream (k inputs read once, R outputs written once, coalesced 16 B/lane).
//
// Work decomposition: a "wave tile" is U x 1 KiB of one shard column
// (64 lanes x 16 B per KiB) across all K inputs of one object.  Waves walk
// tiles grid-stride; tile -> (object, offset) is one scalar division per tile.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <cstring>

#include "gf_device.h"
#include "kernels.h"

namespace hbec {

template <int K, int R, int U>
__device__ __forceinline__ void process_tile(const PassArgs& a, const Tables<K, R>& tb, uint64_t obj,
                                             uint64_t off0, bool full, bool accumulate) {
    // Issue every load of the tile first (K x U x 16 B per lane in flight),
    // then retire one 1 KiB sub-tile at a time so only its accumulators and
    // selectors are live.  Loads are branch-free: lanes past the shard end
    // read its last 16 B (never stored), so no exec branch splits the loads.
    u32x4 x[U][K];
    const uint64_t last = a.shard_len - 16u;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint64_t off = off0 + (uint64_t)u * 1024u;
        if (!full) off = off < last ? off : last;
#pragma unroll
        for (int j = 0; j < K; ++j) x[u][j] = ld16(a.in[j] + obj * a.in_stride[j] + off);
    }
    u32x4 old[U][R];
    if (accumulate) {  // wave-uniform: read-modify-write passes (inputs beyond kMaxK)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint64_t off = off0 + (uint64_t)u * 1024u;
            if (!full) off = off < last ? off : last;
#pragma unroll
            for (int r = 0; r < R; ++r) old[u][r] = *reinterpret_cast<const u32x4*>(a.out[r] + obj * a.out_stride[r] + off);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t off = off0 + (uint64_t)u * 1024u;
        const bool live = full || off < a.shard_len;
        u32x4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = accumulate ? old[u][r] : u32x4{0, 0, 0, 0};
        {
            u32x4 xs[K];
#pragma unroll
            for (int j = 0; j < K; ++j) xs[j] = x[u][j];
            gf_dot<K, R>(acc, xs, a.tab, tb);
        }
        if (live) {
#pragma unroll
            for (int r = 0; r < R; ++r) st16(a.out[r] + obj * a.out_stride[r] + off, acc[r]);
        }
    }
}

// Sub-tiles (1 KiB each) per wave tile: keeps K*U*4 load VGPRs <= 32 (tuning.h).
__host__ __device__ constexpr int tile_kib(int k) {
    return k <= 2 ? HBEC_TILE_SMALL : (k <= 4 ? HBEC_TILE_MID : HBEC_TILE_BIG);
}

// Vector path: every base 16-B aligned, every stride and shard_len % 16 == 0.
template <int K, int R>
__global__ __launch_bounds__(kBlockThreads, kVecWavesPerSimd) void gf_apply_vec(PassArgs a) {
    constexpr int U = tile_kib(K);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave =
        __builtin_amdgcn_readfirstlane(xcd_block() * (kBlockThreads / 64) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (kBlockThreads / 64);
    const uint32_t tpo = a.tiles_per_obj;
    const bool accumulate = a.accumulate != 0;
    const Tables<K, R> tb = load_tables<K, R>(a.tab);
    for (uint32_t t = wave; t < a.n_tiles; t += nwaves) {
        const uint32_t obj = t / tpo;
        const uint32_t tile = t - obj * tpo;
        const uint64_t tile_base = (uint64_t)tile * (uint64_t)(U * 1024);
        const uint64_t off0 = tile_base + lane * 16u;
        if (tile_base + (uint64_t)(U * 1024) <= a.shard_len) {
            process_tile<K, R, U>(a, tb, obj, off0, true, accumulate);
        } else {
            process_tile<K, R, U>(a, tb, obj, off0, false, accumulate);
        }
    }
}

// Pipelined vec path: few waves per CU (HBM works best with ~16-64 KiB of
// loads in flight per CU, hbm_probe copy/xor sweeps), each wave keeping the
// NEXT tile's loads in flight while it computes and stores the current one.
// Tile = U x 1 KiB of each of the K inputs, U = 16 / K (K*U = 16 loads).

// Branch-free tile load: lanes past the end of a partial tile read the last
// 16 B of the shard instead (always in bounds); their results are never
// stored.  No per-load exec branches, so the compiler keeps counted waits.
template <int K, int R, int U>
__device__ __forceinline__ void load_tile(u32x4 (&x)[U][K], const PassArgs& a, uint64_t obj, uint64_t off0) {
    const uint64_t last = a.shard_len - 16u;
#pragma unroll
    for (int q = 0; q < U * K; ++q) {
        const int u = HBEC_PIPE_IMAJ ? q % U : q / K, j = HBEC_PIPE_IMAJ ? q / U : q % K;
        uint64_t off = off0 + (uint64_t)u * 1024u;
        off = off < last ? off : last;
        const uint8_t* p = a.in[j] + obj * a.in_stride[j] + off;
        x[u][j] = HBEC_PIPE_TEMP ? ld16_addr_t(reinterpret_cast<uint64_t>(p)) : ld16(p);
    }
}

template <int K, int R, int U>
__device__ __forceinline__ void compute_store_tile(const u32x4 (&x)[U][K], const PassArgs& a, const Tables<K, R>& tb,
                                                   uint64_t obj, uint64_t off0, bool full) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t off = off0 + (uint64_t)u * 1024u;
        u32x4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
        gf_dot<K, R>(acc, x[u], a.tab, tb);
        if (full || off < a.shard_len) {
#pragma unroll
            for (int r = 0; r < R; ++r) st16(a.out[r] + obj * a.out_stride[r] + off, acc[r]);
        }
    }
}

template <int K, int R>
__global__ __launch_bounds__(kPipeBlockThreads, 1) void gf_apply_vec_pipe(PassArgs a) {
    // never launched with a.accumulate (launch_vec routes those to gf_apply_vec)
    constexpr int U = pipe_u(K);
    constexpr uint64_t TILE = (uint64_t)U * 1024u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nwaves = gridDim.x * (kPipeBlockThreads / 64);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(xcd_block() * (kPipeBlockThreads / 64) + (threadIdx.x >> 6));
    const uint32_t tpo = a.tiles_per_obj;
    const Tables<K, R> tb = load_tables<K, R>(a.tab);
    uint32_t t = wave;
    if (t >= a.n_tiles) return;
    u32x4 cur[U][K];
    uint32_t obj = t / tpo;
    uint64_t base = (uint64_t)(t - obj * tpo) * TILE;
    load_tile<K, R, U>(cur, a, obj, base + lane * 16u);
    // steady state: next tile's loads in flight while this tile computes
    for (uint32_t tn = t + nwaves; tn < a.n_tiles; tn += nwaves) {
        u32x4 nxt[U][K];
        const uint32_t obj_n = tn / tpo;
        const uint64_t base_n = (uint64_t)(tn - obj_n * tpo) * TILE;
        load_tile<K, R, U>(nxt, a, obj_n, base_n + lane * 16u);
        // Pace the wave: ~380 cycles of s_sleep after issuing the next tile's
        // loads lowers the requests in flight at the HBM; 4+2: +1.0-1.5 %
        // (flat from 6 to 8, a cliff from 12), 8+3 (longer tiles): no effect
        // (profiles/r01_tune_sleep.jsonl)
        if (K <= 4) __builtin_amdgcn_s_sleep(HBEC_PIPE_SLEEP);
        if (base + TILE <= a.shard_len)
            compute_store_tile<K, R, U>(cur, a, tb, obj, base + lane * 16u, true);
        else
            compute_store_tile<K, R, U>(cur, a, tb, obj, base + lane * 16u, false);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) cur[u][j] = nxt[u][j];
        obj = obj_n;
        base = base_n;
    }
    if (base + TILE <= a.shard_len)
        compute_store_tile<K, R, U>(cur, a, tb, obj, base + lane * 16u, true);
    else
        compute_store_tile<K, R, U>(cur, a, tb, obj, base + lane * 16u, false);
}

// gf_apply_vec_pipe2: the pipelined kernel in the stripe-plan kernel's loop
// shape -- every tile's shard bases are scalar values computed one tile ahead
// (the plan kernel loads them as records) and full / partial tiles are a
// uniform branch.  The hot path for K <= 4: +1.6 % over gf_apply_vec_pipe at
// 4+2 in an interleaved A/B (75.3 % vs 74.1 % of 8 TB/s on that box), but
// -7 % at 8+3, which keeps gf_apply_vec_pipe (profiles/r01_tune_pipe2.jsonl).
template <int K, int R>
struct PipeTile {
    uint64_t in[K];
    uint64_t out[R];
    uint32_t valid;  // bytes of the tile inside the shard (load clamp)
    uint32_t live;   // bytes stored: valid, or 0 for a past-the-end stand-in tile
};

template <int K, int R, int U>
__device__ __forceinline__ void pipe_tile_coords(PipeTile<K, R>& b, const PassArgs& a, uint32_t t, uint32_t tpo) {
    constexpr uint64_t TILE = (uint64_t)U * 1024u;
    const uint32_t obj = t / tpo;
    const uint64_t off = (uint64_t)(t - obj * tpo) * TILE;
#pragma unroll
    for (int j = 0; j < K; ++j) b.in[j] = reinterpret_cast<uint64_t>(a.in[j]) + obj * a.in_stride[j] + off;
#pragma unroll
    for (int r = 0; r < R; ++r) b.out[r] = reinterpret_cast<uint64_t>(a.out[r]) + obj * a.out_stride[r] + off;
    const uint64_t left = a.shard_len - off;
    b.valid = (uint32_t)(left < TILE ? left : TILE);
    b.live = b.valid;
}

template <int K, int R, int U>
__device__ __forceinline__ void pipe2_load(u32x4 (&x)[U][K], const PipeTile<K, R>& b, uint32_t lane) {
    const uint64_t last = (uint64_t)b.valid - 16u;
#pragma unroll
    for (int q = 0; q < U * K; ++q) {
        const int u = HBEC_PIPE_IMAJ ? q % U : q / K, j = HBEC_PIPE_IMAJ ? q / U : q % K;
        uint64_t off = (uint64_t)lane * 16u + (uint64_t)u * 1024u;
        off = off < last ? off : last;
        x[u][j] = HBEC_PIPE_TEMP ? ld16_addr_t(b.in[j] + off) : ld16_addr(b.in[j] + off);
    }
}

template <int K, int R, int U, bool FULL>
__device__ __forceinline__ void pipe2_store_(const u32x4 (&x)[U][K], const PassArgs& a, const Tables<K, R>& tb,
                                             const PipeTile<K, R>& b, uint32_t lane) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t off = (uint64_t)lane * 16u + (uint64_t)u * 1024u;
        u32x4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
        gf_dot<K, R>(acc, x[u], a.tab, tb);
        if (FULL || off < b.live) {
#pragma unroll
            for (int r = 0; r < R; ++r) st16_addr(b.out[r] + off, acc[r]);
        }
    }
}

// Tile t of the launch; past the end, the launch's last tile stands in: it is
// loaded and coded (so the loop keeps one shape) but stores nothing (live =
// 0, the masked partial-tile store path), so a caller whose outputs overlap
// its inputs cannot see a stale re-store.  No branch around the loads: a
// memory op under a branch makes the compiler drain everything in flight
// (vmcnt(0)) at the join, which serialises the pipeline (measured 2x slower).
template <int K, int R, int U>
__device__ __forceinline__ void pipe_tile_at(PipeTile<K, R>& b, const PassArgs& a, uint32_t t, uint32_t n,
                                             uint32_t tpo) {
    pipe_tile_coords<K, R, U>(b, a, t < n ? t : n - 1u, tpo);
    if (t >= n) b.live = 0;
}

template <int K, int R, int U>
__device__ __forceinline__ void pipe2_finish(const u32x4 (&x)[U][K], const PassArgs& a, const Tables<K, R>& tb,
                                             const PipeTile<K, R>& cur, uint32_t lane) {
    if (cur.live >= (uint32_t)U * 1024u)
        pipe2_store_<K, R, U, true>(x, a, tb, cur, lane);
    else
        pipe2_store_<K, R, U, false>(x, a, tb, cur, lane);
}

// Block barrier once per tile, after the next tile's loads are issued and the
// pacing sleep: the block's 4 waves (one per SIMD) then issue their loads and
// stores in step.  With s_sleep 8: +1.1-1.3 % over the barrier-free loop
// with s_sleep 6, on each of three allocations (profiles/r01_tune_barrier.jsonl).  Every wave of a block runs
// the same number of iterations (the loop bound is the block's first wave's
// tile; a wave past the end re-codes the last tile), so the barrier counts
// always match.

template <int K, int R>
__global__ __launch_bounds__(kPipeBlockThreads, 1) void gf_apply_vec_pipe2(PassArgs a) {
    constexpr int U = pipe_u(K);
    constexpr uint32_t WPB = kPipeBlockThreads / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * WPB;
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(xcd_block() * WPB);  // the block's first wave
    const uint32_t dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wave = wave0 + dw;
    const uint32_t tpo = a.tiles_per_obj;
    const uint32_t n = a.n_tiles;
    if (wave0 >= n) return;  // whole blocks only: the loop below has block barriers
    const Tables<K, R> tb = load_tables<K, R>(a.tab);
    PipeTile<K, R> cur, nxt;
    pipe_tile_at<K, R, U>(cur, a, wave, n, tpo);
    u32x4 x[U][K];
    pipe2_load<K, R, U>(x, cur, lane);
    pipe_tile_at<K, R, U>(nxt, a, wave + nw, n, tpo);
    for (uint32_t b0 = wave0 + nw; b0 < n; b0 += nw) {  // block-uniform trip count
        u32x4 y[U][K];
        pipe2_load<K, R, U>(y, nxt, lane);
        if (K <= 4) __builtin_amdgcn_s_sleep(HBEC_PIPE2_SLEEP);
        __builtin_amdgcn_s_barrier();
        PipeTile<K, R> after;
        pipe_tile_at<K, R, U>(after, a, b0 + dw + nw, n, tpo);
        pipe2_finish<K, R, U>(x, a, tb, cur, lane);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) x[u][j] = y[u][j];
        cur = nxt;
        nxt = after;
    }
    pipe2_finish<K, R, U>(x, a, tb, cur, lane);
}

// ---------------------------------------------------------------------------
// gf_apply_packed: short shards (S < one pipelined tile; 8+3 of a 4 KiB
// object has S = 512 B).  The per-object tiles above would leave lanes idle
// (a 1 KiB tile over a 512-B shard loads the same line twice and stores
// half), so here a wave tile is U x 64 consecutive 16-B ELEMENTS of the
// concatenated shard columns of all objects: element e is byte (e % spo)*16
// of object e / spo (spo = S/16).  Lane addresses are per lane (one object
// per half-wave at S = 512 B: 512 contiguous bytes of each shard), and every
// lane loads and stores live bytes.  Same pipeline as gf_apply_vec_pipe2:
// the next tile's loads in flight while this tile computes and stores, one
// block barrier per tile, block-uniform trip count (past-the-end waves load
// the last tile and store nothing).
template <int K, int U>
__device__ __forceinline__ void packed_load(u32x4 (&x)[U][K], const PassArgs& a, const PackedCoord<U>& c) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < K; ++j) x[u][j] = ld16(a.in[j] + (uint64_t)c.obj[u] * a.in_stride[j] + c.off[u]);
}

template <int K, int R, int U, bool FULL>
__device__ __forceinline__ void packed_store_(const u32x4 (&x)[U][K], const PassArgs& a, const Tables<K, R>& tb,
                                              const PackedCoord<U>& c, uint32_t t, uint32_t lane, uint32_t live) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        u32x4 acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
        gf_dot<K, R>(acc, x[u], a.tab, tb);
        if (FULL || (t * (uint32_t)U + (uint32_t)u) * 64u + lane < live) {
#pragma unroll
            for (int r = 0; r < R; ++r) st16(a.out[r] + (uint64_t)c.obj[u] * a.out_stride[r] + c.off[u], acc[r]);
        }
    }
}

// live = elements stored by this tile's lanes: n_elems, or 0 past the end
template <int K, int R, int U>
__device__ __forceinline__ void packed_finish(const u32x4 (&x)[U][K], const PassArgs& a, const Tables<K, R>& tb,
                                              const PackedCoord<U>& c, uint32_t t, uint32_t n, uint32_t lane) {
    const uint32_t live = t < n ? a.n_elems : 0u;
    if (t < n && (t + 1u) * (uint32_t)U * 64u <= a.n_elems)
        packed_store_<K, R, U, true>(x, a, tb, c, t, lane, live);
    else
        packed_store_<K, R, U, false>(x, a, tb, c, t, lane, live);
}


__host__ __device__ constexpr int packed_u(int k) {
    return k > 4 ? HBEC_PACKED_U_BIG : pipe_u(k);
}

template <int K, int R>
__global__ __launch_bounds__(kPipeBlockThreads, 1) void gf_apply_packed(PassArgs a) {
    constexpr int U = packed_u(K);
    constexpr uint32_t WPB = kPipeBlockThreads / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * WPB;
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(xcd_block() * WPB);
    const uint32_t dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n = a.n_tiles;
    if (wave0 >= n) return;  // whole blocks only: the loop below has block barriers
    const Tables<K, R> tb = load_tables<K, R>(a.tab);
    const uint32_t spo = a.elems_per_obj;
    const double inv = 1.0 / (double)spo;
    uint32_t t = wave0 + dw;
    PackedCoord<U> cur;
    packed_coords<U>(cur, t < n ? t : n - 1u, lane, a.n_elems, spo, inv);
    u32x4 x[U][K];
    packed_load<K, U>(x, a, cur);
    for (uint32_t b0 = wave0 + nw; b0 < n; b0 += nw) {  // block-uniform trip count
        const uint32_t tn = b0 + dw;
        PackedCoord<U> nxt;
        packed_coords<U>(nxt, tn < n ? tn : n - 1u, lane, a.n_elems, spo, inv);
        u32x4 y[U][K];
        packed_load<K, U>(y, a, nxt);
        __builtin_amdgcn_s_barrier();
        packed_finish<K, R, U>(x, a, tb, cur, t, n, lane);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) x[u][j] = y[u][j];
        cur = nxt;
        t = tn;
    }
    packed_finish<K, R, U>(x, a, tb, cur, t, n, lane);
}

// Streaming vec path (runtime K): one input shard at a time with the next
// input's loads in flight, coefficient tables fetched per input by scalar
// loads, so registers stay at R x 4 KiB accumulators + 2 x 4 KiB buffers for
// any K.  Used for shapes whose fully unrolled form would spill.
template <int R>
__global__ __launch_bounds__(kBlockThreads, kVecWavesPerSimd) void gf_apply_vec_stream(PassArgs a, int K) {
    constexpr int U = 4;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave =
        __builtin_amdgcn_readfirstlane(xcd_block() * (kBlockThreads / 64) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (kBlockThreads / 64);
    const uint32_t tpo = a.tiles_per_obj;
    for (uint32_t t = wave; t < a.n_tiles; t += nwaves) {
        const uint32_t obj = t / tpo;
        const uint32_t tile = t - obj * tpo;
        const uint64_t off0 = (uint64_t)tile * (uint64_t)(U * 1024) + lane * 16u;
        bool live[U];
#pragma unroll
        for (int u = 0; u < U; ++u) live[u] = off0 + (uint64_t)u * 1024u < a.shard_len;
        u32x4 acc[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                acc[r][u] = u32x4{0, 0, 0, 0};
                if (a.accumulate && live[u])
                    acc[r][u] = *reinterpret_cast<const u32x4*>(a.out[r] + obj * a.out_stride[r] + off0 + u * 1024u);
            }
        u32x4 cur[U];
        {
            const uint8_t* src = a.in[0] + obj * a.in_stride[0] + off0;
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = live[u] ? ld16(src + u * 1024u) : u32x4{0, 0, 0, 0};
        }
#pragma unroll 1
        for (int j = 0; j < K; ++j) {
            u32x4 nxt[U];
            if (j + 1 < K) {
                const uint8_t* src = a.in[j + 1] + obj * a.in_stride[j + 1] + off0;
#pragma unroll
                for (int u = 0; u < U; ++u) nxt[u] = live[u] ? ld16(src + u * 1024u) : u32x4{0, 0, 0, 0};
            }
            uint32_t tb[R][5];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int q = 0; q < 5; ++q) tb[r][q] = a.tab[r][j][q];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const Sel sx = selectors(cur[u][e]);
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        acc[r][u][e] ^= gf_mul_sel(sx, tb[r][0], tb[r][1], tb[r][2], tb[r][3], tb[r][4]);
                }
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (live[u]) st16(a.out[r] + obj * a.out_stride[r] + off0 + u * 1024u, acc[r][u]);
    }
}

// ---------------------------------------------------------------------------
// gf_apply_unaligned: any base alignment, any stride, any shard length.  ecSplit
// sets S = ceil(len / k) (ecutils.go:14-24), so S is a multiple of 16 for only
// 1 object size in 16, and its databuf puts shard i at i*S (ecutils.go:31-35):
// an arbitrary object's shards start at arbitrary byte offsets.  Round 1's
// byte-per-lane kernel coded them at ~20 % of HBM; this one keeps 16-B accesses, and
// every access is 16-B ALIGNED:
//  * input j of an object starts d_j = base & 15 bytes into an aligned block
//    (d_j is wave-uniform: one object per wave tile).  A lane loads the two
//    aligned blocks that cover its 16-B column and shifts the column out of
//    them (v_alignbyte_b32).  Loads are clamped to the shard's last aligned
//    block, so they stay inside blocks that hold shard bytes; clamped bytes
//    feed only positions >= S, which are never stored.
//  * output r's aligned blocks start at shard positions = e_r (mod 16),
//    e_r = -base & 15.  Lane l stores the block [c_l + e_r, c_l + e_r + 16):
//    the high bytes of its own column and the low bytes of lane l+1's
//    (ds_bpermute).  So a window of 64 computed columns (1 KiB) stores 63
//    blocks, and windows step 1008 B.  The shard head [0, e_r) is stored
//    bytewise by lane 0 of window 0, and a block crossing the shard end
//    bytewise by its lane.
// Accumulate passes (inputs beyond kMaxK) read the old output the same way
// as an input.  A window reads output bytes another window stores only in
// the e_r bytes it does not use itself, so the passes are race-free.
// ---------------------------------------------------------------------------
// stored bytes per 64-lane window: 62 blocks, the column's upper block from
// lane l+1 (lane 63's column is partial); one load per input column, +3-9 %
// over two (profiles/r02_tune_unaligned_shfl.jsonl)
constexpr uint32_t kUnalignedWindow = 992;
constexpr uint32_t kUnalignedStoreLanes = 62;
constexpr int kUnalignedU = HBEC_UNALIGNED_U;  // windows per wave tile (loads in flight)

// A view of one object's shard: aligned base, misalignment, last aligned block.
struct UView {
    uint64_t abase;  // base & ~15
    uint64_t last;   // (base + S - 1) & ~15
    uint32_t d;      // base & 15 (wave-uniform)
};

__device__ __forceinline__ UView uview(uint64_t b, uint64_t s) {
    UView v;
    v.abase = b & ~(uint64_t)15;
    v.last = (b + s - 1u) & ~(uint64_t)15;
    v.d = __builtin_amdgcn_readfirstlane((uint32_t)(b & 15u));
    return v;
}

__device__ __forceinline__ void uload(u32x4& lo, u32x4& hi, const UView& v, uint64_t col) {
    const uint64_t x = v.abase + col;
    lo = ld16_addr(x < v.last ? x : v.last);
    hi = lo;  // replaced by lane l+1's block at use (upper)
}

// the column's upper block: lane l+1's lower block
__device__ __forceinline__ u32x4 upper(const u32x4& lo, const u32x4& hi) {
    (void)hi;
    u32x4 h;
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = __shfl_down(lo[i], 1u, 64);
    return h;
}

typedef __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ void store_bytes(uint64_t addr, const u32x4& v, uint64_t n) {
    gu8* p = reinterpret_cast<gu8*>(addr);  // global, not flat: flat stores also count in lgkmcnt
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if ((uint64_t)b < n) p[b] = (uint8_t)(v[b >> 2] >> (8 * (b & 3)));
}

// One wave tile: U windows from shard position p0 of one object / stripe.
// in_base(j) / out_base(r) give the byte address of that object's input j /
// output r shard (wave-uniform); tab(r, j) its coefficient tables.
// VERIFY: compare the coded columns with the stored outputs instead of
// storing them, and OR 1 into *flag on any mismatching byte (Encoder.Verify).
template <int R, bool VERIFY = false, class InBase, class OutBase, class Tab>
__device__ __forceinline__ void unaligned_tile(int K, uint64_t S, uint64_t p0, bool accumulate, uint32_t lane,
                                               InBase in_base, OutBase out_base, Tab tab,
                                               uint32_t* flag = nullptr) {
    constexpr int U = kUnalignedU;
    constexpr uint32_t W = kUnalignedWindow;
    uint64_t col[U];
    bool live[U];  // window-uniform
#pragma unroll
    for (int u = 0; u < U; ++u) {
        col[u] = p0 + (uint64_t)u * W + lane * 16u;
        live[u] = p0 + (uint64_t)u * W < S;
    }
    u32x4 acc[R][U];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const UView ov = uview(out_base(r), S);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc[r][u] = u32x4{0, 0, 0, 0};
            if (accumulate) {  // kernel-uniform; clamped loads need no per-window branch
                u32x4 lo, hi;
                uload(lo, hi, ov, col[u]);
                acc[r][u] = realign16(lo, upper(lo, hi), ov.d);
            }
        }
    }
    u32x4 clo[U], chi[U];
    UView cv = uview(in_base(0), S);
#pragma unroll
    for (int u = 0; u < U; ++u) uload(clo[u], chi[u], cv, col[u]);  // clamped: no branch
#pragma unroll 1
    for (int j = 0; j < K; ++j) {
        u32x4 nlo[U], nhi[U];
        UView nv = cv;
        if (j + 1 < K) {
            nv = uview(in_base(j + 1), S);
#pragma unroll
            for (int u = 0; u < U; ++u) uload(nlo[u], nhi[u], nv, col[u]);
        }
        uint32_t tb[R][5];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 5; ++q) tb[r][q] = tab(r, j)[q];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32x4 x = realign16(clo[u], upper(clo[u], chi[u]), cv.d);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const Sel sx = selectors(x[e]);
#pragma unroll
                for (int r = 0; r < R; ++r)
                    acc[r][u][e] ^= gf_mul_sel(sx, tb[r][0], tb[r][1], tb[r][2], tb[r][3], tb[r][4]);
            }
        }
        if (j + 1 < K) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                clo[u] = nlo[u];
                chi[u] = nhi[u];
            }
            cv = nv;
        }
    }
    if constexpr (VERIFY) {
        bool bad = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const UView ov = uview(out_base(r), S);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!live[u]) continue;  // window-uniform (the upper block is a shuffle)
                u32x4 lo, hi;
                uload(lo, hi, ov, col[u]);
                const u32x4 st = realign16(lo, upper(lo, hi), ov.d);
                // columns [c, c + 16) of this window's lanes; bytes at or past S do not count
                const uint64_t nv = col[u] < S ? S - col[u] : 0u;
                if (lane < kUnalignedStoreLanes) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const uint64_t b0 = 4u * e;
                        const uint32_t mask = nv >= b0 + 4u ? 0xFFFFFFFFu
                                              : (nv <= b0 ? 0u : (0xFFFFFFFFu >> (8u * (uint32_t)(b0 + 4u - nv))));
                        bad |= ((acc[r][u][e] ^ st[e]) & mask) != 0u;
                    }
                }
            }
        }
        if (bad) atomicOr(flag, 1u);
        return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint64_t ob = out_base(r);
        const uint32_t e = __builtin_amdgcn_readfirstlane((16u - (uint32_t)(ob & 15u)) & 15u);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;  // window-uniform: every lane takes part in the shuffle
            u32x4 nb;
#pragma unroll
            for (int i = 0; i < 4; ++i) nb[i] = __shfl_down(acc[r][u][i], 1u, 64);
            const u32x4 blk = realign16(acc[r][u], nb, e);
            const uint64_t q = col[u] + e;  // block start (shard position); ob + q is 16-B aligned
            if (lane < kUnalignedStoreLanes && q < S) {
                if (q + 16u <= S)
                    st16_addr(ob + q, blk);
                else
                    store_bytes(ob + q, blk, S - q);
            }
            if (lane == 0u && col[u] == 0u && e > 0u) store_bytes(ob, acc[r][u], e < S ? e : S);  // head
        }
    }
}

template <int R>
__global__ __launch_bounds__(kBlockThreads) void gf_apply_unaligned(PassArgs a, int K) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave =
        __builtin_amdgcn_readfirstlane(xcd_block() * (kBlockThreads / 64) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (kBlockThreads / 64);
    const uint32_t tpo = a.tiles_per_obj;
    for (uint32_t t = wave; t < a.n_tiles; t += nwaves) {
        const uint32_t obj = t / tpo;
        const uint64_t p0 = (uint64_t)(t - obj * tpo) * (kUnalignedU * kUnalignedWindow);
        unaligned_tile<R>(
            K, a.shard_len, p0, a.accumulate != 0, lane,
            [&](int j) { return reinterpret_cast<uint64_t>(a.in[j]) + (uint64_t)obj * a.in_stride[j]; },
            [&](int r) { return reinterpret_cast<uint64_t>(a.out[r]) + (uint64_t)obj * a.out_stride[r]; },
            [&](int r, int j) { return a.tab[r][j]; });
    }
}

// Encoder.Verify of views at any alignment: recompute every parity column
// and compare it with the stored one in the same pass (nothing written).
template <int R>
__global__ __launch_bounds__(kBlockThreads) void gf_verify_unaligned(PassArgs a, int K, uint32_t* flags) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave =
        __builtin_amdgcn_readfirstlane(xcd_block() * (kBlockThreads / 64) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (kBlockThreads / 64);
    const uint32_t tpo = a.tiles_per_obj;
    for (uint32_t t = wave; t < a.n_tiles; t += nwaves) {
        const uint32_t obj = t / tpo;
        const uint64_t p0 = (uint64_t)(t - obj * tpo) * (kUnalignedU * kUnalignedWindow);
        unaligned_tile<R, true>(
            K, a.shard_len, p0, false, lane,
            [&](int j) { return reinterpret_cast<uint64_t>(a.in[j]) + (uint64_t)obj * a.in_stride[j]; },
            [&](int r) { return reinterpret_cast<uint64_t>(a.out[r]) + (uint64_t)obj * a.out_stride[r]; },
            [&](int r, int j) { return a.tab[r][j]; }, flags + obj);
    }
}

// Plans over stripes / objects of mixed shard lengths at any alignment: one
// record per wave tile (URec).  Input j of a tile's stripe starts at
// (bit j of in_sel ? b : a) + in_idx[j] * S; outputs likewise.
template <int R>
__global__ __launch_bounds__(kBlockThreads) void gf_apply_unaligned_plan(UPlanArgs p, int K) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave =
        __builtin_amdgcn_readfirstlane(xcd_block() * (kBlockThreads / 64) + (threadIdx.x >> 6));
    const uint32_t nwaves = gridDim.x * (kBlockThreads / 64);
    for (uint32_t t = wave; t < p.n_recs; t += nwaves) {
        const URec rec = p.recs[t];
        const uint64_t S = rec.shard_len;
        unaligned_tile<R>(
            K, S, rec.p0, p.accumulate != 0, lane,
            [&](int j) { return (((p.in_sel >> j) & 1u) ? rec.b : rec.a) + (uint64_t)p.in_idx[j] * S; },
            [&](int r) { return (((p.out_sel >> r) & 1u) ? rec.b : rec.a) + (uint64_t)p.out_idx[r] * S; },
            [&](int r, int j) { return p.tab[r][j]; });
    }
}

// Synthetic objects: object i's bytes are the little-endian
// splitmix64 stream seeded with base_seed ^ (i * golden).  splitmix64 is
// counter based, so each 8-byte word is computed independently.
__global__ __launch_bounds__(kBlockThreads) void fill_splitmix(uint8_t* dst, uint64_t n_obj, uint64_t obj_len,
                                                             uint64_t obj_stride, uint64_t base_seed,
                                                             uint64_t first) {
    const uint64_t words = (obj_len + 7) / 8;
    const uint64_t total = words * n_obj;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total;
         v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t obj = v / words;
        const uint64_t w = v - obj * words;
        const uint64_t seed = base_seed ^ ((first + obj) * 0x9E3779B97F4A7C15ull);
        uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        uint8_t* d = dst + obj * obj_stride + w * 8;
        const uint64_t rem = obj_len - w * 8;
        if (rem >= 8 && (reinterpret_cast<uintptr_t>(d) & 7u) == 0) {
            *reinterpret_cast<uint64_t*>(d) = z;
        } else {
            const int nb = rem >= 8 ? 8 : (int)rem;
            for (int b = 0; b < nb; ++b) d[b] = (uint8_t)(z >> (8 * b));
        }
    }
}

// ---------------------------------------------------------------------------
// Host-side launch table
// ---------------------------------------------------------------------------
template <int K, int R>
static const void* vec_kernel_ptr(bool pipe) {
    if (pipe) return K <= HBEC_PIPE_V2_MAXK ? reinterpret_cast<const void*>(&gf_apply_vec_pipe2<K, R>)
                                              : reinterpret_cast<const void*>(&gf_apply_vec_pipe<K, R>);
    return reinterpret_cast<const void*>(&gf_apply_vec<K, R>);
}

// Fully unrolled instantiations that compile spill-free (checked with
// -Rpass-analysis=kernel-resource-usage); other shapes use the streaming kernel.
template <int K>
static const void* vec_kernel_for_r(int r, bool pipe) {
    switch (r) {
        case 1: return vec_kernel_ptr<K, 1>(pipe);
        case 2: return vec_kernel_ptr<K, 2>(pipe);
        case 3: return vec_kernel_ptr<K, 3>(pipe);
    }
    return nullptr;
}

static const void* unrolled_kernel(int k, int r, bool pipe) {
    switch (k) {
        case 1: return vec_kernel_for_r<1>(r, pipe);
        case 2: return vec_kernel_for_r<2>(r, pipe);
        case 3: return vec_kernel_for_r<3>(r, pipe);
        case 4: return vec_kernel_for_r<4>(r, pipe);
        case 5: return vec_kernel_for_r<5>(r, pipe);
        case 6: return vec_kernel_for_r<6>(r, pipe);
        case 7: return vec_kernel_for_r<7>(r, pipe);
        case 8: return vec_kernel_for_r<8>(r, pipe);
    }
    return nullptr;
}

static const void* stream_kernel(int r) {
    switch (r) {
        case 1: return reinterpret_cast<const void*>(&gf_apply_vec_stream<1>);
        case 2: return reinterpret_cast<const void*>(&gf_apply_vec_stream<2>);
        case 3: return reinterpret_cast<const void*>(&gf_apply_vec_stream<3>);
        case 4: return reinterpret_cast<const void*>(&gf_apply_vec_stream<4>);
    }
    return nullptr;
}

int is_streaming_shape(int k, int r, int force_stream) {
    return (force_stream || !unrolled_kernel(k, r, false)) ? 1 : 0;
}


template <int K>
static const void* packed_for_r(int r) {
    switch (r) {
        case 1: return reinterpret_cast<const void*>(&gf_apply_packed<K, 1>);
        case 2: return reinterpret_cast<const void*>(&gf_apply_packed<K, 2>);
        case 3: return reinterpret_cast<const void*>(&gf_apply_packed<K, 3>);
    }
    return nullptr;
}

static const void* packed_kernel(int k, int r) {
    switch (k) {
        case 1: return packed_for_r<1>(r);
        case 2: return packed_for_r<2>(r);
        case 3: return packed_for_r<3>(r);
        case 4: return packed_for_r<4>(r);
        case 5: return packed_for_r<5>(r);
        case 6: return packed_for_r<6>(r);
        case 7: return packed_for_r<7>(r);
        case 8: return packed_for_r<8>(r);
    }
    return nullptr;
}

int packed_tile_elems(int k) { return packed_u(k) * 64; }

// Shards shorter than this take the packed kernel: below one pipelined tile
// it is the only full-lane kernel (8+3 @ 4 KiB: 70 % vs 7 % of 8 TB/s); for
// K <= 4 it also beats gf_apply_vec_pipe2 up to S = 1 KiB (4+2 @ 4 KiB:
// 72.6 % vs 69.3 %), while at S = 256 KiB it loses (68-72 % vs 74 %)
// (profiles/r02_tune_packed3_*.jsonl).  5 <= K <= 8 up to S = 32 KiB
// (HBEC_PACKED_MAX_BIG): the pipelined kernel's 3 KiB tiles leave most of a
// tile idle when S mod 3 KiB is small, packed tiles never do; 16 384 8+3
// objects at S = 4 / 8 / 12 / 16 / 32 KiB 50.5 / 56.5 / 67.2 / 67.7 / 74.8 %
// -> 71.0 / 56.2 / 67.7 / 72.5 / 75.4 % (profiles/r06_ab_packed.jsonl); 4+2
// loses at 8-16 KiB (69.9 -> 67.9, 72.8 -> 70.4 %) and keeps one tile.
static uint64_t packed_max_shard(int k) {
    if (k > 4) return HBEC_PACKED_MAX_BIG;
    const uint64_t tile = (uint64_t)pipe_u(k) * 1024u;
    return tile > 2048u ? tile : 2048u;
}

// Tuning knobs: HBEC_PACKED=0 sends short shards back to gf_apply_vec (A/B);
// HBEC_PACKED_MAX_SHARD=B takes shards shorter than B bytes (instead of
// shorter than one pipelined tile) through the packed kernel.
static const bool g_packed_on = tune_knob("HBEC_PACKED", 1) != 0;
static const uint64_t g_packed_max = (uint64_t)std::max(0LL, tune_knob("HBEC_PACKED_MAX_SHARD", 0));

int is_packed_shape(int k, int r, uint64_t shard_len, int accumulate, int force_stream) {
    return (g_packed_on && !force_stream && !accumulate && shard_len >= 16 && shard_len % 16 == 0 &&
            shard_len < (g_packed_max ? g_packed_max : packed_max_shard(k)) &&
            packed_kernel(k, r) != nullptr)
               ? 1
               : 0;
}

hipError_t launch_packed(int k, int r, const PassArgs& a, int grid, hipStream_t stream) {
    const void* fn = packed_kernel(k, r);
    if (!fn) return hipErrorInvalidValue;
    void* args[] = {const_cast<PassArgs*>(&a)};
    return hipLaunchKernel(fn, dim3(grid), dim3(kPipeBlockThreads), args, 0, stream);
}

// Resident 4-wave blocks per CU for the packed kernel: K <= 4 streams best
// with 2 (short tiles: more waves keep enough bytes in flight), K > 4 with 1
// (profiles/r02_tune_packed*.jsonl).

hipError_t packed_occupancy(int k, int r, int* blocks_per_cu) {
    const void* fn = packed_kernel(k, r);
    if (!fn) return hipErrorInvalidValue;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, kPipeBlockThreads, 0);
    const int cap = k <= 4 ? HBEC_PACKED_BLOCKS_SMALL : HBEC_PACKED_BLOCKS_BIG;
    if (e == hipSuccess && cap > 0 && *blocks_per_cu > cap) *blocks_per_cu = cap;
    return e;
}

// The pipelined kernel wants whole tiles; short shards (e.g. 8+3 of a 4 KiB
// object: 512 B) take the 1 KiB-tile kernel so fewer lanes idle.
static bool use_pipe(int k, uint64_t shard_len, bool accumulate) {
    return !accumulate && shard_len >= (uint64_t)pipe_u(k) * 1024u;
}

int is_pipe_shape(int k, int r, uint64_t shard_len, int force_stream) {
    return (!is_streaming_shape(k, r, force_stream) && use_pipe(k, shard_len, false)) ? 1 : 0;
}

int vec_tile_bytes(int k, int r, uint64_t shard_len, int accumulate, int force_stream) {
    if (!force_stream && unrolled_kernel(k, r, false))
        return (use_pipe(k, shard_len, accumulate != 0) ? pipe_u(k) : tile_kib(k)) * 1024;
    return 4 * 1024;
}

int vec_block_threads(int k, int r, uint64_t shard_len, int accumulate, int force_stream) {
    return (!is_streaming_shape(k, r, force_stream) && use_pipe(k, shard_len, accumulate != 0)) ? kPipeBlockThreads
                                                                                               : kBlockThreads;
}

hipError_t launch_vec(int k, int r, const PassArgs& a, int grid, hipStream_t stream, int force_stream) {
    // accumulate passes (inputs beyond kMaxK) need the output read-back, which
    // the pipelined kernel does not do: they take the plain unrolled kernel.
    const bool pipe = use_pipe(k, a.shard_len, a.accumulate != 0);
    const void* fn = force_stream ? nullptr : unrolled_kernel(k, r, pipe);
    if (fn) {
        void* args[] = {const_cast<PassArgs*>(&a)};
        return hipLaunchKernel(fn, dim3(grid), dim3(pipe ? kPipeBlockThreads : kBlockThreads), args, 0, stream);
    }
    fn = stream_kernel(r);
    if (!fn || k < 1 || k > kMaxK) return hipErrorInvalidValue;
    void* args[] = {const_cast<PassArgs*>(&a), &k};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}


static const void* unaligned_kernel(int r) {
    switch (r) {
        case 1: return reinterpret_cast<const void*>(&gf_apply_unaligned<1>);
        case 2: return reinterpret_cast<const void*>(&gf_apply_unaligned<2>);
        case 3: return reinterpret_cast<const void*>(&gf_apply_unaligned<3>);
        case 4: return reinterpret_cast<const void*>(&gf_apply_unaligned<4>);
    }
    return nullptr;
}

uint32_t unaligned_tiles_per_obj(uint64_t shard_len) {
    const uint64_t windows = (shard_len + kUnalignedWindow - 1) / kUnalignedWindow;
    return (uint32_t)((windows + kUnalignedU - 1) / kUnalignedU);
}

hipError_t launch_unaligned(int k, int r, const PassArgs& a, int grid, hipStream_t stream) {
    const void* fn = unaligned_kernel(r);
    if (!fn || k < 1 || k > kMaxK) return hipErrorInvalidValue;
    void* args[] = {const_cast<PassArgs*>(&a), &k};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

static const void* unaligned_plan_kernel(int r) {
    switch (r) {
        case 1: return reinterpret_cast<const void*>(&gf_apply_unaligned_plan<1>);
        case 2: return reinterpret_cast<const void*>(&gf_apply_unaligned_plan<2>);
        case 3: return reinterpret_cast<const void*>(&gf_apply_unaligned_plan<3>);
        case 4: return reinterpret_cast<const void*>(&gf_apply_unaligned_plan<4>);
    }
    return nullptr;
}

hipError_t launch_verify_unaligned(int k, int r, const PassArgs& a, uint32_t* flags, int grid, hipStream_t stream) {
    const void* fn = nullptr;
    switch (r) {
        case 1: fn = reinterpret_cast<const void*>(&gf_verify_unaligned<1>); break;
        case 2: fn = reinterpret_cast<const void*>(&gf_verify_unaligned<2>); break;
        case 3: fn = reinterpret_cast<const void*>(&gf_verify_unaligned<3>); break;
        case 4: fn = reinterpret_cast<const void*>(&gf_verify_unaligned<4>); break;
    }
    if (!fn || k < 1 || k > kMaxK) return hipErrorInvalidValue;
    void* args[] = {const_cast<PassArgs*>(&a), &k, &flags};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

uint32_t unaligned_tile_bytes() { return (uint32_t)kUnalignedU * kUnalignedWindow; }

hipError_t launch_unaligned_plan(int k, int r, const UPlanArgs& a, int grid, hipStream_t stream) {
    const void* fn = unaligned_plan_kernel(r);
    if (!fn || k < 1 || k > kMaxK) return hipErrorInvalidValue;
    void* args[] = {const_cast<UPlanArgs*>(&a), &k};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

hipError_t unaligned_occupancy(int r, int* blocks_per_cu) {
    const void* fn = unaligned_kernel(r);
    if (!fn) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, kBlockThreads, 0);
}

hipError_t launch_fill(uint8_t* dst, uint64_t n_obj, uint64_t obj_len, uint64_t obj_stride, uint64_t base_seed,
                       uint64_t first, int grid, hipStream_t stream) {
    hipLaunchKernelGGL(fill_splitmix, dim3(grid), dim3(kBlockThreads), 0, stream, dst, n_obj, obj_len, obj_stride,
                       base_seed, first);
    return hipGetLastError();
}

// Host words to device memory in stream order, carried in the kernel
// arguments (which the runtime copies at launch): nothing on the host has to
// outlive the call and the stream is never synchronised.
struct PutWords {
    uint32_t n;
    uint32_t w[kPutWordsMax];
};
__global__ __launch_bounds__(kBlockThreads) void put_words(uint32_t* __restrict__ dst, PutWords a) {
    for (uint32_t i = threadIdx.x; i < a.n; i += blockDim.x) dst[i] = a.w[i];
}

hipError_t launch_put_words(void* dst, const void* src, size_t bytes, hipStream_t stream) {
    if (bytes % 4 != 0) return hipErrorInvalidValue;
    const uint32_t* w = static_cast<const uint32_t*>(src);
    uint32_t* d = static_cast<uint32_t*>(dst);
    for (size_t i = 0, n = bytes / 4; i < n; i += kPutWordsMax) {
        PutWords a;
        a.n = (uint32_t)std::min<size_t>(kPutWordsMax, n - i);
        std::memcpy(a.w, w + i, (size_t)a.n * 4);
        hipLaunchKernelGGL(put_words, dim3(1), dim3(kBlockThreads), 0, stream, d + i, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t vec_occupancy(int k, int r, int pipe, int force_stream, int* blocks_per_cu) {
    const void* fn = force_stream ? nullptr : unrolled_kernel(k, r, pipe != 0);
    const bool is_pipe = fn && pipe;
    if (!fn) fn = stream_kernel(r);
    if (!fn) return hipErrorInvalidValue;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn,
                                                                is_pipe ? kPipeBlockThreads : kBlockThreads, 0);
    if (e == hipSuccess && is_pipe && kPipeBlocksPerCu > 0 && *blocks_per_cu > kPipeBlocksPerCu)
        *blocks_per_cu = kPipeBlocksPerCu;
    return e;
}

}  // namespace hbec
