// stripes.hip — one-launch GF(2^8) apply over a batch of stripes of MIXED
// shard lengths (BASELINE config 4: 8+3 over 4 KiB and 1 MiB objects; and
// the batching unit for many concurrent ecSplit stripes, ecutils.go:38-70).
//
// A stripe is ecSplit's databuf layout (ecutils.go:31-35,55-58): k+m shards of
// shard_len bytes back to back at `base`, data first.  The host plan cuts
// every stripe into tiles of TILE = stripes_u(k) KiB of shard column and writes
// one 32-B record per tile (kernels.h TileRec: input/output base, strides,
// valid bytes).  For a stripe, shard i of the tile starts at addr +
// i*shard_len.  Waves walk
// the tile list grid-stride with the same pipeline as gf_apply_vec_pipe: the
// NEXT tile's data loads and the tile record after that are in flight while
// the current tile computes and stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "gf_device.h"
#include "kernels.h"

namespace hbec {

// Per-tile shard bases, wave-uniform (scalar): inputs src[j], outputs dst[r].
template <int K, int R, bool SPLIT>
__device__ __forceinline__ void tile_bases(uint64_t (&src)[K], uint64_t (&dst)[R], const StripeArgs& a,
                                           const TileRec& t) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const bool b = SPLIT && ((a.in_sel >> j) & 1u);
        src[j] = b ? t.out_addr + (uint64_t)a.in_idx[j] * t.out_stride : t.in_addr + (uint64_t)a.in_idx[j] * t.in_stride;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const bool b = SPLIT && ((a.out_sel >> r) & 1u);
        dst[r] = b ? t.in_addr + (uint64_t)a.out_idx[r] * t.in_stride : t.out_addr + (uint64_t)a.out_idx[r] * t.out_stride;
    }
}

template <int K, int U>
__device__ __forceinline__ void load_stripe_tile(u32x4 (&x)[U][K], const uint64_t (&src)[K], uint32_t valid,
                                                 uint32_t lane) {
    const uint64_t last = (uint64_t)valid - 16u;  // valid >= 16, multiple of 16
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint64_t off = (uint64_t)lane * 16u + (uint64_t)u * 1024u;
        off = off < last ? off : last;
#pragma unroll
        for (int j = 0; j < K; ++j) x[u][j] = ld16_addr(src[j] + off);
    }
}

// ACC: a later pass over inputs beyond the first 8 (k > 8): the outputs
// already hold the earlier passes' partial sums and are read back and
// XOR-accumulated (clamped to the tile's `valid` bytes like the input loads).
// `live` = bytes this wave stores: the tile's valid bytes, or 0 for a
// past-the-end stand-in tile (block-uniform trip count below).
template <int K, int R, int U, bool FULL, bool ACC>
__device__ __forceinline__ void store_stripe_tile_(const u32x4 (&x)[U][K], const StripeArgs& a,
                                                   const Tables<K, R>& tb, const uint64_t (&dst)[R], uint32_t valid,
                                                   uint32_t live, uint32_t lane) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t off = (uint64_t)lane * 16u + (uint64_t)u * 1024u;
        u32x4 acc[R];
        if constexpr (ACC) {
            const uint64_t last = (uint64_t)valid - 16u;
            const uint64_t ro = off < last ? off : last;
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = ld16_addr(dst[r] + ro);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
        }
        gf_dot<K, R>(acc, x[u], a.tab, tb);
        if (FULL || off < live) {
#pragma unroll
            for (int r = 0; r < R; ++r) st16_addr(dst[r] + off, acc[r]);
        }
    }
}

template <int K, int R, int U, bool ACC>
__device__ __forceinline__ void store_stripe_tile(const u32x4 (&x)[U][K], const StripeArgs& a, const Tables<K, R>& tb,
                                                  const uint64_t (&dst)[R], uint32_t valid, uint32_t live,
                                                  uint32_t lane) {
    if (live >= (uint32_t)U * 1024u)  // wave-uniform: whole tile live
        store_stripe_tile_<K, R, U, true, ACC>(x, a, tb, dst, valid, live, lane);
    else
        store_stripe_tile_<K, R, U, false, ACC>(x, a, tb, dst, valid, live, lane);
}

// MIRROR (hbec_encode_host_md5 on pinned stripes): the tile codes its stripe
// in place over PCIe as the zero-copy path does (inputs and outputs at
// in_addr + idx*in_stride, host-mapped), and also stores every input and
// output column it holds to a device arena at out_addr + idx*out_stride, so
// ShardHash reads the shards from HBM without a second pass over PCIe.
template <int K, int R>
__device__ __forceinline__ void mirror_bases(uint64_t (&min_)[K], uint64_t (&mout)[R], const StripeArgs& a,
                                             const TileRec& t) {
#pragma unroll
    for (int j = 0; j < K; ++j) min_[j] = t.out_addr + (uint64_t)a.in_idx[j] * t.out_stride;
#pragma unroll
    for (int r = 0; r < R; ++r) mout[r] = t.out_addr + (uint64_t)a.out_idx[r] * t.out_stride;
}

template <int K, int R, int U, bool FULL, bool ACC>
__device__ __forceinline__ void store_mirror_tile_(const u32x4 (&x)[U][K], const StripeArgs& a,
                                                   const Tables<K, R>& tb, const uint64_t (&dst)[R],
                                                   const uint64_t (&min_)[K], const uint64_t (&mout)[R],
                                                   uint32_t valid, uint32_t live, uint32_t lane) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t off = (uint64_t)lane * 16u + (uint64_t)u * 1024u;
        u32x4 acc[R];
        if constexpr (ACC) {
            const uint64_t last = (uint64_t)valid - 16u;
            const uint64_t ro = off < last ? off : last;
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = ld16_addr(dst[r] + ro);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
        }
        gf_dot<K, R>(acc, x[u], a.tab, tb);
        if (FULL || off < live) {
#pragma unroll
            for (int r = 0; r < R; ++r) st16_addr(dst[r] + off, acc[r]);
#pragma unroll
            for (int j = 0; j < K; ++j) st16_addr(min_[j] + off, x[u][j]);
#pragma unroll
            for (int r = 0; r < R; ++r) st16_addr(mout[r] + off, acc[r]);
        }
    }
}

template <int K, int R, int U, bool ACC>
__device__ __forceinline__ void store_mirror_tile(const u32x4 (&x)[U][K], const StripeArgs& a, const Tables<K, R>& tb,
                                                  const uint64_t (&dst)[R], const uint64_t (&min_)[K],
                                                  const uint64_t (&mout)[R], uint32_t valid, uint32_t live,
                                                  uint32_t lane) {
    if (live >= (uint32_t)U * 1024u)
        store_mirror_tile_<K, R, U, true, ACC>(x, a, tb, dst, min_, mout, valid, live, lane);
    else
        store_mirror_tile_<K, R, U, false, ACC>(x, a, tb, dst, min_, mout, valid, live, lane);
}

// Tile records are read-only for the whole launch and passed as a separate
// __restrict__ argument, so the wave-uniform loads below become scalar loads.
__device__ __forceinline__ TileRec load_rec(const TileRec* __restrict__ recs, uint32_t i) {
    return recs[i];
}

// Pacing as in gf_apply_vec_pipe2 (DESIGN.md §4 ladder steps 7 and 9): one
// block barrier per tile after the next tile's loads are issued, so a
// block's 4 waves load and store in step, and an optional s_sleep (x 64
// cycles) before it.  The trip count is block-uniform: waves past the end
// load a stand-in tile (the last one) and store nothing.

template <int K, int R, bool SPLIT, bool ACC = false, bool MIRROR = false>
__global__ __launch_bounds__(kBlockThreads, 1) void gf_apply_stripes(StripeArgs a,
                                                                     const TileRec* __restrict__ tiles) {
    // accumulate passes follow a first pass of exactly kStripeMaxK inputs: same tiles
    constexpr int U = ACC ? stripes_u(kStripeMaxK) : stripes_u(K);
    constexpr uint32_t WPB = kBlockThreads / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(xcd_block() * WPB);
    const uint32_t dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * WPB;
    const uint32_t n = a.n_tiles;
    if (wave0 >= n) return;  // whole blocks only: the loop below has block barriers
    const Tables<K, R> tb = load_tables<K, R>(a.tab);
    uint32_t t = wave0 + dw;
    TileRec cur = load_rec(tiles, t < n ? t : n - 1u);
    uint64_t src[K], dst[R], min_[MIRROR ? K : 1], mout[MIRROR ? R : 1];
    auto bases = [&](uint64_t (&s_)[K], uint64_t (&d_)[R], const TileRec& r) {
        if constexpr (MIRROR) {  // in place in the (host-mapped) stripe: in_addr for inputs and outputs
            TileRec in_place = r;
            in_place.out_addr = r.in_addr;
            in_place.out_stride = r.in_stride;
            tile_bases<K, R, false>(s_, d_, a, in_place);
        } else {
            tile_bases<K, R, SPLIT>(s_, d_, a, r);
        }
    };
    bases(src, dst, cur);
    if constexpr (MIRROR) mirror_bases<K, R>(min_, mout, a, cur);
    u32x4 x[U][K];
    load_stripe_tile<K, U>(x, src, cur.valid, lane);
    uint32_t tn = t + nw;
    TileRec nxt = load_rec(tiles, tn < n ? tn : n - 1u);
    for (uint32_t b0 = wave0 + nw; b0 < n; b0 += nw) {  // block-uniform trip count
        tn = b0 + dw;
        u32x4 y[U][K];
        uint64_t nsrc[K], ndst[R];
        bases(nsrc, ndst, nxt);
        load_stripe_tile<K, U>(y, nsrc, nxt.valid, lane);  // data one tile ahead
        // record two tiles ahead, issued after the data loads: scalar loads
        // return out of order, so waiting for `nxt` is an lgkmcnt(0)
        const uint32_t t2 = tn + nw;
        const TileRec after = load_rec(tiles, t2 < n ? t2 : n - 1u);
        __builtin_amdgcn_s_barrier();
        if constexpr (MIRROR) {
            store_mirror_tile<K, R, U, ACC>(x, a, tb, dst, min_, mout, cur.valid, t < n ? cur.valid : 0u, lane);
            mirror_bases<K, R>(min_, mout, a, nxt);
        } else {
            store_stripe_tile<K, R, U, ACC>(x, a, tb, dst, cur.valid, t < n ? cur.valid : 0u, lane);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) x[u][j] = y[u][j];
#pragma unroll
        for (int r = 0; r < R; ++r) dst[r] = ndst[r];
        cur = nxt;
        nxt = after;
        t = tn;
    }
    if constexpr (MIRROR)
        store_mirror_tile<K, R, U, ACC>(x, a, tb, dst, min_, mout, cur.valid, t < n ? cur.valid : 0u, lane);
    else
        store_stripe_tile<K, R, U, ACC>(x, a, tb, dst, cur.valid, t < n ? cur.valid : 0u, lane);
}

template <int K, bool SPLIT, bool ACC, bool MIRROR>
static const void* stripes_for_r(int r) {
    switch (r) {
        case 1: return reinterpret_cast<const void*>(&gf_apply_stripes<K, 1, SPLIT, ACC, MIRROR>);
        case 2: return reinterpret_cast<const void*>(&gf_apply_stripes<K, 2, SPLIT, ACC, MIRROR>);
        case 3: return reinterpret_cast<const void*>(&gf_apply_stripes<K, 3, SPLIT, ACC, MIRROR>);
    }
    return nullptr;
}

template <bool SPLIT, bool ACC, bool MIRROR = false>
static const void* stripes_kernel_(int k, int r) {
    switch (k) {
        case 1: return stripes_for_r<1, SPLIT, ACC, MIRROR>(r);
        case 2: return stripes_for_r<2, SPLIT, ACC, MIRROR>(r);
        case 3: return stripes_for_r<3, SPLIT, ACC, MIRROR>(r);
        case 4: return stripes_for_r<4, SPLIT, ACC, MIRROR>(r);
        case 5: return stripes_for_r<5, SPLIT, ACC, MIRROR>(r);
        case 6: return stripes_for_r<6, SPLIT, ACC, MIRROR>(r);
        case 7: return stripes_for_r<7, SPLIT, ACC, MIRROR>(r);
        case 8: return stripes_for_r<8, SPLIT, ACC, MIRROR>(r);
    }
    return nullptr;
}

// accumulate passes (k > 8) exist for stripe plans and the host ring, not for
// object plans (split), which never exceed 8 inputs per pass; mirrored
// (zero-copy + device copy for hashing) launches are never split
static const void* stripes_kernel(int k, int r, bool split = false, bool acc = false, bool mirror = false) {
    if (mirror) {
        if (split) return nullptr;
        return acc ? stripes_kernel_<false, true, true>(k, r) : stripes_kernel_<false, false, true>(k, r);
    }
    if (acc) return split ? nullptr : stripes_kernel_<false, true>(k, r);
    return split ? stripes_kernel_<true, false>(k, r) : stripes_kernel_<false, false>(k, r);
}

int stripes_tile_bytes(int k) { return stripes_u(k) * 1024; }

bool stripes_supported(int k, int r) { return stripes_kernel(k, r) != nullptr; }

hipError_t launch_stripes(int k, int r, const StripeArgs& a, int grid, hipStream_t stream) {
    const void* fn = stripes_kernel(k, r, a.split != 0, a.accumulate != 0, a.mirror != 0);
    if (!fn) return hipErrorInvalidValue;
    const TileRec* tiles = a.tiles;
    void* args[] = {const_cast<StripeArgs*>(&a), &tiles};
    return hipLaunchKernel(fn, dim3(grid), dim3(kBlockThreads), args, 0, stream);
}

hipError_t stripes_occupancy(int k, int r, int* blocks_per_cu) {
    // per (k, r), asked of the runtime once: the host paths size a grid per chunk
    static std::atomic<int> cache[kMaxK + 1][kMaxR + 1] = {};
    if (k < 1 || k > kMaxK || r < 1 || r > kMaxR) return hipErrorInvalidValue;
    const int hit = cache[k][r].load(std::memory_order_relaxed);
    if (hit > 0) {
        *blocks_per_cu = hit;
        return hipSuccess;
    }
    const void* fn = stripes_kernel(k, r);
    if (!fn) return hipErrorInvalidValue;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, kBlockThreads, 0);
    if (e == hipSuccess && *blocks_per_cu > 0) cache[k][r].store(*blocks_per_cu, std::memory_order_relaxed);
    return e;
}

}  // namespace hbec
