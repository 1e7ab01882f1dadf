// wide.hip — Encoder.Verify for any number of data shards (k > 16 included)
// at any alignment, in ONE read-only pass: recompute each parity column in
// registers, compare it with the stored one, flag the object.  The `hec`
// policy accepts any data_shards (objectserver/ecengine.go:719-724) and
// klauspost's Verify has no size cliff; the round-2 path for k > 16 coded
// parity into scratch and compared it bytewise (two extra passes over R*S).
//
// Design (the per-tile unit is one wave window of 62 compared 16-B columns,
// frame = shard position 0, columns at 16 i):
//  * One continuous element stream per wave: tile t's K input columns, then
//    its R stored parity columns, then tile t + (waves in grid)'s ... .  A
//    ring of D = 4 loads runs ahead of the consumer ACROSS tile boundaries, so
//    the next tile's first inputs are in flight while this tile's parity is
//    compared: runtime K with no tail bubble and no wasted prefetch.
//  * Input / parity columns are dword-aligned 16-B loads shifted into the
//    frame (one DPP lane shift + 4 v_alignbyte), as gf_odd (odd.hip).
//  * The v_perm tables of all K x R coefficients live in LDS (K = 256, R = 8:
//    40 KiB); each input's R x 5 words are broadcast-read when it is consumed.
//  * Columns 16 i + 16 <= S - 16 are compared here; the last < 32 bytes of
//    each parity shard by gf_verify_wide_tail (byte per thread).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf_device.h"
#include "kernels.h"

namespace hbec {

constexpr uint32_t kWideStore = 62;             // compared columns per 64-lane window
constexpr uint32_t kWideWin = kWideStore * 16;  // shard bytes per window
constexpr int kWideU = HBEC_WIDE_U;
constexpr uint32_t kWideTile = kWideU * kWideWin;  // shard bytes per tile
constexpr int kWideD = HBEC_WIDE_D;

// LDS per element j of a tile (inputs 0..K-1, then stored parity K..K+R-1):
// 4 words {base lo, base hi, stride lo, stride hi}; then per input j the R
// coefficient tables, 5 words each, padded to a multiple of 4 words
__host__ __device__ constexpr uint32_t wide_tab_stride(int r) { return (uint32_t)((r * 5 + 3) & ~3); }

// shard columns 16 i + 16 <= S - 16 are compared by the main kernel
__host__ __device__ inline uint64_t wide_main_bytes(uint64_t S) { return S >= 32 ? ((S - 16) / 16) * 16 : 0; }

__device__ __forceinline__ u32x4 wide_shift(const u32x4& v, uint32_t sh) {
    const uint32_t n0 = lane_next(v[0]);
    return u32x4{__builtin_amdgcn_alignbyte(v[1], v[0], sh), __builtin_amdgcn_alignbyte(v[2], v[1], sh),
                 __builtin_amdgcn_alignbyte(v[3], v[2], sh), __builtin_amdgcn_alignbyte(n0, v[3], sh)};
}

// Stream pointer: element j of tile t (object obj, tile ti within it).
struct WidePtr {
    uint32_t t, obj, ti, j;
};

__device__ __forceinline__ void wide_set(WidePtr& p, uint32_t t, uint32_t tpo) {
    p.t = t;
    p.obj = t / tpo;
    p.ti = t - p.obj * tpo;
    p.j = 0;
}

__device__ __forceinline__ uint64_t wide_base(const uint32_t* e4, uint32_t obj) {
    const u32x4 e = *reinterpret_cast<const u32x4*>(e4);
    return ((uint64_t)e[1] << 32 | e[0]) + (uint64_t)obj * ((uint64_t)e[3] << 32 | e[2]);
}

// Frame of a tile: shard position of its first column.  Verify: 16 B
// columns from position 0.  Apply: output 0's 16-B blocks (gf_odd's frame,
// c0 = -32 + (-out0 mod 16)), windows of 62 stored blocks.
template <bool APPLY>
__device__ __forceinline__ int32_t wide_c(const uint32_t* lds_addr, uint32_t K, uint32_t obj, uint32_t ti) {
    if constexpr (!APPLY) return (int32_t)(ti * kWideTile);
    const uint32_t o0 = (uint32_t)wide_base(lds_addr + 4 * K, obj);
    return (int32_t)((16u - (o0 & 15u)) & 15u) - 32 + (int32_t)(ti * kWideTile);
}

// Element addresses and tables come from LDS (ds_read, in order with the
// table reads): no scalar memory load inside the loop, whose out-of-order
// returns would force lgkmcnt(0) waits on every LDS read.
//   verify (APPLY = false): elements per tile = K inputs + R stored parity
//     columns; flags objects whose parity differs (main columns only).
//   apply (APPLY = true): elements per tile = K inputs; after the K-th, the R
//     outputs are stored as 16-B-aligned blocks inside the guard band
//     [kWideGuard, S - kWideGuard) (the rest: gf_apply_wide_edges).
constexpr int32_t kWideGuard = 48;

template <int R, bool APPLY>
__global__ __launch_bounds__(kPipeBlockThreads) void gf_wide(WideArgs a, uint32_t* flags) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t K = a.K, L = APPLY ? K : K + R;  // elements per tile
    const uint32_t ts = wide_tab_stride(R);
    uint32_t* lds_addr = lds;              // [K + R][4]
    uint32_t* lds_tab = lds + 4 * (K + R);  // [K][ts]
    for (uint32_t i = threadIdx.x; i < K + R; i += blockDim.x) {
        const uint64_t b = i < K ? a.in_base[i] : a.out[i - K];
        const uint64_t st = i < K ? a.in_stride[i] : a.out_stride[i - K];
        lds_addr[4 * i] = (uint32_t)b;
        lds_addr[4 * i + 1] = (uint32_t)(b >> 32);
        lds_addr[4 * i + 2] = (uint32_t)st;
        lds_addr[4 * i + 3] = (uint32_t)(st >> 32);
    }
    for (uint32_t i = threadIdx.x; i < K * ts; i += blockDim.x) lds_tab[i] = a.tab[i];
    __syncthreads();

    constexpr uint32_t WPB = kPipeBlockThreads / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * WPB;
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * WPB + (threadIdx.x >> 6));
    const uint32_t n = a.n_tiles, tpo = a.tiles_per_obj;
    if (w >= n) return;
    const uint32_t total = ((n - 1u - w) / nw + 1u) * L;  // this wave's elements
    const int32_t S = (int32_t)a.shard_len;
    const int32_t main_end = (int32_t)wide_main_bytes(a.shard_len);
    const int32_t hi = S - kWideGuard - 16;  // apply: last block start stored

    // producer: loads run kWideD elements ahead of the consumer, across tile
    // boundaries; past the wave's last element it reloads that element
    WidePtr pp, cp;
    wide_set(pp, w, tpo);
    wide_set(cp, w, tpo);
    int32_t pc = wide_c<APPLY>(lds_addr, K, pp.obj, pp.ti);
    uint32_t issued = 0;
    auto issue = [&](u32x4 (&buf)[kWideU], uint32_t& sh) {
        const uint64_t base = wide_base(lds_addr + 4 * pp.j, pp.obj);
        const int32_t l4 = (int32_t)((uint32_t)base & 3u);
        const int32_t t = l4 + pc;
        sh = (uint32_t)t & 3u;
        const int32_t lim = ((l4 + S + 3) & ~3) - 16;
#pragma unroll
        for (int u = 0; u < kWideU; ++u) {
            int32_t v = t - (int32_t)sh + 16 * (int32_t)lane + u * (int32_t)kWideWin;
            v = v < 0 ? 0 : (v > lim ? lim : v);
            buf[u] = ld16_addr((base & ~(uint64_t)3) + (uint64_t)(uint32_t)v);
        }
        if (++issued < total) {
            if (++pp.j == L) {
                wide_set(pp, pp.t + nw, tpo);
                pc = wide_c<APPLY>(lds_addr, K, pp.obj, pp.ti);
            }
        }
    };
    u32x4 ring[kWideD][kWideU];
    uint32_t rsh[kWideD];
#pragma unroll
    for (int i = 0; i < kWideD; ++i) issue(ring[i], rsh[i]);

    u32x4 acc[kWideU][R];
#pragma unroll
    for (int u = 0; u < kWideU; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[u][r] = u32x4{0, 0, 0, 0};
    bool bad = false;
    for (uint32_t p0 = 0; p0 < total; p0 += kWideD) {
#pragma unroll
        for (int i = 0; i < kWideD; ++i) {
            u32x4 xs[kWideU];
#pragma unroll
            for (int u = 0; u < kWideU; ++u) xs[u] = wide_shift(ring[i][u], rsh[i]);
            // the reload reuses ring[i]'s registers only after x is computed:
            // a load hoisted above lands in fresh registers that the loop's
            // back edge must copy back, i.e. waits for (vmcnt(0) per turn)
            __builtin_amdgcn_sched_barrier(0);
            issue(ring[i], rsh[i]);  // unconditional: no load under a branch
            if (p0 + (uint32_t)i < total) {  // wave-uniform; no global loads inside
                const uint32_t j = cp.j;
                if (j < K) {
                    const u32x4* tp = reinterpret_cast<const u32x4*>(lds_tab + j * ts);
                    uint32_t tw[(R * 5 + 3) & ~3];
#pragma unroll
                    for (int q = 0; q < (int)((R * 5 + 3) / 4); ++q) {
                        const u32x4 v = tp[q];
                        tw[4 * q] = v[0];
                        tw[4 * q + 1] = v[1];
                        tw[4 * q + 2] = v[2];
                        tw[4 * q + 3] = v[3];
                    }
#pragma unroll
                    for (int u = 0; u < kWideU; ++u)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const Sel sx = selectors(xs[u][e]);
#pragma unroll
                            for (int r = 0; r < R; ++r)
                                acc[u][r][e] ^= gf_mul_sel(sx, tw[5 * r], tw[5 * r + 1], tw[5 * r + 2], tw[5 * r + 3],
                                                           tw[5 * r + 4]);
                        }
                    if (APPLY && j == K - 1u) {
                        // tile done: each output's 16-B-aligned blocks in the band
                        const int32_t c = wide_c<APPLY>(lds_addr, K, cp.obj, cp.ti);
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const uint64_t ob = wide_base(lds_addr + 4 * (K + r), cp.obj);
                            const uint32_t dl = __builtin_amdgcn_readfirstlane((16u - (((uint32_t)ob + (uint32_t)c) & 15u)) & 15u);
#pragma unroll
                            for (int u = 0; u < kWideU; ++u) {
                                const u32x4 blk = realign16(acc[u][r], lane_next4(acc[u][r]), dl);
                                const int32_t q = c + (int32_t)(u * kWideWin) + 16 * (int32_t)lane + (int32_t)dl;
                                if (lane < kWideStore && q >= kWideGuard && q <= hi)
                                    st16_addr(ob + (uint64_t)(int64_t)q, blk);
                                acc[u][r] = u32x4{0, 0, 0, 0};
                            }
                        }
                    }
                } else if constexpr (!APPLY) {
                    // stored parity r0 = j - K against the recomputed column
                    const uint32_t r0 = j - K;
#pragma unroll
                    for (int u = 0; u < kWideU; ++u) {
                        const int32_t cpos = (int32_t)(cp.ti * kWideTile + u * kWideWin) + 16 * (int32_t)lane;
                        const bool mine = lane < kWideStore && cpos + 16 <= main_end;
                        u32x4 want = acc[u][0];
#pragma unroll
                        for (int r = 1; r < R; ++r)
                            if (r0 == (uint32_t)r) want = acc[u][r];
                        const u32x4 df = want ^ xs[u];
                        bad |= mine && (df[0] | df[1] | df[2] | df[3]) != 0u;
                    }
                    if (r0 == R - 1u) {
                        if (__any(bad) && lane == 0u) atomicOr(flags + cp.obj, 1u);
                        bad = false;
#pragma unroll
                        for (int u = 0; u < kWideU; ++u)
#pragma unroll
                            for (int r = 0; r < R; ++r) acc[u][r] = u32x4{0, 0, 0, 0};
                    }
                }
                if (++cp.j == L) wide_set(cp, cp.t + nw, tpo);
            }
        }
    }
}

// The guard-band bytes of every output shard of an apply (positions gf_wide
// leaves: [0, qmin) and [qmax + 16, S) of output r's aligned blocks; all of
// a shard of S <= 160), byte by thread with runtime K.
constexpr int32_t kWideEdgeSlots = 160;

template <int R>
__global__ __launch_bounds__(kBlockThreads) void gf_apply_wide_edges(WideArgs a) {
    const uint64_t per = (uint64_t)R * kWideEdgeSlots;
    const uint64_t total = a.n_obj * per;
    const int32_t S = (int32_t)a.shard_len;
    const uint32_t ts = wide_tab_stride(R);
    typedef __attribute__((address_space(1))) uint8_t gu8;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t obj = v / per;
        const uint32_t rs = (uint32_t)(v - obj * per);
        const uint32_t r = rs / kWideEdgeSlots;
        const int32_t slot = (int32_t)(rs - r * kWideEdgeSlots);
        const uint64_t out = a.out[r] + obj * a.out_stride[r];
        int32_t pos;
        if (S <= kWideEdgeSlots) {
            if (slot >= S) continue;
            pos = slot;
        } else {
            const int32_t e = (int32_t)((16u - ((uint32_t)out & 15u)) & 15u);
            const int32_t qmin = kWideGuard + e, top = S - kWideGuard - 16, qmax = top - ((top - e) & 15);
            if (slot < kWideEdgeSlots / 2) {
                pos = slot;
                if (pos >= qmin) continue;
            } else {
                pos = S - kWideEdgeSlots + slot;
                if (pos < qmax + 16) continue;
            }
        }
        uint32_t x = 0;
        for (uint32_t j = 0; j < a.K; ++j) {
            const uint32_t b = *reinterpret_cast<const gu8*>(a.in_base[j] + obj * a.in_stride[j] + (uint64_t)pos);
            const uint32_t* t = a.tab + j * ts + 5 * r;
            x ^= gf_mul_sel(selectors(b), t[0], t[1], t[2], t[3], t[4]);
        }
        *reinterpret_cast<gu8*>(out + (uint64_t)pos) = (uint8_t)x;
    }
}

// The last (S - wide_main_bytes(S)) bytes of every parity shard, byte by
// thread: v = XOR_j C[r][j] * in_j[q], compared with the stored byte.
template <int R>
__global__ __launch_bounds__(kBlockThreads) void gf_verify_wide_tail(WideArgs a, uint32_t* flags) {
    const uint64_t S = a.shard_len, q0 = wide_main_bytes(S), nb = S - q0;
    const uint64_t total = (uint64_t)a.n_obj * R * nb;
    const uint32_t ts = wide_tab_stride(R);
    typedef __attribute__((address_space(1))) const uint8_t gu8_c;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < total; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t obj = v / (R * nb);
        const uint32_t rem = (uint32_t)(v - obj * R * nb);
        const uint32_t r = rem / (uint32_t)nb;
        const uint64_t q = q0 + (rem - r * (uint32_t)nb);
        uint32_t x = 0;
        for (uint32_t j = 0; j < a.K; ++j) {
            const uint32_t b = *reinterpret_cast<gu8_c*>(a.in_base[j] + obj * a.in_stride[j] + q);
            const uint32_t* t = a.tab + j * ts + 5 * r;
            x ^= gf_mul_sel(selectors(b), t[0], t[1], t[2], t[3], t[4]);
        }
        const uint32_t s = *reinterpret_cast<gu8_c*>(a.out[r] + obj * a.out_stride[r] + q);
        if (((x ^ s) & 0xFFu) != 0u) atomicOr(flags + obj, 1u);
    }
}

static size_t wide_lds_bytes(uint32_t K, int R) { return ((size_t)(K + R) * 4 + (size_t)K * wide_tab_stride(R)) * 4; }

template <int R>
static hipError_t launch_wide_r(const WideArgs& a, uint32_t* flags, int grid, hipStream_t stream) {
    WideArgs c = a;
    void* args[] = {&c, &flags};
    hipError_t e = hipSuccess;
    if (a.n_tiles > 0)
        e = hipLaunchKernel((const void*)&gf_wide<R, false>, dim3(grid), dim3(kPipeBlockThreads), args,
                            wide_lds_bytes(a.K, R), stream);
    if (e != hipSuccess) return e;
    const uint64_t tail = (uint64_t)a.n_obj * R * (a.shard_len - wide_main_bytes(a.shard_len));
    if (tail == 0) return hipSuccess;
    const int tg = (int)std::min<uint64_t>((tail + kBlockThreads - 1) / kBlockThreads, 4096);
    return hipLaunchKernel((const void*)&gf_verify_wide_tail<R>, dim3(tg), dim3(kBlockThreads), args, 0, stream);
}

template <int R>
static hipError_t launch_apply_wide_r(const WideArgs& a, int grid, hipStream_t stream) {
    WideArgs c = a;
    uint32_t* none = nullptr;
    void* args[] = {&c, &none};
    hipError_t e = hipSuccess;
    if (a.n_tiles > 0)
        e = hipLaunchKernel((const void*)&gf_wide<R, true>, dim3(grid), dim3(kPipeBlockThreads), args,
                            wide_lds_bytes(a.K, R), stream);
    if (e != hipSuccess || a.n_obj == 0) return e;
    const uint64_t total = a.n_obj * (uint64_t)R * kWideEdgeSlots;
    const int tg = (int)std::min<uint64_t>((total + kBlockThreads - 1) / kBlockThreads, 4096);
    void* eargs[] = {&c};
    return hipLaunchKernel((const void*)&gf_apply_wide_edges<R>, dim3(tg), dim3(kBlockThreads), eargs, 0, stream);
}

uint32_t wide_tab_words(int r) { return wide_tab_stride(r); }
uint32_t wide_tile_bytes() { return kWideTile; }
uint64_t wide_main_len(uint64_t shard_len) { return wide_main_bytes(shard_len); }

hipError_t launch_verify_wide(int r, const WideArgs& a, uint32_t* flags, int grid, hipStream_t stream) {
    if (a.K < 1 || a.K > 256 || !pos32_shard(a.shard_len)) return hipErrorInvalidValue;
    switch (r) {
        case 1: return launch_wide_r<1>(a, flags, grid, stream);
        case 2: return launch_wide_r<2>(a, flags, grid, stream);
        case 3: return launch_wide_r<3>(a, flags, grid, stream);
        case 4: return launch_wide_r<4>(a, flags, grid, stream);
        case 5: return launch_wide_r<5>(a, flags, grid, stream);
        case 6: return launch_wide_r<6>(a, flags, grid, stream);
        case 7: return launch_wide_r<7>(a, flags, grid, stream);
        case 8: return launch_wide_r<8>(a, flags, grid, stream);
    }
    return hipErrorInvalidValue;
}

uint32_t wide_apply_tiles_per_obj(uint64_t shard_len) {
    return shard_len > (uint64_t)kWideEdgeSlots ? (uint32_t)((shard_len + 32 + kWideTile - 1) / kWideTile) : 0u;
}

hipError_t launch_apply_wide(int r, const WideArgs& a, int grid, hipStream_t stream) {
    if (a.K < 1 || a.K > 256 || !pos32_shard(a.shard_len)) return hipErrorInvalidValue;
    switch (r) {
        case 1: return launch_apply_wide_r<1>(a, grid, stream);
        case 2: return launch_apply_wide_r<2>(a, grid, stream);
        case 3: return launch_apply_wide_r<3>(a, grid, stream);
        case 4: return launch_apply_wide_r<4>(a, grid, stream);
        case 5: return launch_apply_wide_r<5>(a, grid, stream);
        case 6: return launch_apply_wide_r<6>(a, grid, stream);
        case 7: return launch_apply_wide_r<7>(a, grid, stream);
        case 8: return launch_apply_wide_r<8>(a, grid, stream);
    }
    return hipErrorInvalidValue;
}

}  // namespace hbec
