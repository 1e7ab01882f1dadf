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

constexpr uint32_t kWideStore = 62;           // compared columns per 64-lane window
constexpr uint32_t kWideWin = kWideStore * 16;  // shard bytes per tile
constexpr int kWideD = 4;                     // loads in flight per lane (ring depth)

__host__ __device__ constexpr uint32_t wide_tab_stride(int r) { return (uint32_t)((r * 5 + 3) & ~3); }

// shard columns 16 i + 16 <= S - 16 are compared by the main kernel
__host__ __device__ inline uint64_t wide_main_bytes(uint64_t S) { return S >= 32 ? ((S - 16) / 16) * 16 : 0; }

struct WideLd {
    uint64_t base4;
    int32_t off, lim;
    uint32_t sh;
};

__device__ __forceinline__ WideLd wide_in(uint64_t base, int32_t S, int32_t c) {
    const int32_t l4 = (int32_t)((uint32_t)base & 3u);
    const int32_t t = l4 + c;
    WideLd o;
    o.base4 = base & ~(uint64_t)3;
    o.sh = (uint32_t)t & 3u;
    o.off = t - (int32_t)o.sh;
    o.lim = ((l4 + S + 3) & ~3) - 16;
    return o;
}

__device__ __forceinline__ u32x4 wide_ld(const WideLd& o, uint32_t lane) {
    int32_t v = o.off + 16 * (int32_t)lane;
    v = v < 0 ? 0 : (v > o.lim ? o.lim : v);
    return ld16_addr(o.base4 + (uint64_t)(uint32_t)v);
}

__device__ __forceinline__ u32x4 wide_shift(const u32x4& v, uint32_t sh) {
    const uint32_t n0 = lane_next(v[0]);
    return u32x4{__builtin_amdgcn_alignbyte(v[1], v[0], sh), __builtin_amdgcn_alignbyte(v[2], v[1], sh),
                 __builtin_amdgcn_alignbyte(v[3], v[2], sh), __builtin_amdgcn_alignbyte(n0, v[3], sh)};
}

// Stream pointer: element j of tile t (object obj, tile ti within it);
// element j < K of a tile is input j, element K + r stored parity r.
struct WidePtr {
    uint32_t t, obj, ti, j;
};

__device__ __forceinline__ void wide_set(WidePtr& p, uint32_t t, uint32_t tpo) {
    p.t = t;
    p.obj = t / tpo;
    p.ti = t - p.obj * tpo;
    p.j = 0;
}

template <int R>
__global__ __launch_bounds__(kPipeBlockThreads) void gf_verify_wide(WideArgs a, uint32_t* flags) {
    extern __shared__ uint32_t lds_tab[];
    const uint32_t ts = wide_tab_stride(R);
    for (uint32_t i = threadIdx.x; i < a.K * ts; i += blockDim.x) lds_tab[i] = a.tab[i];
    __syncthreads();

    constexpr uint32_t WPB = kPipeBlockThreads / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * WPB;
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * WPB + (threadIdx.x >> 6));
    const uint32_t n = a.n_tiles, tpo = a.tiles_per_obj, K = a.K;
    if (w >= n) return;
    const uint32_t L = K + R;                          // elements per tile
    const uint32_t total = ((n - 1u - w) / nw + 1u) * L;  // this wave's elements
    const int32_t S = (int32_t)a.shard_len;
    const int32_t main_end = (int32_t)wide_main_bytes(a.shard_len);

    // producer: loads run kWideD elements ahead of the consumer, across tile
    // boundaries; past the wave's last element it reloads that element
    WidePtr pp, cp;
    wide_set(pp, w, tpo);
    wide_set(cp, w, tpo);
    uint32_t issued = 0;
    auto issue = [&](u32x4& buf, uint32_t& sh) {
        const uint32_t j = pp.j;
        const uint64_t base = j < K ? a.in_base[j] + (uint64_t)pp.obj * a.in_stride[j]
                                    : a.out[j - K] + (uint64_t)pp.obj * a.out_stride[j - K];
        const WideLd o = wide_in(base, S, (int32_t)(pp.ti * kWideWin));
        buf = wide_ld(o, lane);
        sh = __builtin_amdgcn_readfirstlane(o.sh);
        if (++issued < total) {
            if (++pp.j == L) wide_set(pp, pp.t + nw, tpo);
        }
    };
    u32x4 ring[kWideD];
    uint32_t rsh[kWideD];
#pragma unroll
    for (int i = 0; i < kWideD; ++i) issue(ring[i], rsh[i]);

    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
    bool bad = false;
    for (uint32_t p0 = 0; p0 < total; p0 += kWideD) {
#pragma unroll
        for (int i = 0; i < kWideD; ++i) {
            const u32x4 x = wide_shift(ring[i], rsh[i]);
            issue(ring[i], rsh[i]);  // unconditional: no load under a branch
            if (p0 + (uint32_t)i < total) {  // wave-uniform; no global loads inside
                const uint32_t j = cp.j;
                if (j < K) {
                    const uint32_t* tp = lds_tab + j * ts;
                    uint32_t t5[R][5];
#pragma unroll
                    for (int r = 0; r < R; ++r)
#pragma unroll
                        for (int q = 0; q < 5; ++q) t5[r][q] = tp[5 * r + q];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const Sel sx = selectors(x[e]);
#pragma unroll
                        for (int r = 0; r < R; ++r)
                            acc[r][e] ^= gf_mul_sel(sx, t5[r][0], t5[r][1], t5[r][2], t5[r][3], t5[r][4]);
                    }
                } else {
                    // stored parity r0 = j - K against the recomputed column
                    const uint32_t r0 = j - K;
                    const int32_t cpos = (int32_t)(cp.ti * kWideWin) + 16 * (int32_t)lane;
                    const bool mine = lane < kWideStore && cpos + 16 <= main_end;
                    u32x4 want = acc[0];
#pragma unroll
                    for (int r = 1; r < R; ++r)
                        if (r0 == (uint32_t)r) want = acc[r];
                    const u32x4 df = want ^ x;
                    bad |= mine && (df[0] | df[1] | df[2] | df[3]) != 0u;
                    if (r0 == R - 1u) {
                        if (__any(bad) && lane == 0u) atomicOr(flags + cp.obj, 1u);
                        bad = false;
#pragma unroll
                        for (int r = 0; r < R; ++r) acc[r] = u32x4{0, 0, 0, 0};
                    }
                }
                if (++cp.j == L) wide_set(cp, cp.t + nw, tpo);
            }
        }
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

template <int R>
static hipError_t launch_wide_r(const WideArgs& a, uint32_t* flags, int grid, hipStream_t stream) {
    WideArgs c = a;
    void* args[] = {&c, &flags};
    hipError_t e = hipSuccess;
    const size_t lds = (size_t)a.K * wide_tab_stride(R) * 4;
    if (a.n_tiles > 0) e = hipLaunchKernel((const void*)&gf_verify_wide<R>, dim3(grid), dim3(kPipeBlockThreads), args, lds, stream);
    if (e != hipSuccess) return e;
    const uint64_t tail = (uint64_t)a.n_obj * R * (a.shard_len - wide_main_bytes(a.shard_len));
    if (tail == 0) return hipSuccess;
    const int tg = (int)std::min<uint64_t>((tail + kBlockThreads - 1) / kBlockThreads, 4096);
    return hipLaunchKernel((const void*)&gf_verify_wide_tail<R>, dim3(tg), dim3(kBlockThreads), args, 0, stream);
}

uint32_t wide_tab_words(int r) { return wide_tab_stride(r); }
uint32_t wide_tile_bytes() { return kWideWin; }
uint64_t wide_main_len(uint64_t shard_len) { return wide_main_bytes(shard_len); }

hipError_t launch_verify_wide(int r, const WideArgs& a, uint32_t* flags, int grid, hipStream_t stream) {
    if (a.K < 1 || a.K > 256 || a.shard_len >= (1ull << 31)) return hipErrorInvalidValue;
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

}  // namespace hbec
