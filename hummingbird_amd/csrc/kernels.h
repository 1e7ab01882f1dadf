// kernels.h — launch interface of the gfx950 GF(2^8) shard kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbec {

constexpr int kMaxK = 16;         // inputs per kernel pass
constexpr int kMaxR = 4;          // outputs per kernel pass
constexpr int kBlockThreads = 256;
#ifndef HBEC_WAVES_PER_SIMD
#define HBEC_WAVES_PER_SIMD 4
#endif
constexpr int kVecWavesPerSimd = HBEC_WAVES_PER_SIMD;  // occupancy floor for the vec kernels

// One pass: out[r] (^)= XOR_{j<K} C[r][j] * in[j] over n_obj objects.
// Input j of object o starts at in[j] + o*in_stride[j]; likewise outputs.
struct PassArgs {
    const uint8_t* in[kMaxK];
    uint64_t in_stride[kMaxK];
    uint8_t* out[kMaxR];
    uint64_t out_stride[kMaxR];
    uint32_t tab[kMaxR][kMaxK][5];  // v_perm tables per coefficient (gf256.h perm_table)
    uint64_t n_obj;
    uint64_t shard_len;     // bytes per shard processed by this pass
    uint32_t tiles_per_obj; // vec path: ceil(shard_len / vec_tile_bytes)
    uint32_t n_tiles;       // vec path: n_obj * tiles_per_obj (< 2^32)
    uint32_t accumulate;    // 1: out ^= result (passes 2.. over >kMaxK inputs)
    uint32_t pad_;
};

// Vec path launch: fully unrolled kernel for small shapes, streaming otherwise.
int vec_tile_bytes(int k, int r, uint64_t shard_len, int accumulate, int force_stream);
int is_streaming_shape(int k, int r, int force_stream);
int is_pipe_shape(int k, int r, uint64_t shard_len, int force_stream);
// Pipelined kernels: U = 16/K KiB of each input per wave tile (K*U = 16 loads).
__host__ __device__ constexpr int pipe_u(int k) { return k >= 16 ? 1 : (16 / k > 4 ? 4 : 16 / k); }

hipError_t launch_vec(int k, int r, const PassArgs& a, int grid, hipStream_t stream, int force_stream);
hipError_t launch_bytes(int k, int r, const PassArgs& a, int grid, hipStream_t stream);
hipError_t launch_fill(uint8_t* dst, uint64_t n_obj, uint64_t obj_len, uint64_t obj_stride, uint64_t base_seed,
                       uint64_t first, int grid, hipStream_t stream);
hipError_t vec_occupancy(int k, int r, int pipe, int force_stream, int* blocks_per_cu);

// ---- stripes (stripes.hip): mixed shard lengths in one launch ----
// One record per tile: shard i of the tile starts at addr + i*shard_len;
// lanes at offsets >= valid are masked on store.
struct TileRec {
    uint64_t addr;
    uint32_t shard_len;
    uint32_t valid;
};

struct StripeArgs {
    const TileRec* tiles;
    uint32_t n_tiles;
    uint32_t pad_;
    uint32_t in_idx[kMaxK];   // shard index read as input j
    uint32_t out_idx[kMaxR];  // shard index written as output r
    uint32_t tab[kMaxR][kMaxK][5];
};

int stripes_tile_bytes(int k);
bool stripes_supported(int k, int r);
hipError_t launch_stripes(int k, int r, const StripeArgs& a, int grid, hipStream_t stream);
hipError_t stripes_occupancy(int k, int r, int* blocks_per_cu);

}  // namespace hbec
