// hbm_probe.hip — HBM ceilings on MI355X for the EC access pattern (tuning aid,
// not product).  Kernels: read-only, write-only, copy, and a GF-free
// "xor k->r" with exactly the encode kernel's views and tile walk.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// objs [n][K*S], out [n][R*S]; out[r] = XOR_j in[j] ^ r  (no field arithmetic)
template <int K, int R>
__device__ void xor_body(const uint8_t* objs, uint8_t* out, uint32_t n_obj, uint32_t S, uint32_t mode) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * 4;
    const uint32_t tpo = S / 1024;
    const uint32_t nt = n_obj * tpo;
    for (uint32_t t = wave; t < nt; t += nw) {
        uint32_t o, tile;
        if (mode == 0) { o = t / tpo; tile = t - o * tpo; }            // object-major (product)
        else { tile = t / n_obj; o = t - tile * n_obj; }               // offset-major
        const uint64_t off = (uint64_t)tile * 1024 + lane * 16;
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            x[j] = __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(objs + (uint64_t)o * K * S + (uint64_t)j * S + off));
#pragma unroll
        for (int r = 0; r < R; ++r) {
            u32x4 a = {(uint32_t)r, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < K; ++j) a ^= x[j];
            __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(out + (uint64_t)o * R * S + (uint64_t)r * S + off));
        }
    }
}


extern "C" {
int probe_write_variant(int v, void* dst, uint64_t n, int grid, void* stream);

__global__ __launch_bounds__(256) void probe_read(const uint8_t* src, uint64_t n16, uint32_t* sink) {
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

__global__ __launch_bounds__(256) void probe_write(uint8_t* dst, uint64_t n16) {
    const u32x4 v = {1, 2, 3, 4};
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst) + i);
}

__global__ __launch_bounds__(256) void probe_copy(const uint8_t* src, uint8_t* dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i);
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst) + i);
    }
}

__global__ __launch_bounds__(256) void probe_xor42(const uint8_t* objs, uint8_t* out, uint32_t n_obj, uint32_t S,
                                                    uint32_t mode) {
    xor_body<4, 2>(objs, out, n_obj, S, mode);
}

__global__ __launch_bounds__(256) void probe_xor40(const uint8_t* objs, uint8_t* out, uint32_t n_obj, uint32_t S,
                                                    uint32_t mode) {
    // read-only variant of the same walk: one word per wave written
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * 4;
    const uint32_t tpo = S / 1024;
    const uint32_t nt = n_obj * tpo;
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t t = wave; t < nt; t += nw) {
        const uint32_t o = t / tpo, tile = t - o * tpo;
        const uint64_t off = (uint64_t)tile * 1024 + lane * 16;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc ^= __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(objs + (uint64_t)o * 4 * S + (uint64_t)j * S + off));
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

}  // extern "C"

// 6-stream xor probe with U consecutive 1 KiB tiles per wave iteration
template <int U>
__global__ __launch_bounds__(256) void probe_xor42u(const uint8_t* objs, uint8_t* out, uint32_t n_obj, uint32_t S) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * 4;
    const uint32_t tpo = S / (1024 * U);
    const uint32_t nt = n_obj * tpo;
    for (uint32_t t = wave; t < nt; t += nw) {
        const uint32_t o = t / tpo, tile = t - o * tpo;
        const uint64_t off = (uint64_t)tile * 1024 * U + lane * 16;
        u32x4 x[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                x[u][j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                    objs + (uint64_t)o * 4 * S + (uint64_t)j * S + off + u * 1024));
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                u32x4 a = {(uint32_t)r, 0, 0, 0};
#pragma unroll
                for (int j = 0; j < 4; ++j) a ^= x[u][j];
                __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(out + (uint64_t)o * 2 * S + (uint64_t)r * S + off + u * 1024));
            }
    }
}

// same 4->2 XOR but shard-INTERLEAVED layout: per object, per 1 KiB column
// block, the 4 input blocks are adjacent (in [n][S/1K][4][1K]) and so are the
// 2 outputs (out [n][S/1K][2][1K]): 2 streams instead of 6.
__global__ __launch_bounds__(256) void probe_xor42_il(const uint8_t* objs, uint8_t* out, uint32_t n_obj, uint32_t S) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * 4;
    const uint64_t nt = (uint64_t)n_obj * (S / 1024);
    for (uint64_t t = wave; t < nt; t += nw) {
        const u32x4* src = reinterpret_cast<const u32x4*>(objs + t * 4096) + lane;
        u32x4 x0 = __builtin_nontemporal_load(src), x1 = __builtin_nontemporal_load(src + 64),
              x2 = __builtin_nontemporal_load(src + 128), x3 = __builtin_nontemporal_load(src + 192);
        u32x4* dst = reinterpret_cast<u32x4*>(out + t * 2048) + lane;
        u32x4 a = x0 ^ x1 ^ x2 ^ x3;
        __builtin_nontemporal_store(a, dst);
        a.x ^= 1u;
        __builtin_nontemporal_store(a, dst + 64);
    }
}

// store-flavour probes: aux bits of the buffer store (1 = sc0, 2 = nt, 16 = sc1)
template <int AUX, int UNR>
__global__ __launch_bounds__(256) void probe_write_buf(uint8_t* dst, uint64_t n16) {
    const u32x4 v = {1, 2, 3, 4};
    // one 4 GiB-capable descriptor per 2 GiB window
    const uint64_t per_block = (uint64_t)UNR * 256;
    for (uint64_t base = (uint64_t)blockIdx.x * per_block; base < n16; base += (uint64_t)gridDim.x * per_block) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + base * 16, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint32_t off = (uint32_t)((u * 256 + threadIdx.x) * 16);
            if (base + u * 256 + threadIdx.x < n16) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, AUX);
        }
    }
}

template <int MODE, int UNR>
__global__ __launch_bounds__(256) void probe_write_flat(uint8_t* dst, uint64_t n16) {
    const u32x4 v = {1, 2, 3, 4};
    const uint64_t per_block = (uint64_t)UNR * 256;
    for (uint64_t base = (uint64_t)blockIdx.x * per_block; base < n16; base += (uint64_t)gridDim.x * per_block) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const uint64_t i = base + u * 256 + threadIdx.x;
            if (i < n16) {
                if (MODE == 0) *(reinterpret_cast<u32x4*>(dst) + i) = v;
                else __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst) + i);
            }
        }
    }
}

// copy sweep: block-contiguous chunk of U x blockDim float4 per iteration,
// all U loads issued before the U stores.
template <int U, int NT>
__global__ void probe_copy_u(const uint8_t* src, uint8_t* dst, uint64_t n16) {
    const u32x4* s = reinterpret_cast<const u32x4*>(src);
    u32x4* d = reinterpret_cast<u32x4*>(dst);
    const uint64_t chunk = (uint64_t)U * blockDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * chunk; base < n16; base += (uint64_t)gridDim.x * chunk) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * blockDim.x + threadIdx.x;
            if (NT) v[u] = __builtin_nontemporal_load(s + i); else v[u] = s[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + (uint64_t)u * blockDim.x + threadIdx.x;
            if (NT) __builtin_nontemporal_store(v[u], d + i); else d[i] = v[u];
        }
    }
}

extern "C" {
int probe_xor_variant(int u, const void* src, void* dst, uint32_t n_obj, uint32_t S, int grid, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const uint8_t* a = (const uint8_t*)src;
    uint8_t* b = (uint8_t*)dst;
    if (u == 0) hipLaunchKernelGGL(probe_xor42_il, dim3(grid), dim3(256), 0, st, a, b, n_obj, S);
    else if (u == 1) hipLaunchKernelGGL((probe_xor42u<1>), dim3(grid), dim3(256), 0, st, a, b, n_obj, S);
    else if (u == 2) hipLaunchKernelGGL((probe_xor42u<2>), dim3(grid), dim3(256), 0, st, a, b, n_obj, S);
    else if (u == 4) hipLaunchKernelGGL((probe_xor42u<4>), dim3(grid), dim3(256), 0, st, a, b, n_obj, S);
    else return -1;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
int probe_copy_variant(int u, int nt, const void* src, void* dst, uint64_t n, int grid, int block, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const uint8_t* a = (const uint8_t*)src;
    uint8_t* b = (uint8_t*)dst;
    const uint64_t n16 = n / 16;
    if (n16 % ((uint64_t)u * block)) return -3;
#define CASE(U, NT) if (u == U && nt == NT) hipLaunchKernelGGL((probe_copy_u<U, NT>), dim3(grid), dim3(block), 0, st, a, b, n16);
    CASE(1, 0) CASE(2, 0) CASE(4, 0) CASE(8, 0) CASE(1, 1) CASE(2, 1) CASE(4, 1) CASE(8, 1)
#undef CASE
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
static int grid_for(int blocks) { return blocks; }

int probe_write_variant(int v, void* dst, uint64_t n, int grid, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    uint8_t* d = (uint8_t*)dst;
    const uint64_t n16 = n / 16;
    switch (v) {
        case 0: hipLaunchKernelGGL((probe_write_flat<0, 1>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 1: hipLaunchKernelGGL((probe_write_flat<1, 1>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 2: hipLaunchKernelGGL((probe_write_flat<0, 4>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 3: hipLaunchKernelGGL((probe_write_flat<1, 4>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 4: hipLaunchKernelGGL((probe_write_buf<0, 4>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 5: hipLaunchKernelGGL((probe_write_buf<2, 4>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 6: hipLaunchKernelGGL((probe_write_buf<16, 4>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 7: hipLaunchKernelGGL((probe_write_buf<17, 4>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 8: hipLaunchKernelGGL((probe_write_buf<18, 4>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 9: hipLaunchKernelGGL((probe_write_buf<1, 4>), dim3(grid), dim3(256), 0, st, d, n16); break;
        case 10: hipLaunchKernelGGL((probe_write_flat<1, 8>), dim3(grid), dim3(256), 0, st, d, n16); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int probe_launch(int which, const void* a, void* b, uint64_t n, uint32_t n_obj, uint32_t S, uint32_t mode, int grid,
                 void* stream) {
    hipStream_t st = (hipStream_t)stream;
    switch (which) {
        case 0: hipLaunchKernelGGL(probe_read, dim3(grid_for(grid)), dim3(256), 0, st, (const uint8_t*)a, n / 16, (uint32_t*)b); break;
        case 1: hipLaunchKernelGGL(probe_write, dim3(grid), dim3(256), 0, st, (uint8_t*)b, n / 16); break;
        case 2: hipLaunchKernelGGL(probe_copy, dim3(grid), dim3(256), 0, st, (const uint8_t*)a, (uint8_t*)b, n / 16); break;
        case 3: hipLaunchKernelGGL(probe_xor42, dim3(grid), dim3(256), 0, st, (const uint8_t*)a, (uint8_t*)b, n_obj, S, mode); break;
        case 4: hipLaunchKernelGGL(probe_xor40, dim3(grid), dim3(256), 0, st, (const uint8_t*)a, (uint8_t*)b, n_obj, S, mode); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
}
