// layout_probe.hip — tuning aid, not product.  Why do
// ecSplit databufs (shard j of object o at o*6S + j*S, parity in the same row,
// objectserver/ecutils.go:31-35) stream slower than data and parity in
// separate arrays, with the same bytes moved (PMC: 1.000x in both)?  One
// GF-free 4-in / 2-out kernel (the product's pipelined schedule: next tile's
// loads in flight, one block barrier per tile, 1 block of 4 waves per CU,
// s_sleep pacing, XCD-grouped blocks), S = 256 KiB, 4096 objects, five
// placements, interleaved over rounds:
//   split     : in  = A + o*4S + j*S,      out = B + o*2S + r*S
//   databuf   : in  = A + o*6S + j*S,      out = A + o*6S + (4+r)*S
//   rowpitch  : in  = A + o*6S + j*S,      out = B + o*6S + (4+r)*S  (databuf pitch, separate arrays)
//   inpitch6  : in  = A + o*6S + j*S,      out = B + o*2S + r*S      (databuf input pitch only)
//   outpitch6 : in  = A + o*4S + j*S,      out = B + o*6S + (4+r)*S  (databuf output pitch only)
// Prints one JSON line per (round, placement): ms and % of 8 TB/s.
//   hipcc --offload-arch=gfx950 -O3 scripts/layout_probe.hip -o scripts/layout_probe.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gc;
typedef __attribute__((address_space(1))) u32x4 gv;

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(3);                                                                      \
        }                                                                                 \
    } while (0)

struct Place {
    uint64_t in_base, in_pitch, out_base, out_pitch, out_off;  // out r at out_base + o*out_pitch + out_off + r*S
};

__device__ __forceinline__ u32x4 ld(uint64_t a) { return __builtin_nontemporal_load(reinterpret_cast<gc*>(a)); }
__device__ __forceinline__ void st(uint64_t a, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<gv*>(a)); }

__global__ __launch_bounds__(256, 1) void xor42(Place p, uint64_t S, uint32_t tpo, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nb = gridDim.x;
    const uint32_t blk = (nb % 8u == 0u) ? (blockIdx.x % 8u) * (nb / 8u) + blockIdx.x / 8u : blockIdx.x;
    const uint32_t nw = nb * 4;
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(blk * 4);
    const uint32_t dw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w0 >= n) return;
    auto base = [&](uint32_t i, uint64_t& ib, uint64_t& ob, uint64_t& off) {
        const uint32_t ii = i < n ? i : n - 1;
        const uint32_t o = ii / tpo;
        off = (uint64_t)(ii - o * tpo) * 1024u + lane * 16u;
        ib = p.in_base + (uint64_t)o * p.in_pitch;
        ob = p.out_base + (uint64_t)o * p.out_pitch + p.out_off;
    };
    uint64_t ib, ob, off;
    base(w0 + dw, ib, ob, off);
    u32x4 x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = ld(ib + j * S + off);
    uint32_t t = w0 + dw;
    for (uint32_t b0 = w0 + nw; b0 < n; b0 += nw) {
        uint64_t ib2, ob2, off2;
        base(b0 + dw, ib2, ob2, off2);
        u32x4 y[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = ld(ib2 + j * S + off2);
        __builtin_amdgcn_s_sleep(8);
        __builtin_amdgcn_s_barrier();
        u32x4 a = x[0] ^ x[1] ^ x[2] ^ x[3];
        if (t < n) {
            st(ob + off, a);
            a.x ^= 1u;
            st(ob + S + off, a);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = y[j];
        ib = ib2;
        ob = ob2;
        off = off2;
        t = b0 + dw;
    }
    u32x4 a = x[0] ^ x[1] ^ x[2] ^ x[3];
    if (t < n) {
        st(ob + off, a);
        a.x ^= 1u;
        st(ob + S + off, a);
    }
}

int main() {
    const uint64_t S = 262144, nobj = 4096;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *A, *B;
    CK(hipMalloc(&A, nobj * 6 * S));
    CK(hipMalloc(&B, nobj * 6 * S));
    CK(hipMemset(A, 0x5A, nobj * 6 * S));
    CK(hipMemset(B, 0, nobj * 6 * S));
    const uint64_t a = (uint64_t)A, b = (uint64_t)B;
    struct Named {
        const char* name;
        Place p;
    };
    const Named places[] = {{"split", {a, 4 * S, b, 2 * S, 0}},
                            {"databuf", {a, 6 * S, a, 6 * S, 4 * S}},
                            {"rowpitch", {a, 6 * S, b, 6 * S, 4 * S}},
                            {"inpitch6", {a, 6 * S, b, 2 * S, 0}},
                            {"outpitch6", {a, 4 * S, b, 6 * S, 4 * S}}};
    const uint32_t tpo = (uint32_t)(S / 1024), n = (uint32_t)(nobj * tpo);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 40; ++w) hipLaunchKernelGGL(xor42, dim3(cus), dim3(256), 0, 0, places[0].p, S, tpo, n);
    CK(hipDeviceSynchronize());
    for (int round = 0; round < 4; ++round)
        for (const Named& pl : places) {
            std::vector<float> ts;
            for (int r = 0; r < 13; ++r) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(xor42, dim3(cus), dim3(256), 0, 0, pl.p, S, tpo, n);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 3) ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            const float ms = ts[ts.size() / 2];
            const double gbs = (double)nobj * 6 * S / (ms * 1e-3) / 1e9;
            printf("{\"probe\": \"layout xor42\", \"round\": %d, \"placement\": \"%s\", \"ms\": %.4f, \"GB_s\": %.1f, "
                   "\"frac\": %.4f}\n",
                   round, pl.name, ms, gbs, gbs / 8000.0);
            fflush(stdout);
        }
    return 0;
}
