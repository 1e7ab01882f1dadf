// oob_probe.hip — tuning aid, not product.  What does a 16-B raw buffer load
// return when it straddles the descriptor's num_records (partly in range)?
// Per-dword range checking would return the in-range dwords and zeros for
// the rest; whole-access checking returns all zeros.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const uint8_t* base, uint32_t nrec, uint32_t* out) {
    const uint32_t lane = threadIdx.x;  // offset = lane (bytes)
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nrec, 0x00020000);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane, 0, 0);
    out[lane * 4 + 0] = v[0];
    out[lane * 4 + 1] = v[1];
    out[lane * 4 + 2] = v[2];
    out[lane * 4 + 3] = v[3];
}

int main() {
    uint8_t* d;
    uint32_t* o;
    if (hipMalloc(&d, 4096) != hipSuccess || hipMalloc(&o, 64 * 16) != hipSuccess) return 3;
    uint8_t h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i + 1);
    if (hipMemcpy(d, h, 4096, hipMemcpyHostToDevice) != hipSuccess) return 5;
    const uint32_t nrec = 40;  // bytes in range
    hipLaunchKernelGGL(k, dim3(1), dim3(48), 0, 0, d, nrec, o);
    uint32_t r[48 * 4];
    if (hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) return 4;
    printf("{\"probe\": \"buffer_load_dwordx4 straddling num_records=%u\", \"rows\": [", nrec);
    for (int off = 16; off < 44; ++off) {
        // which of the 4 dwords came back nonzero, and is dword 0 the true bytes
        uint32_t want0 = 0;
        for (int b = 0; b < 4; ++b) want0 |= (uint32_t)(uint8_t)(off + b + 1) << (8 * b);
        printf("%s{\"off\": %d, \"dw\": [%u, %u, %u, %u], \"dw0_ok\": %s}", off > 16 ? ", " : "", off,
               r[off * 4], r[off * 4 + 1], r[off * 4 + 2], r[off * 4 + 3], r[off * 4] == want0 ? "true" : "false");
    }
    printf("]}\n");
    return 0;
}
