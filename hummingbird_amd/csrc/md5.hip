// md5.hip — ShardHash on the GPU.
//
// The object server keys every stored shard by the MD5 of its whole body,
// hex-encoded (objectserver/indexdb.go:746-753, StablePut: md5.New() fed by
// common.Copy of the request body), and the auditor re-hashes shard files
// against it (objectserver/auditor.go:100-156).  A shard file is the
// concatenation of its per-stripe sub-chunks (ecutils.go:55-69), so the hash
// of a multi-stripe shard is one MD5 chain fed stripe by stripe.
//
// MD5 (RFC 1321) is a strict chain over 64-byte blocks: nothing inside one
// message parallelises.  The GPU's parallelism is across chains — one LANE
// per (object, shard) chain, 64 chains per wave — and a chain's speed is one
// wave's VALU issue rate: 64 steps x 5 VALU ops (v_bfi / v_bitop3 / v_xor3,
// v_add3, v_alignbit, v_add) per block at 4 cycles per instruction for a lone
// wave.  Blocks are loaded D at a time, one group ahead of the compression, so
// the loads' HBM latency hides behind ~D x 1300 cycles of arithmetic.
//
// Grid: x = groups of 64 objects, y = view (so a wave reads ONE view and the
// view's base/stride come from SGPRs).  Chain index (digest/state slot) is
// obj * chain_stride + view0 + view.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf_device.h"
#include "kernels.h"

namespace hbec {

__device__ constexpr uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};

__device__ constexpr int md5_shift(int i) {
    constexpr int s[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    return s[(i >> 4) * 4 + (i & 3)];
}

__device__ constexpr int md5_word(int i) {
    return i < 16 ? i : i < 32 ? (5 * i + 1) & 15 : i < 48 ? (3 * i + 5) & 15 : (7 * i) & 15;
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

// One 64-byte block.  Plain C logic: the compiler maps F/G and I to
// v_bitop3_b32 (gfx950) and a + f + (m + K) to v_add3_u32; H is written as an
// explicit XOR3 (the compiler emitted two v_xor_b32 for b ^ c ^ d).
__device__ __forceinline__ void md5_compress(uint32_t (&h)[4], const uint32_t (&m)[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t f;
        if (i < 16)
            f = d ^ (b & (c ^ d));
        else if (i < 32)
            f = c ^ (d & (b ^ c));
        else if (i < 48)
            f = xor3(b, c, d);  // one v_bitop3 (plain C became two v_xor_b32)
        else
            f = c ^ (b | ~d);
        const uint32_t t = a + f + (m[md5_word(i)] + kMd5K[i]);
        a = d;
        d = c;
        c = b;
        b = b + rotl(t, md5_shift(i));
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

__device__ __forceinline__ void md5_compress4(uint32_t (&h)[4], const u32x4 (&q)[4]) {
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        m[4 * j + 0] = q[j].x;
        m[4 * j + 1] = q[j].y;
        m[4 * j + 2] = q[j].z;
        m[4 * j + 3] = q[j].w;
    }
    md5_compress(h, m);
}

// Byte q (< carry + len) of the pending stream = carried tail ++ this call's data.
struct Pending {
    const uint8_t* tail;  // carried bytes (state), may be null when carry == 0
    const uint8_t* data;
    uint32_t carry;
    __device__ __forceinline__ uint32_t at(uint64_t q) const { return q < carry ? tail[q] : data[q - carry]; }
};

// Block of 16 words from pending bytes [off, off + n) followed by the MD5 pad
// byte 0x80 at n (when pad) and zeros; bit length in words 14-15 when len_words.
__device__ __forceinline__ void assemble(uint32_t (&m)[16], const Pending& p, uint64_t off, uint32_t n, bool pad) {
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t q = 4 * w + j;
            const uint32_t byte = q < n ? p.at(off + q) : (pad && q == n ? 0x80u : 0u);
            x |= byte << (8 * j);
        }
        m[w] = x;
    }
}

struct Md5State {
    uint32_t h[4];
    uint8_t tail[64];
};  // 80 B per chain; the carried length is uniform and kept on the host

constexpr int kMd5MaxViews = 32;
constexpr uint32_t kMd5Init = 1u, kMd5Final = 2u;

struct Md5Args {
    const uint8_t* base[kMd5MaxViews];
    uint64_t stride[kMd5MaxViews];
    Md5State* state;   // per chain; unused when flags == init|final
    uint8_t* digest;   // per chain 16 B, written on final
    uint64_t n_obj;
    uint64_t len;      // bytes per chain in this call
    uint64_t total;    // bytes per chain before this call
    uint32_t chain_stride;  // chains per object
    uint32_t view0;         // chain index of view 0 of this launch
    uint32_t flags;
    uint32_t pad_;
};


template <bool ALIGNED, int D>
__global__ __launch_bounds__(HBEC_MD5_BLOCK) void md5_chains(Md5Args a) {
    const uint32_t v = blockIdx.y;
    const uint64_t o = (uint64_t)blockIdx.x * HBEC_MD5_BLOCK + threadIdx.x;
    if (o >= a.n_obj) return;
    const uint8_t* p = a.base[v] + o * a.stride[v];
    const uint64_t chain = o * a.chain_stride + a.view0 + v;
    Md5State* st = a.state ? a.state + chain : nullptr;

    uint32_t h[4];
    if (a.flags & kMd5Init) {
        h[0] = 0x67452301u;
        h[1] = 0xefcdab89u;
        h[2] = 0x98badcfeu;
        h[3] = 0x10325476u;
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = st->h[i];
    }
    const uint32_t carry = (uint32_t)(a.total & 63u);
    Pending pend{st ? st->tail : nullptr, p, carry};
    const uint64_t lv = carry + a.len;  // pending bytes
    const uint64_t nv = lv / 64u;       // whole blocks among them
    uint64_t b0 = 0;                    // first block not yet compressed
    if (carry != 0 && nv > 0) {         // block straddling the carried tail
        uint32_t m[16];
        assemble(m, pend, 0, 64, false);
        md5_compress(h, m);
        b0 = 1;
    }
    // Blocks b0..nv-1 lie wholly in this call's data at data offset 64*b - carry.
    const uint64_t nb = nv - b0;
    if (nb > 0) {
        const uint8_t* q0 = p + (64u * b0 - carry);
        const uint64_t groups = (nb + D - 1) / D;
        u32x4 cur[D][4];
        auto load_group = [&](u32x4 (&dst)[D][4], uint64_t g) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                uint64_t blk = g * D + j;
                blk = blk < nb ? blk : nb - 1;  // clamp: always a valid address
                const uint8_t* bp = q0 + 64u * blk;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    if (ALIGNED) {
                        dst[j][w] = *reinterpret_cast<const u32x4*>(bp + 16 * w);
                    } else {
                        u32x4 x;
                        uint32_t e[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint8_t* c = bp + 16 * w + 4 * k;
                            e[k] = (uint32_t)c[0] | ((uint32_t)c[1] << 8) | ((uint32_t)c[2] << 16) |
                                   ((uint32_t)c[3] << 24);
                        }
                        x.x = e[0];
                        x.y = e[1];
                        x.z = e[2];
                        x.w = e[3];
                        dst[j][w] = x;
                    }
                }
            }
        };
        // ping-pong between two register groups: group g+1 loads while g
        // compresses, without copying registers; loads past the end re-read
        // the last group (clamped), compressions past it are skipped.
        u32x4 grp_b[D][4];
        load_group(cur, 0);
        for (uint64_t g = 0; g < groups; g += 2) {
            load_group(grp_b, g + 1 < groups ? g + 1 : g);
#pragma unroll
            for (int j = 0; j < D; ++j)
                if (g * D + j < nb) md5_compress4(h, cur[j]);
            load_group(cur, g + 2 < groups ? g + 2 : groups - 1);
#pragma unroll
            for (int j = 0; j < D; ++j)
                if ((g + 1) * D + j < nb) md5_compress4(h, grp_b[j]);
        }

    }
    const uint32_t rv = (uint32_t)(lv - nv * 64u);  // pending bytes left (< 64)
    if (a.flags & kMd5Final) {
        const uint64_t bits = (a.total + a.len) * 8u;
        uint32_t m[16];
        assemble(m, pend, nv * 64u, rv, true);
        if (rv >= 56) {
            md5_compress(h, m);
#pragma unroll
            for (int w = 0; w < 14; ++w) m[w] = 0;
        }
        m[14] = (uint32_t)bits;
        m[15] = (uint32_t)(bits >> 32);
        md5_compress(h, m);
        uint32_t* out = reinterpret_cast<uint32_t*>(a.digest + chain * 16u);
#pragma unroll
        for (int i = 0; i < 4; ++i) out[i] = h[i];
    } else {
        // carry the leftover bytes; reading pend.at(nv*64 + q) never touches a
        // tail byte this loop has already overwritten (nv > 0: data only;
        // nv == 0: byte q maps onto itself)
        for (uint32_t q = 0; q < rv; ++q) st->tail[q] = (uint8_t)pend.at(nv * 64u + q);
#pragma unroll
        for (int i = 0; i < 4; ++i) st->h[i] = h[i];
    }
}

// ---------------------------------------------------------------------------
// md5_list: one-shot MD5 of independent buffers of ANY lengths (shard files for
// an auditor pass, the shards of a host-path chunk).  One lane per chain, the
// chain described by a 32-B record; the host sorts records by length so a
// wave's lanes run similar trip counts (a wave lasts as long as its longest
// chain).  Same compression and load pipeline as md5_chains.
// ---------------------------------------------------------------------------
struct Md5ListRec {
    uint64_t addr;
    uint64_t len;
    uint64_t slot;  // digest index
    uint64_t pad_;
};

__device__ uint8_t kMd5ZeroBlock[64 * HBEC_MD5_DEPTH_LIST];  // load target of empty chains

// The loop runs the WAVE's longest chain (uniform trip count, so loads stay
// pipelined: divergent per-lane loops made the compiler wait for every load
// before each block); lanes past their own end compress clamped blocks and
// keep their state with a select.
template <bool ALIGNED>
__global__ __launch_bounds__(64) void md5_list(const Md5ListRec* __restrict__ recs, uint64_t n, uint8_t* digest) {
    constexpr int D = HBEC_MD5_DEPTH_LIST;
    const uint64_t c = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    const bool live = c < n;
    Md5ListRec r{0, 0, 0, 0};
    if (live) r = recs[c];
    const uint8_t* p = reinterpret_cast<const uint8_t*>(r.addr);
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    const uint64_t nb = r.len / 64u;
    uint64_t nb_max = nb;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = (uint64_t)__shfl_xor((long long)nb_max, off, 64);
        nb_max = o > nb_max ? o : nb_max;
    }
    nb_max = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(nb_max >> 32)) << 32) |
             __builtin_amdgcn_readfirstlane((uint32_t)nb_max);
    // integer addresses + address_space(1) loads: a generic pointer here makes
    // the compiler emit flat loads, whose lgkmcnt share forces full waits
    const uint64_t base = nb > 0 ? r.addr : reinterpret_cast<uint64_t>(kMd5ZeroBlock);
    const uint64_t last = nb > 0 ? nb - 1 : 0;
    if (nb_max > 0) {
        const uint64_t groups = (nb_max + D - 1) / D;
        auto load_group = [&](u32x4 (&dst)[D][4], uint64_t g) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                uint64_t blk = g * D + j;
                blk = blk < last ? blk : last;  // clamp to this lane's chain
                const uint64_t bp = base + 64u * blk;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    if (ALIGNED) {
                        dst[j][w] = *reinterpret_cast<gu32x4_c*>(bp + 16 * w);
                    } else {
                        typedef __attribute__((address_space(1))) const uint8_t gu8_c;
                        uint32_t e[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            gu8_c* q = reinterpret_cast<gu8_c*>(bp + 16 * w + 4 * k);
                            e[k] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) |
                                   ((uint32_t)q[3] << 24);
                        }
                        dst[j][w] = u32x4{e[0], e[1], e[2], e[3]};
                    }
                }
            }
        };
        auto step = [&](const u32x4 (&q)[4], uint64_t blk) {
            uint32_t t[4] = {h[0], h[1], h[2], h[3]};
            md5_compress4(t, q);
            const bool keep = blk < nb;
#pragma unroll
            for (int i = 0; i < 4; ++i) h[i] = keep ? t[i] : h[i];
        };
        u32x4 ga[D][4], gb[D][4];
        load_group(ga, 0);
        for (uint64_t g = 0; g < groups; g += 2) {  // uniform: groups from the wave maximum
            load_group(gb, g + 1 < groups ? g + 1 : g);
#pragma unroll
            for (int j = 0; j < D; ++j)
                if (g * D + j < nb_max) step(ga[j], g * D + j);
            load_group(ga, g + 2 < groups ? g + 2 : groups - 1);
#pragma unroll
            for (int j = 0; j < D; ++j)
                if ((g + 1) * D + j < nb_max) step(gb[j], (g + 1) * D + j);
        }
    }
    if (!live) return;
    const uint32_t rv = (uint32_t)(r.len - nb * 64u);
    const Pending pend{nullptr, p, 0};
    uint32_t m[16];
    assemble(m, pend, nb * 64u, rv, true);
    if (rv >= 56) {
        md5_compress(h, m);
#pragma unroll
        for (int w = 0; w < 14; ++w) m[w] = 0;
    }
    const uint64_t bits = r.len * 8u;
    m[14] = (uint32_t)bits;
    m[15] = (uint32_t)(bits >> 32);
    md5_compress(h, m);
    uint32_t* out = reinterpret_cast<uint32_t*>(digest + r.slot * 16u);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = h[i];
}

// Blocks per load group and the buffer scheme, from the depth sweep on MI355X
// (profiles/r01_md5_sweep.jsonl).

uint64_t md5_state_bytes() { return sizeof(Md5State); }

// recs: device array of n records ({addr, len, slot, 0}); aligned = every addr 16-B aligned.
hipError_t launch_md5_list(const void* recs, uint64_t n, uint8_t* digest, bool aligned, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 63) / 64));
    const Md5ListRec* r = static_cast<const Md5ListRec*>(recs);
    if (aligned)
        hipLaunchKernelGGL(md5_list<true>, grid, dim3(64), 0, stream, r, n, digest);
    else
        hipLaunchKernelGGL(md5_list<false>, grid, dim3(64), 0, stream, r, n, digest);
    return hipGetLastError();
}

// views: n_views (base, stride) pairs (<= kMd5MaxViews per launch; callers
// split), chain (o, view0 + v) of chain_stride chains per object.
hipError_t launch_md5(const void* const* bases, const uint64_t* strides, int n_views, uint32_t chain_stride,
                      uint32_t view0, uint64_t n_obj, uint64_t len, uint64_t total, uint32_t flags, void* state,
                      uint8_t* digest, bool aligned, hipStream_t stream) {
    if (n_views <= 0 || n_views > kMd5MaxViews || n_obj == 0) return hipErrorInvalidValue;
    Md5Args a{};
    for (int v = 0; v < n_views; ++v) {
        a.base[v] = static_cast<const uint8_t*>(bases[v]);
        a.stride[v] = strides[v];
    }
    a.state = static_cast<Md5State*>(state);
    a.digest = digest;
    a.n_obj = n_obj;
    a.len = len;
    a.total = total;
    a.chain_stride = chain_stride;
    a.view0 = view0;
    a.flags = flags;
    const dim3 grid((unsigned)((n_obj + HBEC_MD5_BLOCK - 1) / HBEC_MD5_BLOCK), (unsigned)n_views);
    if (aligned)
        hipLaunchKernelGGL((md5_chains<true, HBEC_MD5_DEPTH>), grid, dim3(HBEC_MD5_BLOCK), 0, stream, a);
    else
        hipLaunchKernelGGL((md5_chains<false, 1>), grid, dim3(HBEC_MD5_BLOCK), 0, stream, a);
    return hipGetLastError();
}

}  // namespace hbec
