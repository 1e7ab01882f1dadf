// gf256.h — host-side GF(2^8) field and coding-matrix construction.
//
// Restates the codec of github.com/klauspost/reedsolomon that
// objectserver/ecutils.go:27,77,135 builds with reedsolomon.New(k, m):
//   field   : poly 0x11D, generator 2 (klauspost galois.go)
//   matrix  : Vandermonde(k+m, k) x inv(top k x k) (klauspost matrix.go buildMatrix)
//   inverse : Gauss-Jordan (matrix.go Invert); unique, so only the result matters.
// This is product code (it runs on the host beside the kernels); the oracle in
// oracle/ is an independent restatement used only by the tests.
#pragma once
#include <stdint.h>

#include <cstring>
#include <vector>

namespace hbec {

struct Field {
    uint8_t exp[510];
    uint8_t log[256];
    Field() {
        int x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = exp[i + 255] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a == 0 || b == 0) ? 0 : exp[log[a] + log[b]]; }
    uint8_t div(uint8_t a, uint8_t b) const {
        if (a == 0) return 0;
        int d = (int)log[a] - (int)log[b];
        if (d < 0) d += 255;
        return exp[d];
    }
    uint8_t pow(uint8_t a, int n) const {  // galExp
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[(log[a] * n) % 255];
    }
};

inline const Field& field() {
    static const Field f;
    return f;
}

// Row-major n x n inverse over GF(2^8).  Returns false if singular.
inline bool invert(int n, const uint8_t* in, uint8_t* out) {
    const Field& F = field();
    const int w = 2 * n;
    std::vector<uint8_t> a((size_t)n * w, 0);
    for (int r = 0; r < n; ++r) {
        std::memcpy(&a[(size_t)r * w], in + (size_t)r * n, n);
        a[(size_t)r * w + n + r] = 1;
    }
    for (int r = 0; r < n; ++r) {
        uint8_t* row = &a[(size_t)r * w];
        if (row[r] == 0) {
            for (int b = r + 1; b < n; ++b) {
                uint8_t* rb = &a[(size_t)b * w];
                if (rb[r] != 0) {
                    for (int c = 0; c < w; ++c) std::swap(row[c], rb[c]);
                    break;
                }
            }
        }
        if (row[r] == 0) return false;
        if (row[r] != 1) {
            const uint8_t s = F.div(1, row[r]);
            for (int c = 0; c < w; ++c) row[c] = F.mul(s, row[c]);
        }
        for (int b = r + 1; b < n; ++b) {
            uint8_t* rb = &a[(size_t)b * w];
            const uint8_t s = rb[r];
            if (s)
                for (int c = 0; c < w; ++c) rb[c] ^= F.mul(s, row[c]);
        }
    }
    for (int d = 0; d < n; ++d)
        for (int ab = 0; ab < d; ++ab) {
            uint8_t* ra = &a[(size_t)ab * w];
            const uint8_t s = ra[d];
            if (s) {
                const uint8_t* rd = &a[(size_t)d * w];
                for (int c = 0; c < w; ++c) ra[c] ^= F.mul(s, rd[c]);
            }
        }
    for (int r = 0; r < n; ++r) std::memcpy(out + (size_t)r * n, &a[(size_t)r * w + n], n);
    return true;
}

// (k+m) x k systematic coding matrix (klauspost buildMatrix).
inline bool build_matrix(int k, int m, std::vector<uint8_t>& out) {
    const Field& F = field();
    const int total = k + m;
    std::vector<uint8_t> vm((size_t)total * k), inv((size_t)k * k);
    for (int r = 0; r < total; ++r)
        for (int c = 0; c < k; ++c) vm[(size_t)r * k + c] = F.pow((uint8_t)r, c);
    if (!invert(k, vm.data(), inv.data())) return false;
    out.assign((size_t)total * k, 0);
    for (int r = 0; r < total; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t v = 0;
            for (int i = 0; i < k; ++i) v ^= F.mul(vm[(size_t)r * k + i], inv[(size_t)i * k + c]);
            out[(size_t)r * k + c] = v;
        }
    return true;
}

// v_perm_b32 lookup tables for multiplication by c (kernels.hip gf_mul_sel):
//   t[0..1] : c * b        for b = 0..7   (bytes 0-3 in t[0], 4-7 in t[1])
//   t[2..3] : c * (b << 3) for b = 0..7
//   t[4]    : c * (b << 6) for b = 0..3
inline void perm_table(uint8_t c, uint32_t t[5]) {
    const Field& F = field();
    uint8_t b0[8], b1[8], b2[4];
    for (int b = 0; b < 8; ++b) {
        b0[b] = F.mul(c, (uint8_t)b);
        b1[b] = F.mul(c, (uint8_t)(b << 3));
    }
    for (int b = 0; b < 4; ++b) b2[b] = F.mul(c, (uint8_t)(b << 6));
    auto pack = [](const uint8_t* p) {
        return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    };
    t[0] = pack(b0);
    t[1] = pack(b0 + 4);
    t[2] = pack(b1);
    t[3] = pack(b1 + 4);
    t[4] = pack(b2);
}

}  // namespace hbec
