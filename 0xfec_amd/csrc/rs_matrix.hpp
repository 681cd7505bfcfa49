// rs_matrix.hpp — host-side construction of the systematic Reed-Solomon matrix.
//
// Produces the same matrix as github.com/klauspost/reedsolomon v1.12.4 `New(k, m)` with
// default options (reference call site internal/fec/reed_solomon.go:16, manager.go:60,83):
//   vandermonde(n, k)[r][c] = r^c   (galExp semantics: 0^0 = 1)
//   M = vandermonde * inverse(top k x k of vandermonde)
// Any k rows of M are linearly independent (row-equivalent to a Vandermonde matrix with
// distinct evaluation points), which the reconstruct plan relies on.
#pragma once

#include <stdint.h>

#include <vector>

#include "gf256.h"

namespace rs {

// Invert an n x n matrix in place (row-major). Returns false if singular.
inline bool invert(int n, uint8_t* m) {
    const int w = 2 * n;
    std::vector<uint8_t> a((size_t)n * w, 0);
    for (int r = 0; r < n; ++r) {
        for (int c = 0; c < n; ++c) a[(size_t)r * w + c] = m[(size_t)r * n + c];
        a[(size_t)r * w + n + r] = 1;
    }
    for (int col = 0; col < n; ++col) {
        int piv = -1;
        for (int r = col; r < n; ++r)
            if (a[(size_t)r * w + col]) { piv = r; break; }
        if (piv < 0) return false;
        if (piv != col)
            for (int c = 0; c < w; ++c) std::swap(a[(size_t)piv * w + c], a[(size_t)col * w + c]);
        const uint8_t s = gf::inv(a[(size_t)col * w + col]);
        for (int c = 0; c < w; ++c) a[(size_t)col * w + c] = gf::mul(s, a[(size_t)col * w + c]);
        for (int r = 0; r < n; ++r) {
            if (r == col) continue;
            const uint8_t f = a[(size_t)r * w + col];
            if (!f) continue;
            for (int c = 0; c < w; ++c) a[(size_t)r * w + c] ^= gf::mul(f, a[(size_t)col * w + c]);
        }
    }
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) m[(size_t)r * n + c] = a[(size_t)r * w + n + c];
    return true;
}

// n x k systematic encoding matrix, row-major. Empty on failure.
inline std::vector<uint8_t> build_matrix(int k, int n) {
    std::vector<uint8_t> out;
    if (k <= 0 || n < k || n > 256) return out;
    std::vector<uint8_t> vm((size_t)n * k), top((size_t)k * k);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) vm[(size_t)r * k + c] = gf::exp_pow((uint8_t)r, c);
    for (size_t i = 0; i < top.size(); ++i) top[i] = vm[i];
    if (!invert(k, top.data())) return out;
    out.assign((size_t)n * k, 0);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int t = 0; t < k; ++t) acc ^= gf::mul(vm[(size_t)r * k + t], top[(size_t)t * k + c]);
            out[(size_t)r * k + c] = acc;
        }
    return out;
}

}  // namespace rs
