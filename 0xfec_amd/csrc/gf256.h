// gf256.h — GF(2^8) arithmetic for the MI355X FEC engine (host + device).
//
// Field: x^8+x^4+x^3+x^2+1 (0x11D), generator 2 — the field of
// github.com/klauspost/reedsolomon v1.12.4, which the reference calls from
// internal/fec/reed_solomon.go:16,51,124.
//
// Device multiply-by-constant uses three v_perm_b32 byte lookups per packed dword
// (see PermTab below): a coefficient c becomes five dwords of 8/8/4-entry product
// tables, and c*x for four packed bytes x is
//     perm(T0, x & 7) ^ perm(T1, (x >> 3) & 7) ^ perm(T2, (x >> 6) & 3)
// which is exact because x -> c*x is linear over GF(2).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define GF_HD __host__ __device__
#else
#define GF_HD
#endif

namespace gf {

struct alignas(16) Tables {   // aligned: kernels stage exp | log into LDS as dwords
    uint8_t exp[512];
    uint8_t log[256];
};

constexpr Tables make_tables() {
    Tables t{};
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
        t.exp[i] = (uint8_t)x;
        t.exp[i + 255] = (uint8_t)x;
        t.log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    t.exp[510] = t.exp[0];
    t.exp[511] = t.exp[1];
    return t;
}

inline constexpr Tables kTables = make_tables();

// Multiply without tables (russian peasant). Usable anywhere, constexpr.
GF_HD constexpr inline uint8_t mul_slow(uint8_t a, uint8_t b) {
    unsigned r = 0, x = a;
    for (int i = 0; i < 8; ++i) {
        if (b & (1u << i)) r ^= x;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    return (uint8_t)r;
}

inline uint8_t mul(uint8_t a, uint8_t b) {
    if (a == 0 || b == 0) return 0;
    return kTables.exp[kTables.log[a] + kTables.log[b]];
}

inline uint8_t inv(uint8_t a) {  // a != 0
    return kTables.exp[255 - kTables.log[a]];
}

// klauspost galExp: n == 0 -> 1 (also for a == 0), a == 0 -> 0.
inline uint8_t exp_pow(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return kTables.exp[((int)kTables.log[a] * n) % 255];
}

// Five-dword v_perm product table for one coefficient, padded to 8 dwords so a
// lane can fetch it with one ds_read_b128 + one ds_read_b32 from LDS.
struct alignas(16) PermTab {
    uint32_t t0lo, t0hi;  // c * {0..7}
    uint32_t t1lo, t1hi;  // c * {0, 8, 16, .., 56}
    uint32_t t2;          // c * {0, 64, 128, 192}
    uint32_t pad0, pad1, pad2;
};
static_assert(sizeof(PermTab) == 32, "PermTab must be 32 bytes");

GF_HD inline uint32_t pack4(uint8_t a, uint8_t b, uint8_t c, uint8_t d) {
    return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}

// Build the table from the 8 powers c*2^b (b = 0..7), by linearity.
GF_HD inline PermTab make_permtab(uint8_t c) {
    uint8_t p[8];
    unsigned x = c;
    for (int b = 0; b < 8; ++b) {
        p[b] = (uint8_t)x;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    uint8_t t0[8], t1[8], t2[4];
    for (int i = 0; i < 8; ++i) {
        t0[i] = (uint8_t)(((i & 1) ? p[0] : 0) ^ ((i & 2) ? p[1] : 0) ^ ((i & 4) ? p[2] : 0));
        t1[i] = (uint8_t)(((i & 1) ? p[3] : 0) ^ ((i & 2) ? p[4] : 0) ^ ((i & 4) ? p[5] : 0));
    }
    for (int i = 0; i < 4; ++i) t2[i] = (uint8_t)(((i & 1) ? p[6] : 0) ^ ((i & 2) ? p[7] : 0));
    PermTab t{};
    t.t0lo = pack4(t0[0], t0[1], t0[2], t0[3]);
    t.t0hi = pack4(t0[4], t0[5], t0[6], t0[7]);
    t.t1lo = pack4(t1[0], t1[1], t1[2], t1[3]);
    t.t1hi = pack4(t1[4], t1[5], t1[6], t1[7]);
    t.t2 = pack4(t2[0], t2[1], t2[2], t2[3]);
    return t;
}

// v_perm_b32: byte i of the result is byte sel_i of {s0 (bytes 4-7), s1 (bytes 0-3)}, 0x0c -> 0x00
// (the selector values this file uses). Host restatement for the self-test.
GF_HD inline uint32_t perm_b32(uint32_t s0, uint32_t s1, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(s0, s1, sel);
#else
    const uint64_t v = ((uint64_t)s0 << 32) | s1;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t b = (sel >> (8 * i)) & 0xFFu;
        r |= (b < 8 ? (uint32_t)((v >> (8 * b)) & 0xFFu) : 0u) << (8 * i);
    }
    return r;
#endif
}

// make_permtab in 32-bit lane arithmetic (the rebuild kernels expand coefficient rows with it):
// the doubling chain p_b = c * 2^b (3 ops a step), packed into q = p0..p3 and r = p4..p7, then
// each table from two byte permutes and XORs. ~40 VALU against ~75 for the byte-wise form.
GF_HD inline PermTab make_permtab_fast(uint32_t c) {
    // x * 2 for x < 256: bit 7 sign-extended (v_bfe_i32) selects the reduction, one 3-input op
    auto dbl = [](uint32_t x) -> uint32_t { return (x << 1) ^ ((uint32_t)((int32_t)(x << 24) >> 31) & 0x11Du); };
    const uint32_t p0 = c & 0xFFu, p1 = dbl(p0), p2 = dbl(p1), p3 = dbl(p2);
    const uint32_t p4 = dbl(p3), p5 = dbl(p4), p6 = dbl(p5), p7 = dbl(p6);
    const uint32_t q = p0 | (p1 << 8) | (p2 << 16) | (p3 << 24);
    const uint32_t r = p4 | (p5 << 8) | (p6 << 16) | (p7 << 24);
    PermTab t{};
    t.t0lo = perm_b32(q, q, 0x0001000cu) ^ perm_b32(q, q, 0x010c0c0cu);   // 0, p0, p1, p0^p1
    t.t0hi = t.t0lo ^ perm_b32(q, q, 0x02020202u);                         // ^ p2
    t.t1lo = perm_b32(r, q, 0x0304030cu) ^ perm_b32(r, q, 0x040c0c0cu);   // 0, p3, p4, p3^p4
    t.t1hi = t.t1lo ^ perm_b32(r, q, 0x05050505u);                         // ^ p5
    t.t2 = perm_b32(r, q, 0x0607060cu) ^ perm_b32(r, q, 0x070c0c0cu);     // 0, p6, p7, p6^p7
    return t;
}

}  // namespace gf
