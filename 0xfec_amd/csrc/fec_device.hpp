// fec_device.hpp — device-side helpers shared by the gfx950 FEC kernels (fec_encode.hip,
// fec_decode.hip, fec_xor.hip): 16-byte streaming loads/stores, the v_perm GF(2^8) product
// (gf256.h PermTab), the three-input XOR, XCD-contiguous workgroup order.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>

#include "fec_kernels.hpp"
#include "gf256.h"

namespace fk {

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    const uint32_t t = __umulhi(n, f.magic);
    return (uint32_t)(((uint64_t)t + n) >> f.shift);
}

// Workgroup index in XCD-contiguous order. Dispatch deals workgroups round-robin over the 8
// XCDs (MI355X_MICROARCH.md, workgroup dispatch); here the workgroups one XCD receives take one
// contiguous eighth of the grid, so each XCD streams its own contiguous address range (speed
// only: any bijection is correct; DESIGN.md 3: +5-9 % encode, +2-3.5 % decode). Workgroups past
// the last multiple of 8 keep their index.
__device__ __forceinline__ uint32_t xcd_order_of(uint32_t wg, uint32_t G) {
    const uint32_t full = G & ~7u;
    if (wg >= full) return wg;
    return (wg & 7u) * (full >> 3) + (wg >> 3);
}
__device__ __forceinline__ uint32_t xcd_order() { return xcd_order_of(blockIdx.x, gridDim.x); }

struct Idx {
    uint32_t a, b, c;
};

__device__ __forceinline__ Idx split(uint32_t x) {
    return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// c * x for four packed bytes, c given by its PermTab words.
__device__ __forceinline__ uint32_t gmul(const Idx& i, uint32_t t0lo, uint32_t t0hi, uint32_t t1lo,
                                         uint32_t t1hi, uint32_t t2) {
    return __builtin_amdgcn_perm(t0hi, t0lo, i.a) ^ __builtin_amdgcn_perm(t1hi, t1lo, i.b) ^
           __builtin_amdgcn_perm(t2, t2, i.c);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    if constexpr (NT) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *reinterpret_cast<const uint4*>(p);
    }
}

template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, const uint4& v) {
    if constexpr (NT) {
        const u32x4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
    } else {
        *reinterpret_cast<uint4*>(p) = v;
    }
}

// 16-byte store with cache policy SP (measurement knob st_pol): 0 nt (st16<true>), 1 sc1, 2 sc0 sc1,
// 3 nt sc1. sc1 / sc0 sc1 stores drop the line from the XCD's L2 (MI355X_MICROARCH.md, stores of
// each flavour). The asm stores are not in the compiler's wait counts, which no kernel here needs:
// nothing reads what a kernel stores before the kernel ends.
template <int SP>
__device__ __forceinline__ void st16p(uint8_t* p, const uint4& v) {
    if constexpr (SP == 0) {
        st16<true>(p, v);
    } else {
        const u32x4 w = {v.x, v.y, v.z, v.w};
        if constexpr (SP == 1)
            asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 0" ::"v"(p), "v"(w) : "memory");
        else if constexpr (SP == 2)
            asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 0" ::"v"(p), "v"(w) : "memory");
        else
            asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 0" ::"v"(p), "v"(w) : "memory");
    }
}

__device__ __forceinline__ uint32_t word_of(const uint4& v, int d) {
    return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

// Keep only the first nb bytes of v (zero the rest).
__device__ __forceinline__ uint4 keep_bytes(const uint4& v, uint32_t nb) {
    auto m = [nb](int d) -> uint32_t {
        const int rem = (int)nb - 4 * d;
        return rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * rem));
    };
    return make_uint4(v.x & m(0), v.y & m(1), v.z & m(2), v.w & m(3));
}

// Store one output chunk holding nb valid bytes. A partial tail chunk is one full 16-byte store
// with the bytes past nb zeroed: the slot padding up to the 16-byte boundary is written as zeros
// ("Whole-chunk outputs"), which avoids partially written cache lines (+3-4 %
// encode, +1 % decode against byte-exact partial stores).
template <bool NT>
__device__ __forceinline__ void store_chunk(uint8_t* p, const uint4& v, uint32_t nb) {
    st16<NT>(p, nb >= 16 ? v : keep_bytes(v, nb));
}

// a ^ b ^ c in one VALU op. gfx950 has no v_xor3_b32; v_bitop3_b32 with truth table 0x96 is
// the three-input XOR. As inline asm it also pins the accumulation order: left to the compiler,
// long XOR chains are reassociated into trees that keep every product live at once.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// The three v_perm products of c * x (x one packed dword, c by its PermTab words).
struct Prod3 {
    uint32_t p0, p1, p2;
};
__device__ __forceinline__ Prod3 gprod(const Idx& i, const uint4& lo, uint32_t t2) {
    return {__builtin_amdgcn_perm(lo.y, lo.x, i.a), __builtin_amdgcn_perm(lo.w, lo.z, i.b),
            __builtin_amdgcn_perm(t2, t2, i.c)};
}

// acc ^= c_a * x_a ^ c_b * x_b for one 16-byte chunk of two inputs: six v_perm products per
// dword folded with three 3-input XORs.
__device__ __forceinline__ void mac2(uint32_t (&acc)[4], const Idx (&ia)[4], const Idx (&ib)[4],
                                     const gf::PermTab* ta, const gf::PermTab* tb) {
    const uint4 la = *reinterpret_cast<const uint4*>(ta);
    const uint4 lb = *reinterpret_cast<const uint4*>(tb);
    const uint32_t a2 = ta->t2, b2 = tb->t2;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const Prod3 p = gprod(ia[d], la, a2);
        const Prod3 q = gprod(ib[d], lb, b2);
        acc[d] = xor3(xor3(xor3(acc[d], p.p0, p.p1), p.p2, q.p0), q.p1, q.p2);
    }
}

// acc ^= c * x for one 16-byte chunk of one input.
__device__ __forceinline__ void mac1(uint32_t (&acc)[4], const Idx (&ia)[4], const gf::PermTab* ta) {
    const uint4 la = *reinterpret_cast<const uint4*>(ta);
    const uint32_t a2 = ta->t2;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const Prod3 p = gprod(ia[d], la, a2);
        acc[d] = xor3(acc[d], p.p0, p.p1) ^ p.p2;
    }
}

__device__ __forceinline__ void split4(Idx (&ix)[4], const uint4& x) {
    ix[0] = split(x.x);
    ix[1] = split(x.y);
    ix[2] = split(x.z);
    ix[3] = split(x.w);
}

// err |= bit from the lanes that reach this point together, as one atomic per wave: the library
// is built without the compiler's atomic combining (_build.py), and per-lane atomics on one
// address serialise at L2 (XOR(2,1) with U{1..2} losses, half the blocks failing: 5.97 ms with an
// atomic per failing block, 0.48 ms with one per wave; profiles/r05/xor_ab_r05g.log).
__device__ __forceinline__ void wave_flag(int* err, int bit) {
    const uint64_t act = __ballot(1);
    if (__lane_id() == (uint32_t)__ffsll((unsigned long long)act) - 1) atomicOr(err, bit);
}

// The wave's <= 3 block masks (blocks bfirst, +1, +2, clamped to the batch; a wave of 64 items
// spans at most 3 blocks when cps >= 32) by scalar loads: wave-uniform addresses through the
// constant cache, which the scalar unit turns into shard addresses while the vector memory path is
// free (a vector load of the masks puts a dependent vector round trip in front of the shard loads).
struct WaveMasks {
    uint32_t m0, m1, m2;
    __device__ __forceinline__ uint32_t of(uint32_t g) const { return g == 0 ? m0 : g == 1 ? m1 : m2; }
};
__device__ __forceinline__ WaveMasks wave_masks(const uint32_t* masks, uint32_t bfirst, uint32_t nblocks) {
    typedef __attribute__((address_space(4))) const uint32_t ConstU32;
    ConstU32* cm = (ConstU32*)masks;
    const uint32_t bf = (uint32_t)__builtin_amdgcn_readfirstlane((int)bfirst), last = nblocks - 1;
    return {cm[bf], cm[(uint32_t)__builtin_amdgcn_readfirstlane((int)min(bf + 1, last))],
            cm[(uint32_t)__builtin_amdgcn_readfirstlane((int)min(bf + 2, last))]};
}

__device__ __forceinline__ uint4 as_uint4(const uint32_t (&v)[4]) { return make_uint4(v[0], v[1], v[2], v[3]); }

}  // namespace fk
