// fec_kernels.hip — gfx950 (MI355X, CDNA4) kernels for block FEC.
//
// Hot path of ddritzenhoff/0xFEC internal/fec (reed_solomon.go:51 Encode, :124
// ReconstructData; xor.go:28-33, :80-86), rebuilt for CDNA4:
//   * byte-wise GF(2^8) work on packed dwords with v_perm_b32 product tables
//     (three lookups per dword per coefficient; no MFMA — this is not a contraction)
//   * every lane owns one 16-byte column chunk of a block and streams the k input
//     shards of that chunk with global_load_dwordx4 (a wave covers 1 KiB contiguous
//     per input shard), accumulating all outputs in VGPRs, so each input byte is read
//     from HBM exactly once and each output byte written once
//   * coefficient tables sit in LDS and are read wave-uniform (broadcast)
//   * decode solves only the e x e system of the erased data shards per block
//     (rs_plan_kernel), which is the same linear solution klauspost computes from the
//     full k x k inverse of the first k present rows.
// Grid shapes, non-temporal access and tail-store form were chosen by measurement
// (tools/kbench.py; DESIGN.md "Kernel tuning").
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fec_kernels.hpp"
#include "gf256.h"

namespace fk {

Tuning g_tune;

FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{d, 0, 0};
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.shift = l;
    f.magic = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    return f;
}

PlanLayout plan_layout(uint32_t k, uint32_t maxe) {
    PlanLayout l;
    l.in_off = 0;
    l.out_off = (k + 7) & ~7u;                       // in slots, read 8 at a time
    l.nout_off = l.out_off + maxe;
    l.coef_off = (l.nout_off + 1 + 3) & ~3u;
    l.stride = (l.coef_off + maxe * k + 15) & ~15u;
    return l;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    const uint32_t t = __umulhi(n, f.magic);
    return (uint32_t)(((uint64_t)t + n) >> f.shift);
}

// Item order inside a block: the first `rot` items take the last `rot` chunks of the shard,
// so a shard's tail and the next shard's head — which share a 128-byte line when the shard
// stride is an odd multiple of 64 (1216 = 9.5 lines) — are loaded by neighbouring lanes of
// one wave on consecutive instructions, and the line is fetched from HBM once.
__device__ __forceinline__ uint32_t rotate_chunk(uint32_t c, uint32_t cps, uint32_t rot) {
    return c < rot ? c + (cps - rot) : c - rot;
}

// Workgroup index in XCD-contiguous order. Dispatch deals workgroups round-robin over the 8
// XCDs (MI355X_MICROARCH.md, workgroup dispatch); with swz the workgroups one XCD receives take
// one contiguous eighth of the grid, so each XCD streams its own contiguous address range
// (speed only: any bijection is correct). Workgroups past the last multiple of 8 keep their index.
__device__ __forceinline__ uint32_t xcd_order(uint32_t swz) {
    const uint32_t wg = blockIdx.x, G = gridDim.x;
    if (!swz) return wg;
    const uint32_t full = G & ~7u;
    if (wg >= full) return wg;
    return (wg & 7u) * (full >> 3) + (wg >> 3);
}

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

__device__ __forceinline__ uint32_t word_of(const uint4& v, int d) {
    return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

// Store the first nb (< 16) bytes of v, byte-exact.
__device__ __forceinline__ void st_partial(uint8_t* p, const uint4& v, uint32_t nb) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t w = word_of(v, d);
        if (4u * d + 4u <= nb) {
            *reinterpret_cast<uint32_t*>(p + 4 * d) = w;
        } else if (4u * d < nb) {
            const uint32_t rem = nb - 4u * d;
            if (rem >= 2) *reinterpret_cast<uint16_t*>(p + 4 * d) = (uint16_t)w;
            if (rem & 1) p[4 * d + (rem & 2)] = (uint8_t)(w >> (8 * (rem & 2)));
        }
    }
}

// Keep only the first nb bytes of v (zero the rest).
__device__ __forceinline__ uint4 keep_bytes(const uint4& v, uint32_t nb) {
    auto m = [nb](int d) -> uint32_t {
        const int rem = (int)nb - 4 * d;
        return rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * rem));
    };
    return make_uint4(v.x & m(0), v.y & m(1), v.z & m(2), v.w & m(3));
}

// Store one output chunk holding nb valid bytes. A partial tail chunk is either one full
// 16-byte store with the bytes past nb zeroed (pad_zero: the slot padding up to the 16-byte
// boundary is written as zeros, which avoids partially written cache lines) or a byte-exact
// partial store.
template <bool NT>
__device__ __forceinline__ void store_chunk(uint8_t* p, const uint4& v, uint32_t nb, uint32_t pad_zero) {
    if (nb >= 16)
        st16<NT>(p, v);
    else if (pad_zero)
        st16<NT>(p, keep_bytes(v, nb));
    else
        st_partial(p, v, nb);
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

__device__ __forceinline__ uint4 as_uint4(const uint32_t (&v)[4]) { return make_uint4(v[0], v[1], v[2], v[3]); }

// ------------------------------------------------------------------ RS encode
// One lane = one 16-byte column chunk of one block; all m parities accumulate in VGPRs.
// Inputs are loaded 8 shards at a time (clamped, so loads are never predicated), then
// each input updates every parity accumulator with its LDS-broadcast PermTab.
// POL: bit 0 non-temporal loads, bit 1 non-temporal stores.
template <int MAXM, bool LDS_TABS, int POL>
__global__ __launch_bounds__(kThreads) void rs_encode_kernel(EncodeArgs a) {
    constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const gf::PermTab* tabs;
    if constexpr (LDS_TABS) {
        uint32_t* dst = reinterpret_cast<uint32_t*>(smem);
        const uint32_t nw = a.m * a.k * 8;
        for (uint32_t i = threadIdx.x; i < nw; i += kThreads) dst[i] = a.tabs[i];
        __syncthreads();
        tabs = reinterpret_cast<const gf::PermTab*>(smem);
    } else {
        tabs = reinterpret_cast<const gf::PermTab*>(a.tabs);
    }
    const uint32_t k = a.k, m = a.m;
    const uint32_t stride = gridDim.x * kThreads;
    for (uint32_t item = xcd_order(a.swz) * kThreads + threadIdx.x; item < a.total; item += stride) {
        const uint32_t b = fdiv(item, a.div_cps);
        const uint32_t c = rotate_chunk(item - b * a.cps, a.cps, a.rot);
        const uint8_t* src = a.in + (uint64_t)b * a.in_bs + (uint64_t)c * kChunk;
        uint32_t acc[MAXM][4];
#pragma unroll
        for (int r = 0; r < MAXM; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0;
        for (uint32_t j0 = 0; j0 < k; j0 += kInGroup) {
            uint4 x[kInGroup];
#pragma unroll
            for (int jj = 0; jj < kInGroup; ++jj)   // uniform predicate: no loads past shard k-1
                x[jj] = j0 + jj < k ? ld16<NTL>(src + (uint64_t)(j0 + jj) * a.ss) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int jj = 0; jj < kInGroup; jj += 2) {
                const uint32_t j = j0 + jj;
                if (j + 1 < k) {
                    Idx ia[4], ib[4];
                    split4(ia, x[jj]);
                    split4(ib, x[jj + 1]);
#pragma unroll
                    for (int r = 0; r < MAXM; ++r)
                        if (r < (int)m) mac2(acc[r], ia, ib, tabs + r * k + j, tabs + r * k + j + 1);
                } else if (j < k) {
                    Idx ia[4];
                    split4(ia, x[jj]);
#pragma unroll
                    for (int r = 0; r < MAXM; ++r)
                        if (r < (int)m) mac1(acc[r], ia, tabs + r * k + j);
                }
            }
        }
        uint8_t* dst = a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk;
        const uint32_t nb = a.len - c * kChunk;
#pragma unroll
        for (int r = 0; r < MAXM; ++r)
            if (r < (int)m) store_chunk<NTS>(dst + (uint64_t)r * a.ss, as_uint4(acc[r]), nb, a.pad_zero);
    }
}

// ------------------------------------------------------------------ dyadic encode
// For k = 2^a and m = 2^b (m <= k) klauspost's systematic matrix is dyadic: parity row i,
// column j holds g(i ^ j) with g = parity row 0. (Its rows are the Lagrange basis on the
// additive subgroup {0..k-1} of GF(2^8) evaluated at k ^ i; the subgroup's vanishing polynomial
// is GF(2)-linear, so L_j(k ^ i) = W(k) / (K (k ^ i ^ j)) depends on i ^ j only.) With
// j = h*m + v (v < m): parity_i = sum_h conv(G_h, D_h)[i], conv(C, D)[i] = sum_v C[v ^ i] D[v],
// a convolution over the group Z_2^b. Split on the top index bit, with P = conv(C0, D0),
// Q = conv(C1, D1), R = conv(C0 ^ C1, D0 ^ D1) over half the size:
//   conv(C, D) = (P ^ Q, R ^ P ^ Q)
// (field arithmetic is exact, so this is the same bytes as the matrix product). Recursing, a
// group costs 3^b field products instead of 4^b: RS(8,12) 18 instead of 32, RS(16,24) 54
// instead of 128. Products are linear in the data, so the split of D0 ^ D1 is the XOR of the
// splits (3 ops, not 5). Leaf constants (C0 ^ C1 combinations) come from the host in the
// recursion's order: P's leaves, Q's, R's (dyadic_leaf_tables()).
template <int B>
struct Pow3 {
    static constexpr int v = 3 * Pow3<B - 1>::v;
};
template <>
struct Pow3<0> {
    static constexpr int v = 1;
};

template <int NC>
__device__ __forceinline__ void dy_leaf(const Idx (&d)[NC], const gf::PermTab* t, uint32_t (&y)[NC]) {
    const uint4 lo = *reinterpret_cast<const uint4*>(t);
    const uint32_t t2 = t->t2;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const Prod3 p = gprod(d[c], lo, t2);
        y[c] = xor3(p.p0, p.p1, p.p2);
    }
}

// Y[i] = sum_l C[l ^ i] * D[l], i, l < 2^B, for NC dword columns; C by its leaf tables T.
template <int B, int NC>
__device__ __forceinline__ void dy_conv(const Idx (*D)[NC], const gf::PermTab* T, uint32_t (*Y)[NC]) {
    if constexpr (B == 0) {
        dy_leaf<NC>(D[0], T, Y[0]);
    } else {
        constexpr int H = 1 << (B - 1), L = Pow3<B - 1>::v;
        uint32_t P[H][NC], R[H][NC];
        dy_conv<B - 1, NC>(D, T, P);
        dy_conv<B - 1, NC>(D + H, T + L, Y);   // Q, in the low half of Y
        {
            Idx S[H][NC];
#pragma unroll
            for (int i = 0; i < H; ++i)
#pragma unroll
                for (int c = 0; c < NC; ++c)
                    S[i][c] = {D[i][c].a ^ D[i + H][c].a, D[i][c].b ^ D[i + H][c].b, D[i][c].c ^ D[i + H][c].c};
            dy_conv<B - 1, NC>(S, T + 2 * L, R);
        }
#pragma unroll
        for (int i = 0; i < H; ++i)
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const uint32_t q = Y[i][c];
                Y[i][c] = P[i][c] ^ q;
                Y[i + H][c] = xor3(R[i][c], P[i][c], q);
            }
    }
}

// ------------------------------------------------------------------ RS encode, fixed shape
// The code shapes the reference benchmarks, with K and M compile-time: one lane = one 16-byte
// column chunk, the K loads issued back to back, inputs folded in pairs (mac2), no runtime
// guards. Tail chunks are stored whole with the pad bytes zeroed.
template <int K, int M, int POL>
struct FixedEncode {
    static constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    const EncodeArgs& a;
    const gf::PermTab* T;

    __device__ __forceinline__ void load(uint4 (&x)[K], uint32_t it) const {
        const uint32_t b = fdiv(it, a.div_cps);
        const uint32_t c = it - b * a.cps;
        const uint8_t* src = a.in + (uint64_t)b * a.in_bs + (uint64_t)c * kChunk;
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = ld16<NTL>(src + (uint64_t)j * a.ss);
    }

    __device__ __forceinline__ void compute_store(const uint4 (&x)[K], uint32_t it) const {
        // opaque zero: keeps the table reads next to their use (hoisted out of a loop they
        // would hold 5*M*K VGPRs)
        uint32_t toff = 0;
        asm volatile("" : "+s"(toff));
        const gf::PermTab* t = T + toff;
        uint32_t acc[M][4];
#pragma unroll
        for (int r = 0; r < M; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0;
        if constexpr ((POL & 4) != 0) {   // diagnostics (knob enc_diag): traffic only, no field math
#pragma unroll
            for (int j = 0; j < K; ++j)
#pragma unroll
                for (int d = 0; d < 4; ++d) acc[j % M][d] ^= word_of(x[j], d);
        } else if constexpr ((POL & 8) != 0) {   // dyadic code: T holds the leaf tables
            constexpr int B = M == 1 ? 0 : M == 2 ? 1 : M == 4 ? 2 : M == 8 ? 3 : 4;
            constexpr int L = Pow3<B>::v;
            constexpr int NC = K >= 16 ? 1 : 4;   // dword columns per pass (registers)
#pragma unroll
            for (int c0 = 0; c0 < 4; c0 += NC) {
                // opaque zero per pass: the table reads stay in their pass (shared across
                // passes they would be hoisted and held: 5 VGPRs per leaf)
                uint32_t poff = 0;
                asm volatile("" : "+s"(poff));
                const gf::PermTab* tp = t + poff;
#pragma unroll
                for (int h = 0; h < K / M; ++h) {
                    Idx D[M][NC];
#pragma unroll
                    for (int v = 0; v < M; ++v)
#pragma unroll
                        for (int c = 0; c < NC; ++c) D[v][c] = split(word_of(x[h * M + v], c0 + c));
                    uint32_t Y[M][NC];
                    dy_conv<B, NC>(D, tp + h * L, Y);
#pragma unroll
                    for (int i = 0; i < M; ++i)
#pragma unroll
                        for (int c = 0; c < NC; ++c) acc[i][c0 + c] = h ? acc[i][c0 + c] ^ Y[i][c] : Y[i][c];
                }
            }
        } else
#pragma unroll
        for (int j = 0; j < K; j += 2) {
            Idx ia[4], ib[4];
            split4(ia, x[j]);
            if (j + 1 < K) split4(ib, x[j + 1 < K ? j + 1 : j]);
#pragma unroll
            for (int r = 0; r < M; ++r) {
                if (j + 1 < K) mac2(acc[r], ia, ib, t + r * K + j, t + r * K + j + 1);
                else mac1(acc[r], ia, t + r * K + j);
            }
        }
        const uint32_t b = fdiv(it, a.div_cps);
        const uint32_t c = it - b * a.cps;
        uint8_t* dst = a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk;
        const uint32_t nb = min(a.len - c * kChunk, (uint32_t)kChunk);
#pragma unroll
        for (int r = 0; r < M; ++r) st16<NTS>(dst + (uint64_t)r * a.ss, keep_bytes(as_uint4(acc[r]), nb));
    }
};

template <int K, int M>
__device__ __forceinline__ const gf::PermTab* stage_tabs(uint8_t* smem, const uint32_t* tabs) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(smem);
    for (uint32_t i = threadIdx.x; i < (uint32_t)(M * K * 8); i += kThreads) dst[i] = tabs[i];
    __syncthreads();
    return reinterpret_cast<const gf::PermTab*>(smem);
}

// Flat launch: one item per lane, XCD-contiguous workgroup order.
template <int K, int M, int POL>
__global__ __launch_bounds__(kThreads) void rs_encode_fixed_kernel(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const FixedEncode<K, M, POL> f{a, stage_tabs<K, M>(smem, a.tabs)};
    const uint32_t it = xcd_order(a.swz) * kThreads + threadIdx.x;
    if (it >= a.total) return;
    uint4 x[K];
    f.load(x, it);
    f.compute_store(x, it);
}

// Persistent ticket-queue launch (the default for the fixed shapes). The items are split into
// 8 contiguous ranges; the workgroups with blockIdx % 8 == x own range x (the grid is a multiple
// of 8, so every range has owners: correctness never depends on placement) and draw 256-item
// chunks of it in order from ticket counter x. Round-robin dispatch puts those workgroups on one
// XCD, so each XCD streams one compact window of addresses: measured as fast as a flat grid for
// pure traffic, where a static persistent sweep lets the windows drift apart and loses ~20 %
// (tools/mix_probe.py persist). Each lane loads its next chunk's K inputs and draws the ticket
// after it before it computes and stores the current chunk (ping-pong register sets), so two
// resident workgroups per CU keep HBM busy while the field arithmetic runs.
template <int K, int M, int POL, int D>
__global__ __launch_bounds__(kThreads) void rs_encode_queue_kernel(EncodeArgs a) {
    static_assert(D == 1 || D == 2, "prefetch depth");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // tk[2..2+D]: the first D+1 tickets (never rewritten); tk[t & 1]: the ticket drawn in stage
    // t, read after that stage's barrier and rewritten two stages later, after a barrier every
    // reader has passed
    __shared__ uint32_t tk[2 + D + 1];
    uint32_t* ctr = a.ctr + (blockIdx.x & 7u) * kCtrStride;
    if (threadIdx.x == 0)
        for (int i = 0; i <= D; ++i) tk[2 + i] = atomicAdd(ctr, 1u);
    const FixedEncode<K, M, POL> f{a, stage_tabs<K, M>(smem, a.tabs)};   // barrier inside
    const uint32_t lo = (blockIdx.x & 7u) * a.per_xcd;
    const uint32_t hi = min(a.total, lo + a.per_xcd);
    // chunk bases in flight (uniform over the workgroup): q[0] is computed, q[D] is loaded next
    uint32_t q[D + 1];
#pragma unroll
    for (int i = 0; i <= D; ++i) q[i] = lo + tk[2 + i] * kThreads;
    const uint32_t last = hi - 1;           // loads clamp to the range's last item
    const uint32_t lane = threadIdx.x;
    uint4 xs[D + 1][K];
    // one stage: draw the ticket D+1 chunks ahead, issue the loads of chunk q[D], compute and
    // store chunk q[0], publish the ticket. The barrier waits for LDS only (HIP's __syncthreads
    // would also drain vmcnt, i.e. wait for the prefetched loads).
    auto stage = [&](uint4 (&now)[K], uint4 (&fill)[K], uint32_t slot) {
        uint32_t drawn = 0;
        if (lane == 0) drawn = atomicAdd(ctr, 1u);
        f.load(fill, min(q[D] + lane, last));   // clamped: unconditional, no merge of old values
        if (q[0] + lane < hi) f.compute_store(now, q[0] + lane);
        if (lane == 0) tk[slot] = drawn;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int i = 0; i < D; ++i) q[i] = q[i + 1];
        q[D] = lo + tk[slot] * kThreads;
    };
    if (q[0] < hi) {
#pragma unroll
        for (int i = 0; i < D; ++i) f.load(xs[i], min(q[i] + lane, last));
        if constexpr (D == 1) {
            while (q[0] < hi) {
                stage(xs[0], xs[1], 0);
                if (q[0] >= hi) break;
                stage(xs[1], xs[0], 1);
            }
        } else {
            while (q[0] < hi) {
                stage(xs[0], xs[2], 0);
                if (q[0] >= hi) break;
                stage(xs[1], xs[0], 1);
                if (q[0] >= hi) break;
                stage(xs[2], xs[1], 0);
                if (q[0] >= hi) break;
                stage(xs[0], xs[2], 1);
                if (q[0] >= hi) break;
                stage(xs[1], xs[0], 0);
                if (q[0] >= hi) break;
                stage(xs[2], xs[1], 1);
            }
        }
    }
    // The last workgroup to finish rewinds the counters for the next launch on this stream
    // (every workgroup's draws precede its arrival, released by the fence).
    if (threadIdx.x == 0) {
        __threadfence();
        uint32_t* done = a.ctr + 8 * kCtrStride;
        if (atomicAdd(done, 1u) == gridDim.x - 1) {
            for (int x = 0; x < 8; ++x) atomicExch(a.ctr + x * kCtrStride, 0u);
            atomicExch(done, 0u);
        }
    }
}

// Ticket queue without prefetch (prefetch depth 0): draw, barrier, load, compute, store.
// DRAIN: the barrier is HIP's __syncthreads, which also waits for the workgroup's stores.
template <int K, int M, int POL, bool DRAIN>
__global__ __launch_bounds__(kThreads) void rs_encode_queue0_kernel(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint32_t tk[2];
    uint32_t* ctr = a.ctr + (blockIdx.x & 7u) * kCtrStride;
    const FixedEncode<K, M, POL> f{a, stage_tabs<K, M>(smem, a.tabs)};
    const uint32_t lo = (blockIdx.x & 7u) * a.per_xcd;
    const uint32_t hi = min(a.total, lo + a.per_xcd);
    for (uint32_t t = 0;; ++t) {
        if (threadIdx.x == 0) tk[t & 1] = atomicAdd(ctr, 1u);
        if constexpr (DRAIN) __syncthreads();
        else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const uint32_t base = lo + tk[t & 1] * kThreads;
        if (base >= hi) break;
        const uint32_t it = base + threadIdx.x;
        if (it < hi) {
            uint4 x[K];
            f.load(x, it);
            f.compute_store(x, it);
        }
    }
    if (threadIdx.x == 0) {
        __threadfence();
        uint32_t* done = a.ctr + 8 * kCtrStride;
        if (atomicAdd(done, 1u) == gridDim.x - 1) {
            for (int x = 0; x < 8; ++x) atomicExch(a.ctr + x * kCtrStride, 0u);
            atomicExch(done, 0u);
        }
    }
}

// ------------------------------------------------------------------ RS reconstruct plan
// One thread per block, one wave per workgroup. From the present mask: E = erased data
// shards (e of them); the inputs are the first k present shards in index order (as in
// klauspost ReconstructData). One erasure: a single parity row solves it. Two or more: the
// coefficients come from Lagrange interpolation over the shard indices (below). Each lane
// assembles its record in LDS (byte writes), then the wave copies its 64 consecutive records
// to HBM with 16-byte stores.
constexpr int kPlanThreads = 64;

// LDS of one plan workgroup: exp/log tables, the parity rows, the records.
struct PlanLds {
    size_t prows, recs, total;
};
__host__ __device__ inline PlanLds plan_lds(uint32_t m, uint32_t k, uint32_t stride) {
    PlanLds l;
    l.prows = 768;
    l.recs = (l.prows + m * k + 15) & ~(size_t)15;
    l.total = l.recs + (size_t)kPlanThreads * stride;
    return l;
}

__global__ __launch_bounds__(kPlanThreads) void rs_plan_kernel(PlanArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const PlanLds L = plan_lds(a.m, a.k, a.lay.stride);
    uint8_t* s_exp = smem;                 // 512
    uint8_t* s_log = smem + 512;           // 256
    uint8_t* s_prows = smem + L.prows;     // m x k
    uint8_t* recs = smem + L.recs;         // kPlanThreads * stride
    for (int i = threadIdx.x; i < 512; i += kPlanThreads) s_exp[i] = gf::kTables.exp[i];
    for (int i = threadIdx.x; i < 256; i += kPlanThreads) s_log[i] = gf::kTables.log[i];
    for (uint32_t i = threadIdx.x; i < a.m * a.k; i += kPlanThreads) s_prows[i] = a.prows[i];
    __syncthreads();
    auto mul = [&](uint32_t x, uint32_t y) -> uint32_t {
        return (x && y) ? s_exp[s_log[x] + s_log[y]] : 0u;
    };
    const PlanLayout lay = a.lay;
    const uint32_t b0 = blockIdx.x * kPlanThreads;
    const uint32_t b = b0 + threadIdx.x;
    uint8_t* P = recs + threadIdx.x * lay.stride;
    const uint32_t k = a.k, m = a.m, n = k + m;
    if (b < a.nblocks) {
        const uint32_t all = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
        const uint32_t mask = a.masks[b] & all;
        const uint32_t kmask = (1u << k) - 1u;   // k <= 31
        const uint32_t e = k - __popc(mask & kmask);
        int32_t st = a.max_out ? (int32_t)e : 0;   // recover reports the rebuilt count
        if (e == 0) {
            P[lay.nout_off] = 0;
        } else if ((uint32_t)__popc(mask) < k) {
            P[lay.nout_off] = 0;
            st = -4;  // FEC_ERR_TOO_FEW_SHARDS
            atomicOr(a.err, 1);
        } else if (a.max_out && e > a.max_out) {
            P[lay.nout_off] = 0;
            st = -1;  // FEC_ERR_INVALID_ARG: more erasures than output slots
            atomicOr(a.err, 2);
        } else if (e == 1) {
            // one erasure: x_E = inv(A[R0][E0]) * (p_R0 ^ sum_j A[R0][j] x_j)
            const uint32_t E0 = __ffs(~mask & kmask) - 1;
            const uint32_t R0 = __ffs(mask >> k) - 1;
            const uint8_t* row = s_prows + R0 * k;
            const uint32_t inv = s_exp[255 - s_log[row[E0]]];
            for (uint32_t j = 0, pos = 0; j < k; ++j) {
                if (j == E0) continue;
                P[lay.in_off + pos] = (uint8_t)j;
                P[lay.coef_off + pos] = (uint8_t)mul(inv, row[j]);
                ++pos;
            }
            P[lay.in_off + k - 1] = (uint8_t)(k + R0);
            P[lay.coef_off + k - 1] = (uint8_t)inv;
            P[lay.out_off] = (uint8_t)E0;
            P[lay.nout_off] = 1;
        } else {
            // e >= 2, by Lagrange interpolation instead of inverting the e x e system. The
            // systematic matrix is M = V inv(V_top) with V[r][c] = r^c (klauspost buildMatrix),
            // so every shard is y_r = p(r) for one polynomial p of degree < k, and an erased
            // data shard is x_i = p(i) = sum over the first k present shards s of
            //   y_s * prod_{t != s} (i ^ t) / (s ^ t)
            // (nodes are the shard indices as field elements, all distinct). This is the same
            // unique solution ReconstructData computes; in the log domain it is sums of table
            // lookups with no serial dependence: k^2 + 3ek lookups per block.
            uint8_t* S = P + lay.in_off;
            uint8_t* C = P + lay.coef_off;
            uint32_t pos = 0;
            for (uint32_t idx = 0; idx < n && pos < k; ++idx)
                if ((mask >> idx) & 1u) S[pos++] = (uint8_t)idx;
            for (uint32_t i = 0, r = 0; i < k; ++i)
                if (!((mask >> i) & 1u)) P[lay.out_off + r++] = (uint8_t)i;
            // D_p = sum_{q != p} log(s_p ^ s_q) mod 255, kept in row 0 of the coefficients
            for (uint32_t p = 0; p < k; ++p) {
                const uint32_t sp = S[p];
                uint32_t d = 0;
                for (uint32_t q = 0; q < k; ++q)
                    if (q != p) d += s_log[sp ^ S[q]];
                C[p] = (uint8_t)(d % 255u);
            }
            // rows high to low: row 0 overwrites each D_p right after reading it
            for (uint32_t r = e; r-- > 0;) {
                const uint32_t i = P[lay.out_off + r];
                uint32_t nsum = 0;
                for (uint32_t q = 0; q < k; ++q) nsum += s_log[i ^ S[q]];
                for (uint32_t p = 0; p < k; ++p) {
                    const uint32_t v = nsum + 2u * 255u - s_log[i ^ S[p]] - C[p];
                    C[r * k + p] = s_exp[v % 255u];
                }
            }
            P[lay.nout_off] = (uint8_t)e;
        }
        if (a.status) a.status[b] = st;
    }
    __syncthreads();
    const uint32_t nrec = min((uint32_t)kPlanThreads, a.nblocks - b0);
    const uint32_t nw = nrec * lay.stride / 16;
    const uint4* src = reinterpret_cast<const uint4*>(recs);
    uint4* dst = reinterpret_cast<uint4*>(a.plans + (uint64_t)b0 * lay.stride);
    for (uint32_t i = threadIdx.x; i < nw; i += kPlanThreads) dst[i] = src[i];
}

// ------------------------------------------------------------------ RS reconstruct
// One (block, chunk) item: load the k input shards named by the plan record P, fold them with
// the block's PermTabs T (row r = erased shard r), store the rebuilt chunks. `rows` is
// wave-uniform (the wave's largest erasure count), so the loop bounds never diverge.
template <int MAXE, bool NTL, bool NTS>
__device__ __forceinline__ void recon_item(const ReconArgs& a, const uint8_t* P, const gf::PermTab* T,
                                           uint32_t blk, uint32_t c, uint32_t rows, uint32_t nout) {
    const uint32_t k = a.k;
    const PlanLayout& lay = a.lay;
    uint8_t* dblk = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    const uint8_t* pblk = a.parity + (uint64_t)blk * a.pbs + (uint64_t)c * kChunk;
    uint32_t acc[MAXE][4];
#pragma unroll
    for (int r = 0; r < MAXE; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0;
    for (uint32_t j0 = 0; j0 < k; j0 += kInGroup) {
        // the 8 input slots of this group, one ds_read_b64
        const uint2 sl = *reinterpret_cast<const uint2*>(P + lay.in_off + j0);
        uint4 x[kInGroup];
#pragma unroll
        for (int jj = 0; jj < kInGroup; ++jj) {
            const uint32_t w = jj < 4 ? sl.x : sl.y;
            const uint32_t slot = (w >> (8 * (jj & 3))) & 0xFFu;
            x[jj] = j0 + jj < k   // uniform predicate: no loads past input k-1
                        ? ld16<NTL>(slot < k ? dblk + (uint64_t)slot * a.ss : pblk + (uint64_t)(slot - k) * a.ss)
                        : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int jj = 0; jj < kInGroup; jj += 2) {
            const uint32_t j = j0 + jj;
            if (j + 1 < k) {
                Idx ia[4], ib[4];
                split4(ia, x[jj]);
                split4(ib, x[jj + 1]);
#pragma unroll
                for (int r = 0; r < MAXE; ++r)
                    if (r < (int)rows) mac2(acc[r], ia, ib, T + r * k + j, T + r * k + j + 1);
            } else if (j < k) {
                Idx ia[4];
                split4(ia, x[jj]);
#pragma unroll
                for (int r = 0; r < MAXE; ++r)
                    if (r < (int)rows) mac1(acc[r], ia, T + r * k + j);
            }
        }
    }
    const uint32_t nb = a.len - c * kChunk;
    const uint8_t* out_idx = P + lay.out_off;
    uint8_t* oblk = a.out ? a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk : nullptr;
#pragma unroll
    for (int r = 0; r < MAXE; ++r)
        if (r < (int)nout)
            store_chunk<NTS>(oblk ? oblk + (uint64_t)r * a.ss : dblk + (uint64_t)out_idx[r] * a.ss, as_uint4(acc[r]),
                             nb, a.pad_zero);
}

template <int MAXE>
__device__ __forceinline__ uint32_t wave_rows(uint32_t nout) {
    uint32_t rows = 0;
#pragma unroll
    for (int r = 0; r < MAXE; ++r)
        if (__any((int)nout > r)) rows = r + 1;
    return rows;
}

// Two items per lane (the lane's chunk in this wave's first and second 64-item run): both
// items' k loads are issued before either is folded, so a wave keeps twice the bytes in flight
// behind one plan stage. Items of blocks with nothing to rebuild (nout == 0) load nothing.
template <int MAXE, bool NTL, bool NTS>
__device__ __forceinline__ void recon_pair(const ReconArgs& a, const uint8_t* PA, const gf::PermTab* TA,
                                           uint32_t blkA, uint32_t cA, uint32_t rowsA, uint32_t noutA,
                                           const uint8_t* PB, const gf::PermTab* TB, uint32_t blkB, uint32_t cB,
                                           uint32_t rowsB, uint32_t noutB) {
    const uint32_t k = a.k;
    const PlanLayout& lay = a.lay;
    uint8_t* dA = a.data + (uint64_t)blkA * a.dbs + (uint64_t)cA * kChunk;
    const uint8_t* pA = a.parity + (uint64_t)blkA * a.pbs + (uint64_t)cA * kChunk;
    uint8_t* dB = a.data + (uint64_t)blkB * a.dbs + (uint64_t)cB * kChunk;
    const uint8_t* pB = a.parity + (uint64_t)blkB * a.pbs + (uint64_t)cB * kChunk;
    uint32_t accA[MAXE][4], accB[MAXE][4];
#pragma unroll
    for (int r = 0; r < MAXE; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) accA[r][q] = accB[r][q] = 0;
    for (uint32_t j0 = 0; j0 < k; j0 += kInGroup) {
        const uint2 slA = *reinterpret_cast<const uint2*>(PA + lay.in_off + j0);
        const uint2 slB = *reinterpret_cast<const uint2*>(PB + lay.in_off + j0);
        uint4 xa[kInGroup], xb[kInGroup];
#pragma unroll
        for (int jj = 0; jj < kInGroup; ++jj) {
            const uint32_t sa = ((jj < 4 ? slA.x : slA.y) >> (8 * (jj & 3))) & 0xFFu;
            const uint32_t sb = ((jj < 4 ? slB.x : slB.y) >> (8 * (jj & 3))) & 0xFFu;
            xa[jj] = j0 + jj < k && noutA
                         ? ld16<NTL>(sa < k ? dA + (uint64_t)sa * a.ss : pA + (uint64_t)(sa - k) * a.ss)
                         : make_uint4(0, 0, 0, 0);
            xb[jj] = j0 + jj < k && noutB
                         ? ld16<NTL>(sb < k ? dB + (uint64_t)sb * a.ss : pB + (uint64_t)(sb - k) * a.ss)
                         : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int jj = 0; jj < kInGroup; jj += 2) {
            const uint32_t j = j0 + jj;
            if (j + 1 < k) {
                Idx ia[4], ib[4];
                split4(ia, xa[jj]);
                split4(ib, xa[jj + 1]);
#pragma unroll
                for (int r = 0; r < MAXE; ++r)
                    if (r < (int)rowsA) mac2(accA[r], ia, ib, TA + r * k + j, TA + r * k + j + 1);
                split4(ia, xb[jj]);
                split4(ib, xb[jj + 1]);
#pragma unroll
                for (int r = 0; r < MAXE; ++r)
                    if (r < (int)rowsB) mac2(accB[r], ia, ib, TB + r * k + j, TB + r * k + j + 1);
            } else if (j < k) {
                Idx ia[4];
                split4(ia, xa[jj]);
#pragma unroll
                for (int r = 0; r < MAXE; ++r)
                    if (r < (int)rowsA) mac1(accA[r], ia, TA + r * k + j);
                split4(ia, xb[jj]);
#pragma unroll
                for (int r = 0; r < MAXE; ++r)
                    if (r < (int)rowsB) mac1(accB[r], ia, TB + r * k + j);
            }
        }
    }
    const uint8_t* oiA = PA + lay.out_off;
    const uint8_t* oiB = PB + lay.out_off;
    uint8_t* oA = a.out ? a.out + (uint64_t)blkA * a.out_bs + (uint64_t)cA * kChunk : nullptr;
    uint8_t* oB = a.out ? a.out + (uint64_t)blkB * a.out_bs + (uint64_t)cB * kChunk : nullptr;
#pragma unroll
    for (int r = 0; r < MAXE; ++r)
        if (r < (int)noutA)
            store_chunk<NTS>(oA ? oA + (uint64_t)r * a.ss : dA + (uint64_t)oiA[r] * a.ss, as_uint4(accA[r]),
                             a.len - cA * kChunk, a.pad_zero);
#pragma unroll
    for (int r = 0; r < MAXE; ++r)
        if (r < (int)noutB)
            store_chunk<NTS>(oB ? oB + (uint64_t)r * a.ss : dB + (uint64_t)oiB[r] * a.ss, as_uint4(accB[r]),
                             a.len - cB * kChunk, a.pad_zero);
}

// Tile form: a workgroup takes tiles of G consecutive blocks: it stages their plans in LDS,
// expands every coefficient to its PermTab once, then lanes sweep the G*cps (block, chunk)
// items. Rows beyond a block's own erasure count carry zero tables, and each item loops only
// to the wave's largest erasure count (ballot), so one-erasure batches do one row of work.
// Used for short shards (fewer than 32 chunks: many blocks per wave).
template <int MAXE, int POL>
__global__ __launch_bounds__(kThreads) void rs_reconstruct_kernel(ReconArgs a) {
    constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t k = a.k, G = a.g, maxe = a.maxe;
    const PlanLayout lay = a.lay;
    gf::PermTab* tabs = reinterpret_cast<gf::PermTab*>(smem);                // G*maxe*k
    uint8_t* plans = smem + (size_t)G * maxe * k * sizeof(gf::PermTab);      // G*stride
    for (uint32_t tile = xcd_order(a.swz); tile < a.ntiles; tile += gridDim.x) {
        const uint32_t b0 = tile * G;
        const uint32_t gt = min(G, a.nblocks - b0);
        __syncthreads();   // previous tile fully consumed
        {
            const uint32_t nw = gt * lay.stride / 16;
            const uint4* src = reinterpret_cast<const uint4*>(a.plans + (uint64_t)b0 * lay.stride);
            uint4* dst = reinterpret_cast<uint4*>(plans);
            for (uint32_t i = threadIdx.x; i < nw; i += kThreads) dst[i] = src[i];
        }
        __syncthreads();
        {
            const uint32_t ne = gt * maxe * k;
            for (uint32_t i = threadIdx.x; i < ne; i += kThreads) {
                const uint32_t g = i / (maxe * k);
                const uint32_t rem = i - g * maxe * k;
                const uint32_t r = rem / k, j = rem - r * k;
                const uint8_t* P = plans + g * lay.stride;
                const uint8_t c = r < P[lay.nout_off] ? P[lay.coef_off + r * k + j] : 0;
                tabs[i] = gf::make_permtab(c);
            }
        }
        __syncthreads();
        const uint32_t nitems = gt * a.cps;
        for (uint32_t base = 0; base < nitems; base += kThreads) {
            const uint32_t t = base + threadIdx.x;
            const bool inr = t < nitems;
            const uint32_t g = inr ? fdiv(t, a.div_cps) : 0;
            const uint32_t c = rotate_chunk(t - g * a.cps, a.cps, a.rot);
            const uint8_t* P = plans + g * lay.stride;
            const uint32_t nout = inr ? P[lay.nout_off] : 0;
            const uint32_t rows = wave_rows<MAXE>(nout);
            if (nout == 0) continue;
            recon_item<MAXE, NTL, NTS>(a, P, tabs + g * maxe * k, b0 + g, c, rows, nout);
        }
    }
}

// Wave form (shards of 32+ chunks, i.e. at most 3 blocks per wave): flat grid, one item per
// lane; each wave stages the plan records of its own blocks and expands only the PermTabs of
// rows those blocks rebuild, in a wave-private LDS slice, so no workgroup barrier stands
// between a wave's plan load and its data loads.
constexpr uint32_t kWaveBlocks = 3;

__host__ __device__ inline size_t wave_slice_bytes(uint32_t k, uint32_t maxe, uint32_t stride) {
    return (size_t)kWaveBlocks * maxe * k * 32 + (size_t)kWaveBlocks * stride;
}

// Fused form: the wave also builds its blocks' plan records (the work of rs_plan_kernel) from
// the present masks, lanes in parallel: slots and erased indices by prefix popcounts, one
// erasure by the single-parity-row solution, several by the Lagrange coefficients (see
// rs_plan_kernel) with the k^2 + e*k lookups spread over the 64 lanes. No plan kernel, no plan
// buffer round trip through HBM.
struct FusedLds {
    size_t prows, slices, slice;   // offsets: exp [0,512), log [512,768), prows, wave slices
};
__host__ __device__ inline size_t fused_slice_bytes(uint32_t k, uint32_t maxe, uint32_t stride) {
    return (wave_slice_bytes(k, maxe, stride) + (size_t)k + maxe + 15) & ~(size_t)15;
}
__host__ __device__ inline FusedLds fused_lds(uint32_t m, uint32_t k, uint32_t maxe, uint32_t stride) {
    FusedLds l;
    l.prows = 768;
    l.slices = (l.prows + (size_t)m * k + 15) & ~(size_t)15;
    l.slice = fused_slice_bytes(k, maxe, stride);
    return l;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int MAXE, int POL, bool FUSED, int IPL>
__global__ __launch_bounds__(kThreads) void rs_reconstruct_wave_kernel(ReconArgs a) {
    constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t k = a.k, maxe = a.maxe;
    const PlanLayout lay = a.lay;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* slice;
    const uint8_t *s_exp = nullptr, *s_log = nullptr, *s_prows = nullptr;
    if constexpr (FUSED) {
        const FusedLds L = fused_lds(a.m, k, maxe, lay.stride);
        uint8_t* e8 = smem;
        uint8_t* l8 = smem + 512;
        uint8_t* p8 = smem + L.prows;
        for (uint32_t i = threadIdx.x; i < 512; i += kThreads) e8[i] = gf::kTables.exp[i];
        for (uint32_t i = threadIdx.x; i < 256; i += kThreads) l8[i] = gf::kTables.log[i];
        for (uint32_t i = threadIdx.x; i < a.m * k; i += kThreads) p8[i] = a.prows[i];
        __syncthreads();
        s_exp = e8;
        s_log = l8;
        s_prows = p8;
        slice = smem + L.slices + (size_t)wave * L.slice;
    } else {
        slice = smem + (size_t)wave * wave_slice_bytes(k, maxe, lay.stride);
    }
    gf::PermTab* tabs = reinterpret_cast<gf::PermTab*>(slice);                      // 3*maxe*k
    uint8_t* plans = slice + (size_t)kWaveBlocks * maxe * k * sizeof(gf::PermTab);  // 3*stride
    const uint32_t total = a.nblocks * a.cps;
    constexpr uint32_t NI = IPL < 0 ? -IPL : IPL;   // items per lane; IPL < 0: one after the other
    const uint32_t i0 = (xcd_order(a.swz) * kThreads + (wave << 6)) * NI;
    if (i0 >= total) return;
    const uint32_t bfirst = fdiv(i0, a.div_cps);
    const uint32_t nb = fdiv(min(i0 + 64u * NI - 1u, total - 1u), a.div_cps) - bfirst + 1;   // <= 3
    if constexpr (!FUSED) {
        const uint32_t nw = nb * lay.stride / 16;
        const uint4* src = reinterpret_cast<const uint4*>(a.plans + (a.diag ? 0 : (uint64_t)bfirst * lay.stride));
        if (lane < nw) reinterpret_cast<uint4*>(plans)[lane] = src[lane];
    } else {
        uint8_t* Dt = plans + (size_t)kWaveBlocks * lay.stride;   // k bytes
        uint8_t* Nt = Dt + k;                                       // maxe bytes
        const uint32_t m = a.m, n = k + m;
        const uint32_t all = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
        const uint32_t kmask = (1u << k) - 1u;
        auto mul = [&](uint32_t x, uint32_t y) -> uint32_t { return (x && y) ? s_exp[s_log[x] + s_log[y]] : 0u; };
        // the wave's (<= 3) masks in one load, then broadcast
        const uint32_t mine = lane < nb ? a.masks[bfirst + lane] : 0u;
        for (uint32_t g = 0; g < nb; ++g) {
            const uint32_t b = bfirst + g;
            uint8_t* P = plans + g * lay.stride;
            const uint32_t mask = (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)g) & all;
            const uint32_t e = k - __popc(mask & kmask);
            int32_t st = a.max_out ? (int32_t)e : 0;
            uint32_t nout = 0;
            if (e != 0) {
                if ((uint32_t)__popc(mask) < k) {
                    st = -4;   // FEC_ERR_TOO_FEW_SHARDS
                    if (lane == 0) atomicOr(a.err, 1);
                } else if (a.max_out && e > a.max_out) {
                    st = -1;   // FEC_ERR_INVALID_ARG: more erasures than output slots
                    if (lane == 0) atomicOr(a.err, 2);
                } else {
                    nout = e;
                }
            }
            if (lane == 0) {
                P[lay.nout_off] = (uint8_t)nout;
                if (a.status) a.status[b] = st;
            }
            if (nout) {
                // the first k present shards (index order) and the erased data shards
                const uint32_t below = lane < 32 ? ((1u << lane) - 1u) : 0xFFFFFFFFu;
                if (lane < n && ((mask >> lane) & 1u)) {
                    const uint32_t pos = __popc(mask & below);
                    if (pos < k) P[lay.in_off + pos] = (uint8_t)lane;
                }
                if (lane < k && !((mask >> lane) & 1u)) P[lay.out_off + (lane - __popc(mask & kmask & below))] = (uint8_t)lane;
                wave_sync();
                const uint8_t* S = P + lay.in_off;
                uint8_t* C = P + lay.coef_off;
                if (e == 1) {
                    const uint32_t E0 = __ffs(~mask & kmask) - 1;
                    const uint32_t R0 = __ffs(mask >> k) - 1;
                    const uint8_t* row = s_prows + R0 * k;
                    const uint32_t inv = s_exp[255 - s_log[row[E0]]];
                    if (lane < k) {
                        const uint32_t sj = S[lane];
                        C[lane] = (uint8_t)(sj < k ? mul(inv, row[sj]) : inv);
                    }
                } else {
                    if (lane < k) {
                        const uint32_t sp = S[lane];
                        uint32_t d = 0;
                        for (uint32_t q = 0; q < k; ++q)
                            if (q != lane) d += s_log[sp ^ S[q]];
                        Dt[lane] = (uint8_t)(d % 255u);
                    }
                    if (lane < e) {
                        const uint32_t i = P[lay.out_off + lane];
                        uint32_t ns = 0;
                        for (uint32_t q = 0; q < k; ++q) ns += s_log[i ^ S[q]];
                        Nt[lane] = (uint8_t)(ns % 255u);
                    }
                    wave_sync();
                    for (uint32_t t = lane; t < e * k; t += 64) {
                        const uint32_t r = t / k, p = t - r * k;
                        const uint32_t v = Nt[r] + 2u * 255u - s_log[P[lay.out_off + r] ^ S[p]] - Dt[p];
                        C[r * k + p] = s_exp[v % 255u];
                    }
                }
            }
            wave_sync();
        }
    }
    wave_sync();
    {
        const uint32_t ne = nb * maxe * k;
        for (uint32_t i = lane; i < ne; i += 64) {
            const uint32_t g = i / (maxe * k);
            const uint32_t rem = i - g * maxe * k;
            const uint32_t r = rem / k, j = rem - r * k;
            const uint8_t* P = plans + g * lay.stride;
            if (r < P[lay.nout_off]) tabs[i] = gf::make_permtab(P[lay.coef_off + r * k + j]);
        }
    }
    wave_sync();
    if constexpr (IPL < 0) {
        // the wave's items one 64-item run after the other, behind one plan stage
        for (uint32_t u = 0; u < NI; ++u) {
            const uint32_t item = i0 + u * 64 + lane;
            const bool inr = item < total;
            const uint32_t blk = inr ? fdiv(item, a.div_cps) : bfirst;
            const uint32_t g = blk - bfirst;
            const uint32_t c = item - blk * a.cps;
            const uint8_t* P = plans + g * lay.stride;
            const uint32_t nout = inr ? P[lay.nout_off] : 0;
            const uint32_t rows = wave_rows<MAXE>(nout);
            if (nout) recon_item<MAXE, NTL, NTS>(a, P, tabs + g * maxe * k, blk, c, rows, nout);
        }
    } else if constexpr (IPL == 1) {
        const uint32_t item = i0 + lane;
        const bool inr = item < total;
        const uint32_t blk = inr ? fdiv(item, a.div_cps) : bfirst;
        const uint32_t g = blk - bfirst;
        const uint32_t c = item - blk * a.cps;
        const uint8_t* P = plans + g * lay.stride;
        const uint32_t nout = inr ? P[lay.nout_off] : 0;
        const uint32_t rows = wave_rows<MAXE>(nout);
        if (nout == 0) return;
        recon_item<MAXE, NTL, NTS>(a, P, tabs + g * maxe * k, blk, c, rows, nout);
    } else {
        const uint32_t itA = i0 + lane, itB = itA + 64;
        const bool inA = itA < total, inB = itB < total;
        const uint32_t bA = inA ? fdiv(itA, a.div_cps) : bfirst;
        const uint32_t bB = inB ? fdiv(itB, a.div_cps) : bfirst;
        const uint8_t* PA = plans + (bA - bfirst) * lay.stride;
        const uint8_t* PB = plans + (bB - bfirst) * lay.stride;
        const uint32_t nA = inA ? PA[lay.nout_off] : 0, nB = inB ? PB[lay.nout_off] : 0;
        const uint32_t rA = wave_rows<MAXE>(nA), rB = wave_rows<MAXE>(nB);
        if ((nA | nB) == 0) return;
        recon_pair<MAXE, NTL, NTS>(a, PA, tabs + (bA - bfirst) * maxe * k, bA, itA - bA * a.cps, rA, nA, PB,
                                   tabs + (bB - bfirst) * maxe * k, bB, itB - bB * a.cps, rB, nB);
    }
}

// ------------------------------------------------------------------ XOR
// KG = inputs loaded back to back per group (2, 4 or 8, the smallest that covers k, or 8 for
// k > 8): a group issues exactly the loads it uses except for clamped repeats in the last
// group, so XOR(2,1) issues 2 loads per item, not 8.
template <int KG>
__device__ __forceinline__ void xor_fold(uint4& acc, const uint4 (&x)[KG], uint32_t valid) {
#pragma unroll
    for (int jj = 0; jj < KG; ++jj)
        if ((uint32_t)jj < valid) {
            acc.x ^= x[jj].x;
            acc.y ^= x[jj].y;
            acc.z ^= x[jj].z;
            acc.w ^= x[jj].w;
        }
}

template <int POL, int KG>
__global__ __launch_bounds__(kThreads) void xor_encode_kernel(XorArgs a) {
    constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    const uint32_t k = a.k;
    const uint32_t stride = gridDim.x * kThreads;
    for (uint32_t item = xcd_order(a.swz) * kThreads + threadIdx.x; item < a.total; item += stride) {
        const uint32_t b = fdiv(item, a.div_cps);
        const uint32_t c = rotate_chunk(item - b * a.cps, a.cps, a.rot);
        const uint8_t* src = a.in + (uint64_t)b * a.in_bs + (uint64_t)c * kChunk;
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (uint32_t j0 = 0; j0 < k; j0 += KG) {
            uint4 x[KG];
#pragma unroll
            for (int jj = 0; jj < KG; ++jj) x[jj] = ld16<NTL>(src + (uint64_t)min(j0 + jj, k - 1) * a.ss);
            xor_fold<KG>(acc, x, k - j0);
        }
        store_chunk<NTS>(a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk, acc, a.len - c * kChunk, a.pad_zero);
    }
}

template <int POL, int KG>
__global__ __launch_bounds__(kThreads) void xor_reconstruct_kernel(XorArgs a) {
    constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    const uint32_t k = a.k, n = k + 1;
    const uint32_t all = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
    const uint32_t stride = gridDim.x * kThreads;
    for (uint32_t item = xcd_order(a.swz) * kThreads + threadIdx.x; item < a.total; item += stride) {
        const uint32_t b = fdiv(item, a.div_cps);
        const uint32_t c = rotate_chunk(item - b * a.cps, a.cps, a.rot);
        const uint32_t miss = ~a.masks[b] & all;
        const uint32_t nmiss = __popc(miss);
        const uint32_t mi = miss ? (uint32_t)__ffs(miss) - 1 : 0;
        const bool work = nmiss == 1 && mi < k;
        const bool fail = nmiss > 1 && (miss & ((1u << k) - 1u));
        if (c == 0) {
            if (a.status) a.status[b] = fail ? -4 : 0;
            if (fail) atomicOr(a.err, 1);
        }
        if (!work) continue;
        uint8_t* blk = a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk;
        const uint8_t* par = a.parity + (uint64_t)b * a.par_bs + (uint64_t)c * kChunk;
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (uint32_t j0 = 0; j0 < k; j0 += KG) {
            uint4 x[KG];
#pragma unroll
            for (int jj = 0; jj < KG; ++jj) {
                const uint32_t j = min(j0 + jj, k - 1);
                const uint32_t s = j + (j >= mi);     // the k shards other than the missing one
                x[jj] = ld16<NTL>(s < k ? blk + (uint64_t)s * a.ss : par);
            }
            xor_fold<KG>(acc, x, k - j0);
        }
        store_chunk<NTS>(blk + (uint64_t)mi * a.ss, acc, a.len - c * kChunk, a.pad_zero);
    }
}

// ------------------------------------------------------------------ launchers
template <int MAXM, int POL>
static hipError_t enc_dispatch2(const EncodeArgs& a, int grid, hipStream_t s) {
    const bool lds_tabs = a.m * a.k <= (uint32_t)kMaxLdsTabs;
    if (lds_tabs) {
        const size_t lds = occupancy_lds(g_tune.gen_wpc, (size_t)a.m * a.k * sizeof(gf::PermTab));
        hipLaunchKernelGGL((rs_encode_kernel<MAXM, true, POL>), dim3(grid), dim3(kThreads), lds, s, a);
    } else {
        const size_t lds = occupancy_lds(g_tune.gen_wpc, 0);
        hipLaunchKernelGGL((rs_encode_kernel<MAXM, false, POL>), dim3(grid), dim3(kThreads), lds, s, a);
    }
    return hipGetLastError();
}

template <int MAXM>
static hipError_t enc_dispatch(const EncodeArgs& a, int grid, hipStream_t s) {
    switch (g_tune.enc_nt & 3) {
        case 0: return enc_dispatch2<MAXM, 0>(a, grid, s);
        case 1: return enc_dispatch2<MAXM, 1>(a, grid, s);
        case 2: return enc_dispatch2<MAXM, 2>(a, grid, s);
        default: return enc_dispatch2<MAXM, 3>(a, grid, s);
    }
}

hipError_t launch_rs_encode(const EncodeArgs& a, int grid, hipStream_t s) {
    if (a.m <= 1) return enc_dispatch<1>(a, grid, s);
    if (a.m <= 2) return enc_dispatch<2>(a, grid, s);
    if (a.m <= 4) return enc_dispatch<4>(a, grid, s);
    if (a.m <= 8) return enc_dispatch<8>(a, grid, s);
    return enc_dispatch<16>(a, grid, s);   // caller splits m > 16
}

// (k, m) shapes with a fixed-shape encode instance: the reference's benchmark codes RS(2,3),
// RS(8,12), RS(16,24). Any other shape runs the generic kernel.
bool fixed_encode_applies(uint32_t k, uint32_t m) {
    if (!g_tune.enc_fixed) return false;
    return (k == 2 && m == 1) || (k == 8 && m == 4) || (k == 16 && m == 8);
}

template <int K, int M>
static hipError_t enc_fixed_dispatch(const EncodeArgs& a, int grid, size_t lds, bool queue, hipStream_t s) {
    if (queue) {
        if (g_tune.enc_qdepth == 0 && g_tune.enc_diag)
            hipLaunchKernelGGL((rs_encode_queue0_kernel<K, M, 7, true>), dim3(grid), dim3(kThreads), lds, s, a);
        else if (g_tune.enc_qdepth == 0)
            hipLaunchKernelGGL((rs_encode_queue0_kernel<K, M, 3, true>), dim3(grid), dim3(kThreads), lds, s, a);
        else if (g_tune.enc_qdepth < 0)
            hipLaunchKernelGGL((rs_encode_queue0_kernel<K, M, 3, false>), dim3(grid), dim3(kThreads), lds, s, a);
        else if (g_tune.enc_diag)
            hipLaunchKernelGGL((rs_encode_queue_kernel<K, M, 7, 1>), dim3(grid), dim3(kThreads), lds, s, a);
        else if (g_tune.enc_qdepth >= 2 && K <= 8)   // K = 16 at depth 2 exceeds the register file
            hipLaunchKernelGGL((rs_encode_queue_kernel<K, M, 3, (K <= 8 ? 2 : 1)>), dim3(grid), dim3(kThreads), lds, s, a);
        else
            hipLaunchKernelGGL((rs_encode_queue_kernel<K, M, 3, 1>), dim3(grid), dim3(kThreads), lds, s, a);
    } else if (g_tune.enc_dyadic && a.dytabs && K >= 4) {
        EncodeArgs d = a;
        d.tabs = a.dytabs;
        if (g_tune.enc_nt & 1)
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 11>), dim3(grid), dim3(kThreads), lds, s, d);
        else
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 10>), dim3(grid), dim3(kThreads), lds, s, d);
    } else {
        if (g_tune.enc_nt & 1)
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 3>), dim3(grid), dim3(kThreads), lds, s, a);
        else
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 2>), dim3(grid), dim3(kThreads), lds, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_rs_encode_fixed(EncodeArgs a, int ncu, hipStream_t s) {
    const uint32_t chunks = (a.total + kThreads - 1) / kThreads;
    if (chunks == 0) return hipSuccess;
    // Per shape (measured): RS(8,12) and RS(16,24) run the flat grid at
    // g_tune.enc_wpc (3) workgroups per CU; RS(2,3) (2 loads per lane: little in flight per
    // wave) at full residency. The ticket-queue form stays selectable (enc_queue).
    const bool queue = g_tune.enc_queue && a.ctr != nullptr && a.k == 8;
    int grid = (int)chunks;
    int wpc = a.k == 2 ? 0 : g_tune.enc_wpc;
    if (queue) {
        wpc = g_tune.enc_qwpc > 0 ? g_tune.enc_qwpc : 2;
        grid = ncu * wpc;
        // no more owners per range than the range has chunks; a multiple of 8 (every range owned)
        const int per_range = (int)((chunks + 7) / 8);
        grid = std::min(grid / 8, per_range) * 8;
        if (grid < 8) grid = 8;
        a.per_xcd = ((a.total + 7) / 8 + kThreads - 1) / kThreads * kThreads;
    }
    const size_t lds = occupancy_lds(wpc, (size_t)a.m * a.k * sizeof(gf::PermTab));
    if (a.k == 2 && a.m == 1) return enc_fixed_dispatch<2, 1>(a, grid, lds, queue, s);
    if (a.k == 8 && a.m == 4) return enc_fixed_dispatch<8, 4>(a, grid, lds, queue, s);
    if (a.k == 16 && a.m == 8) return enc_fixed_dispatch<16, 8>(a, grid, lds, queue, s);
    return hipErrorInvalidValue;
}

hipError_t launch_rs_plan(const PlanArgs& a, hipStream_t s) {
    const int grid = (int)((a.nblocks + kPlanThreads - 1) / kPlanThreads);
    if (grid == 0) return hipSuccess;
    const size_t lds = plan_lds(a.m, a.k, a.lay.stride).total;
    const dim3 g(grid), t(kPlanThreads);
    hipLaunchKernelGGL(rs_plan_kernel, g, t, lds, s, a);
    return hipGetLastError();
}

size_t recon_lds_bytes(uint32_t g, uint32_t k, uint32_t maxe, const PlanLayout& lay) {
    return (size_t)g * maxe * k * sizeof(gf::PermTab) + (size_t)g * lay.stride;
}

template <int POL>
static hipError_t recon_dispatch(const ReconArgs& a, int grid, hipStream_t s) {
    const size_t lds = occupancy_lds(g_tune.dec_wpc, recon_lds_bytes(a.g, a.k, a.maxe, a.lay));
    if (a.maxe <= 1) hipLaunchKernelGGL((rs_reconstruct_kernel<1, POL>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (a.maxe <= 2) hipLaunchKernelGGL((rs_reconstruct_kernel<2, POL>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (a.maxe <= 4) hipLaunchKernelGGL((rs_reconstruct_kernel<4, POL>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (a.maxe <= 8) hipLaunchKernelGGL((rs_reconstruct_kernel<8, POL>), dim3(grid), dim3(kThreads), lds, s, a);
    else hipLaunchKernelGGL((rs_reconstruct_kernel<16, POL>), dim3(grid), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

// The wave form applies to shards of 32+ chunks (at most 3 blocks per wave) while its LDS
// (4 wave slices per workgroup) stays within 64 KiB.
bool wave_recon_applies(uint32_t cps, uint32_t k, uint32_t maxe, uint32_t stride) {
    return g_tune.dec_wave && cps >= 32 && 4 * fused_slice_bytes(k, maxe, stride) + 2048 <= 65536;
}

template <int POL, bool FUSED, int IPL>
static hipError_t recon_wave_dispatch(const ReconArgs& a, hipStream_t s) {
    const uint64_t per_wg = (uint64_t)kThreads * (IPL < 0 ? -IPL : IPL);
    const int grid = (int)(((uint64_t)a.nblocks * a.cps + per_wg - 1) / per_wg);
    if (grid == 0) return hipSuccess;
    size_t own = 4 * wave_slice_bytes(a.k, a.maxe, a.lay.stride);
    if (FUSED) {
        const FusedLds L = fused_lds(a.m, a.k, a.maxe, a.lay.stride);
        own = L.slices + 4 * L.slice;
    }
    const size_t lds = occupancy_lds(g_tune.dec_wpc, own);
#define FEC_WAVE_LAUNCH(E) \
    hipLaunchKernelGGL((rs_reconstruct_wave_kernel<E, POL, FUSED, IPL>), dim3(grid), dim3(kThreads), lds, s, a)
    if (a.maxe <= 1) FEC_WAVE_LAUNCH(1);
    else if (a.maxe <= 2) FEC_WAVE_LAUNCH(2);
    else if (a.maxe <= 4) FEC_WAVE_LAUNCH(4);
    else if constexpr (IPL != 2) {   // the pair form is only built for up to 4 rows
        if (a.maxe <= 8) FEC_WAVE_LAUNCH(8);
        else FEC_WAVE_LAUNCH(16);
    } else {
        return hipErrorInvalidValue;
    }
#undef FEC_WAVE_LAUNCH
    return hipGetLastError();
}

// Items per lane of the wave form (knob dec_ipl: 0 auto, 1, 2). Two items per lane pay for
// latency-bound shapes (RS(2,3): 57 -> 51.5 us per 2^16 blocks) and cost 17 % where HBM is
// the bound (RS(8,12)), so auto picks 2 for k <= 4. Two need at most 4 rebuilt rows (registers)
// and shards of 64+ chunks (the 128-item span then still covers at most 3 blocks).
template <int POL, bool FUSED>
static hipError_t recon_wave_ipl(const ReconArgs& a, hipStream_t s) {
    const int ipl = g_tune.dec_ipl ? g_tune.dec_ipl : (a.k <= 4 ? 2 : 1);
    if (ipl == 2 && a.maxe <= 4 && a.cps >= 64) return recon_wave_dispatch<POL, FUSED, 2>(a, s);
    if (ipl == 3 && a.cps >= 64) return recon_wave_dispatch<POL, FUSED, -2>(a, s);
    return recon_wave_dispatch<POL, FUSED, 1>(a, s);
}

hipError_t launch_rs_reconstruct_wave(const ReconArgs& a, hipStream_t s) {
    switch (g_tune.dec_nt & 3) {
        case 0: return recon_wave_ipl<0, false>(a, s);
        case 1: return recon_wave_ipl<1, false>(a, s);
        case 2: return recon_wave_ipl<2, false>(a, s);
        default: return recon_wave_ipl<3, false>(a, s);
    }
}

hipError_t launch_rs_recover_fused(const ReconArgs& a, hipStream_t s) {
    return (g_tune.dec_nt & 3) == 3 ? recon_wave_ipl<3, true>(a, s) : recon_wave_ipl<0, true>(a, s);
}

hipError_t launch_rs_reconstruct(const ReconArgs& a, int grid, hipStream_t s) {
    switch (g_tune.dec_nt & 3) {
        case 0: return recon_dispatch<0>(a, grid, s);
        case 1: return recon_dispatch<1>(a, grid, s);
        case 2: return recon_dispatch<2>(a, grid, s);
        default: return recon_dispatch<3>(a, grid, s);
    }
}

template <int KG>
static void xor_launch(const XorArgs& a, int grid, size_t lds, bool nt, bool encode, hipStream_t s) {
    if (encode) {
        if (nt) hipLaunchKernelGGL((xor_encode_kernel<3, KG>), dim3(grid), dim3(kThreads), lds, s, a);
        else hipLaunchKernelGGL((xor_encode_kernel<0, KG>), dim3(grid), dim3(kThreads), lds, s, a);
    } else {
        if (nt) hipLaunchKernelGGL((xor_reconstruct_kernel<3, KG>), dim3(grid), dim3(kThreads), lds, s, a);
        else hipLaunchKernelGGL((xor_reconstruct_kernel<0, KG>), dim3(grid), dim3(kThreads), lds, s, a);
    }
}

static hipError_t xor_dispatch(const XorArgs& a, int grid, size_t lds, bool nt, bool encode, hipStream_t s) {
    if (a.k <= 2) xor_launch<2>(a, grid, lds, nt, encode, s);
    else if (a.k <= 4) xor_launch<4>(a, grid, lds, nt, encode, s);
    else xor_launch<8>(a, grid, lds, nt, encode, s);
    return hipGetLastError();
}

hipError_t launch_xor_encode(const XorArgs& a, int grid, hipStream_t s) {
    return xor_dispatch(a, grid, occupancy_lds(g_tune.gen_wpc, 0), (g_tune.enc_nt & 3) != 0, true, s);
}

hipError_t launch_xor_reconstruct(const XorArgs& a, int grid, hipStream_t s) {
    return xor_dispatch(a, grid, occupancy_lds(g_tune.dec_wpc, 0), (g_tune.dec_nt & 3) != 0, false, s);
}

uint32_t pick_tile_blocks(uint32_t cps, uint32_t k, uint32_t maxe, const PlanLayout& lay) {
    // Blocks per tile: the smallest count that reaches the best lane utilisation of the
    // G*cps items over 256 lanes within dec_max_rounds rounds, bounded by 48 KiB of LDS.
    const size_t per_block = recon_lds_bytes(1, k, maxe, lay);
    uint32_t gmax = (uint32_t)((48u * 1024u) / per_block);
    if (gmax < 1) gmax = 1;
    if (gmax > 256) gmax = 256;
    uint32_t best = 1;
    double best_u = -1.0;
    for (uint32_t g = 1; g <= gmax; ++g) {
        const uint32_t items = g * cps;
        const uint32_t rounds = (items + kThreads - 1) / kThreads;
        if (rounds > (uint32_t)g_tune.dec_max_rounds && g > 1) break;
        const double u = (double)items / (double)(rounds * kThreads);
        if (u > best_u + 1e-3) {
            best = g;
            best_u = u;
        }
    }
    return best;
}

int occupancy_grid(int device, int which, uint32_t sel, size_t lds) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0)
        ncu = 256;
    int per = 0;
    const void* fn = nullptr;
    if (which == 0) {
        if (sel <= 1) fn = (const void*)rs_encode_kernel<1, true, 3>;
        else if (sel <= 2) fn = (const void*)rs_encode_kernel<2, true, 3>;
        else if (sel <= 4) fn = (const void*)rs_encode_kernel<4, true, 3>;
        else if (sel <= 8) fn = (const void*)rs_encode_kernel<8, true, 3>;
        else fn = (const void*)rs_encode_kernel<16, true, 3>;
    } else if (which == 1) {
        if (sel <= 1) fn = (const void*)rs_reconstruct_kernel<1, 3>;
        else if (sel <= 2) fn = (const void*)rs_reconstruct_kernel<2, 3>;
        else if (sel <= 4) fn = (const void*)rs_reconstruct_kernel<4, 3>;
        else if (sel <= 8) fn = (const void*)rs_reconstruct_kernel<8, 3>;
        else fn = (const void*)rs_reconstruct_kernel<16, 3>;
    } else {
        fn = (const void*)xor_encode_kernel<3, 8>;
    }
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, kThreads, lds) != hipSuccess || per <= 0)
        per = 4;
    if (per > 8) per = 8;
    return ncu * per;
}

}  // namespace fk
