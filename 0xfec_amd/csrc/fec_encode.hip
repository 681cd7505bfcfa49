// fec_encode.hip — RS encode kernels for gfx950 (reed_solomon.go:51 Encode): generic (k, m),
// fixed compile-time shapes (RS(2,3), RS(8,12), RS(16,24)) with the dyadic split-recursive body,
// and the persistent ticket-queue form (knob enc_queue). See fec_kernels.hip for the overview.
#include "fec_device.hpp"

namespace fk {

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

// Flat launch: one item per lane, XCD-contiguous workgroup order. POL bit 4 (knob enc_early): the
// table words' loads go out first, then the item's K shard loads, and the tables reach LDS behind an
// LDS-only barrier, so the shard loads are in flight while the tables stage (without it the
// workgroup's __syncthreads waits for the table loads before any shard load is issued: one memory
// round trip per workgroup, which a 40-us RS(2,3) launch of ~20 000 workgroups feels).
template <int K, int M, int POL>
__global__ __launch_bounds__(kThreads) void rs_encode_fixed_kernel(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t it = xcd_order(a.swz) * kThreads + threadIdx.x;
    if constexpr ((POL & 16) != 0) {
        constexpr uint32_t W = M * K * 8, R = (W + kThreads - 1) / kThreads;   // table dwords, per lane
        uint32_t tw[R];
#pragma unroll
        for (uint32_t q = 0; q < R; ++q) {
            const uint32_t i = threadIdx.x + q * kThreads;
            tw[q] = i < W ? a.tabs[i] : 0u;
        }
        const FixedEncode<K, M, POL> f{a, reinterpret_cast<const gf::PermTab*>(smem)};
        uint4 x[K];
        if (it < a.total) f.load(x, it);
#pragma unroll
        for (uint32_t q = 0; q < R; ++q) {
            const uint32_t i = threadIdx.x + q * kThreads;
            if (i < W) reinterpret_cast<uint32_t*>(smem)[i] = tw[q];
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (it >= a.total) return;
        f.compute_store(x, it);
    } else {
        const FixedEncode<K, M, POL> f{a, stage_tabs<K, M>(smem, a.tabs)};
        if (it >= a.total) return;
        uint4 x[K];
        f.load(x, it);
        f.compute_store(x, it);
    }
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

// ------------------------------------------------------------------ RS encode, bit-sliced
// The fixed shapes as one XOR network over bit planes (gen_bitslice.py): a lane takes two
// 16-byte chunks of every data shard, turns each shard's 8 dwords into 8 bit planes (plane b holds bit b of the 32 bytes), runs the compile-time network
// (shared sub-sums, three-input XORs, no tables), and turns the parity planes back into bytes.
// RS(16,24): 2 x 48 ops of transposes per shard plus 1202 network ops per 32 bytes, against 54
// v_perm products of the dyadic body per 16 bytes.
template <int K, int M>
struct BsShape;   // G: shards per network group
template <int K, int M, int GI>
__device__ __forceinline__ void bs_grp(const uint32_t (&x)[BsShape<K, M>::G][8], uint32_t (&y)[M][8]);
#include "fec_bitslice.inc"

// In every byte column q of the 8 dwords, transpose the 8x8 bit block (row = dword i, column =
// bit b): afterwards bit 8q + i of w[b] is what was bit 8q + b of w[i]. Three delta swaps (block
// sizes 4, 2, 1), two ops per register per stage. A transpose is its own inverse.
// (a & m) | (b & ~m) as one v_bfi_b32 (left to the compiler, the masks are merged into the
// neighbouring XORs as AND + three-input ops: more instructions)
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(d) : "s"(m), "v"(a), "v"(b));
    return d;
}
template <int S>
__device__ __forceinline__ void delta_swap8(uint32_t (&w)[8]) {
    constexpr uint32_t lo = S == 4 ? 0x0F0F0F0Fu : S == 2 ? 0x33333333u : 0x55555555u;   // bits with (b & S) == 0
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i & S) continue;
        const uint32_t a = w[i], c = w[i + S];
        w[i] = bfi(lo, a, c << S);
        w[i + S] = bfi(lo, a >> S, c);
    }
}
__device__ __forceinline__ void bit_transpose8(uint32_t (&w)[8]) {
    delta_swap8<4>(w);
    delta_swap8<2>(w);
    delta_swap8<1>(w);
}

// Group GI of the network: transpose the group's raw chunks into planes, fold them into y.
// STREAM: the next group's loads are issued first, behind an opaque dependence on the previous
// group's last output, so only two groups of inputs are ever held (fewer VGPRs, more waves) and
// every wave keeps loads in flight while it computes.
template <int K, int M, int POL, bool STREAM, int GI>
__device__ __forceinline__ void bs_stream(const uint8_t* s0, const uint8_t* s1, uint64_t ss,
                                          uint4 (&cur)[BsShape<K, M>::G][2], uint32_t (&y)[M][8]) {
    constexpr int G = BsShape<K, M>::G, NG = K / G;
    constexpr bool NTL = POL & 1;
    uint4 nxt[G][2];
    if constexpr (STREAM && GI + 1 < NG) {
        uint64_t off = (uint64_t)(GI + 1) * G * ss;
        if constexpr (GI > 0) asm volatile("" : "+v"(off) : "v"(y[M - 1][7]));
#pragma unroll
        for (int j = 0; j < G; ++j) {
            nxt[j][0] = ld16<NTL>(s0 + off + (uint64_t)j * ss);
            nxt[j][1] = ld16<NTL>(s1 + off + (uint64_t)j * ss);
        }
    }
    uint32_t x[G][8];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        x[j][0] = cur[j][0].x, x[j][1] = cur[j][0].y, x[j][2] = cur[j][0].z, x[j][3] = cur[j][0].w;
        x[j][4] = cur[j][1].x, x[j][5] = cur[j][1].y, x[j][6] = cur[j][1].z, x[j][7] = cur[j][1].w;
        bit_transpose8(x[j]);
    }
    bs_grp<K, M, GI>(x, y);
    if constexpr (GI + 1 < NG) {
        if constexpr (!STREAM) {
#pragma unroll
            for (int j = 0; j < G; ++j) {
                nxt[j][0] = ld16<NTL>(s0 + (uint64_t)((GI + 1) * G + j) * ss);
                nxt[j][1] = ld16<NTL>(s1 + (uint64_t)((GI + 1) * G + j) * ss);
            }
        }
        bs_stream<K, M, POL, STREAM, GI + 1>(s0, s1, ss, nxt, y);
    }
}

template <int K, int M, int POL>
__global__ __launch_bounds__(kThreads) void rs_encode_bits_kernel(EncodeArgs a) {
    constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    // A wave takes 128 consecutive (block, chunk) items: lane l items w*128 + l and w*128 + 64 + l,
    // so each load and store instruction covers 64 consecutive chunks, as in the one-chunk
    // kernels. The two chunks of a lane may belong to different blocks: the network treats every
    // byte column alike.
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t f0 = (xcd_order(a.swz) * kThreads + (threadIdx.x & ~63u)) * 2u + lane;
    if (f0 >= a.total) return;
    const uint32_t f1 = f0 + 64u;
    const bool two = f1 < a.total;
    const uint32_t b0 = fdiv(f0, a.div_cps), c0 = f0 - b0 * a.cps;
    const uint32_t fb = two ? f1 : f0;   // without a second item the first is loaded again (no
    const uint32_t b1 = fdiv(fb, a.div_cps), c1 = fb - b1 * a.cps;   // branch); its outputs are not stored
    const uint8_t* s0 = a.in + (uint64_t)b0 * a.in_bs + (uint64_t)c0 * kChunk;
    const uint8_t* s1 = a.in + (uint64_t)b1 * a.in_bs + (uint64_t)c1 * kChunk;
    constexpr int G = BsShape<K, M>::G;
    uint4 g0[G][2];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        g0[j][0] = ld16<NTL>(s0 + (uint64_t)j * a.ss);
        g0[j][1] = ld16<NTL>(s1 + (uint64_t)j * a.ss);
    }
    uint32_t y[M][8];
    bs_stream<K, M, POL, (POL & 16) != 0, 0>(s0, s1, a.ss, g0, y);
    uint8_t* d0 = a.out + (uint64_t)b0 * a.out_bs + (uint64_t)c0 * kChunk;
    uint8_t* d1 = a.out + (uint64_t)b1 * a.out_bs + (uint64_t)c1 * kChunk;
    const uint32_t nb0 = min(a.len - c0 * kChunk, (uint32_t)kChunk);
    const uint32_t nb1 = min(a.len - c1 * kChunk, (uint32_t)kChunk);
#pragma unroll
    for (int r = 0; r < M; ++r) {
        bit_transpose8(y[r]);
        st16<NTS>(d0 + (uint64_t)r * a.ss, keep_bytes(make_uint4(y[r][0], y[r][1], y[r][2], y[r][3]), nb0));
        if (two) st16<NTS>(d1 + (uint64_t)r * a.ss, keep_bytes(make_uint4(y[r][4], y[r][5], y[r][6], y[r][7]), nb1));
    }
}

template <int K, int M>
static hipError_t enc_bits_dispatch(const EncodeArgs& a, hipStream_t s) {
    const int grid = (int)((a.total + 2 * kThreads - 1) / (2 * kThreads));
    if (grid == 0) return hipSuccess;
    const size_t lds = occupancy_lds(g_tune.enc_bwpc, 0);
    const bool nt = g_tune.enc_nt & 1, stream = g_tune.enc_bits & 4;
    if (stream && nt) hipLaunchKernelGGL((rs_encode_bits_kernel<K, M, 19>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (stream) hipLaunchKernelGGL((rs_encode_bits_kernel<K, M, 18>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (nt) hipLaunchKernelGGL((rs_encode_bits_kernel<K, M, 3>), dim3(grid), dim3(kThreads), lds, s, a);
    else hipLaunchKernelGGL((rs_encode_bits_kernel<K, M, 2>), dim3(grid), dim3(kThreads), lds, s, a);
    return hipGetLastError();
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
    // cache policy: plain, or non-temporal loads and stores (the mixed forms measured no better)
    return (g_tune.enc_nt & 3) ? enc_dispatch2<MAXM, 3>(a, grid, s) : enc_dispatch2<MAXM, 0>(a, grid, s);
}

hipError_t launch_rs_encode(const EncodeArgs& a, int grid, hipStream_t s) {
    if (a.m <= 1) return enc_dispatch<1>(a, grid, s);
    if (a.m <= 2) return enc_dispatch<2>(a, grid, s);
    if (a.m <= 4) return enc_dispatch<4>(a, grid, s);
    if (a.m <= 8) return enc_dispatch<8>(a, grid, s);
    return enc_dispatch<16>(a, grid, s);   // caller splits m > 16
}

// (k, m) shapes with a fixed-shape encode instance: the reference's benchmark codes RS(2,3),
// RS(8,12), RS(16,24), and (bit-sliced) its sender's RS(20,30). Any other shape runs the
// generic kernel.
bool fixed_encode_applies(uint32_t k, uint32_t m) {
    if (!g_tune.enc_fixed) return false;
    return (k == 2 && m == 1) || (k == 8 && m == 4) || (k == 16 && m == 8) ||
           (k == 20 && m == 10 && (g_tune.enc_bits & 8));   // bit-sliced only
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
        if ((g_tune.enc_early == 1 || (g_tune.enc_early == 2 && K == 2)) && (g_tune.enc_nt & 1))
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 27>), dim3(grid), dim3(kThreads), lds, s, d);
        else if (g_tune.enc_nt & 1)
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 11>), dim3(grid), dim3(kThreads), lds, s, d);
        else
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 10>), dim3(grid), dim3(kThreads), lds, s, d);
    } else {
        if ((g_tune.enc_early == 1 || (g_tune.enc_early == 2 && K == 2)) && (g_tune.enc_nt & 1))
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 19>), dim3(grid), dim3(kThreads), lds, s, a);
        else if (g_tune.enc_nt & 1)
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 3>), dim3(grid), dim3(kThreads), lds, s, a);
        else
            hipLaunchKernelGGL((rs_encode_fixed_kernel<K, M, 2>), dim3(grid), dim3(kThreads), lds, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_rs_encode_fixed(EncodeArgs a, int ncu, hipStream_t s) {
    const uint32_t chunks = (a.total + kThreads - 1) / kThreads;
    if (chunks == 0) return hipSuccess;
    // bit-sliced network (knob enc_bits: bit 0 RS(16,24), bit 1 RS(8,12), bit 2 streamed loads,
    // bit 3 RS(20,30), the reference's own sender code, manager.go:80)
    if (a.k == 16 && a.m == 8 && (g_tune.enc_bits & 1)) return enc_bits_dispatch<16, 8>(a, s);
    if (a.k == 8 && a.m == 4 && (g_tune.enc_bits & 2)) return enc_bits_dispatch<8, 4>(a, s);
    if (a.k == 20 && a.m == 10 && (g_tune.enc_bits & 8)) return enc_bits_dispatch<20, 10>(a, s);
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
    if (!queue && rs_encode23_applies(a.k, a.m)) return launch_rs_encode23(a, s);
    if (a.k == 2 && a.m == 1) return enc_fixed_dispatch<2, 1>(a, grid, lds, queue, s);
    if (a.k == 8 && a.m == 4) return enc_fixed_dispatch<8, 4>(a, grid, lds, queue, s);
    if (a.k == 16 && a.m == 8) return enc_fixed_dispatch<16, 8>(a, grid, lds, queue, s);
    return hipErrorInvalidValue;
}

const void* encode_occupancy_kernel(uint32_t sel) {
    if (sel <= 1) return (const void*)rs_encode_kernel<1, true, 3>;
    if (sel <= 2) return (const void*)rs_encode_kernel<2, true, 3>;
    if (sel <= 4) return (const void*)rs_encode_kernel<4, true, 3>;
    if (sel <= 8) return (const void*)rs_encode_kernel<8, true, 3>;
    return (const void*)rs_encode_kernel<16, true, 3>;
}

}  // namespace fk
