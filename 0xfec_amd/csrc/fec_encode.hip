// fec_encode.hip — RS encode kernels for gfx950 (reed_solomon.go:51 Encode): generic (k, m), RS(8,12)
// by the dyadic split-recursive body, RS(16,24) / RS(20,30) by the bit-sliced XOR network (RS(2,3):
// fec_encode23.hip). See fec_kernels.hip for the overview.
#include "fec_device.hpp"

namespace fk {

// ------------------------------------------------------------------ RS encode
// One lane = one 16-byte column chunk of one block; all m parities accumulate in VGPRs.
// Inputs are loaded 8 shards at a time (clamped, so loads are never predicated), then
// each input updates every parity accumulator with its LDS-broadcast PermTab. Non-temporal loads
// and stores (+2-5 %).
template <int MAXM, bool LDS_TABS>
__global__ __launch_bounds__(kThreads) void rs_encode_kernel(EncodeArgs a) {
    constexpr bool NTL = true, NTS = true;
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
    for (uint32_t item = xcd_order() * kThreads + threadIdx.x; item < a.total; item += stride) {
        const uint32_t b = fdiv(item, a.div_cps);
        const uint32_t c = item - b * a.cps;
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
            if (r < (int)m) store_chunk<NTS>(dst + (uint64_t)r * a.ss, as_uint4(acc[r]), nb);
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

// The dyadic body: the M parity chunks of one 16-byte column from its K data chunks, the leaf
// tables at `tabs` (LDS).
template <int K, int M>
__device__ __forceinline__ void dy_encode_chunk(const uint4 (&x)[K], const uint8_t* tabs, uint32_t (&acc)[M][4]) {
    static_assert((K & (K - 1)) == 0 && (M & (M - 1)) == 0 && M <= K, "dyadic codes: powers of two, m <= k");
    // opaque zero: keeps the table reads next to their use (hoisted out of a loop they would hold
    // 5*M*K VGPRs)
    uint32_t toff = 0;
    asm volatile("" : "+s"(toff));
    const gf::PermTab* t = reinterpret_cast<const gf::PermTab*>(tabs) + toff;
    constexpr int B = M == 1 ? 0 : M == 2 ? 1 : M == 4 ? 2 : M == 8 ? 3 : 4;
    constexpr int L = Pow3<B>::v;
    constexpr int NC = K >= 16 ? 1 : 4;   // dword columns per pass (registers)
#pragma unroll
    for (int c0 = 0; c0 < 4; c0 += NC) {
        // opaque zero per pass: the table reads stay in their pass (shared across passes they
        // would be hoisted and held: 5 VGPRs per leaf)
        uint32_t poff = 0;
        asm volatile("" : "+s"(poff));
        const gf::PermTab* tp = t + poff;
#pragma unroll
        for (int h = 0; h < K / M; ++h) {
            Idx D[M][NC];
#pragma unroll
            for (int v = 0; v < M; ++v)
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) D[v][cc] = split(word_of(x[h * M + v], c0 + cc));
            uint32_t Y[M][NC];
            dy_conv<B, NC>(D, tp + h * L, Y);
#pragma unroll
            for (int i = 0; i < M; ++i)
#pragma unroll
                for (int cc = 0; cc < NC; ++cc) acc[i][c0 + cc] = h ? acc[i][c0 + cc] ^ Y[i][cc] : Y[i][cc];
        }
    }
}

// ------------------------------------------------------------------ RS encode, fixed shape
// RS(8,12), the headline code, with K and M compile-time and the dyadic body: one lane = one
// 16-byte column chunk, the K loads issued back to back, no runtime guards; the workgroup stages
// the leaf tables (dyadic_leaves(), fec_capi.cpp) in LDS. Non-temporal loads; stores by policy SP
// (fec_device.hpp st16p; the launch's default sc1). Tail chunks are stored whole with the pad
// bytes zeroed. (Round 6 measured a form with its loads decoupled from its arithmetic, each wave
// walking T tiles with the next D tiles' shard chunks in flight as LDS-DMA loads into a ring:
// 7-17 % slower than this flat grid at every residency, its traffic twin 7.5-9 % below the flat
// twin; the kernel is in commit f1dd58a. A body with half the VALU ran no faster at 2 workgroups/CU
// and slower at 3; leaf tables by scalar loads, with no LDS staging and no barrier, ran 5 % faster
// at 2 and level at 3, where this kernel runs: DESIGN.md 3, r6 rows.)
// WW < 4 (knob enc_ww, default 3): WW waves of each workgroup take items (the workgroup covers
// WW * 64), the others stage their table words and exit after the barrier; the working lanes issue
// their shard loads before the table staging and the barrier, so the prologue runs under them.
template <int K, int M, int SP = 0, int WW = 4>
__global__ __launch_bounds__(kThreads) void rs_encode_fixed_kernel(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint4 x[K];
    uint32_t b, c;
    if constexpr (WW < kThreads / 64) {
        static_assert(M * K * 8 == kThreads, "one leaf-table word per thread");
        const uint32_t wave = threadIdx.x >> 6;
        // every kernel argument in one scalar round trip
        const uint32_t order = xcd_order();
        asm volatile("" ::"s"(a.in), "s"(a.in_bs), "s"(a.ss), "s"(a.total), "s"(a.cps), "s"(a.div_cps.magic),
                     "s"(a.div_cps.shift), "s"(a.dytabs), "s"(order));
        const uint32_t tw = a.dytabs[threadIdx.x];
        const uint32_t it = order * (WW * 64u) + threadIdx.x;
        const bool live = wave < (uint32_t)WW && it < a.total;
        const uint32_t itc = min(it, a.total - 1u);
        b = fdiv(itc, a.div_cps);
        c = itc - b * a.cps;
        // unconditional loads (a lane past the end re-reads the last item, an idle wave one table
        // line): the table word's wait then counts only itself (vmcnt K), not the shard loads
        const bool work = wave < (uint32_t)WW;
        const uint8_t* src = work ? a.in + (uint64_t)b * a.in_bs + (uint64_t)c * kChunk
                                  : reinterpret_cast<const uint8_t*>(a.dytabs);
        const uint64_t ss = work ? a.ss : 0;
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = ld16<true>(src + (uint64_t)j * ss);
        reinterpret_cast<uint32_t*>(smem)[threadIdx.x] = tw;
        __syncthreads();
        if (!live) return;
    } else {
        {
            uint32_t* dst = reinterpret_cast<uint32_t*>(smem);
            for (uint32_t i = threadIdx.x; i < (uint32_t)(M * K * 8); i += kThreads) dst[i] = a.dytabs[i];
            __syncthreads();
        }
        const uint32_t it = xcd_order() * kThreads + threadIdx.x;
        if (it >= a.total) return;
        b = fdiv(it, a.div_cps);
        c = it - b * a.cps;
        const uint8_t* src = a.in + (uint64_t)b * a.in_bs + (uint64_t)c * kChunk;
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = ld16<true>(src + (uint64_t)j * a.ss);
    }
    uint32_t acc[M][4];
    dy_encode_chunk<K, M>(x, smem, acc);
    uint8_t* dst = a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk;
    const uint32_t nb = min(a.len - c * kChunk, (uint32_t)kChunk);
#pragma unroll
    for (int r = 0; r < M; ++r) st16p<SP>(dst + (uint64_t)r * a.ss, keep_bytes(as_uint4(acc[r]), nb));
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

// Group GI of the network: transpose the group's raw chunks into planes, fold them into y, then
// load the next group (streaming the next group's loads ahead of this one's network measured -0.2 %,
// r02).
template <int K, int M, int GI>
__device__ __forceinline__ void bs_stream(const uint8_t* s0, const uint8_t* s1, uint64_t ss,
                                          uint4 (&cur)[BsShape<K, M>::G][2], uint32_t (&y)[M][8]) {
    constexpr int G = BsShape<K, M>::G, NG = K / G;
    uint4 nxt[G][2];
    uint32_t x[G][8];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        x[j][0] = cur[j][0].x, x[j][1] = cur[j][0].y, x[j][2] = cur[j][0].z, x[j][3] = cur[j][0].w;
        x[j][4] = cur[j][1].x, x[j][5] = cur[j][1].y, x[j][6] = cur[j][1].z, x[j][7] = cur[j][1].w;
        bit_transpose8(x[j]);
    }
    bs_grp<K, M, GI>(x, y);
    if constexpr (GI + 1 < NG) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
            nxt[j][0] = ld16<true>(s0 + (uint64_t)((GI + 1) * G + j) * ss);
            nxt[j][1] = ld16<true>(s1 + (uint64_t)((GI + 1) * G + j) * ss);
        }
        bs_stream<K, M, GI + 1>(s0, s1, ss, nxt, y);
    }
}

template <int K, int M, int SP>
__global__ __launch_bounds__(kThreads) void rs_encode_bits_kernel(EncodeArgs a) {
    constexpr bool NTL = true;
    // A wave takes 128 consecutive (block, chunk) items: lane l items w*128 + l and w*128 + 64 + l,
    // so each load and store instruction covers 64 consecutive chunks, as in the one-chunk
    // kernels. The two chunks of a lane may belong to different blocks: the network treats every
    // byte column alike.
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t f0 = (xcd_order() * kThreads + (threadIdx.x & ~63u)) * 2u + lane;
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
    bs_stream<K, M, 0>(s0, s1, a.ss, g0, y);
    uint8_t* d0 = a.out + (uint64_t)b0 * a.out_bs + (uint64_t)c0 * kChunk;
    uint8_t* d1 = a.out + (uint64_t)b1 * a.out_bs + (uint64_t)c1 * kChunk;
    const uint32_t nb0 = min(a.len - c0 * kChunk, (uint32_t)kChunk);
    const uint32_t nb1 = min(a.len - c1 * kChunk, (uint32_t)kChunk);
#pragma unroll
    for (int r = 0; r < M; ++r) {
        bit_transpose8(y[r]);
        st16p<SP>(d0 + (uint64_t)r * a.ss, keep_bytes(make_uint4(y[r][0], y[r][1], y[r][2], y[r][3]), nb0));
        if (two) st16p<SP>(d1 + (uint64_t)r * a.ss, keep_bytes(make_uint4(y[r][4], y[r][5], y[r][6], y[r][7]), nb1));
    }
}

template <int K, int M>
static hipError_t enc_bits_dispatch(const EncodeArgs& a, hipStream_t s) {
    const int grid = (int)((a.total + 2 * kThreads - 1) / (2 * kThreads));
    if (grid == 0) return hipSuccess;
    const size_t lds = occupancy_lds(g_tune.enc_bwpc, 0);
    if (a.sp == 1) hipLaunchKernelGGL((rs_encode_bits_kernel<K, M, 1>), dim3(grid), dim3(kThreads), lds, s, a);
    else hipLaunchKernelGGL((rs_encode_bits_kernel<K, M, 0>), dim3(grid), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------ launchers
template <int MAXM>
static hipError_t enc_dispatch(const EncodeArgs& a, int grid, hipStream_t s) {
    const bool lds_tabs = a.m * a.k <= (uint32_t)kMaxLdsTabs;
    if (lds_tabs) {
        const size_t lds = occupancy_lds(g_tune.gen_wpc, (size_t)a.m * a.k * sizeof(gf::PermTab));
        hipLaunchKernelGGL((rs_encode_kernel<MAXM, true>), dim3(grid), dim3(kThreads), lds, s, a);
    } else {
        const size_t lds = occupancy_lds(g_tune.gen_wpc, 0);
        hipLaunchKernelGGL((rs_encode_kernel<MAXM, false>), dim3(grid), dim3(kThreads), lds, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_rs_encode(const EncodeArgs& a, int grid, hipStream_t s) {
    if (a.m <= 1) return enc_dispatch<1>(a, grid, s);
    if (a.m <= 2) return enc_dispatch<2>(a, grid, s);
    if (a.m <= 4) return enc_dispatch<4>(a, grid, s);
    if (a.m <= 8) return enc_dispatch<8>(a, grid, s);
    return enc_dispatch<16>(a, grid, s);   // caller splits m > 16
}

// (k, m) shapes with an encode of their own: the reference's benchmark codes RS(2,3) (its parity
// row, fec_encode23.hip), RS(8,12) (dyadic), RS(16,24) and its sender's RS(20,30) (bit-sliced).
// Any other shape runs the generic kernel.
bool fixed_encode_applies(uint32_t k, uint32_t m, bool dyadic) {
    if (!g_tune.enc_fixed) return false;
    return rs_encode23_applies(k, m) || (k == 8 && m == 4 && dyadic) || (k == 16 && m == 8) || (k == 20 && m == 10);
}

hipError_t launch_rs_encode_fixed(const EncodeArgs& a, hipStream_t s) {
    if (a.total == 0) return hipSuccess;
    if (rs_encode23_applies(a.k, a.m)) return launch_rs_encode23(a, s);
    if (a.k == 16 && a.m == 8) return enc_bits_dispatch<16, 8>(a, s);
    if (a.k == 20 && a.m == 10) return enc_bits_dispatch<20, 10>(a, s);
    if (a.k == 8 && a.m == 4 && a.dytabs) {
        // 3 workgroups per CU (knob enc_wpc; DESIGN.md 3: the flat grid at 3 beats 2, 4 and uncapped),
        // three of each workgroup's waves taking items (knob enc_ww): 9 working waves per CU with
        // the shard loads issued before the table staging and barrier, -1.1 / -1.3 / -1.1 % time
        // against four waves on three boxes (profiles/r06/enc_ww_ab_r06ww.log, _r06ww2,
        // enc_ww_stpol_ab_r06st.log); 2 working waves at 3 / 4
        // workgroups per CU +11 / +4 %
        const int grid = (int)((a.total + kThreads - 1) / kThreads);
        const size_t lds = occupancy_lds(g_tune.enc_wpc, (size_t)a.m * a.k * sizeof(gf::PermTab));
        // parity stored with sc1 (a.sp 1, encode_store_policy: the line leaves the XCD's L2; -1.4 to
        // -2.1 % time against nt stores on three boxes, profiles/r06/stpol_ab_*.log), or nt
        // (workgroups of 2 or 1 waves, residency in steps of 8 / 4 waves per CU: 2.49-2.67 ms against
        // 2.43 at 3 workgroups of 4 waves, profiles/r06/enc_nt_ab_r06h.log)
        if (a.sp == 1) {
            const int ww = g_tune.enc_ww;
            if (ww == 2 || ww == 3) {
                const int g2 = (int)((a.total + 64u * ww - 1) / (64u * ww));
                if (ww == 2)
                    hipLaunchKernelGGL((rs_encode_fixed_kernel<8, 4, 1, 2>), dim3(g2), dim3(kThreads), lds, s, a);
                else
                    hipLaunchKernelGGL((rs_encode_fixed_kernel<8, 4, 1, 3>), dim3(g2), dim3(kThreads), lds, s, a);
            } else {
                hipLaunchKernelGGL((rs_encode_fixed_kernel<8, 4, 1>), dim3(grid), dim3(kThreads), lds, s, a);
            }
        } else {
            hipLaunchKernelGGL((rs_encode_fixed_kernel<8, 4>), dim3(grid), dim3(kThreads), lds, s, a);
        }
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

}  // namespace fk
