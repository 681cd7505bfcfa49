// fec_decode.hip — RS reconstruct kernels for gfx950 (reed_solomon.go:124 ReconstructData):
// per-block plan (single parity row or Lagrange coefficients), the wave-private-plan rebuild
// (default for long shards), the workgroup-tile rebuild (short shards) and the fused form.
#include "fec_recon.hpp"

namespace fk {

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
        const uint32_t all = low_mask(n);
        const uint32_t mask = a.masks[b] & all;
        const uint32_t kmask = low_mask(k);   // k = 32 when m = 0
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
            const uint32_t R0 = __ffs(k < 32 ? mask >> k : 0u) - 1;
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
                         ? ld16<NTL>(slot_addr(dA, parity_base(pA, k, a.pss), sa, k, (uint32_t)a.ss, (uint32_t)a.pss))
                         : make_uint4(0, 0, 0, 0);
            xb[jj] = j0 + jj < k && noutB
                         ? ld16<NTL>(slot_addr(dB, parity_base(pB, k, a.pss), sb, k, (uint32_t)a.ss, (uint32_t)a.pss))
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
                tabs[i] = gf::make_permtab_fast(c);
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

// K: compile-time data shard count for the IPL = 1 body (0: runtime a.k); W > 0: that body with a
// rolling window of W loaded inputs (recon_item_roll) instead of all K up front.
template <int MAXE, int POL, bool FUSED, int IPL, int K = 0, int W = 0, bool RP = false>
__global__ __launch_bounds__(kThreads) void rs_reconstruct_wave_kernel(ReconArgs a) {
    constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    // blocks per wave slice: the rolling form is launched for shards of 64+ chunks only, where
    // 64 consecutive items span at most 2 blocks (smaller slices: more workgroups per CU)
    constexpr uint32_t WB = W > 0 ? 2u : kWaveBlocks;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (a.gate && *a.gate != a.gate_want) return;   // the classify kernel picked the direct path
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
        slice = smem + (size_t)wave * wave_slice_bytes(k, maxe, lay.stride, WB);
    }
    gf::PermTab* tabs = reinterpret_cast<gf::PermTab*>(slice);             // WB*maxe*k
    uint8_t* plans = slice + (size_t)WB * maxe * k * sizeof(gf::PermTab);  // WB*stride
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
        // the wave's (<= 3) masks in one load, then broadcast
        const uint32_t mine = lane < nb ? a.masks[bfirst + lane] : 0u;
        build_wave_plans(a, plans, bfirst, nb, lane, mine, s_exp, s_log, s_prows);
    }
    wave_sync();
    {
        // expand only the rows the blocks rebuild: entry i of c0 + c1 + c2 (c_g = nout_g * k)
        const uint32_t c0 = plans[lay.nout_off] * k;
        const uint32_t c1 = nb > 1 ? plans[lay.stride + lay.nout_off] * k : 0u;
        const uint32_t c2 = nb > 2 ? plans[2 * lay.stride + lay.nout_off] * k : 0u;
        const uint32_t kk = K > 0 ? (uint32_t)K : k;   // compile-time k: the division is a shift
        for (uint32_t i = lane; i < c0 + c1 + c2; i += 64) {
            const uint32_t g = (i >= c0) + (i >= c0 + c1);
            const uint32_t rem = i - (g == 0 ? 0u : g == 1 ? c0 : c0 + c1);
            const uint32_t r = rem / kk, j = rem - r * kk;
            const uint8_t* P = plans + g * lay.stride;
            tabs[g * maxe * k + rem] = gf::make_permtab_fast(P[lay.coef_off + r * k + j]);
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
            const uint32_t rb = a.sorted ? *reinterpret_cast<const uint32_t*>(P + lay.blk_off) : blk;
            if (nout) recon_item<MAXE, NTL, NTS>(a, P, tabs + g * maxe * k, rb, c, rows, nout);
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
        const uint32_t rb = a.sorted ? *reinterpret_cast<const uint32_t*>(P + lay.blk_off) : blk;
        if constexpr (K > 0 && W > 0)
            recon_item_roll<K, MAXE, W, NTL, NTS, RP>(a, P, tabs + g * maxe * k, rb, c, rows, nout);
        else if constexpr (K > 0) recon_item_k<K, MAXE, NTL, NTS>(a, P, tabs + g * maxe * k, rb, c, rows, nout);
        else recon_item<MAXE, NTL, NTS>(a, P, tabs + g * maxe * k, rb, c, rows, nout);
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
        const uint32_t rbA = a.sorted ? *reinterpret_cast<const uint32_t*>(PA + lay.blk_off) : bA;
        const uint32_t rbB = a.sorted ? *reinterpret_cast<const uint32_t*>(PB + lay.blk_off) : bB;
        recon_pair<MAXE, NTL, NTS>(a, PA, tabs + (bA - bfirst) * maxe * k, rbA, itA - bA * a.cps, rA, nA, PB,
                                   tabs + (bB - bfirst) * maxe * k, rbB, itB - bB * a.cps, rB, nB);
    }
}

// ------------------------------------------------------------------ tiered rebuild
// A wave's registers are sized for the largest row count its kernel can meet (RS(20,30): ten
// rebuilt rows, 208 VGPRs, 2 waves per SIMD), even when almost every wave rebuilds one or two
// rows. So the rebuild runs in two launches: tier A carries row bodies 1..RT only (RT = knob
// dec_tier), with a rolling load window, at more resident waves; a wave whose blocks rebuild
// more than RT rows goes on the worklist (a.hard, as the direct decode's hard waves) and a
// persistent tier-B launch with every row body rebuilds those waves. A single-erasure batch
// never reaches tier B (its grid finds an empty list and exits).
//
// One wave's rebuild of the 64 items from i0, plans from the (sorted) plan buffer: stage the
// blocks' records, expand the PermTabs of the rows they rebuild, one item per lane. RT > 0:
// waves needing more rows are deferred to the worklist instead.
template <int MAXE, int POL, int K, int W, int RT>
__device__ __forceinline__ void tier_wave(const ReconArgs& a, uint8_t* slice, uint32_t i0, uint32_t lane) {
    constexpr bool NTL = POL & 1, NTS = (POL & 2) != 0;
    constexpr uint32_t WB = W > 0 ? 2u : kWaveBlocks;
    // PermTab rows per block in the slice: tier A never expands more than RT
    const uint32_t k = K, maxe = RT > 0 ? (uint32_t)RT : a.maxe;
    const PlanLayout lay = a.lay;
    gf::PermTab* tabs = reinterpret_cast<gf::PermTab*>(slice);
    uint8_t* plans = slice + (size_t)WB * maxe * k * sizeof(gf::PermTab);
    const uint32_t total = a.nblocks * a.cps;
    const uint32_t bfirst = fdiv(i0, a.div_cps);
    const uint32_t nb = fdiv(min(i0 + 63u, total - 1u), a.div_cps) - bfirst + 1;   // <= WB
    {
        const uint32_t nw = nb * lay.stride / 16;
        const uint4* src = reinterpret_cast<const uint4*>(a.plans + (uint64_t)bfirst * lay.stride);
        if (lane < nw) reinterpret_cast<uint4*>(plans)[lane] = src[lane];
    }
    wave_sync();
    const uint32_t n0 = plans[lay.nout_off];
    const uint32_t n1 = nb > 1 ? plans[lay.stride + lay.nout_off] : 0u;
    const uint32_t n2 = (WB > 2 && nb > 2) ? plans[2 * lay.stride + lay.nout_off] : 0u;
    if constexpr (RT > 0) {
        if (max(n0, max(n1, n2)) > (uint32_t)RT) {   // wave-uniform: the whole wave goes to tier B
            if (lane == 0) {
                const uint32_t slot = atomicAdd(a.hard, 1u);
                if (slot < a.hard_cap) a.hard[kHardList + slot] = i0;
                else atomicOr(a.err, 4);   // never expected: the list holds one entry per wave
            }
            return;
        }
    }
    {
        // only the rows the blocks rebuild: entry i of c0 + c1 + c2 (c_g = nout_g * k)
        const uint32_t c0 = n0 * k, c1 = n1 * k, c2 = n2 * k;
        for (uint32_t i = lane; i < c0 + c1 + c2; i += 64) {
            const uint32_t g = (i >= c0) + (i >= c0 + c1);
            const uint32_t rem = i - (g == 0 ? 0u : g == 1 ? c0 : c0 + c1);
            const uint32_t r = rem / k, j = rem - r * k;
            const uint8_t* P = plans + g * lay.stride;
            tabs[g * maxe * k + rem] = gf::make_permtab_fast(P[lay.coef_off + r * k + j]);
        }
    }
    wave_sync();
    const uint32_t item = i0 + lane;
    const bool inr = item < total;
    const uint32_t blk = inr ? fdiv(item, a.div_cps) : bfirst;
    const uint32_t g = blk - bfirst;
    const uint32_t c = item - blk * a.cps;
    const uint8_t* P = plans + g * lay.stride;
    const uint32_t nout = inr ? P[lay.nout_off] : 0;
    const uint32_t rows = wave_rows<MAXE>(nout);
    if (nout == 0) return;
    const uint32_t rb = a.sorted ? *reinterpret_cast<const uint32_t*>(P + lay.blk_off) : blk;
    if constexpr (W > 0) recon_item_roll<K, MAXE, W, NTL, NTS>(a, P, tabs + g * maxe * k, rb, c, rows, nout);
    else recon_item_k<K, MAXE, NTL, NTS>(a, P, tabs + g * maxe * k, rb, c, rows, nout);
}

// Tier A: flat grid, one wave per 64 items, row bodies 1..RT.
template <int RT, int POL, int K, int W>
__global__ __launch_bounds__(kThreads) void rs_reconstruct_tier_kernel(ReconArgs a) {
    constexpr uint32_t WB = W > 0 ? 2u : kWaveBlocks;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (a.gate && *a.gate != a.gate_want) return;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* slice = smem + (size_t)wave * wave_slice_bytes(K, RT, a.lay.stride, WB);
    const uint32_t i0 = xcd_order(a.swz) * kThreads + (wave << 6);
    if (i0 >= a.nblocks * a.cps) return;
    tier_wave<RT, POL, K, W, RT>(a, slice, i0, lane);
}

// Tier B: a persistent grid of waves takes the deferred waves in turn, every row body; with an
// empty list every wave exits at once. The last workgroup to finish rewinds the list.
template <int MAXE, int POL, int K, int W>
__global__ __launch_bounds__(kThreads) void rs_reconstruct_list_kernel(ReconArgs a) {
    constexpr uint32_t WB = W > 0 ? 2u : kWaveBlocks;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* slice = smem + (size_t)wave * wave_slice_bytes(K, a.maxe, a.lay.stride, WB);
    const uint32_t count = min(__hip_atomic_load(a.hard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), a.hard_cap);
    const uint32_t nw = gridDim.x * (kThreads / 64);
    for (uint32_t t = blockIdx.x * (kThreads / 64) + wave; t < count; t += nw) {
        wave_sync();   // the previous wave's reads of the slice are done
        tier_wave<MAXE, POL, K, W, 0>(a, slice, a.hard[kHardList + t], lane);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(a.hard + kHardDone, 1u) == gridDim.x - 1) {
            atomicExch(a.hard, 0u);
            atomicExch(a.hard + kHardDone, 0u);
        }
    }
}

template <int K, int MAXE, int WA, int WB_, int POL>
static hipError_t tier_launch(const ReconArgs& a, uint32_t rt, hipStream_t s) {
    const uint64_t total = (uint64_t)a.nblocks * a.cps;
    const int grid = (int)((total + kThreads - 1) / kThreads);
    if (grid == 0) return hipSuccess;
    const size_t ldsB = 4 * wave_slice_bytes(K, a.maxe, a.lay.stride, WB_ > 0 ? 2 : 3);
#define FEC_TIER_A(R)                                                                                          \
    hipLaunchKernelGGL((rs_reconstruct_tier_kernel<R, POL, K, WA>), dim3(grid), dim3(kThreads),                \
                       occupancy_lds(g_tune.dec_wpc, 4 * wave_slice_bytes(K, R, a.lay.stride, WA > 0 ? 2 : 3)), s, \
                       a)
    if (rt <= 1) FEC_TIER_A(1);
    else if (rt <= 2) FEC_TIER_A(2);
    else FEC_TIER_A(4);
#undef FEC_TIER_A
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const void* fb = (const void*)rs_reconstruct_list_kernel<MAXE, POL, K, WB_>;
    const int gridB = std::max<int>(1, (int)a.list_grid / 4) * resident_per_cu(fb, ldsB);   // list_grid: 4 x CUs
    hipLaunchKernelGGL((rs_reconstruct_list_kernel<MAXE, POL, K, WB_>), dim3(gridB), dim3(kThreads), ldsB, s, a);
    return hipGetLastError();
}

bool tier_recon_applies(uint32_t k, uint32_t maxe, uint32_t cps) {
    return g_tune.dec_tier > 0 && g_tune.dec_fixk && (g_tune.dec_nt & 3) && cps >= 64 &&
           ((k == 16 && maxe == 8) || (k == 20 && maxe == 10));
}

hipError_t launch_rs_reconstruct_tiered(const ReconArgs& a, hipStream_t s) {
    const uint32_t rt = (uint32_t)g_tune.dec_tier;
    if (a.k == 16) return tier_launch<16, 8, 8, 8, 3>(a, rt, s);
    return tier_launch<20, 16, 8, 0, 3>(a, rt, s);
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
// (4 wave slices per workgroup) fits a workgroup (gfx950: 160 KiB; RS(20,30) needs 80 KiB).
bool wave_recon_applies(uint32_t cps, uint32_t k, uint32_t maxe, uint32_t stride) {
    return g_tune.dec_wave && cps >= 32 && 4 * fused_slice_bytes(k, maxe, stride) + 2048 <= g_max_lds;
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
    // the benchmark's multi-erasure code RS(16,24) with its K known at compile time
    if constexpr (IPL == 1 && !FUSED) {
        // rolling load window (dec_fixk 2): 120 instead of 163 VGPRs and 2-block wave slices, so
        // 4 instead of 3 workgroups per CU; RS(16,24) +1.7 % (dec_select.py, interleaved A/B)
        // (dec_fixk 4, fec_rebuild.hip, falls back here for plain loads / stores: the window form)
        const bool roll = (g_tune.dec_fixk == 2 || g_tune.dec_fixk == 4) && a.cps >= 64;
        const size_t lds2 = occupancy_lds(g_tune.dec_wpc, 4 * wave_slice_bytes(a.k, a.maxe, a.lay.stride, 2));
        // (always flat: wrapped in a persistent loop for gated launches, these bodies lost their
        // register allocation, K = 20 248 VGPRs + 408 B/lane of scratch, 3.5x slower, r03h)
#define FEC_K_LAUNCH(KERN, L) hipLaunchKernelGGL(KERN, dim3(grid), dim3(kThreads), L, s, a)
        if (a.k == 16 && a.maxe == 8 && g_tune.dec_fixk) {
            if (roll && g_tune.dec_fixk == 3)   // 130 VGPRs, 3 waves/SIMD: -2.6 % here (r03f)
                FEC_K_LAUNCH((rs_reconstruct_wave_kernel<8, POL, false, 1, 16, 8, true>), lds2);
            else if (roll)
                FEC_K_LAUNCH((rs_reconstruct_wave_kernel<8, POL, false, 1, 16, 8>), lds2);
            else
                FEC_K_LAUNCH((rs_reconstruct_wave_kernel<8, POL, false, 1, 16>), lds);
            return hipGetLastError();
        }
        // the reference's own receiver code RS(20,30) (manager.go:80-90)
        if (a.k == 20 && a.maxe == 10 && g_tune.dec_fixk) {
            // rolling window + row-pipelined table reads (and no switch-prefix hoisting): 208 -> 141
            // VGPRs, 3 instead of 2 waves/SIMD, +15 % (dec_select.py r03f: 4056 -> 3528 us for
            // 2^19 blocks, e ~ U{1..10}); the window alone measured -0.8 % (203 VGPRs)
            if (g_tune.dec_fixk >= 2 && a.cps >= 64)
                FEC_K_LAUNCH((rs_reconstruct_wave_kernel<16, POL, false, 1, 20, 8, true>), lds2);
            else
                FEC_K_LAUNCH((rs_reconstruct_wave_kernel<16, POL, false, 1, 20>), lds);
            return hipGetLastError();
        }
#undef FEC_K_LAUNCH
    }
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
    // cache policy: plain, or non-temporal loads and stores (the mixed forms measured no better)
    return (g_tune.dec_nt & 3) ? recon_wave_ipl<3, false>(a, s) : recon_wave_ipl<0, false>(a, s);
}

hipError_t launch_rs_recover_fused(const ReconArgs& a, hipStream_t s) {
    return (g_tune.dec_nt & 3) ? recon_wave_ipl<3, true>(a, s) : recon_wave_ipl<0, true>(a, s);
}

hipError_t launch_rs_reconstruct(const ReconArgs& a, int grid, hipStream_t s) {
    return (g_tune.dec_nt & 3) ? recon_dispatch<3>(a, grid, s) : recon_dispatch<0>(a, grid, s);
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

const void* recon_occupancy_kernel(uint32_t sel) {
    if (sel <= 1) return (const void*)rs_reconstruct_kernel<1, 3>;
    if (sel <= 2) return (const void*)rs_reconstruct_kernel<2, 3>;
    if (sel <= 4) return (const void*)rs_reconstruct_kernel<4, 3>;
    if (sel <= 8) return (const void*)rs_reconstruct_kernel<8, 3>;
    return (const void*)rs_reconstruct_kernel<16, 3>;
}

}  // namespace fk
