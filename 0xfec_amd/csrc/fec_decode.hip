// fec_decode.hip — RS reconstruct kernels for gfx950 (reed_solomon.go:124 ReconstructData):
// per-block plan in block order (single parity row or Lagrange coefficients), the wave-private-plan
// rebuild (shards of 32+ chunks, sorted plans from fec_plan.hip) and the workgroup-tile rebuild
// (short shards).
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
            wave_flag(a.err, 1);
        } else if (a.max_out && e > a.max_out) {
            P[lay.nout_off] = 0;
            st = -1;  // FEC_ERR_INVALID_ARG: more erasures than output slots
            wave_flag(a.err, 2);
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
// Tile form: a workgroup takes tiles of G consecutive blocks: it stages their plans in LDS,
// expands every coefficient to its PermTab once, then lanes sweep the G*cps (block, chunk)
// items. Rows beyond a block's own erasure count carry zero tables, and each item loops only
// to the wave's largest erasure count (ballot), so one-erasure batches do one row of work.
// Used for short shards (fewer than 32 chunks: many blocks per wave). One tile per workgroup.
template <int MAXE>
__global__ __launch_bounds__(kThreads) void rs_reconstruct_kernel(ReconArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t k = a.k, G = a.g, maxe = a.maxe;
    const PlanLayout lay = a.lay;
    gf::PermTab* tabs = reinterpret_cast<gf::PermTab*>(smem);                // G*maxe*k
    uint8_t* plans = smem + (size_t)G * maxe * k * sizeof(gf::PermTab);      // G*stride
    for (uint32_t tile = xcd_order(); tile < a.ntiles; tile += gridDim.x) {
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
            const uint32_t c = t - g * a.cps;
            const uint8_t* P = plans + g * lay.stride;
            const uint32_t nout = inr ? P[lay.nout_off] : 0;
            const uint32_t rows = wave_rows<MAXE>(nout);
            if (nout == 0) continue;
            recon_item<MAXE>(a, P, tabs + g * maxe * k, b0 + g, c, rows, nout);
        }
    }
}

// Wave form (shards of 32+ chunks): one wave per 64 consecutive items of the sorted plan order
// (the body, wave_body, is in fec_recon.hpp).
template <int MAXE, int K = 0>
__global__ __launch_bounds__(kThreads) void rs_reconstruct_wave_kernel(ReconArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    wave_body<MAXE, K>(a, smem, xcd_order());
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

hipError_t launch_rs_reconstruct(const ReconArgs& a, int grid, hipStream_t s) {
    const size_t lds = occupancy_lds(g_tune.dec_wpc, recon_lds_bytes(a.g, a.k, a.maxe, a.lay));
    if (a.maxe <= 1) hipLaunchKernelGGL((rs_reconstruct_kernel<1>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (a.maxe <= 2) hipLaunchKernelGGL((rs_reconstruct_kernel<2>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (a.maxe <= 4) hipLaunchKernelGGL((rs_reconstruct_kernel<4>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (a.maxe <= 8) hipLaunchKernelGGL((rs_reconstruct_kernel<8>), dim3(grid), dim3(kThreads), lds, s, a);
    else hipLaunchKernelGGL((rs_reconstruct_kernel<16>), dim3(grid), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

// The wave form applies to shards of 32+ chunks (at most 3 blocks per wave) while its LDS
// (4 wave slices per workgroup) fits a workgroup (gfx950: 160 KiB; RS(20,30) needs 80 KiB).
bool wave_recon_applies(uint32_t cps, uint32_t k, uint32_t maxe, uint32_t stride) {
    return g_tune.dec_wave && cps >= 32 && 4 * wave_slice_bytes(k, maxe, stride) + 2048 <= g_max_lds;
}

hipError_t launch_rs_reconstruct_wave(const ReconArgs& a, hipStream_t s) {
    const int grid = (int)(((uint64_t)a.nblocks * a.cps + kThreads - 1) / kThreads);
    if (grid == 0) return hipSuccess;
    const size_t lds = occupancy_lds(g_tune.dec_wpc, 4 * wave_slice_bytes(a.k, a.maxe, a.lay.stride));
#define FEC_WAVE_LAUNCH(...) hipLaunchKernelGGL((rs_reconstruct_wave_kernel<__VA_ARGS__>), dim3(grid), dim3(kThreads), lds, s, a)
    // the benchmark's multi-erasure code RS(16,24) and the reference's own RS(20,30)
    // (manager.go:80-90) with k at compile time; with shards of 64+ chunks both run
    // rs_rebuild_k_kernel (fec_rebuild.hip) instead
    if (a.k == 16 && a.maxe == 8) FEC_WAVE_LAUNCH(8, 16);
    else if (a.k == 20 && a.maxe == 10) FEC_WAVE_LAUNCH(16, 20);
    else if (a.maxe <= 1) FEC_WAVE_LAUNCH(1);
    else if (a.maxe <= 2) FEC_WAVE_LAUNCH(2);
    else if (a.maxe <= 4) FEC_WAVE_LAUNCH(4);
    else if (a.maxe <= 8) FEC_WAVE_LAUNCH(8);
    else FEC_WAVE_LAUNCH(16);
#undef FEC_WAVE_LAUNCH
    return hipGetLastError();
}

uint32_t pick_tile_blocks(uint32_t cps, uint32_t k, uint32_t maxe, const PlanLayout& lay) {
    // Blocks per tile: the smallest count that reaches the best lane utilisation of the G*cps
    // items over 256 lanes within 8 rounds, bounded by 48 KiB of LDS.
    constexpr uint32_t kMaxRounds = 8;
    const size_t per_block = recon_lds_bytes(1, k, maxe, lay);
    uint32_t gmax = (uint32_t)((48u * 1024u) / per_block);
    if (gmax < 1) gmax = 1;
    if (gmax > 256) gmax = 256;
    uint32_t best = 1;
    double best_u = -1.0;
    for (uint32_t g = 1; g <= gmax; ++g) {
        const uint32_t items = g * cps;
        const uint32_t rounds = (items + kThreads - 1) / kThreads;
        if (rounds > kMaxRounds && g > 1) break;
        const double u = (double)items / (double)(rounds * kThreads);
        if (u > best_u + 1e-3) {
            best = g;
            best_u = u;
        }
    }
    return best;
}

}  // namespace fk
