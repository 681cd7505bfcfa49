// fec_recover.hip — direct RS reconstruct for gfx950 (reed_solomon.go:124 ReconstructData, and the
// copy-out of recoverSymbolPayloads, :126-135), for codes whose single-erasure coefficient tables
// are small (k*m*k PermTabs <= 16 KiB: RS(2,3), RS(8,12), ...).
//
// A block with one erased data shard E0 is rebuilt from the first k present shards in index
// order — the k-1 other data shards and the first present parity R0 — with the coefficients of
// parity row R0 (x_E0 = inv(A[R0][E0]) * (p_R0 ^ sum_j A[R0][j] x_j)). Those coefficients depend
// on (E0, R0) only, so every one of the k*m plans is expanded to PermTabs once per code on the
// host (a table of k*m*k*32 bytes that stays in L2): a lane reads its block's present mask,
// derives (E0, R0) and its input slots from it with a few scalar-width ops and issues its k loads
// straight away, while its wave copies the <= 3 table rows it needs into LDS. No plan kernel, no
// plan records in HBM, no PermTab expansion on the device.
//
// The direct form serves calls where no block can need a multi-erasure rebuild: one output
// slot per block, or one parity shard (m = 1: two erasures leave too few shards). A block with
// more erasures than that is an error the kernel reports itself. Multi-slot and in-place calls
// of the codes with m >= 2 take the sorted-plan route (fec_plan.hip + fec_decode.hip) instead:
// on batches with multi-erasure blocks mixed in, a direct kernel that handed such waves to a
// second, multi-erasure kernel ran at half that route's rate, and on single-erasure batches
// gained only 2.4 % over it (round 5, profiles/r05/mixed_route_*_r05g.log).
#include <string.h>

#include <algorithm>

#include "fec_recon.hpp"

namespace fk {

// LDS of one direct wave (4 per workgroup, no workgroup-level staging, no barrier): the PermTab
// rows of its <= 3 blocks.
__host__ __device__ inline size_t direct_wave_bytes(uint32_t k) { return (size_t)kWaveBlocks * k * sizeof(gf::PermTab); }

constexpr size_t kDirectTableBytes = 16 * 1024;

// The fetched 16-byte table pieces of a wave (NT per lane) into its LDS rows, then a wave barrier.
template <int NT>
__device__ __forceinline__ void rows_to_lds(gf::PermTab* wt, const uint4 (&tv)[NT], uint32_t lane, uint32_t n) {
    uint4* w = reinterpret_cast<uint4*>(wt);
#pragma unroll
    for (int q = 0; q < NT; ++q)
        if (lane + 64u * q < n) w[lane + 64u * q] = tv[q];
    wave_sync();
}

// The single-erasure coefficient bytes of a small code ((k*m) rows of ceil(k/4) dwords), passed
// by value: the kernel reads them from its argument segment with scalar loads.
constexpr uint32_t kCoefWords = 128;
struct CoefWords {
    uint32_t w[kCoefWords];
};

// Statuses (recover: e rebuilt; in place: 0; failures as rs_plan_kernel reports them) and failure
// flags of blocks [64 w, 64 w + 64), w = the calling wave's launch index: one coalesced mask load
// and one coalesced status store per 64 blocks. (Stored by the waves of each block, the 4-byte
// statuses of neighbouring blocks were scattered partial-line stores from different waves: RS(2,3)
// 45 -> 57 us with a status array.)
__device__ __forceinline__ void direct_status_pass(const ReconArgs& a, uint32_t k, uint32_t w, uint32_t lane) {
    if (w * 64u >= a.nblocks) return;   // wave-uniform
    const uint32_t all = low_mask(k + a.m), kmask = low_mask(k);
    const uint32_t b = w * 64u + lane;
    uint32_t bad = 0;
    if (b < a.nblocks) {
        const uint32_t mask = a.masks[b] & all;
        const uint32_t e = k - __popc(mask & kmask);
        int32_t st = a.max_out ? (int32_t)e : 0;
        if (e != 0 && (uint32_t)__popc(mask) < k) {
            st = -4;   // FEC_ERR_TOO_FEW_SHARDS
            bad = 1;
        } else if (a.max_out && e > a.max_out) {
            st = -1;   // FEC_ERR_INVALID_ARG: more erasures than output slots
            bad = 2;
        }
        if (a.status) a.status[b] = st;
    }
    const bool f1 = __ballot(bad == 1) != 0, f2 = __ballot(bad == 2) != 0;
    if (lane == 0 && (f1 || f2)) atomicOr(a.err, (f1 ? 1 : 0) | (f2 ? 2 : 0));
}

// K: compile-time data shard count (0: runtime a.k). TAB: how a wave gets the PermTabs of its
// blocks' rows: 0 copies them from the code's PermTab table (one vector load per wave, L1/L2
// hits); 1 reads the rows' coefficient bytes from the kernel arguments (scalar loads, off the
// vector memory path) and expands them on the lanes (gf::make_permtab); 2 as 1 with the bytes
// read from the code's coefficient table in device memory (a.single_coef, through the constant
// address space: scalar loads), for codes whose rows do not fit the argument (RS(20,30): 1000
// dwords).
// WW: waves of the workgroup that take items (4: all; fewer: the others exit at once and the
// workgroup covers WW * 64 items).
template <int K, int TAB, int SP = 0, int WW = 4>
__device__ __forceinline__ void direct_body(const ReconArgs& a, const CoefWords& cwords, uint8_t* smem) {
    constexpr bool NTL = true, NTS = true;   // non-temporal loads and stores (see launch_rs_recover_direct)
    {
        const uint32_t vb = blockIdx.x;
        const uint32_t k = K ? (uint32_t)K : a.k, m = a.m;
        const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        if (WW < kThreads / 64 && wave >= (uint32_t)WW) return;
        uint8_t* slice = smem + (size_t)wave * direct_wave_bytes(k);
        const uint32_t total = a.nblocks * a.cps;
        const uint32_t all = low_mask(k + m), kmask = low_mask(k);
        direct_status_pass(a, k, vb * WW + wave, lane);
        const uint32_t i0 = xcd_order() * (WW * 64u) + (wave << 6);
        if (i0 >= total) return;
        const uint32_t bfirst = fdiv(i0, a.div_cps);
        const uint32_t nb = fdiv(min(i0 + 63u, total - 1u), a.div_cps) - bfirst + 1;   // <= 3
        // The wave's <= 3 masks by scalar loads (wave-uniform addresses, the constant cache), which
        // the scalar unit turns into shard addresses while the vector memory path is free: a
        // vector load of the masks put a dependent vector round trip in front of every wave's
        // shard loads (decode twin at 4 workgroups/CU: 5.73 TB/s with a vector mask load, 5.84
        // with scalar ones, 5.85 with no mask at all; with the field arithmetic 5.70 / 5.83 /
        // 5.87; profiles/r05/dec_twin_r05b.log)
        const WaveMasks wm = wave_masks(a.masks, bfirst, a.nblocks);
        auto mask_of = [&](uint32_t g) { return wm.of(g); };   // g < nb

        // Per block (uniform): the table row (E0 * m + R0) of a single-erasure block.
        uint32_t row[kWaveBlocks] = {0, 0, 0};
        bool any = false;
    #pragma unroll
        for (uint32_t g = 0; g < kWaveBlocks; ++g) {
            if (g >= nb) break;
            const uint32_t mask = mask_of(g) & all;
            const uint32_t e = k - __popc(mask & kmask);
            if (e == 1 && (uint32_t)__popc(mask) >= k && !(a.max_out && e > a.max_out)) {
                row[g] = (__ffs(~mask & kmask) - 1) * m + (__ffs(mask >> k) - 1);   // m >= 1 here: k < 32
                any = true;
            }
        }
        // a wave none of whose blocks has one erased data shard (nothing erased, or failed) issues
        // no loads (wave-uniform: the masks are scalar)
        if (!any) return;
        // The PermTab rows of the wave's blocks into its LDS slice, prepared while the data loads are
        // in flight (vector loads return in order: LDS writes that wait for a row load wait for that
        // load only, and scalar loads are counted apart).
        gf::PermTab* wt = reinterpret_cast<gf::PermTab*>(slice);
        // TAB 0: pieces per lane: 3 blocks * 2k 16-byte pieces (<= 64 for k <= 10, the compile-time shapes)
        constexpr int NT = (K > 0 && K <= 10) ? 1 : 3;
        uint4 tv[NT];
        if constexpr (TAB == 0) {
            // unconditional loads (a lane past the wave's pieces re-reads a valid piece): no branch,
            // so nothing makes the compiler wait for them before the data loads
            const uint4* src = reinterpret_cast<const uint4*>(a.single);
            const uint32_t np = nb * 2 * k;
    #pragma unroll
            for (int q = 0; q < NT; ++q) {
                const uint32_t t = min(lane + 64u * q, np - 1u);
                const uint32_t g = t / (2 * k), r = t - g * 2 * k;
                const uint32_t rw = g == 0 ? row[0] : g == 1 ? row[1] : row[2];
                tv[q] = src[(size_t)rw * 2 * k + r];
            }
        }
        // TAB 1: the rows' coefficient words by scalar loads (uniform addresses, constant cache), then
        // lane l < nb*k expands coefficient j = l % k of block g = l / k into wt[l]
        constexpr uint32_t KW = K > 0 ? (K + 3) / 4 : 8;   // coefficient dwords per row (k <= 32)
        uint32_t cw[kWaveBlocks][KW];
        if constexpr (TAB >= 1) {
            // a kernel argument, or device memory read as constant: scalar loads either way
            typedef __attribute__((address_space(4))) const uint32_t ConstU32;
            ConstU32* ct = TAB == 1 ? (ConstU32*)cwords.w : (ConstU32*)a.single_coef;
            const uint32_t kw = (k + 3) / 4;
    #pragma unroll
            for (uint32_t g = 0; g < kWaveBlocks; ++g)
    #pragma unroll
                for (uint32_t q = 0; q < KW; ++q) {
                    // the index is wave-uniform; readfirstlane makes that visible, so the load is scalar
                    const uint32_t at = (uint32_t)__builtin_amdgcn_readfirstlane((int)(row[g] * kw + q));
                    cw[g][q] = q < kw ? ct[at] : 0u;
                }
        }
        auto expand_rows = [&]() {
            for (uint32_t l = lane; l < nb * k; l += 64) {
                const uint32_t lg = l / k, lj = l - lg * k;
                uint32_t coef = 0;
    #pragma unroll
                for (uint32_t g = 0; g < kWaveBlocks; ++g)
    #pragma unroll
                    for (uint32_t q = 0; q < KW; ++q)
                        if (lg == g && (lj >> 2) == q) coef = (cw[g][q] >> (8 * (lj & 3))) & 0xFFu;
                wt[l] = gf::make_permtab((uint8_t)coef);   // the lane form measured 0-1 % slower here
            }
            wave_sync();
        };
        const uint32_t item = i0 + lane;
        const bool inr = item < total;
        const uint32_t blk = inr ? fdiv(item, a.div_cps) : bfirst;
        const uint32_t g = blk - bfirst;
        const uint32_t c = item - blk * a.cps;
        const uint32_t mask = mask_of(g) & all;
        const bool work = inr && k - __popc(mask & kmask) == 1 && (uint32_t)__popc(mask) >= k;
        const uint32_t E0 = __ffs(~mask & kmask) - 1;
        const uint32_t R0 = work ? __ffs(mask >> k) - 1 : 0;
        const gf::PermTab* T = wt + g * k;
        const uint8_t* dblk = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
        const uint8_t* par = a.parity + (uint64_t)blk * a.pbs + (uint64_t)R0 * a.pss + (uint64_t)c * kChunk;
        uint32_t acc[4] = {0, 0, 0, 0};
        if constexpr (K > 0) {
            // unconditional loads (a lane with nothing to rebuild reads one L2-resident table line
            // instead): no branch around them, so the row pieces' LDS writes wait for the row loads
            // only (vmcnt counts in order), not for the data
            const uint8_t* idle = reinterpret_cast<const uint8_t*>(TAB == 2 ? a.single_coef : a.single);
            const uint64_t ss = work ? a.ss : 0;
            const uint8_t* d0 = work ? dblk : idle;
            const uint8_t* p0 = work ? par : idle;
            uint4 x[K];
    #pragma unroll
            for (int j = 0; j < K - 1; ++j) x[j] = ld16<NTL>(d0 + (uint64_t)(j + (j >= (int)E0)) * ss);
            x[K - 1] = ld16<NTL>(p0);
            if constexpr (TAB == 0) rows_to_lds(wt, tv, lane, nb * 2 * k);
            else expand_rows();
            if (!work) return;
    #pragma unroll
            for (int j = 0; j < K; j += 2) {
                Idx ia[4], ib[4];
                split4(ia, x[j]);
                if (j + 1 < K) {
                    split4(ib, x[j + 1]);
                    mac2(acc, ia, ib, T + j, T + j + 1);
                } else {
                    mac1(acc, ia, T + j);
                }
            }
        } else {
            if constexpr (TAB == 0) rows_to_lds(wt, tv, lane, nb * 2 * k);
            else expand_rows();
            if (!work) return;
            for (uint32_t j0 = 0; j0 < k; j0 += kInGroup) {
                uint4 x[kInGroup];
    #pragma unroll
                for (int jj = 0; jj < kInGroup; ++jj) {
                    const uint32_t j = j0 + jj;
                    x[jj] = j + 1 < k ? ld16<NTL>(dblk + (uint64_t)(j + (j >= E0)) * a.ss)
                                      : (j + 1 == k ? ld16<NTL>(par) : make_uint4(0, 0, 0, 0));
                }
    #pragma unroll
                for (int jj = 0; jj < kInGroup; jj += 2) {
                    const uint32_t j = j0 + jj;
                    if (j + 1 < k) {
                        Idx ia[4], ib[4];
                        split4(ia, x[jj]);
                        split4(ib, x[jj + 1]);
                        mac2(acc, ia, ib, T + j, T + j + 1);
                    } else if (j < k) {
                        Idx ia[4];
                        split4(ia, x[jj]);
                        mac1(acc, ia, T + j);
                    }
                }
            }
        }
        uint8_t* dst = a.out ? a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk
                             : const_cast<uint8_t*>(dblk) + (uint64_t)E0 * a.ss;
        const uint32_t nbytes = a.len - c * kChunk;
        if constexpr (SP == 0) store_chunk<NTS>(dst, as_uint4(acc), nbytes);
        else st16p<SP>(dst, nbytes >= 16 ? as_uint4(acc) : keep_bytes(as_uint4(acc), nbytes));
    }
}

template <int K, int TAB, int SP = 0>
__global__ __launch_bounds__(kThreads) void rs_recover_direct_kernel(ReconArgs a, CoefWords cwords) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    direct_body<K, TAB, SP>(a, cwords, smem);
}

// ------------------------------------------------------------------ routed in-place reconstruct
// In-place calls (fec_rs_reconstruct_batch) of RS(8,12) cannot know before the kernels run whether
// a block has two or more erased data shards: the masks are device memory. A classify pass reduces
// the masks to one word (route: nonzero if some recoverable block has >= 2 erased data shards); the
// sorted plan kernel then exits at once when it is zero, and this kernel runs the direct
// single-erasure body (no plan records) when it is zero and the wave rebuild of the sorted plans
// when it is not: one launch of the flat grid either way, no empty grid on either route.
// One workgroup per CU sweeps the masks; a workgroup that finds such a block sets the word with one
// atomic (an atomic per wave on one address, 8192 of them on a mixed 2^20-block batch, serialised
// at L2 for ~90 us).
__global__ __launch_bounds__(256) void rs_route_classify_kernel(const uint32_t* masks, uint32_t nblocks, uint32_t k,
                                                                 uint32_t m, uint32_t* route) {
    __shared__ uint32_t found;
    if (threadIdx.x == 0) found = 0;
    __syncthreads();
    const uint32_t all = low_mask(k + m), kmask = low_mask(k);
    bool multi = false;
    for (uint32_t b = blockIdx.x * 256u + threadIdx.x; b < nblocks; b += gridDim.x * 256u) {
        const uint32_t mask = masks[b] & all;
        multi |= k - __popc(mask & kmask) >= 2 && (uint32_t)__popc(mask) >= k;
    }
    if (__ballot(multi) != 0 && __lane_id() == 0) found = 1;   // plain LDS store: any writer wins
    __syncthreads();
    if (threadIdx.x == 0 && found) atomicOr(route, 1u);
}

// WW < 4 (knob route_ww): the direct route runs WW waves of each workgroup over a grid of
// total / (WW * 64) workgroups; the plan route runs the first total / 256 of them, all four waves
// each, in XCD order among themselves, and the rest exit at once.
template <int MAXE, int DK, int TAB, int SP, int WW = 4>
__global__ __launch_bounds__(kThreads) void rs_reconstruct_routed_kernel(ReconArgs a, CoefWords cwords) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    typedef __attribute__((address_space(4))) const uint32_t ConstU32;
    if (*(ConstU32*)a.route == 0) {
        direct_body<DK, TAB, SP, WW>(a, cwords, smem);
    } else if constexpr (WW == kThreads / 64) {
        wave_body<MAXE, 0>(a, smem, xcd_order());
    } else {
        const uint32_t g4 = (a.nblocks * a.cps + kThreads - 1) / kThreads;
        if (blockIdx.x >= g4) return;
        wave_body<MAXE, 0>(a, smem, xcd_order_of(blockIdx.x, g4));
    }
}

// RS(2,3) (k = 2, m = 1): a block is rebuilt from its other data shard and the parity with the
// two coefficients of its erased shard's row, x_E0 = c[E0][0] * x_other ^ c[E0][1] * p. Both rows'
// PermTabs (4 x 32 bytes) arrive as a kernel argument, so a lane picks its row's words from scalar
// registers with v_cndmask: no LDS, no wave barrier and no per-wave table expansion between the
// two shard loads and the store (the general kernel's <2, 1> form expands 2 rows per block on the
// lanes and synchronises the wave before the products).
struct K2Rows {
    gf::PermTab t[2][2];   // [E0][input: 0 the other data shard, 1 the parity]
};

__global__ __launch_bounds__(kThreads) void rs_recover_k2m1_kernel(ReconArgs a, K2Rows rows) {
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t total = a.nblocks * a.cps;
    direct_status_pass(a, 2, blockIdx.x * (kThreads / 64) + wave, lane);
    const uint32_t i0 = xcd_order() * kThreads + (wave << 6);
    if (i0 >= total) return;
    const uint32_t bfirst = fdiv(i0, a.div_cps);
    const WaveMasks wm = wave_masks(a.masks, bfirst, a.nblocks);
    const uint32_t item = i0 + lane;
    if (item >= total) return;
    const uint32_t blk = fdiv(item, a.div_cps), c = item - blk * a.cps;
    const uint32_t mask = wm.of(blk - bfirst) & 7u;
    // one data shard lost and the parity present (6: x0 lost, 5: x1 lost); any other mask has
    // nothing to rebuild or too few shards (the status pass reports those)
    if (mask != 5u && mask != 6u) return;
    const bool e1 = mask == 5u;
    const uint8_t* dblk = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    const uint4 x = ld16<true>(dblk + (e1 ? 0 : a.ss));
    const uint4 p = ld16<true>(a.parity + (uint64_t)blk * a.pbs + (uint64_t)c * kChunk);
    const gf::PermTab &ta0 = rows.t[0][0], &ta1 = rows.t[1][0], &tb0 = rows.t[0][1], &tb1 = rows.t[1][1];
    const uint4 la = make_uint4(e1 ? ta1.t0lo : ta0.t0lo, e1 ? ta1.t0hi : ta0.t0hi, e1 ? ta1.t1lo : ta0.t1lo,
                                e1 ? ta1.t1hi : ta0.t1hi);
    const uint4 lb = make_uint4(e1 ? tb1.t0lo : tb0.t0lo, e1 ? tb1.t0hi : tb0.t0hi, e1 ? tb1.t1lo : tb0.t1lo,
                                e1 ? tb1.t1hi : tb0.t1hi);
    const uint32_t a2 = e1 ? ta1.t2 : ta0.t2, b2 = e1 ? tb1.t2 : tb0.t2;
    Idx ia[4], ib[4];
    split4(ia, x);
    split4(ib, p);
    uint32_t acc[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const Prod3 u = gprod(ia[d], la, a2), v = gprod(ib[d], lb, b2);
        acc[d] = xor3(xor3(u.p0, u.p1, u.p2), v.p0, v.p1) ^ v.p2;
    }
    uint8_t* dst = a.out ? a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk
                         : const_cast<uint8_t*>(dblk) + (e1 ? a.ss : 0);
    store_chunk<true>(dst, as_uint4(acc), a.len - c * kChunk);
}

size_t direct_table_words(uint32_t k, uint32_t m) { return (size_t)k * m * k * 8; }

bool direct_recon_applies(uint32_t k, uint32_t m, uint32_t cps, bool single_slot) {
    if (!g_tune.dec_direct || m == 0 || k + m > 32 || cps < 32) return false;
    // only where no block can need a multi-erasure rebuild (one output slot, or one parity shard:
    // more erasures are an error the kernel reports itself; see the top of this file), for small
    // codes (their PermTab table fits) and RS(20,30) / RS(16,24) with their rows read from device
    // memory
    if (!single_slot && m != 1) return false;
    const bool small = (size_t)k * m * k * sizeof(gf::PermTab) <= kDirectTableBytes;
    const bool big = (k == 20 && m == 10) || (k == 16 && m == 8);
    return (small || big) && 4 * direct_wave_bytes(k) <= g_max_lds;
}

bool routed_recon_applies(uint32_t k, uint32_t m, uint32_t cps, uint32_t maxe, uint32_t stride) {
    // RS(8,12)-shaped codes in place (the headline code: the direct body with k at compile time and
    // its rows from the kernel argument), when the wave rebuild serves their plan route
    return g_tune.dec_route && g_tune.dec_direct == 1 && k == 8 && m >= 2 && maxe <= 8 &&
           (size_t)k * m * ((k + 3) / 4) <= kCoefWords && (size_t)k * m * k * sizeof(gf::PermTab) <= kDirectTableBytes &&
           wave_recon_applies(cps, k, maxe, stride);
}

hipError_t launch_rs_route_classify(const ReconArgs& a, uint32_t* route, hipStream_t s) {
    if (a.nblocks == 0) return hipSuccess;
    if (hipMemsetAsync(route, 0, 4, s) != hipSuccess) return hipGetLastError();
    const int grid = (int)std::min<uint64_t>(256, ((uint64_t)a.nblocks + 255) / 256);
    hipLaunchKernelGGL(rs_route_classify_kernel, dim3(grid), dim3(256), 0, s, a.masks, a.nblocks, a.k, a.m, route);
    return hipGetLastError();
}

hipError_t launch_rs_reconstruct_routed(const ReconArgs& a, hipStream_t s) {
    const uint64_t total = (uint64_t)a.nblocks * a.cps;
    const bool w3 = g_tune.route_ww == 3;
    const int flat = (int)((total + (w3 ? 191 : kThreads - 1)) / (w3 ? 192 : kThreads));
    if (flat == 0) return hipSuccess;
    CoefWords cw{};
    memcpy(cw.w, a.single_coef_host, (size_t)a.k * a.m * ((a.k + 3) / 4) * 4);
    // residency (knob route_wpc): 4 workgroups per CU. The direct body alone runs best at 3, the wave
    // body at its VGPR limit of 5: at 3 the plan route lost 8-10 % on mixed batches, at 5 / uncapped
    // the direct route kept only 0.4-2.9 % of its gain; at 4 single-erasure batches run 2.2-3.9 %
    // faster than round 5's sorted-plan route and mixed ones within +-3 % of it
    // (profiles/r06/inplace_route_r06g.log, _r06j). With three of each workgroup's waves on the
    // direct route (knob route_ww 3, the default) the direct route runs at its own best residency
    // (12 waves per CU) and the plan route keeps 16: one data shard lost 1.971 -> 1.930 ms (the
    // out-of-place decode 1.896), U{1..4} 2.107 -> 2.063, U{1..2} level (inplace_ww3_r06r.log)
    const int wpc = g_tune.route_wpc;
    const size_t own = std::max(4 * direct_wave_bytes(a.k), 4 * wave_slice_bytes(a.k, a.maxe, a.lay.stride));
    const size_t lds = occupancy_lds(wpc, own);
    // in place: nt stores (decode_store_policy)
    if (w3) {
        if (a.maxe <= 4)
            hipLaunchKernelGGL((rs_reconstruct_routed_kernel<4, 8, 1, 0, 3>), dim3(flat), dim3(kThreads), lds, s, a, cw);
        else
            hipLaunchKernelGGL((rs_reconstruct_routed_kernel<8, 8, 1, 0, 3>), dim3(flat), dim3(kThreads), lds, s, a, cw);
    } else if (a.maxe <= 4) {
        hipLaunchKernelGGL((rs_reconstruct_routed_kernel<4, 8, 1, 0>), dim3(flat), dim3(kThreads), lds, s, a, cw);
    } else {
        hipLaunchKernelGGL((rs_reconstruct_routed_kernel<8, 8, 1, 0>), dim3(flat), dim3(kThreads), lds, s, a, cw);
    }
    return hipGetLastError();
}

template <int K, int TAB, int SP = 0>
static hipError_t direct_launch(const ReconArgs& a0, const CoefWords& cw, hipStream_t s) {
    const uint64_t total = (uint64_t)a0.nblocks * a0.cps;
    const int flat = (int)((total + kThreads - 1) / kThreads);
    if (flat == 0) return hipSuccess;
    // residency by shape: 3 workgroups/CU for k >= 8 (RS(8,12) with the masks by scalar loads,
    // profiles/r05/dec_twin_r05c.log: 5.88 TB/s at 3 against 5.82 at 4, 5.76 at 5, 5.37 at 2; with
    // a vector mask load 4 had been best, +3.6 % over uncapped; RS(16,24) / RS(20,30) 3, +1 %, r03i),
    // small codes uncapped
    const int wpc = g_tune.dir_wpc >= 0 ? (int)g_tune.dir_wpc : (a0.k >= 8 ? 3 : 0);
    // (workgroups of 2 waves at 5 / 6 / 7 per CU: +2.1 / +0.5 / +1.1 % time, r06i)
    const size_t lds = occupancy_lds(wpc, 4 * direct_wave_bytes(a0.k));
    hipLaunchKernelGGL((rs_recover_direct_kernel<K, TAB, SP>), dim3(flat), dim3(kThreads), lds, s, a0, cw);
    return hipGetLastError();
}

hipError_t launch_rs_recover_direct(const ReconArgs& a, hipStream_t s) {
    // the reference's benchmark shapes at compile time, the rest by runtime k. Non-temporal loads
    // and stores for every code: plain loads measured +8 % for RS(2,3) (r02), but only because its
    // 65 536-block batch (239 MB) fits the 256 MiB Infinity Cache and back-to-back launches re-read
    // it from there (the encode's plain-load A/B, r04, showed the same +11 %); shards streamed in
    // once do not come back, so the decode streams as the encode does (round 5)
    hipError_t e;
    CoefWords cw{};
    const size_t kw = (a.k + 3) / 4, words = (size_t)a.k * a.m * kw;
    const bool by_arg = g_tune.dec_direct != 2 && a.single_coef_host && words <= kCoefWords;
    if (by_arg) memcpy(cw.w, a.single_coef_host, words * 4);
    if (a.k == 20)   // RS(20,30), RS(16,24): rows from the device coefficient table
        e = direct_launch<20, 2>(a, cw, s);
    else if (a.k == 16)
        e = direct_launch<16, 2>(a, cw, s);
    else if (a.k == 8 && by_arg && a.sp == 3)   // nt sc1 stores (decode_store_policy; else nt)
        e = direct_launch<8, 1, 3>(a, cw, s);
    else if (a.k == 8)
        e = by_arg ? direct_launch<8, 1>(a, cw, s) : direct_launch<8, 0>(a, cw, s);
    else if (a.k == 2 && a.m == 1 && by_arg) {
        K2Rows rows;
        for (int e0 = 0; e0 < 2; ++e0)
            for (int j = 0; j < 2; ++j) rows.t[e0][j] = gf::make_permtab((uint8_t)(cw.w[e0] >> (8 * j)));
        const uint64_t total = (uint64_t)a.nblocks * a.cps;
        const int flat = (int)((total + kThreads - 1) / kThreads);
        if (flat == 0) return hipSuccess;
        const int wpc = g_tune.dir_wpc >= 0 ? (int)g_tune.dir_wpc : 0;
        hipLaunchKernelGGL(rs_recover_k2m1_kernel, dim3(flat), dim3(kThreads), occupancy_lds(wpc, 0), s, a, rows);
        e = hipGetLastError();
    } else if (a.k == 2)
        e = by_arg ? direct_launch<2, 1>(a, cw, s) : direct_launch<2, 0>(a, cw, s);
    else
        e = by_arg ? direct_launch<0, 1>(a, cw, s) : direct_launch<0, 0>(a, cw, s);
    return e;
}

}  // namespace fk
