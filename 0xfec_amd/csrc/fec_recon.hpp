// fec_recon.hpp — device pieces shared by the reconstruct kernels (fec_decode.hip: plan + wave /
// tile rebuild; fec_recover.hip: direct single-erasure rebuild; fec_rebuild.hip): the per-item
// rebuild and the wave slice layout.
#pragma once

#include "fec_device.hpp"

namespace fk {

// Input slot `slot` of an item (< k: data shard slot, else parity shard slot - k): one 64-bit
// base select, one stride select and one 32 x 32 + 64 multiply-add (v_mad_u64_u32). pbase is
// the item's parity address minus k parity strides; shard strides are below 4 GiB (checked by
// the host). Selecting between two full 64-bit products instead costs ~13 VALU per input.
// (Pointer arithmetic, not integer casts: the loads must stay global_load, not flat_load.)
__device__ __forceinline__ const uint8_t* slot_addr(const uint8_t* dblk, const uint8_t* pbase, uint32_t slot,
                                                    uint32_t k, uint32_t ss, uint32_t pss) {
    const bool d = slot < k;
    return (d ? dblk : pbase) + (uint64_t)slot * (d ? ss : pss);
}
__device__ __forceinline__ const uint8_t* parity_base(const uint8_t* pblk, uint32_t k, uint64_t pss) {
    return pblk - (uint64_t)k * pss;
}

// One (block, chunk) item: load the k input shards named by the plan record P, fold them with
// the block's PermTabs T (row r = erased shard r), store the rebuilt chunks. `rows` is
// wave-uniform (the wave's largest erasure count), so the loop bounds never diverge.
// Non-temporal loads and stores throughout the reconstruct kernels.
constexpr bool kNT = true;

template <int MAXE>
__device__ __forceinline__ void recon_item(const ReconArgs& a, const uint8_t* P, const gf::PermTab* T,
                                           uint32_t blk, uint32_t c, uint32_t rows, uint32_t nout) {
    const uint32_t k = a.k;
    const PlanLayout& lay = a.lay;
    uint8_t* dblk = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    const uint8_t* pblk = a.parity + (uint64_t)blk * a.pbs + (uint64_t)c * kChunk;
    const uint8_t* pbase = parity_base(pblk, k, a.pss);
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
                        ? ld16<kNT>(slot_addr(dblk, pbase, slot, k, (uint32_t)a.ss, (uint32_t)a.pss))
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
            store_chunk<kNT>(oblk ? oblk + (uint64_t)r * a.ss : dblk + (uint64_t)out_idx[r] * a.ss, as_uint4(acc[r]),
                             nb);
}

// recon_item with the data shard count K known at compile time: all K input loads are issued
// before any is folded (the runtime-k form issues them 8 at a time, and the second group's
// loads wait for the first group's arithmetic), and the wave-uniform row count selects a
// straight-line body per count (per-row branches inside the fold make the compiler copy the
// accumulators through every branch).
template <int K, int ROWS>
__device__ __forceinline__ void recon_rows_k(const ReconArgs& a, const uint8_t* P, const gf::PermTab* T,
                                             const uint4 (&x)[K], uint8_t* dblk, uint8_t* oblk, uint32_t c,
                                             uint32_t nout) {
    uint32_t acc[ROWS][4];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0;
#pragma unroll
    for (int j = 0; j < K; j += 2) {
        // opaque zero per input pair: keeps the table reads next to their use (hoisted, every
        // pair's tables would be held at once)
        uint32_t toff = 0;
        asm volatile("" : "+s"(toff));
        const gf::PermTab* t = T + toff;
        // the pair's inputs pass through an opaque step here, so their splits are not hoisted
        // ahead of earlier pairs (all splits at once would hold 3 words per input dword)
        const uint4 xa = x[j], xb = x[j + 1];
        __builtin_amdgcn_sched_barrier(0);
        Idx ia[4], ib[4];
        split4(ia, xa);
        split4(ib, xb);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) mac2(acc[r], ia, ib, t + r * K + j, t + r * K + j + 1);
    }
    const uint32_t nb = a.len - c * kChunk;
    const uint8_t* out_idx = P + a.lay.out_off;
#pragma unroll
    for (int r = 0; r < ROWS; ++r)
        if (r < (int)nout)
            store_chunk<kNT>(oblk ? oblk + (uint64_t)r * a.ss : dblk + (uint64_t)out_idx[r] * a.ss, as_uint4(acc[r]),
                             nb);
}

template <int K, int MAXE>
__device__ __forceinline__ void recon_item_k(const ReconArgs& a, const uint8_t* P, const gf::PermTab* T,
                                             uint32_t blk, uint32_t c, uint32_t rows, uint32_t nout) {
    static_assert(K % 2 == 0, "inputs are folded in pairs");
    const PlanLayout& lay = a.lay;
    uint8_t* dblk = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    const uint8_t* pblk = a.parity + (uint64_t)blk * a.pbs + (uint64_t)c * kChunk;
    const uint8_t* pbase = parity_base(pblk, K, a.pss);
    uint4 x[K];
#pragma unroll
    for (int j0 = 0; j0 < K; j0 += 8) {
        const uint2 sl = *reinterpret_cast<const uint2*>(P + lay.in_off + j0);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            if (j0 + jj >= K) break;   // compile-time: the slot area is rounded up to 8 bytes
            const uint32_t slot = ((jj < 4 ? sl.x : sl.y) >> (8 * (jj & 3))) & 0xFFu;
            x[j0 + jj] = ld16<kNT>(slot_addr(dblk, pbase, slot, K, (uint32_t)a.ss, (uint32_t)a.pss));
        }
    }
    uint8_t* oblk = a.out ? a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk : nullptr;
    // row bodies 1..R (R: the code's largest erasure count, min(k, m): RS(16,24) 8, RS(20,30) 10)
    constexpr int R = MAXE < K ? (MAXE <= 8 ? MAXE : 10) : K;
    static_assert(R <= 10, "row bodies 1..10");
    switch (rows) {   // wave-uniform
        case 1: recon_rows_k<K, 1>(a, P, T, x, dblk, oblk, c, nout); break;
        case 2: if constexpr (R >= 2) recon_rows_k<K, 2>(a, P, T, x, dblk, oblk, c, nout); break;
        case 3: if constexpr (R >= 3) recon_rows_k<K, 3>(a, P, T, x, dblk, oblk, c, nout); break;
        case 4: if constexpr (R >= 4) recon_rows_k<K, 4>(a, P, T, x, dblk, oblk, c, nout); break;
        case 5: if constexpr (R >= 5) recon_rows_k<K, 5>(a, P, T, x, dblk, oblk, c, nout); break;
        case 6: if constexpr (R >= 6) recon_rows_k<K, 6>(a, P, T, x, dblk, oblk, c, nout); break;
        case 7: if constexpr (R >= 7) recon_rows_k<K, 7>(a, P, T, x, dblk, oblk, c, nout); break;
        case 8: if constexpr (R >= 8) recon_rows_k<K, 8>(a, P, T, x, dblk, oblk, c, nout); break;
        case 9: if constexpr (R >= 9) recon_rows_k<K, 9>(a, P, T, x, dblk, oblk, c, nout); break;
        default: if constexpr (R >= 10) recon_rows_k<K, 10>(a, P, T, x, dblk, oblk, c, nout); break;
    }
}

template <int MAXE>
__device__ __forceinline__ uint32_t wave_rows(uint32_t nout) {
    uint32_t rows = 0;
#pragma unroll
    for (int r = 0; r < MAXE; ++r)
        if (__any((int)nout > r)) rows = r + 1;
    return rows;
}

// Wave form (shards of 32+ chunks, i.e. at most 3 blocks per wave): flat grid, one item per
// lane; each wave stages the plan records of its own blocks and expands only the PermTabs of
// rows those blocks rebuild, in a wave-private LDS slice, so no workgroup barrier stands
// between a wave's plan load and its data loads.
constexpr uint32_t kWaveBlocks = 3;

__host__ __device__ inline size_t wave_slice_bytes(uint32_t k, uint32_t maxe, uint32_t stride,
                                                   uint32_t nblk = kWaveBlocks) {
    return (size_t)nblk * maxe * k * 32 + (size_t)nblk * stride;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave form (shards of 32+ chunks): one wave per 64 consecutive items of the sorted plan order; the
// wave stages its <= 3 blocks' records and the PermTabs of the rows they rebuild in a wave-private
// LDS slice (no workgroup barrier), one item per lane. K: compile-time data shard count (0: runtime
// a.k), all K input loads in flight before the first is folded (recon_item_k). The body of
// rs_reconstruct_wave_kernel (fec_decode.hip) and of the routed kernel's plan route (fec_recover.hip).
// order: the workgroup's place in the grid's item order (xcd_order() for a grid of exactly the
// plan items' workgroups).
template <int MAXE, int K = 0>
__device__ __forceinline__ void wave_body(const ReconArgs& a, uint8_t* smem, uint32_t order) {
    const uint32_t k = a.k, maxe = a.maxe;
    const PlanLayout lay = a.lay;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* slice = smem + (size_t)wave * wave_slice_bytes(k, maxe, lay.stride);
    gf::PermTab* tabs = reinterpret_cast<gf::PermTab*>(slice);                     // 3*maxe*k
    uint8_t* plans = slice + (size_t)kWaveBlocks * maxe * k * sizeof(gf::PermTab);  // 3*stride
    const uint32_t total = a.nblocks * a.cps;
    const uint32_t i0 = order * kThreads + (wave << 6);
    if (i0 >= total) return;
    const uint32_t bfirst = fdiv(i0, a.div_cps);
    const uint32_t nb = fdiv(min(i0 + 63u, total - 1u), a.div_cps) - bfirst + 1;   // <= 3
    {
        const uint32_t nw = nb * lay.stride / 16;
        const uint4* src = reinterpret_cast<const uint4*>(a.plans + (uint64_t)bfirst * lay.stride);
        if (lane < nw) reinterpret_cast<uint4*>(plans)[lane] = src[lane];
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
    if constexpr (K > 0) recon_item_k<K, MAXE>(a, P, tabs + g * maxe * k, rb, c, rows, nout);
    else recon_item<MAXE>(a, P, tabs + g * maxe * k, rb, c, rows, nout);
}

}  // namespace fk
