// fec_xor.hip — XOR(k,1) encode / single-erasure recovery kernels for gfx950
// (internal/fec/xor.go:28-33, :80-86).
#include "fec_device.hpp"

namespace fk {

// ------------------------------------------------------------------ XOR
// KG = inputs loaded back to back per group (2, 4 or 8, the smallest that covers k, or 8 for
// k > 8): a group issues exactly the loads it uses except for clamped repeats in the last
// group, so XOR(2,1) issues 2 loads per item, not 8.
// BF: branch-free, an input past `valid` (a clamped repeat) is masked out, not skipped. With a
// branch around its fold (BF false) the compiler sinks the load into the branch, so the group's
// loads go out one round trip after another (load, wait, fold, load, wait, fold). The reconstruct
// folds branch-free (at 6 workgroups/CU 0.625 against 0.652 ms, 2^20 XOR(2,1) blocks); the encode
// keeps the branching fold, whose one load at a time runs 1.2 % faster at 6 workgroups/CU (0.601
// against 0.608 ms) though 6 % slower at 4 (profiles/r06/xor_ab_fold_r06u.log, _r06v).
template <int KG, bool BF>
__device__ __forceinline__ void xor_fold(uint4& acc, const uint4 (&x)[KG], uint32_t valid) {
#pragma unroll
    for (int jj = 0; jj < KG; ++jj) {
        if constexpr (!BF) {
            if ((uint32_t)jj < valid) {
                acc.x ^= x[jj].x;
                acc.y ^= x[jj].y;
                acc.z ^= x[jj].z;
                acc.w ^= x[jj].w;
            }
            continue;
        }
        const uint32_t keep = (uint32_t)jj < valid ? ~0u : 0u;
        acc.x ^= x[jj].x & keep;
        acc.y ^= x[jj].y & keep;
        acc.z ^= x[jj].z & keep;
        acc.w ^= x[jj].w & keep;
    }
}

// Flat grids (one item per lane), non-temporal loads and stores.
template <int KG, bool BF>
__global__ __launch_bounds__(kThreads) void xor_encode_kernel(XorArgs a) {
    constexpr bool NTL = true, NTS = true;
    const uint32_t k = a.k;
    const uint32_t item = xcd_order() * kThreads + threadIdx.x;
    if (item < a.total) {
        const uint32_t b = fdiv(item, a.div_cps);
        const uint32_t c = item - b * a.cps;
        const uint8_t* src = a.in + (uint64_t)b * a.in_bs + (uint64_t)c * kChunk;
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (uint32_t j0 = 0; j0 < k; j0 += KG) {
            uint4 x[KG];
#pragma unroll
            for (int jj = 0; jj < KG; ++jj) x[jj] = ld16<NTL>(src + (uint64_t)min(j0 + jj, k - 1) * a.ss);
            xor_fold<KG, BF>(acc, x, k - j0);
        }
        store_chunk<NTS>(a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk, acc, a.len - c * kChunk);
    }
}

template <int KG, bool BF>
__global__ __launch_bounds__(kThreads) void xor_reconstruct_kernel(XorArgs a) {
    constexpr bool NTL = true, NTS = true;
    const uint32_t k = a.k, n = k + 1;
    const uint32_t all = low_mask(n);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // Statuses and failure flags of blocks [64 w, 64 w + 64), w = this wave's launch index: one
    // coalesced mask load and one coalesced status store per 64 blocks (as the direct RS decode)
    {
        const uint32_t w = blockIdx.x * (kThreads / 64) + wave;
        if (w * 64u < a.nblocks) {   // wave-uniform
            const uint32_t b = w * 64u + lane;
            bool fail = false;
            if (b < a.nblocks) {
                const uint32_t miss = ~a.masks[b] & all;
                fail = __popc(miss) > 1 && (miss & low_mask(k));
                if (a.status) a.status[b] = fail ? -4 : 0;
            }
            if (__ballot(fail) != 0 && lane == 0) atomicOr(a.err, 1);
        }
    }
    const uint32_t i0 = xcd_order() * kThreads + (wave << 6);
    if (i0 >= a.total) return;
    const uint32_t item = i0 + lane;
    const uint32_t b = fdiv(min(item, a.total - 1u), a.div_cps);
    uint32_t mk;
    if (a.cps >= 32) {   // the wave's <= 3 masks by scalar loads, off the vector memory path
        const uint32_t bfirst = fdiv(i0, a.div_cps);
        const WaveMasks wm = wave_masks(a.masks, bfirst, a.nblocks);
        // all three in flight together: left alone, the compiler sank the second and third load
        // into the lanes' select branches, one wait each
        asm volatile("" ::"s"(wm.m0), "s"(wm.m1), "s"(wm.m2));
        mk = wm.of(b - bfirst);
    } else {
        mk = a.masks[b];
    }
    if (item >= a.total) return;
    const uint32_t c = item - b * a.cps;
    const uint32_t miss = ~mk & all;
    const uint32_t mi = miss ? (uint32_t)__ffs(miss) - 1 : 0;
    if (__popc(miss) != 1 || mi >= k) return;   // nothing to rebuild, or a failure reported above
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
        xor_fold<KG, BF>(acc, x, k - j0);
    }
    store_chunk<NTS>(blk + (uint64_t)mi * a.ss, acc, a.len - c * kChunk);
}

template <int KG>
static void xor_launch(const XorArgs& a, int grid, size_t lds, bool encode, hipStream_t s) {
    if (encode) hipLaunchKernelGGL((xor_encode_kernel<KG, false>), dim3(grid), dim3(kThreads), lds, s, a);
    else hipLaunchKernelGGL((xor_reconstruct_kernel<KG, true>), dim3(grid), dim3(kThreads), lds, s, a);
}

static hipError_t xor_dispatch(const XorArgs& a, int grid, size_t lds, bool encode, hipStream_t s) {
    if (a.k <= 2) xor_launch<2>(a, grid, lds, encode, s);
    else if (a.k <= 4) xor_launch<4>(a, grid, lds, encode, s);
    else xor_launch<8>(a, grid, lds, encode, s);
    return hipGetLastError();
}

// residency (knob xor_wpc): 6 workgroups/CU for both kernels. XOR(2,1), 2^20 blocks, against as
// many as fit (8): encode 0.601 against 0.618 ms, reconstruct 0.625 against 0.630, its in-place
// traffic twin 0.618 at 6 (profiles/r06/xor_ab_*_r06*.log)
hipError_t launch_xor_encode(const XorArgs& a, int grid, hipStream_t s) {
    return xor_dispatch(a, grid, occupancy_lds(g_tune.xor_wpc, 0), true, s);
}

// (XOR(2,1) by a one-item-per-lane kernel of its own measured 0.7 % slower, r04m: the gap to the
// XOR twin is the in-place write, not the loop)
hipError_t launch_xor_reconstruct(const XorArgs& a, int grid, hipStream_t s) {
    return xor_dispatch(a, grid, occupancy_lds(g_tune.xor_wpc, 0), false, s);
}

}  // namespace fk
