// fec_xor.hip — XOR(k,1) encode / single-erasure recovery kernels for gfx950
// (internal/fec/xor.go:28-33, :80-86).
#include "fec_device.hpp"

namespace fk {

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
    const uint32_t all = low_mask(n);
    const uint32_t stride = gridDim.x * kThreads;
    for (uint32_t item = xcd_order(a.swz) * kThreads + threadIdx.x; item < a.total; item += stride) {
        const uint32_t b = fdiv(item, a.div_cps);
        const uint32_t c = rotate_chunk(item - b * a.cps, a.cps, a.rot);
        const uint32_t miss = ~a.masks[b] & all;
        const uint32_t nmiss = __popc(miss);
        const uint32_t mi = miss ? (uint32_t)__ffs(miss) - 1 : 0;
        const bool work = nmiss == 1 && mi < k;
        const bool fail = nmiss > 1 && (miss & low_mask(k));
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

// XOR(2,1) reconstruct (the reference's XOR code, manager.go:54-56), one item per lane on a flat
// grid (knob xor_fix2, off: measured 0.7 % slower than the generic kernel): the block's lost data
// shard = the other one ^ the parity, written in place, with no loop over input groups.
template <bool NTL, bool NTS>
__global__ __launch_bounds__(kThreads) void xor_reconstruct2_kernel(XorArgs a) {
    const uint32_t item = xcd_order(a.swz) * kThreads + threadIdx.x;
    if (item >= a.total) return;
    const uint32_t b = fdiv(item, a.div_cps);
    const uint32_t c = item - b * a.cps;
    const uint32_t miss = ~a.masks[b] & 7u;
    const uint32_t nmiss = __popc(miss);
    if (c == 0) {
        const bool fail = nmiss > 1;   // two or three of the three shards: a data shard among them
        if (a.status) a.status[b] = fail ? -4 : 0;
        if (fail) atomicOr(a.err, 1);
    }
    if (nmiss != 1 || miss == 4u) return;   // nothing lost, or only the parity
    const uint32_t mi = miss >> 1;           // 1 -> shard 0, 2 -> shard 1
    uint8_t* blk = a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk;
    const uint4 x = ld16<NTL>(blk + (uint64_t)(mi ^ 1u) * a.ss);
    const uint4 p = ld16<NTL>(a.parity + (uint64_t)b * a.par_bs + (uint64_t)c * kChunk);
    const uint4 r = make_uint4(x.x ^ p.x, x.y ^ p.y, x.z ^ p.z, x.w ^ p.w);
    store_chunk<NTS>(blk + (uint64_t)mi * a.ss, r, a.len - c * kChunk, a.pad_zero);
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
    if (a.k == 2 && g_tune.xor_fix2 && a.rot == 0) {
        const uint32_t flat = (a.total + kThreads - 1) / kThreads;
        if (flat == 0) return hipSuccess;
        if (g_tune.dec_nt & 3)
            hipLaunchKernelGGL((xor_reconstruct2_kernel<true, true>), dim3(flat), dim3(kThreads), 0, s, a);
        else
            hipLaunchKernelGGL((xor_reconstruct2_kernel<false, false>), dim3(flat), dim3(kThreads), 0, s, a);
        return hipGetLastError();
    }
    return xor_dispatch(a, grid, occupancy_lds(g_tune.dec_wpc, 0), (g_tune.dec_nt & 3) != 0, false, s);
}

const void* xor_occupancy_kernel() { return (const void*)xor_encode_kernel<3, 8>; }

}  // namespace fk
