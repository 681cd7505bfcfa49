// mix_probe.hip — diagnostics only: how the HBM rate of a mixed read/write stream depends on
// things the codec kernels control (output-buffer offset, workgroup->XCD mapping, resident
// waves per CU, items per lane). Built and run by tools/mix_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t swizzle_wg(uint32_t wg, uint32_t G, int mode) {
    if (mode == 0) return wg;
    // contiguous range of workgroups per XCD (dispatch deals workgroups round-robin over 8)
    const uint32_t full = G & ~7u;
    if (wg >= full) return wg;
    const uint32_t cpx = full >> 3;
    return (wg & 7u) * cpx + (wg >> 3);
}

// item = (block, 16-B chunk). Each lane loads NIN shards of its chunk (stride ss inside the
// input block) and stores NOUT shards (stride ss inside the output block). IPL items per lane,
// all loads issued before the first store.
template <int NIN, int NOUT, int IPL>
__global__ __launch_bounds__(256) void mix_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                  size_t in_bs, size_t out_bs, size_t ss, uint32_t cps,
                                                  uint32_t total, int swz) {
    extern __shared__ uint8_t pad[];
    const uint32_t wg = swizzle_wg(blockIdx.x, gridDim.x, swz);
    u32x4 acc[IPL];
    uint32_t items[IPL];
#pragma unroll
    for (int u = 0; u < IPL; ++u) {
        const uint32_t item = (wg * IPL + u) * 256 + threadIdx.x;
        items[u] = item;
        acc[u] = (u32x4){0, 0, 0, 0};
        if (item < total) {
            const uint32_t b = item / cps, c = item - b * cps;
            const uint8_t* src = in + (size_t)b * in_bs + (size_t)c * 16;
#pragma unroll
            for (int j = 0; j < NIN; ++j)
                acc[u] ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (size_t)j * ss));
        }
    }
#pragma unroll
    for (int u = 0; u < IPL; ++u) {
        const uint32_t item = items[u];
        if (item < total) {
            const uint32_t b = item / cps, c = item - b * cps;
            uint8_t* dst = out + (size_t)b * out_bs + (size_t)c * 16;
#pragma unroll
            for (int r = 0; r < NOUT; ++r) {
                u32x4 v = acc[u];
                v.x ^= r;
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + (size_t)r * ss));
            }
        }
    }
    if (NOUT == 0 && pad[0] == 0x5A && acc[0].x == 0x12345u) out[0] = 1;
}

extern "C" int mix_probe(const void* in, void* out, size_t in_bs, size_t out_bs, size_t ss, unsigned cps,
                         unsigned nblocks, int nin, int nout, int ipl, int swz, size_t lds_pad, void* stream) {
    const uint32_t total = cps * nblocks;
    const uint32_t per_wg = 256u * ipl;
    const int grid = (int)((total + per_wg - 1) / per_wg);
    hipStream_t s = (hipStream_t)stream;
    const uint8_t* i8 = (const uint8_t*)in;
    uint8_t* o8 = (uint8_t*)out;
#define MK(NI, NO, IP)                                                                                        \
    if (nin == NI && nout == NO && ipl == IP) {                                                               \
        hipLaunchKernelGGL((mix_kernel<NI, NO, IP>), dim3(grid), dim3(256), lds_pad, s, i8, o8, in_bs, out_bs, \
                           ss, cps, total, swz);                                                              \
        return (int)hipGetLastError();                                                                        \
    }
    MK(1, 1, 1) MK(1, 1, 2) MK(1, 1, 4) MK(8, 4, 1) MK(8, 4, 2) MK(8, 1, 1) MK(8, 1, 2) MK(8, 0, 1) MK(0, 1, 1)
    MK(0, 1, 4) MK(2, 1, 1) MK(4, 1, 1) MK(2, 2, 1) MK(4, 4, 1) MK(8, 8, 1) MK(8, 2, 1) MK(4, 2, 1) MK(16, 8, 1)
    MK(16, 3, 1) MK(8, 4, 4) MK(8, 1, 4)
    return -1;
}

// One item per lane (IPL 1), XCD-contiguous order, with the store's cache policy varied (round 6,
// what the decode shape's one store per 8 reads costs, and whether a policy
// changes it): POL 0 nt (the codec kernels' form), 1 plain, 2 sc1, 3 sc0 sc1 (the last two drop the
// line from L2: MI355X_MICROARCH.md, stores of each flavour).
template <int POL>
__device__ __forceinline__ void st_pol(uint8_t* p, u32x4 v) {
    if constexpr (POL == 0) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    } else if constexpr (POL == 1) {
        *reinterpret_cast<u32x4*>(p) = v;
    } else if constexpr (POL == 2) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    } else if constexpr (POL == 3) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    } else {
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    }
}

template <int NIN, int NOUT, int POL>
__global__ __launch_bounds__(256) void mix_pol_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                      size_t in_bs, size_t out_bs, size_t ss, uint32_t cps,
                                                      uint32_t total) {
    extern __shared__ uint8_t pad[];
    const uint32_t item = swizzle_wg(blockIdx.x, gridDim.x, 1) * 256 + threadIdx.x;
    if (item >= total) return;
    const uint32_t b = item / cps, c = item - b * cps;
    const uint8_t* src = in + (size_t)b * in_bs + (size_t)c * 16;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < NIN; ++j)
        acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (size_t)j * ss));
    uint8_t* dst = out + (size_t)b * out_bs + (size_t)c * 16;
#pragma unroll
    for (int r = 0; r < NOUT; ++r) {
        u32x4 v = acc;
        v.x ^= r;
        st_pol<POL>(dst + (size_t)r * ss, v);
    }
    if (NOUT == 0 && pad[0] == 0x5A && acc.x == 0x12345u) out[0] = 1;
}

extern "C" int mix_pol_probe(const void* in, void* out, size_t in_bs, size_t out_bs, size_t ss, unsigned cps,
                             unsigned nblocks, int nin, int nout, int pol, size_t lds_pad, void* stream) {
    const uint32_t total = cps * nblocks;
    const int grid = (int)((total + 255) / 256);
    hipStream_t s = (hipStream_t)stream;
    const uint8_t* i8 = (const uint8_t*)in;
    uint8_t* o8 = (uint8_t*)out;
#define MQ(NI, NO, PO)                                                                                           \
    if (nin == NI && nout == NO && pol == PO) {                                                                  \
        hipLaunchKernelGGL((mix_pol_kernel<NI, NO, PO>), dim3(grid), dim3(256), lds_pad, s, i8, o8, in_bs, out_bs, \
                           ss, cps, total);                                                                      \
        return (int)hipGetLastError();                                                                           \
    }
    MQ(8, 1, 0) MQ(8, 1, 1) MQ(8, 1, 2) MQ(8, 1, 3) MQ(8, 4, 0) MQ(8, 4, 1) MQ(8, 4, 2) MQ(8, 4, 3) MQ(8, 0, 0)
    return -1;
}

// Load cache policy (round 6): the 8 shard loads of an item as one asm statement with its own wait
// (the destinations are written at the wait, so the compiler cannot read them early). LP 0 nt,
// 1 plain, 2 sc1, 3 nt sc1, 4 sc0 sc1. Stores by st_pol<SP>. NIN is 8.
#define FEC_LD8(MOD)                                                                                       \
    asm volatile("global_load_dwordx4 %0, %8, off" MOD "\n\t"                                             \
                 "global_load_dwordx4 %1, %8, off offset:1216" MOD "\n\t"                                 \
                 "global_load_dwordx4 %2, %8, off offset:2432" MOD "\n\t"                                 \
                 "global_load_dwordx4 %3, %8, off offset:3648" MOD "\n\t"                                 \
                 "global_load_dwordx4 %4, %9, off" MOD "\n\t"                                             \
                 "global_load_dwordx4 %5, %9, off offset:1216" MOD "\n\t"                                 \
                 "global_load_dwordx4 %6, %9, off offset:2432" MOD "\n\t"                                 \
                 "global_load_dwordx4 %7, %9, off offset:3648" MOD "\n\t"                                 \
                 "s_waitcnt vmcnt(0)"                                                                       \
                 : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), \
                   "=&v"(x[7])                                                                              \
                 : "v"(src), "v"(src + 4 * 1216)                                                            \
                 : "memory")

template <int LP, int NOUT, int SP>
__global__ __launch_bounds__(256) void mix_lp_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                     size_t in_bs, size_t out_bs, size_t ss, uint32_t cps,
                                                     uint32_t total) {
    extern __shared__ uint8_t pad[];
    const uint32_t item = swizzle_wg(blockIdx.x, gridDim.x, 1) * 256 + threadIdx.x;
    if (item >= total) return;
    const uint32_t b = item / cps, c = item - b * cps;
    const uint8_t* src = in + (size_t)b * in_bs + (size_t)c * 16;   // shard stride 1216 (the asm offsets)
    u32x4 x[8];
    if constexpr (LP == 0) FEC_LD8(" nt");
    else if constexpr (LP == 1) FEC_LD8("");
    else if constexpr (LP == 2) FEC_LD8(" sc1");
    else if constexpr (LP == 3) FEC_LD8(" nt sc1");
    else FEC_LD8(" sc0 sc1");
    u32x4 acc = x[0] ^ x[1] ^ x[2] ^ x[3] ^ x[4] ^ x[5] ^ x[6] ^ x[7];
    uint8_t* dst = out + (size_t)b * out_bs + (size_t)c * 16;
#pragma unroll
    for (int r = 0; r < NOUT; ++r) {
        u32x4 v = acc;
        v.x ^= r;
        st_pol<SP>(dst + (size_t)r * ss, v);
    }
    if (pad[0] == 0x5A && acc.x == 0x12345u) out[0] = 1;
}

extern "C" int mix_lp_probe(const void* in, void* out, size_t in_bs, size_t out_bs, size_t ss, unsigned cps,
                            unsigned nblocks, int nout, int lp, int sp, size_t lds_pad, void* stream) {
    if (ss != 1216) return -2;
    const uint32_t total = cps * nblocks;
    const int grid = (int)((total + 255) / 256);
    hipStream_t s = (hipStream_t)stream;
    const uint8_t* i8 = (const uint8_t*)in;
    uint8_t* o8 = (uint8_t*)out;
#define ML(LP, NO, SP)                                                                                          \
    if (lp == LP && nout == NO && sp == SP) {                                                                   \
        hipLaunchKernelGGL((mix_lp_kernel<LP, NO, SP>), dim3(grid), dim3(256), lds_pad, s, i8, o8, in_bs, out_bs, \
                           ss, cps, total);                                                                     \
        return (int)hipGetLastError();                                                                          \
    }
    ML(0, 4, 0) ML(1, 4, 0) ML(2, 4, 0) ML(3, 4, 0) ML(4, 4, 0) ML(0, 4, 2) ML(1, 4, 2) ML(2, 4, 2) ML(3, 4, 2)
    ML(4, 4, 2) ML(0, 1, 0) ML(1, 1, 0) ML(2, 1, 0) ML(3, 1, 0) ML(4, 1, 0) ML(0, 1, 4) ML(1, 1, 4) ML(2, 1, 4)
    ML(3, 1, 4) ML(4, 1, 4)
    return -1;
}

// Persistent forms of the same pattern. MODE 0: static sweep (workgroup j of XCD x takes items
// lo_x + j*256 + t*step); MODE 1: per-XCD ticket counter, one 256-item chunk per workgroup
// ticket (LDS broadcast, one barrier); MODE 2: per-XCD ticket per wave (64 items).
template <int NIN, int NOUT, int MODE>
__global__ __launch_bounds__(256) void mix_persist(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                   size_t in_bs, size_t out_bs, size_t ss, uint32_t cps,
                                                   uint32_t total, uint32_t per_xcd, uint32_t* ctr) {
    extern __shared__ uint8_t pad[];
    __shared__ uint32_t tk[2];
    const uint32_t x = blockIdx.x & 7u;
    const uint32_t lo = x * per_xcd, hi = min(total, lo + per_xcd);
    const uint32_t cpx = gridDim.x >> 3, j = blockIdx.x >> 3;
    uint32_t* c = ctr + x * 32;
    u32x4 keep = {0, 0, 0, 0};
    for (uint32_t t = 0;; ++t) {
        uint32_t base;
        if constexpr (MODE == 0) {
            base = lo + (t * cpx + j) * 256;
        } else if constexpr (MODE == 1) {
            if (threadIdx.x == 0) tk[t & 1] = atomicAdd(c, 1u);
            __syncthreads();
            base = lo + tk[t & 1] * 256;
        } else {
            uint32_t v = 0;
            if ((threadIdx.x & 63) == 0) v = atomicAdd(c, 1u);
            v = __shfl(v, 0);
            base = lo + v * 64 - (threadIdx.x & ~63u);   // + threadIdx.x below
        }
        if (base + (MODE == 2 ? (threadIdx.x & ~63u) : 0) >= hi) break;
        const uint32_t item = base + threadIdx.x;
        if (item < hi) {
            const uint32_t b = item / cps, cc = item - b * cps;
            const uint8_t* src = in + (size_t)b * in_bs + (size_t)cc * 16;
            u32x4 acc = {0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < NIN; ++q)
                acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (size_t)q * ss));
            uint8_t* dst = out + (size_t)b * out_bs + (size_t)cc * 16;
#pragma unroll
            for (int r = 0; r < NOUT; ++r) {
                u32x4 v = acc;
                v.x ^= r;
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + (size_t)r * ss));
            }
            keep ^= acc;
        }
    }
    if (NOUT == 0 && pad[0] == 0x5A && keep.x == 0x12345u) out[0] = 1;
}

extern "C" int mix_persist_probe(const void* in, void* out, size_t in_bs, size_t out_bs, size_t ss, unsigned cps,
                                 unsigned nblocks, int nin, int nout, int mode, int grid, size_t lds_pad,
                                 void* ctr, void* stream) {
    const uint32_t total = cps * nblocks;
    const uint32_t per_xcd = (total + 7) / 8;
    hipStream_t s = (hipStream_t)stream;
    hipMemsetAsync(ctr, 0, 8 * 32 * 4, s);
    const uint8_t* i8 = (const uint8_t*)in;
    uint8_t* o8 = (uint8_t*)out;
#define MP(NI, NO, MD)                                                                                       \
    if (nin == NI && nout == NO && mode == MD) {                                                            \
        hipLaunchKernelGGL((mix_persist<NI, NO, MD>), dim3(grid), dim3(256), lds_pad, s, i8, o8, in_bs, out_bs, \
                           ss, cps, total, per_xcd, (uint32_t*)ctr);                                        \
        return (int)hipGetLastError();                                                                      \
    }
    MP(8, 4, 0) MP(8, 4, 1) MP(8, 4, 2) MP(8, 1, 0) MP(8, 1, 1) MP(8, 1, 2)
    return -1;
}
