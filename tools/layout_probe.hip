// layout_probe.hip — diagnostics only: does the parity layout change the HBM rate of the
// codec's access shapes? Pure traffic (XOR instead of field math), 16 B per lane, nt loads and
// stores, one item per lane, XCD-contiguous workgroup order optional. Parity shard r of block b
// lives at parity + b*pbs + r*pss: [B][m][S] is (pbs, pss) = (m*S, S), [m][B][S] is (S, B*S).
//   encode shape: k data shards read, m parity shards written
//   decode shape: k-1 data shards (shard b % k skipped, as a rotating erasure) + parity 0 read,
//                 one recovered shard written to out[B][S]
// Built and run by tools/layout_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t swizzle_wg(uint32_t wg, uint32_t G, int mode) {
    if (mode == 0) return wg;
    const uint32_t full = G & ~7u;
    if (wg >= full) return wg;
    return (wg & 7u) * (full >> 3) + (wg >> 3);
}

template <int K, int M>
__global__ __launch_bounds__(256) void enc_shape(const uint8_t* __restrict__ data, uint8_t* __restrict__ par,
                                                 size_t dbs, size_t ss, size_t pbs, size_t pss, uint32_t cps,
                                                 uint32_t total, int swz) {
    extern __shared__ uint8_t pad[];
    const uint32_t item = swizzle_wg(blockIdx.x, gridDim.x, swz) * 256 + threadIdx.x;
    if (item >= total) return;
    const uint32_t b = item / cps, c = item - b * cps;
    const uint8_t* src = data + (size_t)b * dbs + (size_t)c * 16;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < K; ++j) acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (size_t)j * ss));
    uint8_t* dst = par + (size_t)b * pbs + (size_t)c * 16;
#pragma unroll
    for (int r = 0; r < M; ++r) {
        u32x4 v = acc;
        v.x ^= r;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + (size_t)r * pss));
    }
    if (pad[0] == 0x5A && acc.y == 0x12345u) par[0] = 1;
}

template <int K>
__global__ __launch_bounds__(256) void dec_shape(const uint8_t* __restrict__ data, const uint8_t* __restrict__ par,
                                                 uint8_t* __restrict__ out, size_t dbs, size_t ss, size_t pbs,
                                                 uint32_t cps, uint32_t total, int swz) {
    extern __shared__ uint8_t pad[];
    const uint32_t item = swizzle_wg(blockIdx.x, gridDim.x, swz) * 256 + threadIdx.x;
    if (item >= total) return;
    const uint32_t b = item / cps, c = item - b * cps;
    const uint32_t e = b % K;
    const uint8_t* src = data + (size_t)b * dbs + (size_t)c * 16;
    u32x4 acc = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(par + (size_t)b * pbs + (size_t)c * 16));
#pragma unroll
    for (int j = 0; j < K - 1; ++j) {
        const uint32_t s = j < (int)e ? j : j + 1;
        acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (size_t)s * ss));
    }
    __builtin_nontemporal_store(acc, reinterpret_cast<u32x4*>(out + (size_t)b * ss + (size_t)c * 16));
    if (pad[0] == 0x5A && acc.y == 0x12345u) out[0] = 1;
}

extern "C" int layout_probe(int shape, const void* data, void* par, void* out, size_t dbs, size_t ss, size_t pbs,
                            size_t pss, unsigned cps, unsigned nblocks, int swz, size_t lds_pad, void* stream) {
    const uint32_t total = cps * nblocks;
    const int grid = (int)((total + 255) / 256);
    hipStream_t s = (hipStream_t)stream;
    if (shape == 0)
        hipLaunchKernelGGL((enc_shape<8, 4>), dim3(grid), dim3(256), lds_pad, s, (const uint8_t*)data, (uint8_t*)par,
                           dbs, ss, pbs, pss, cps, total, swz);
    else
        hipLaunchKernelGGL((dec_shape<8>), dim3(grid), dim3(256), lds_pad, s, (const uint8_t*)data,
                           (const uint8_t*)par, (uint8_t*)out, dbs, ss, pbs, cps, total, swz);
    return (int)hipGetLastError();
}
