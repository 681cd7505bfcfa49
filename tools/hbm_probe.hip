// hbm_probe.hip — diagnostics only: achievable HBM rates on this MI355X for the access
// shapes the FEC kernels use (16-B lanes, streaming). Built and run by tools/hbm_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ src, size_t n, uint32_t* out) {
    u32x4 acc = {0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * 256 * UNROLL;
    for (size_t i = (size_t)blockIdx.x * 256 * UNROLL + threadIdx.x; i < n; i += stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t j = i + (size_t)u * 256;
            if (j < n) v[u] = NT ? __builtin_nontemporal_load(src + j) : src[j];
            else v[u] = acc;
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[blockIdx.x] = 1;
}

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256 * UNROLL;
    for (size_t i = (size_t)blockIdx.x * 256 * UNROLL + threadIdx.x; i < n; i += stride) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t j = i + (size_t)u * 256;
            if (j < n) v[u] = NT ? __builtin_nontemporal_load(src + j) : src[j];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t j = i + (size_t)u * 256;
            if (j < n) {
                if (NT) __builtin_nontemporal_store(v[u], dst + j);
                else dst[j] = v[u];
            }
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void write_kernel(u32x4* __restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256;
    const u32x4 v = {1, 2, 3, 4};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        if (NT) __builtin_nontemporal_store(v, dst + i);
        else dst[i] = v;
    }
}

extern "C" {
int probe_read(const void* src, size_t bytes, void* out, int grid, int unroll, int nt, void* stream) {
    const size_t n = bytes / 16;
    hipStream_t s = (hipStream_t)stream;
#define RK(U)                                                                                        \
    if (unroll == U) {                                                                               \
        if (nt) hipLaunchKernelGGL((read_kernel<U, true>), dim3(grid), dim3(256), 0, s, (const u32x4*)src, n, (uint32_t*)out); \
        else hipLaunchKernelGGL((read_kernel<U, false>), dim3(grid), dim3(256), 0, s, (const u32x4*)src, n, (uint32_t*)out); \
    }
    RK(1) RK(2) RK(4) RK(8)
    return (int)hipGetLastError();
}

int probe_copy(const void* src, void* dst, size_t bytes, int grid, int unroll, int nt, void* stream) {
    const size_t n = bytes / 16;
    hipStream_t s = (hipStream_t)stream;
#define CK(U)                                                                                        \
    if (unroll == U) {                                                                               \
        if (nt) hipLaunchKernelGGL((copy_kernel<U, true>), dim3(grid), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, n); \
        else hipLaunchKernelGGL((copy_kernel<U, false>), dim3(grid), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, n); \
    }
    CK(1) CK(2) CK(4) CK(8)
    return (int)hipGetLastError();
}

int probe_write(void* dst, size_t bytes, int grid, int nt, void* stream) {
    const size_t n = bytes / 16;
    hipStream_t s = (hipStream_t)stream;
    if (nt) hipLaunchKernelGGL((write_kernel<true>), dim3(grid), dim3(256), 0, s, (u32x4*)dst, n);
    else hipLaunchKernelGGL((write_kernel<false>), dim3(grid), dim3(256), 0, s, (u32x4*)dst, n);
    return (int)hipGetLastError();
}
}

// Shard-pattern probe: blocks of `n` slots of `ss` bytes; item = (block, 16-B chunk); each
// lane loads `kin` slots and stores `nout` slots (XOR of the loads), like the codec kernels.
template <bool NT>
__global__ __launch_bounds__(256) void shard_kernel(const uint8_t* __restrict__ base, uint8_t* __restrict__ obase,
                                                    size_t bs, size_t ss, uint32_t cps, uint32_t total,
                                                    int kin, int nout, uint32_t* sink) {
    const uint32_t stride = gridDim.x * 256;
    u32x4 keep = {0, 0, 0, 0};
    for (uint32_t item = blockIdx.x * 256 + threadIdx.x; item < total; item += stride) {
        const uint32_t b = item / cps, c = item - b * cps;
        const uint8_t* src = base + (size_t)b * bs + (size_t)c * 16;
        u32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (j < kin) {
                const u32x4* p = reinterpret_cast<const u32x4*>(src + (size_t)j * ss);
                acc ^= NT ? __builtin_nontemporal_load(p) : *p;
            }
        }
        uint8_t* dst = obase + (size_t)b * bs + (size_t)c * 16;
        for (int r = 0; r < nout; ++r) {
            u32x4* q = reinterpret_cast<u32x4*>(dst + (size_t)r * ss);
            if (NT) __builtin_nontemporal_store(acc, q);
            else *q = acc;
        }
        keep ^= acc;
    }
    if (nout == 0 && (keep.x ^ keep.y ^ keep.z ^ keep.w) == 0x9E3779B9u) sink[0] = 1;
}

extern "C" int probe_shards(const void* base, void* obase, size_t bs, size_t ss, unsigned cps, unsigned nblocks,
                            int kin, int nout, int nt, int grid, void* sink, void* stream) {
    const uint32_t total = cps * nblocks;
    if (grid <= 0) grid = (total + 255) / 256;
    hipStream_t s = (hipStream_t)stream;
    if (nt) hipLaunchKernelGGL(shard_kernel<true>, dim3(grid), dim3(256), 0, s, (const uint8_t*)base, (uint8_t*)obase, bs, ss, cps, total, kin, nout, (uint32_t*)sink);
    else hipLaunchKernelGGL(shard_kernel<false>, dim3(grid), dim3(256), 0, s, (const uint8_t*)base, (uint8_t*)obase, bs, ss, cps, total, kin, nout, (uint32_t*)sink);
    return (int)hipGetLastError();
}

// Store-policy probe: like shard_kernel<NT loads>, with the store's cache-policy bits chosen
// by `pol`: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1, 4 sc1 nt, 5 sc0 sc1 nt.
template <int POL>
__device__ __forceinline__ void st_pol(u32x4* q, u32x4 v) {
    if constexpr (POL == 0) *q = v;
    else if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" :: "v"(q), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(q), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(q), "v"(v) : "memory");
    else if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" :: "v"(q), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" :: "v"(q), "v"(v) : "memory");
}

template <int POL>
__global__ __launch_bounds__(256) void shard_pol_kernel(const uint8_t* __restrict__ base, uint8_t* __restrict__ obase,
                                                        size_t bs, size_t ss, uint32_t cps, uint32_t total,
                                                        int kin, int nout) {
    const uint32_t stride = gridDim.x * 256;
    for (uint32_t item = blockIdx.x * 256 + threadIdx.x; item < total; item += stride) {
        const uint32_t b = item / cps, c = item - b * cps;
        const uint8_t* src = base + (size_t)b * bs + (size_t)c * 16;
        u32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if (j < kin) acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (size_t)j * ss));
        uint8_t* dst = obase + (size_t)b * bs + (size_t)c * 16;
        for (int r = 0; r < nout; ++r) st_pol<POL>(reinterpret_cast<u32x4*>(dst + (size_t)r * ss), acc);
    }
}

extern "C" int probe_store_policy(const void* base, void* obase, size_t bs, size_t ss, unsigned cps, unsigned nblocks,
                                  int kin, int nout, int pol, void* stream) {
    const uint32_t total = cps * nblocks;
    const int grid = (total + 255) / 256;
    hipStream_t s = (hipStream_t)stream;
#define SP(P) if (pol == P) hipLaunchKernelGGL(shard_pol_kernel<P>, dim3(grid), dim3(256), 0, s, (const uint8_t*)base, (uint8_t*)obase, bs, ss, cps, total, kin, nout);
    SP(0) SP(1) SP(2) SP(3) SP(4) SP(5)
    return (int)hipGetLastError();
}
