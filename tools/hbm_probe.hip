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
