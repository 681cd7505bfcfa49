// fec_pack.hip — layout conversion on the device for the host-resident path (fec_capi.cpp).
//
// The caller's host layout is arbitrary (the reference's shards are biggest+2 bytes, e.g. 1202,
// packed back to back); the kernels need 16-byte-aligned shard slots. Rather than moving each
// 1202-byte shard with its own DMA row (2D copies of narrow rows run far below PCIe rate), the
// host path copies the caller's whole span with one linear DMA and converts it here, where
// bandwidth is two orders of magnitude higher than PCIe:
//   span -> stage   dword d of stage slot (b, j) gathers its 4 bytes from the span
//   stage -> packed dword d of the packed [nb][cols][len] image gathers its 4 bytes from stage
#include <hip/hip_runtime.h>

#include "fec_kernels.hpp"

namespace fk {

namespace {

struct PackArgs {
    uint8_t* dst;
    const uint8_t* src;
    uint64_t src_bs, src_ss;   // span: shard j of block b at src + b*src_bs + j*src_ss
    uint64_t st_bs, st_ss;     // stage: slot (b, j) at + b*st_bs + j*st_ss
    uint32_t nb, cols, len, wps;   // wps: dwords per stage slot written (ceil(len / 4))
    uint64_t total;            // dwords to produce
};

__global__ __launch_bounds__(256) void span_to_stage_kernel(PackArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= a.total) return;
    const uint64_t w = t % a.wps, r = t / a.wps;
    const uint64_t j = r % a.cols, b = r / a.cols;
    const uint8_t* s = a.src + b * a.src_bs + j * a.src_ss;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t col = (uint32_t)(4 * w) + q;
        if (col < a.len) v |= (uint32_t)s[col] << (8 * q);
    }
    *reinterpret_cast<uint32_t*>(a.dst + b * a.st_bs + j * a.st_ss + 4 * w) = v;
}

__global__ __launch_bounds__(256) void stage_to_packed_kernel(PackArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= a.total) return;
    const uint64_t bytes = (uint64_t)a.nb * a.cols * a.len;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint64_t i = 4 * t + q;
        if (i < bytes) {
            const uint64_t r = i / a.len, col = i - r * a.len;
            const uint64_t j = r % a.cols, b = r / a.cols;
            v |= (uint32_t)a.src[b * a.st_bs + j * a.st_ss + col] << (8 * q);
        }
    }
    *reinterpret_cast<uint32_t*>(a.dst + 4 * t) = v;   // dst holds round_up(bytes, 4)
}

}  // namespace

hipError_t launch_span_to_stage(uint8_t* stage, uint64_t st_bs, uint64_t st_ss, const uint8_t* span, uint64_t src_bs,
                                uint64_t src_ss, uint32_t nb, uint32_t cols, uint32_t len, hipStream_t s) {
    PackArgs a{};
    a.dst = stage;
    a.src = span;
    a.src_bs = src_bs;
    a.src_ss = src_ss;
    a.st_bs = st_bs;
    a.st_ss = st_ss;
    a.nb = nb;
    a.cols = cols;
    a.len = len;
    a.wps = (len + 3) / 4;
    a.total = (uint64_t)nb * cols * a.wps;
    if (a.total == 0) return hipSuccess;
    hipLaunchKernelGGL(span_to_stage_kernel, dim3((uint32_t)((a.total + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_stage_to_packed(uint8_t* packed, const uint8_t* stage, uint64_t st_bs, uint64_t st_ss, uint32_t nb,
                                  uint32_t cols, uint32_t len, hipStream_t s) {
    PackArgs a{};
    a.dst = packed;
    a.src = stage;
    a.st_bs = st_bs;
    a.st_ss = st_ss;
    a.nb = nb;
    a.cols = cols;
    a.len = len;
    a.total = ((uint64_t)nb * cols * len + 3) / 4;
    if (a.total == 0) return hipSuccess;
    hipLaunchKernelGGL(stage_to_packed_kernel, dim3((uint32_t)((a.total + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace fk
