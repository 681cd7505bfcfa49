// fec_pack.hip — layout conversion on the device for the host-resident path (fec_capi.cpp).
//
// The caller's host layout is arbitrary (the reference's shards are biggest+2 bytes, e.g. 1202,
// packed back to back); the kernels need 16-byte-aligned shard slots. Rather than moving each
// 1202-byte shard with its own DMA row (2D copies of narrow rows run far below PCIe rate), the
// host path copies the caller's whole span with one linear DMA and converts it here, where
// bandwidth is two orders of magnitude higher than PCIe:
//   span -> stage   dword d of stage slot (b, j) gathers its 4 bytes from the span
//   stage -> packed dword d of the packed [nb][cols][len] image gathers its 4 bytes from stage
// and two gathers that read pinned host memory directly (see below).
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

// ---- device-side gather straight out of pinned host memory (no DMA engine, no host memcpy) ----
//
// A kernel load of a pinned, device-mapped host address crosses PCIe by itself; a wave that
// needs one 1202-byte shard reads exactly those bytes (tools/zerocopy_probe.hip measures the
// rate against hipMemcpyAsync). Used where a linear DMA would carry bytes nobody reads (the
// single parity plane a single-erasure decode needs out of a block's m), or where the host would
// otherwise memcpy every payload into a staging buffer first (the Go ABI's registered packet
// buffers, fec_go.h fec_go_encoder_submit_ref).

// 16 output bytes [16c, 16c + 16) of a shard of `len` bytes at src (any 2-byte alignment): the
// aligned dwords covering them, funnel-shifted; bytes at or past len are zero (no load reaches
// an aligned dword that starts at or past src + len, so nothing past the shard's last dword is
// touched).
__device__ __forceinline__ uint4 gather_chunk(const uint8_t* src, uint32_t len, uint32_t c) {
    const uint32_t sh = (uint32_t)((uintptr_t)src & 3u);
    const uint32_t b0 = 16u * c;
    if (b0 >= len) return make_uint4(0, 0, 0, 0);
    uint32_t v[4];
    if (sh == 0 && b0 + 16 <= len) {
        const uint4 x = *reinterpret_cast<const uint4*>(src + b0);
        v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w;
    } else {
        const uint32_t* A = reinterpret_cast<const uint32_t*>(src - sh) + 4 * c;
        const uint32_t lim = len + sh;   // aligned dword q is loaded when 4q < lim
        uint32_t d[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) d[q] = (b0 + 4u * q < lim && (q < 4 || sh)) ? A[q] : 0u;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = sh ? __builtin_amdgcn_alignbyte(d[q + 1], d[q], sh) : d[q];
    }
    if (b0 + 16 > len) {   // bytes at or past len: zero
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int keep = (int)len - (int)(b0 + 4u * q);
            v[q] = keep >= 4 ? v[q] : keep <= 0 ? 0u : (v[q] & ((1u << (8 * keep)) - 1u));
        }
    }
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// BE16(len) at [frame, frame + 2) of the chunk (reed_solomon.go:77-87), when it falls inside.
__device__ __forceinline__ uint4 put_frame(uint4 x, uint32_t c, uint32_t len, uint32_t frame) {
    if (frame == kNoFrame) return x;
    uint32_t v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (uint32_t t = 0; t < 2; ++t) {
        const uint32_t p = frame + t;
        if (p >= 16u * c && p < 16u * c + 16u) {
            const uint32_t byte = t == 0 ? (len >> 8) & 0xFFu : len & 0xFFu;
            const uint32_t q = (p - 16u * c) >> 2, s = 8u * (p & 3u);
            v[q] = (v[q] & ~(0xFFu << s)) | (byte << s);
        }
    }
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// One wave per descriptor: shard i written to dst + i * slot, all `slot` bytes (zeros past the
// framed content).
__global__ __launch_bounds__(256) void gather_desc_kernel(const GatherDesc* __restrict__ desc, uint32_t n,
                                                         uint8_t* __restrict__ dst, uint64_t slot) {
    const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (i >= n) return;
    const GatherDesc d = desc[i];
    const uint8_t* src = reinterpret_cast<const uint8_t*>(d.src);
    uint8_t* out = dst + (uint64_t)i * slot;
    const uint32_t chunks = (uint32_t)(slot >> 4);
    for (uint32_t c = lane; c < chunks; c += 64)
        *reinterpret_cast<uint4*>(out + 16u * c) = put_frame(gather_chunk(src, d.len, c), c, d.len, d.frame);
}

// Parity planes a reconstruct reads, straight from the caller's pinned parity region: plane r of
// block b (base + b*bs + r*ss, len bytes) goes to dst + (r*nb + b)*slot when the block's present
// mask makes parity r one of its first k present shards (klauspost ReconstructData, the first e
// present parities for e erased data shards); other (r, b) are not read or written.
__global__ __launch_bounds__(256) void gather_planes_kernel(const uint8_t* __restrict__ base, uint64_t bs, uint64_t ss,
                                                           uint32_t len, const uint32_t* __restrict__ masks,
                                                           uint32_t nb, uint32_t planes, uint32_t plane_bits,
                                                           uint32_t k, uint8_t* __restrict__ dst, uint64_t slot) {
    const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (i >= nb * planes) return;
    const uint32_t r = i / nb, b = i - r * nb;
    if (!((plane_bits >> r) & 1u)) return;   // a plane the host path moves by DMA
    const uint32_t mask = masks[b];
    const uint32_t e = k - (uint32_t)__popc(mask & low_mask(k));
    const uint32_t par = k < 32 ? mask >> k : 0u;
    if (e == 0 || !((par >> r) & 1u) || (uint32_t)__popc(par & low_mask(r)) >= e) return;
    const uint8_t* src = base + (uint64_t)b * bs + (uint64_t)r * ss;
    uint8_t* out = dst + (uint64_t)i * slot;
    const uint32_t chunks = (uint32_t)(slot >> 4);
    for (uint32_t c = lane; c < chunks; c += 64) *reinterpret_cast<uint4*>(out + 16u * c) = gather_chunk(src, len, c);
}

}  // namespace

hipError_t launch_gather_desc(const GatherDesc* desc, uint32_t n, uint8_t* dst, uint64_t slot, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_desc_kernel, dim3((n + 3) / 4), dim3(256), 0, s, desc, n, dst, slot);
    return hipGetLastError();
}

hipError_t launch_gather_planes(const uint8_t* base, uint64_t bs, uint64_t ss, uint32_t len, const uint32_t* masks,
                                uint32_t nb, uint32_t planes, uint32_t plane_bits, uint32_t k, uint8_t* dst,
                                uint64_t slot, hipStream_t s) {
    const uint64_t n = (uint64_t)nb * planes;
    if (n == 0 || plane_bits == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_planes_kernel, dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, s, base, bs, ss, len, masks,
                       nb, planes, plane_bits, k, dst, slot);
    return hipGetLastError();
}

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
