// fec_synth.hip — synthetic workload generator on the device (bench.py, tests).
//
// BASELINE.md §2 inputs: payload bytes from splitmix64 keyed by (seed, block, shard, word), so
// every rank of a sharded run regenerates exactly its slice of one global batch in HBM, and the
// host restatement (0xfec_amd/shard.py synth_payload_blocks / synth_single_erasures) produces the
// same bytes for the oracle. Not part of the reference's interface: this is the data loader of
// the benchmark, kept on the device so a 2^20-block batch (10 GB) is generated in milliseconds.
#include <hip/hip_runtime.h>

#include "../../include/fec_hip.h"
#include "../../include/fec_synth.h"
#include "fec_kernels.hpp"

namespace fk {

namespace {

constexpr uint64_t kGold = 0x9E3779B97F4A7C15ull;

__host__ __device__ inline uint64_t splitmix_fin(uint64_t x) {
    x += kGold;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// word w of data shard j of global block b (shard.py synth_payload_blocks)
__device__ inline uint64_t synth_word(uint64_t seed, uint64_t b, uint64_t j, uint64_t w) {
    return splitmix_fin((seed * kGold) ^ (b << 24) ^ (j << 16) ^ w);
}

// erased data shard of global block b: a key no data word uses (the low 24 bits of a data key
// are shard << 16 ^ word with word < 2^13)
__device__ inline uint64_t erasure_key(uint64_t seed, uint64_t b) {
    return splitmix_fin((seed * kGold) ^ (b << 24) ^ 0xFFFFFFull);
}

struct SynthArgs {
    uint8_t* data;
    uint64_t bs, ss;
    uint64_t seed, first;
    uint32_t k, len, cps;   // len = payload bytes; cps = 16-byte chunks per shard slot
    uint64_t total;         // nblocks * k * cps
};

// One lane = one 16-byte chunk of one shard slot: payload bytes, then the big-endian uint16
// length trailer at [len, len+2) (reed_solomon.go:77-87), zeros to the end of the slot.
__global__ __launch_bounds__(256) void synth_data_kernel(SynthArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= a.total) return;
    const uint64_t c = t % a.cps;
    const uint64_t bj = t / a.cps;
    const uint64_t j = bj % a.k, b = bj / a.k;
    const uint64_t w0 = synth_word(a.seed, a.first + b, j, 2 * c), w1 = synth_word(a.seed, a.first + b, j, 2 * c + 1);
    uint32_t out[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const uint32_t i = (uint32_t)(16 * c) + 4 * q + y;   // byte index in the shard
            const uint64_t w = (4 * q + y) < 8 ? w0 : w1;
            uint32_t byte = 0;
            if (i < a.len) byte = (uint32_t)(w >> (8 * ((4 * q + y) & 7))) & 0xFF;
            else if (i == a.len) byte = (a.len >> 8) & 0xFF;
            else if (i == a.len + 1) byte = a.len & 0xFF;
            v |= byte << (8 * y);
        }
        out[q] = v;
    }
    *reinterpret_cast<uint4*>(a.data + b * a.bs + j * a.ss + 16 * c) = make_uint4(out[0], out[1], out[2], out[3]);
}

__global__ __launch_bounds__(256) void synth_erasure_kernel(uint64_t seed, uint64_t first, uint64_t nblocks,
                                                            uint32_t k, uint32_t all, uint32_t* masks,
                                                            int32_t* erased) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nblocks) return;
    const uint32_t e = (uint32_t)(erasure_key(seed, first + b) % k);
    masks[b] = all & ~(1u << e);
    if (erased) erased[b] = (int32_t)e;
}

}  // namespace

}  // namespace fk

extern "C" {

int fec_synth_data(fec_ctx* ctx, uint64_t seed, uint64_t first_block, size_t nblocks, int k, size_t payload_len,
                   uint8_t* data, size_t block_stride, size_t shard_stride) {
    if (!ctx || !data || k <= 0 || payload_len > 65535) return FEC_ERR_INVALID_ARG;
    if ((shard_stride & 15) || (block_stride & 15) || ((uintptr_t)data & 15)) return FEC_ERR_ALIGNMENT;
    if (shard_stride < payload_len + 2 || block_stride < (size_t)k * shard_stride) return FEC_ERR_INVALID_ARG;
    if (nblocks == 0) return FEC_OK;
    fk::SynthArgs a{};
    a.data = data;
    a.bs = block_stride;
    a.ss = shard_stride;
    a.seed = seed;
    a.first = first_block;
    a.k = (uint32_t)k;
    a.len = (uint32_t)payload_len;
    a.cps = (uint32_t)(shard_stride / 16);
    a.total = (uint64_t)nblocks * a.k * a.cps;
    hipStream_t s = (hipStream_t)fec_ctx_stream(ctx);
    const uint64_t grid = (a.total + 255) / 256;
    if (grid > 0x7FFFFFFFull) return FEC_ERR_INVALID_ARG;
    hipLaunchKernelGGL(fk::synth_data_kernel, dim3((uint32_t)grid), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

int fec_synth_single_erasures(fec_ctx* ctx, uint64_t seed, uint64_t first_block, size_t nblocks, int k, int m,
                              uint32_t* masks, int32_t* erased) {
    if (!ctx || !masks || k <= 0 || m < 0 || k + m > FEC_MAX_DECODE_SHARDS) return FEC_ERR_INVALID_ARG;
    if (nblocks == 0) return FEC_OK;
    hipStream_t s = (hipStream_t)fec_ctx_stream(ctx);
    const uint64_t grid = (nblocks + 255) / 256;
    if (grid > 0x7FFFFFFFull) return FEC_ERR_INVALID_ARG;
    hipLaunchKernelGGL(fk::synth_erasure_kernel, dim3((uint32_t)grid), dim3(256), 0, s, seed, (uint64_t)first_block,
                       (uint64_t)nblocks, (uint32_t)k, fk::low_mask((uint32_t)(k + m)), masks, erased);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

}  // extern "C"
