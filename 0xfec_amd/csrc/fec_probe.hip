// fec_probe.hip — traffic twins of the headline kernels (measurement only; include/fec_probe.h).
//
// A twin moves exactly the bytes its kernel moves, with the same launch geometry (flat grid, one
// 16-byte chunk per lane, XCD-contiguous workgroup order, the same residency cap through dynamic
// LDS, the same cache policies: non-temporal loads, and the kernel's store policy, zero-padded tail
// chunks) and no field arithmetic: the XOR of
// its inputs stands in for the products. Timed on the same box and buffers right after the
// kernel, its rate is that box's ceiling for the kernel's access shape, so a bench line can say
// how much of a kernel's distance to the 8 TB/s spec is the box and how much is the kernel.
//   encode twin   rs_encode_fixed_kernel<K, M, ..> (fec_encode.hip): K shard loads, M stores
//   recover twin  rs_recover_direct_kernel<K, ..> (fec_recover.hip) on single-erasure blocks:
//                 the k-1 other data shards and the first present parity, one store to `out`
//   rebuild twin  the multi-erasure decode (sorted plans + fec_rebuild.hip) of RS(16,24) / RS(20,30):
//                 per block the first k present shards and one store per erased data shard, in
//                 block order (the rebuild walks the same blocks in plan order within 64-block
//                 windows), at the rebuild's residency; no plan kernel
//   stream        shape-independent reference: nin consecutive shards of each block read, one
//                 store per block, no masks (the simplest mixed read/write stream of the layout)
// Every twin takes a residency (workgroups per CU; -1: the twinned kernel's own), so a caller can
// take each twin's best over residency as the box's ceiling for its access shape.
#include <string.h>

#include <algorithm>
#include <chrono>

#include "../../include/fec_hip.h"
#include "../../include/fec_probe.h"
#include "fec_device.hpp"

namespace fk {
namespace {

// SP: the store policy of the kernel twinned (fec_device.hpp st16p; RS(8,12): knobs st_pol / dst_pol)
template <int K, int M, int SP = 0>
__global__ __launch_bounds__(kThreads) void probe_encode_kernel(EncodeArgs a) {
    extern __shared__ uint8_t smem[];   // residency only, as the encode's staged tables
    const uint32_t it = xcd_order() * kThreads + threadIdx.x;
    if (it >= a.total) return;
    const uint32_t b = fdiv(it, a.div_cps);
    const uint32_t c = it - b * a.cps;
    const uint8_t* src = a.in + (uint64_t)b * a.in_bs + (uint64_t)c * kChunk;
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld16<true>(src + (uint64_t)j * a.ss);
    uint4 acc[M];
#pragma unroll
    for (int r = 0; r < M; ++r) acc[r] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < K; ++j) {
        acc[j % M].x ^= x[j].x;
        acc[j % M].y ^= x[j].y;
        acc[j % M].z ^= x[j].z;
        acc[j % M].w ^= x[j].w;
    }
    uint8_t* dst = a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk;
    const uint32_t nb = min(a.len - c * kChunk, (uint32_t)kChunk);
#pragma unroll
    for (int r = 0; r < M; ++r) st16p<SP>(dst + (uint64_t)r * a.ss, keep_bytes(acc[r], nb));
    if (a.k == 0x5A5A5A5Au) smem[0] = 1;   // never: keeps the LDS allocation
}

struct RecoverProbeArgs {
    const uint8_t* data;
    const uint8_t* parity;
    uint8_t* out;
    const uint32_t* masks;
    uint64_t dbs, pbs, ss, out_bs;
    uint32_t len, cps, total, nblocks, nin;
    FastDiv div_cps;
};

template <int K, int SP = 0>
__global__ __launch_bounds__(kThreads) void probe_recover_kernel(RecoverProbeArgs a, uint32_t m) {
    extern __shared__ uint8_t smem[];   // residency only, as the decode's wave slices
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t i0 = xcd_order() * kThreads + (wave << 6);
    if (i0 >= a.total) return;
    // the wave's <= 3 block masks by scalar loads, as the direct kernel
    const uint32_t bfirst = fdiv(i0, a.div_cps);
    typedef __attribute__((address_space(4))) const uint32_t ConstU32;
    ConstU32* cm = (ConstU32*)a.masks;
    const uint32_t bf = (uint32_t)__builtin_amdgcn_readfirstlane((int)bfirst), last = a.nblocks - 1;
    const uint32_t m0 = cm[bf];
    const uint32_t m1 = cm[(uint32_t)__builtin_amdgcn_readfirstlane((int)min(bf + 1, last))];
    const uint32_t m2 = cm[(uint32_t)__builtin_amdgcn_readfirstlane((int)min(bf + 2, last))];
    const uint32_t item = i0 + lane;
    if (item >= a.total) return;
    const uint32_t blk = fdiv(item, a.div_cps);
    const uint32_t g = blk - bfirst;
    const uint32_t c = item - blk * a.cps;
    const uint32_t mask = (g == 0 ? m0 : g == 1 ? m1 : m2) & low_mask(K + m);
    const uint32_t E0 = __ffs(~mask & low_mask(K)) - 1;
    const uint32_t R0 = __ffs(mask >> K) - 1;
    if (__popc(mask & low_mask(K)) != K - 1 || R0 >= m) return;   // not a single-erasure block: nothing read
    const uint8_t* d0 = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K - 1; ++j) x[j] = ld16<true>(d0 + (uint64_t)(j + (j >= (int)E0)) * a.ss);
    x[K - 1] = ld16<true>(a.parity + (uint64_t)blk * a.pbs + (uint64_t)R0 * a.ss + (uint64_t)c * kChunk);
    uint4 acc = x[0];
#pragma unroll
    for (int j = 1; j < K; ++j) {
        acc.x ^= x[j].x;
        acc.y ^= x[j].y;
        acc.z ^= x[j].z;
        acc.w ^= x[j].w;
    }
    const uint32_t nb = min(a.len - c * kChunk, (uint32_t)kChunk);
    // out == data: in place, into the erased shard's own slot (the routed in-place reconstruct's
    // store); else the separate output (the recover's)
    uint8_t* dst = a.out == a.data ? const_cast<uint8_t*>(d0) + (uint64_t)E0 * a.ss
                                   : a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk;
    st16p<SP>(dst, keep_bytes(acc, nb));
    if (a.nin == 0x5A5A5A5Au) smem[0] = 1;   // never: keeps the LDS allocation
}

template <int K, int R>
__global__ __launch_bounds__(kThreads) void probe_rebuild_kernel(RecoverProbeArgs a, uint32_t m) {
    extern __shared__ uint8_t smem[];   // residency only, as the rebuild's table and wave slices
    const uint32_t item = xcd_order() * kThreads + threadIdx.x;
    if (item >= a.total) return;
    const uint32_t blk = fdiv(item, a.div_cps);
    const uint32_t c = item - blk * a.cps;
    const uint32_t mask = a.masks[blk] & low_mask(K + m);
    const uint32_t e = K - __popc(mask & low_mask(K));
    if (e == 0 || (uint32_t)__popc(mask) < K) return;   // nothing to rebuild / unrecoverable: nothing read
    const uint8_t* d0 = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    const uint8_t* p0 = a.parity + (uint64_t)blk * a.pbs + (uint64_t)c * kChunk;
    uint32_t rest = mask;
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < K; ++j) {   // the first K present shards, in index order
        const uint32_t s = __ffs(rest) - 1;
        rest &= rest - 1;
        const uint4 x = ld16<true>(s < (uint32_t)K ? d0 + (uint64_t)s * a.ss : p0 + (uint64_t)(s - K) * a.ss);
        acc.x ^= x.x;
        acc.y ^= x.y;
        acc.z ^= x.z;
        acc.w ^= x.w;
    }
    const uint32_t nb = min(a.len - c * kChunk, (uint32_t)kChunk);
    uint8_t* o = a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if ((uint32_t)r < e) st16<true>(o + (uint64_t)r * a.ss, keep_bytes(acc, nb));
    if (a.nin == 0x5A5A5A5Au) smem[0] = 1;   // never: keeps the LDS allocation
}

// NIN consecutive shards of the block read (data at stride ss inside the block), their XOR stored
// once per chunk: the simplest mixed read / write stream of the bench layout.
template <int NIN>
__global__ __launch_bounds__(kThreads) void probe_stream_kernel(RecoverProbeArgs a) {
    extern __shared__ uint8_t smem[];   // residency only
    const uint32_t item = xcd_order() * kThreads + threadIdx.x;
    if (item >= a.total) return;
    const uint32_t blk = fdiv(item, a.div_cps);
    const uint32_t c = item - blk * a.cps;
    const uint8_t* d0 = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    uint4 x[NIN];
#pragma unroll
    for (int j = 0; j < NIN; ++j) x[j] = ld16<true>(d0 + (uint64_t)j * a.ss);
    uint4 acc = x[0];
#pragma unroll
    for (int j = 1; j < NIN; ++j) {
        acc.x ^= x[j].x;
        acc.y ^= x[j].y;
        acc.z ^= x[j].z;
        acc.w ^= x[j].w;
    }
    const uint32_t nb = min(a.len - c * kChunk, (uint32_t)kChunk);
    st16<true>(a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk, keep_bytes(acc, nb));
    if (a.nin == 0x5A5A5A5Au) smem[0] = 1;   // never: keeps the LDS allocation
}

int stream_of(fec_ctx* ctx, hipStream_t* s) {
    if (!ctx) return FEC_ERR_INVALID_ARG;
    *s = (hipStream_t)fec_ctx_stream(ctx);
    int dev = 0;
    if (hipStreamGetDevice(*s, &dev) != hipSuccess || hipSetDevice(dev) != hipSuccess) {
        (void)hipGetLastError();
        return FEC_ERR_HIP;
    }
    return FEC_OK;
}

bool layout_ok(const void* p, size_t bs, size_t ss, size_t len) {
    return p && !((uintptr_t)p & 15) && !(bs & 15) && !(ss & 15) && ss >= len;
}

}  // namespace
}  // namespace fk

extern "C" int fec_probe_encode_traffic(fec_ctx* ctx, int k, int m, size_t shard_len, size_t nblocks,
                                        const void* data, size_t dbs, void* parity, size_t pbs, size_t ss, int wpc) {
    using namespace fk;
    hipStream_t s;
    int rc = stream_of(ctx, &s);
    if (rc) return rc;
    if (!((k == 2 && m == 1) || (k == 8 && m == 4) || (k == 16 && m == 8) || (k == 20 && m == 10)))
        return FEC_ERR_INVALID_ARG;
    if (!layout_ok(data, dbs, ss, shard_len) || !layout_ok(parity, pbs, ss, shard_len) || shard_len == 0)
        return FEC_ERR_ALIGNMENT;
    const uint32_t cps = (uint32_t)((shard_len + kChunk - 1) / kChunk);
    if ((uint64_t)nblocks * cps >= (uint64_t(1) << 31)) return FEC_ERR_INVALID_ARG;
    if (nblocks == 0) return FEC_OK;
    EncodeArgs a{};
    a.in = (const uint8_t*)data;
    a.out = (uint8_t*)parity;
    a.in_bs = dbs;
    a.out_bs = pbs;
    a.ss = ss;
    a.k = (uint32_t)k;
    a.m = (uint32_t)m;
    a.len = (uint32_t)shard_len;
    a.cps = cps;
    a.total = (uint32_t)(nblocks * cps);
    a.div_cps = make_fastdiv(cps);
    const int grid = (int)((a.total + kThreads - 1) / kThreads);
    // the encode's own residency (wpc -1): RS(8,12) g_tune.enc_wpc workgroups per CU, RS(2,3)
    // uncapped (no LDS); RS(16,24) and RS(20,30) as the bit-sliced encode (g_tune.enc_bwpc; the
    // bit-sliced kernel takes two chunks a lane, the twin one)
    if (wpc < 0) wpc = k >= 16 ? (int)g_tune.enc_bwpc : k == 2 ? 0 : (int)g_tune.enc_wpc;
    const size_t lds = occupancy_lds(wpc, k == 8 ? (size_t)m * k * 32 : 0);
    // the encodes' store policy for this layout (encode_store_policy)
    a.sp = encode_store_policy(g_tune.st_pol, data, dbs, parity, pbs, nblocks);
#define FEC_ENC_TWIN(K, M)                                                                              \
    do {                                                                                                \
        if (a.sp == 1)                                                                                  \
            hipLaunchKernelGGL((probe_encode_kernel<K, M, 1>), dim3(grid), dim3(kThreads), lds, s, a); \
        else                                                                                            \
            hipLaunchKernelGGL((probe_encode_kernel<K, M, 0>), dim3(grid), dim3(kThreads), lds, s, a); \
    } while (0)
    if (k == 2) FEC_ENC_TWIN(2, 1);
    else if (k == 8) FEC_ENC_TWIN(8, 4);
    else if (k == 16) FEC_ENC_TWIN(16, 8);
    else FEC_ENC_TWIN(20, 10);
#undef FEC_ENC_TWIN
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

extern "C" int fec_probe_recover_traffic(fec_ctx* ctx, int k, int m, size_t shard_len, size_t nblocks,
                                         const void* data, size_t dbs, const void* parity, size_t pbs, size_t ss,
                                         const uint32_t* masks, void* out, size_t out_bs, int wpc) {
    using namespace fk;
    hipStream_t s;
    int rc = stream_of(ctx, &s);
    if (rc) return rc;
    if (!((k == 2 && m == 1) || (k == 8 && m == 4) || (k == 16 && m == 8) || (k == 20 && m == 10)))
        return FEC_ERR_INVALID_ARG;
    if (!masks || !layout_ok(data, dbs, ss, shard_len) || !layout_ok(parity, pbs, ss, shard_len) ||
        !layout_ok(out, out_bs, 16, 0) || shard_len == 0 || out_bs < ((shard_len + 15) & ~size_t(15)))
        return FEC_ERR_ALIGNMENT;
    const uint32_t cps = (uint32_t)((shard_len + kChunk - 1) / kChunk);
    if ((uint64_t)nblocks * cps >= (uint64_t(1) << 31) || cps < 32) return FEC_ERR_INVALID_ARG;
    if (nblocks == 0) return FEC_OK;
    RecoverProbeArgs a{};
    a.data = (const uint8_t*)data;
    a.parity = (const uint8_t*)parity;
    a.out = (uint8_t*)out;
    a.masks = masks;
    a.dbs = dbs;
    a.pbs = pbs;
    a.ss = ss;
    a.out_bs = out_bs;
    a.len = (uint32_t)shard_len;
    a.cps = cps;
    a.total = (uint32_t)(nblocks * cps);
    a.nblocks = (uint32_t)nblocks;
    a.div_cps = make_fastdiv(cps);
    const int grid = (int)((a.total + kThreads - 1) / kThreads);
    // the direct decode's residency (wpc -1; fec_recover.hip direct_launch): 3 workgroups per CU for
    // k >= 8, small codes uncapped; LDS as its four wave slices of 3 blocks' PermTab rows
    if (wpc < 0) wpc = g_tune.dir_wpc >= 0 ? (int)g_tune.dir_wpc : (k >= 8 ? 3 : 0);
    const size_t lds = occupancy_lds(wpc, (size_t)4 * 3 * k * 32);
    const uint32_t um = (uint32_t)m;
    if (k == 2) hipLaunchKernelGGL((probe_recover_kernel<2>), dim3(grid), dim3(kThreads), lds, s, a, um);
    else if (k == 8 && decode_store_policy(g_tune.dst_pol, data, dbs, parity, pbs, out, out_bs, nblocks) == 3)
        hipLaunchKernelGGL((probe_recover_kernel<8, 3>), dim3(grid), dim3(kThreads), lds, s, a, um);
    else if (k == 8) hipLaunchKernelGGL((probe_recover_kernel<8>), dim3(grid), dim3(kThreads), lds, s, a, um);
    else if (k == 16) hipLaunchKernelGGL((probe_recover_kernel<16>), dim3(grid), dim3(kThreads), lds, s, a, um);
    else hipLaunchKernelGGL((probe_recover_kernel<20>), dim3(grid), dim3(kThreads), lds, s, a, um);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

extern "C" int fec_probe_rebuild_traffic(fec_ctx* ctx, int k, int m, size_t shard_len, size_t nblocks,
                                         const void* data, size_t dbs, const void* parity, size_t pbs, size_t ss,
                                         const uint32_t* masks, void* out, size_t out_bs, int wpc) {
    using namespace fk;
    hipStream_t s;
    int rc = stream_of(ctx, &s);
    if (rc) return rc;
    if (!((k == 16 && m == 8) || (k == 20 && m == 10))) return FEC_ERR_INVALID_ARG;
    if (!masks || !layout_ok(data, dbs, ss, shard_len) || !layout_ok(parity, pbs, ss, shard_len) ||
        !layout_ok(out, out_bs, 16, 0) || shard_len == 0 || out_bs < (size_t)m * ((shard_len + 15) & ~size_t(15)) ||
        (ss | out_bs) >> 32)
        return FEC_ERR_ALIGNMENT;
    const uint32_t cps = (uint32_t)((shard_len + kChunk - 1) / kChunk);
    if ((uint64_t)nblocks * cps >= (uint64_t(1) << 31)) return FEC_ERR_INVALID_ARG;
    if (nblocks == 0) return FEC_OK;
    RecoverProbeArgs a{};
    a.data = (const uint8_t*)data;
    a.parity = (const uint8_t*)parity;
    a.out = (uint8_t*)out;
    a.masks = masks;
    a.dbs = dbs;
    a.pbs = pbs;
    a.ss = ss;
    a.out_bs = out_bs;
    a.len = (uint32_t)shard_len;
    a.cps = cps;
    a.total = (uint32_t)(nblocks * cps);
    a.nblocks = (uint32_t)nblocks;
    a.div_cps = make_fastdiv(cps);
    const int grid = (int)((a.total + kThreads - 1) / kThreads);
    // the rebuild's residency (wpc -1): its VGPRs allow 4 workgroups per CU (fec_rebuild.hip, uncapped)
    const size_t lds = occupancy_lds(wpc < 0 ? 4 : wpc, 0);
    const uint32_t um = (uint32_t)m;
    if (k == 16) hipLaunchKernelGGL((probe_rebuild_kernel<16, 8>), dim3(grid), dim3(kThreads), lds, s, a, um);
    else hipLaunchKernelGGL((probe_rebuild_kernel<20, 10>), dim3(grid), dim3(kThreads), lds, s, a, um);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

extern "C" int fec_probe_stream_traffic(fec_ctx* ctx, int nin, size_t shard_len, size_t nblocks, const void* in,
                                        size_t in_bs, void* out, size_t out_bs, size_t ss, int wpc) {
    using namespace fk;
    hipStream_t s;
    int rc = stream_of(ctx, &s);
    if (rc) return rc;
    if (nin != 2 && nin != 8 && nin != 16 && nin != 20) return FEC_ERR_INVALID_ARG;
    if (!layout_ok(in, in_bs, ss, shard_len) || !layout_ok(out, out_bs, 16, 0) || shard_len == 0 ||
        out_bs < ((shard_len + 15) & ~size_t(15)) || in_bs < (size_t)(nin - 1) * ss + shard_len)
        return FEC_ERR_ALIGNMENT;
    const uint32_t cps = (uint32_t)((shard_len + kChunk - 1) / kChunk);
    if ((uint64_t)nblocks * cps >= (uint64_t(1) << 31)) return FEC_ERR_INVALID_ARG;
    if (nblocks == 0) return FEC_OK;
    RecoverProbeArgs a{};
    a.data = (const uint8_t*)in;
    a.out = (uint8_t*)out;
    a.dbs = in_bs;
    a.ss = ss;
    a.out_bs = out_bs;
    a.len = (uint32_t)shard_len;
    a.cps = cps;
    a.total = (uint32_t)(nblocks * cps);
    a.nblocks = (uint32_t)nblocks;
    a.nin = (uint32_t)nin;
    a.div_cps = make_fastdiv(cps);
    const int grid = (int)((a.total + kThreads - 1) / kThreads);
    const size_t lds = occupancy_lds(wpc < 0 ? 0 : wpc, 0);
    if (nin == 2) hipLaunchKernelGGL((probe_stream_kernel<2>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (nin == 8) hipLaunchKernelGGL((probe_stream_kernel<8>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (nin == 16) hipLaunchKernelGGL((probe_stream_kernel<16>), dim3(grid), dim3(kThreads), lds, s, a);
    else hipLaunchKernelGGL((probe_stream_kernel<20>), dim3(grid), dim3(kThreads), lds, s, a);
    return hipGetLastError() == hipSuccess ? FEC_OK : FEC_ERR_HIP;
}

// The host link as the host path drives it (fec_capi.cpp HostPipe): hipMemcpyAsync between pinned
// host and device buffers of `bytes`, H2D alone, D2H alone, and both at once on two non-blocking
// streams; the best of `reps` by host wall clock around a device synchronisation. GB/s into
// out[0..2]. Buffers are allocated and freed here.
extern "C" int fec_probe_link(fec_ctx* ctx, size_t bytes, int reps, double* out) {
    using namespace fk;
    hipStream_t s0;
    int rc = stream_of(ctx, &s0);
    if (rc) return rc;
    if (!out || bytes == 0 || reps <= 0) return FEC_ERR_INVALID_ARG;
    uint8_t *h_up = nullptr, *h_dn = nullptr, *d_up = nullptr, *d_dn = nullptr;
    hipStream_t su = nullptr, sd = nullptr;
    rc = FEC_ERR_HIP;
    auto best = [&](auto fn) -> double {
        fn();
        if (hipDeviceSynchronize() != hipSuccess) return -1.0;
        double b = 1e30;
        for (int r = 0; r < reps; ++r) {
            const auto t0 = std::chrono::steady_clock::now();
            fn();
            if (hipDeviceSynchronize() != hipSuccess) return -1.0;
            b = std::min(b, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        return b;
    };
    if (hipHostMalloc(&h_up, bytes, hipHostMallocDefault) == hipSuccess &&
        hipHostMalloc(&h_dn, bytes, hipHostMallocDefault) == hipSuccess && hipMalloc(&d_up, bytes) == hipSuccess &&
        hipMalloc(&d_dn, bytes) == hipSuccess && hipStreamCreateWithFlags(&su, hipStreamNonBlocking) == hipSuccess &&
        hipStreamCreateWithFlags(&sd, hipStreamNonBlocking) == hipSuccess) {
        memset(h_up, 1, bytes);
        memset(h_dn, 2, bytes);
        (void)hipMemset(d_dn, 3, bytes);
        (void)hipMemset(d_up, 4, bytes);
        (void)hipDeviceSynchronize();
        // both directions first, on the fresh streams: the runtime keeps a stream on the SDMA engine
        // it first got, and two copies issued back to back on fresh streams get different engines
        // (pcie_duplex_probe: 48.6 GB/s each way); streams that each ran a copy alone first can end
        // up sharing one engine (28.7 each way, serialised)
        const double tb = best([&] {
            (void)hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, su);
            (void)hipMemcpyAsync(h_dn, d_dn, bytes, hipMemcpyDeviceToHost, sd);
        });
        const double tu = best([&] { (void)hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, su); });
        const double td = best([&] { (void)hipMemcpyAsync(h_dn, d_dn, bytes, hipMemcpyDeviceToHost, sd); });
        if (tu > 0 && td > 0 && tb > 0) {
            out[0] = (double)bytes / tu / 1e9;
            out[1] = (double)bytes / td / 1e9;
            out[2] = (double)bytes / tb / 1e9;
            rc = FEC_OK;
        }
    }
    for (hipStream_t q : {su, sd})
        if (q) (void)hipStreamDestroy(q);
    for (void* q : {(void*)h_up, (void*)h_dn})
        if (q) (void)hipHostFree(q);
    for (void* q : {(void*)d_up, (void*)d_dn})
        if (q) (void)hipFree(q);
    (void)hipGetLastError();
    return rc;
}
