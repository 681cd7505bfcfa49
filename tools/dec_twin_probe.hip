// dec_twin_probe.hip — diagnostics only (tools/dec_twin_probe.py): what the RS(8,12) single-erasure
// decode's access shape moves with and without the dependent present-mask load in front of each
// wave's shard loads, at every residency, beside the library's own decode.
//
// Every variant is a flat grid, one 16-byte chunk per lane, XCD-contiguous workgroup order,
// non-temporal loads and stores, the bench layout (data [B][8][ss], parity [B][4][ss], out [B][ss]):
//   MODE 0  the wave's <= 3 masks by one vector load, then readlane (rs_recover_direct_kernel's prefix)
//   MODE 1  no mask load: erased index from a hash of the block, first parity (addresses known at launch)
//   MODE 2  the wave's masks by scalar loads (uniform address: the constant cache)
//   MODE 3  shape-independent reference: the block's 8 data shards (no holes, no parity region) + 1 store
// ARITH 0: XOR of the inputs (traffic twin); 1: the decode's field arithmetic (8 v_perm products per
// dword pair from per-wave PermTab rows expanded into LDS, as the direct kernel does).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../0xfec_amd/csrc/fec_device.hpp"

using namespace fk;

struct ProbeArgs {
    const uint8_t* data;
    const uint8_t* parity;
    uint8_t* out;
    const uint32_t* masks;
    uint64_t dbs, pbs, ss, out_bs;
    uint32_t len, cps, total, nblocks;
    FastDiv div_cps;
    uint32_t coef[8];
};

template <int MODE, int ARITH>
__global__ __launch_bounds__(256) void dec_probe_kernel(ProbeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int K = 8;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t i0 = xcd_order() * 256 + (wave << 6);
    if (i0 >= a.total) return;
    const uint32_t bfirst = fdiv(i0, a.div_cps);
    const uint32_t nb = fdiv(min(i0 + 63u, a.total - 1u), a.div_cps) - bfirst + 1;
    uint32_t m0 = 0, m1 = 0, m2 = 0;
    if constexpr (MODE == 0) {
        const uint32_t mine = lane < nb ? a.masks[bfirst + lane] : 0u;
        m0 = (uint32_t)__builtin_amdgcn_readlane((int)mine, 0);
        m1 = (uint32_t)__builtin_amdgcn_readlane((int)mine, 1);
        m2 = (uint32_t)__builtin_amdgcn_readlane((int)mine, 2);
    } else if constexpr (MODE == 2) {
        typedef __attribute__((address_space(4))) const uint32_t CU32;
        CU32* cm = (CU32*)a.masks;
        const uint32_t bf = (uint32_t)__builtin_amdgcn_readfirstlane((int)bfirst);
        const uint32_t last = a.nblocks - 1;
        m0 = cm[bf];
        m1 = cm[(uint32_t)__builtin_amdgcn_readfirstlane((int)min(bf + 1, last))];
        m2 = cm[(uint32_t)__builtin_amdgcn_readfirstlane((int)min(bf + 2, last))];
    }
    const uint32_t item = i0 + lane;
    const bool inr = item < a.total;
    const uint32_t blk = inr ? fdiv(item, a.div_cps) : bfirst;
    const uint32_t g = blk - bfirst;
    const uint32_t c = item - blk * a.cps;
    uint32_t E0, R0;
    if constexpr (MODE == 1 || MODE == 3) {
        E0 = (blk * 2654435761u) >> 29;
        R0 = 0;
    } else {
        const uint32_t mask = (g == 0 ? m0 : g == 1 ? m1 : m2) & 0xFFFu;
        E0 = __ffs(~mask & 0xFFu) - 1;
        R0 = __ffs(mask >> K) - 1;
        if (E0 > 7) E0 = 7;
        if (R0 > 3) R0 = 0;
    }
    const uint8_t* d0 = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    const uint8_t* p0 = a.parity + (uint64_t)blk * a.pbs + (uint64_t)R0 * a.ss + (uint64_t)c * kChunk;
    uint4 x[K];
    if constexpr (MODE == 3) {
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = ld16<true>(d0 + (uint64_t)j * a.ss);
    } else {
#pragma unroll
        for (int j = 0; j < K - 1; ++j) x[j] = ld16<true>(d0 + (uint64_t)(j + (j >= (int)E0)) * a.ss);
        x[K - 1] = ld16<true>(p0);
    }
    uint32_t acc[4] = {0, 0, 0, 0};
    if constexpr (ARITH) {
        // the wave's rows (3 blocks x 8 PermTabs) expanded into its LDS slice while the loads fly
        gf::PermTab* wt = reinterpret_cast<gf::PermTab*>(smem + (size_t)wave * 3 * K * sizeof(gf::PermTab));
        if (lane < nb * K) {
            const uint32_t gg = lane / K, j = lane - gg * K;
            wt[lane] = gf::make_permtab_fast((a.coef[j] + gg * 0x3Bu + E0 * 0x11u) & 0xFFu);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // fec_recon.hpp wave_sync()
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (!inr) return;
        const gf::PermTab* T = wt + g * K;
#pragma unroll
        for (int j = 0; j < K; j += 2) {
            Idx ia[4], ib[4];
            split4(ia, x[j]);
            split4(ib, x[j + 1]);
            mac2(acc, ia, ib, T + j, T + j + 1);
        }
    } else {
        if (!inr) return;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            acc[0] ^= x[j].x;
            acc[1] ^= x[j].y;
            acc[2] ^= x[j].z;
            acc[3] ^= x[j].w;
        }
    }
    const uint32_t nbytes = min(a.len - c * kChunk, (uint32_t)kChunk);
    st16<true>(a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk, keep_bytes(as_uint4(acc), nbytes));
}

static FastDiv host_fastdiv(uint32_t d) {
    // same construction as fec_capi.cpp make_fastdiv: q = (umulhi(n, magic) + n) >> shift
    uint32_t shift = 0;
    while ((1ull << shift) < d) ++shift;
    const uint64_t magic = ((1ull << 32) * ((1ull << shift) - d)) / d + 1;
    return FastDiv{d, (uint32_t)magic, shift};
}

extern "C" int dec_probe(int mode, int arith, int wpc, const void* data, const void* parity, void* out,
                         const uint32_t* masks, size_t dbs, size_t pbs, size_t ss, size_t out_bs, unsigned len,
                         unsigned nblocks, void* stream) {
    ProbeArgs a{};
    a.data = (const uint8_t*)data;
    a.parity = (const uint8_t*)parity;
    a.out = (uint8_t*)out;
    a.masks = masks;
    a.dbs = dbs;
    a.pbs = pbs;
    a.ss = ss;
    a.out_bs = out_bs;
    a.len = len;
    a.cps = (len + 15) / 16;
    a.total = a.cps * nblocks;
    a.nblocks = nblocks;
    a.div_cps = host_fastdiv(a.cps);
    for (int j = 0; j < 8; ++j) a.coef[j] = 0x1Du * (j + 3);
    const int grid = (int)((a.total + 255) / 256);
    const size_t lds = occupancy_lds(wpc, 4 * 3 * 8 * sizeof(gf::PermTab));
    hipStream_t s = (hipStream_t)stream;
#define DP(M, A)                                                                                  \
    if (mode == M && arith == A) {                                                                \
        hipLaunchKernelGGL((dec_probe_kernel<M, A>), dim3(grid), dim3(256), lds, s, a);           \
        return (int)hipGetLastError();                                                            \
    }
    DP(0, 0) DP(1, 0) DP(2, 0) DP(3, 0) DP(0, 1) DP(1, 1) DP(2, 1) DP(3, 1)
    return -1;
}

// ---------------------------------------------------------------- multi-erasure rebuild twins
// RS(16,24) (K = 16, M = 8): per block the first K present shards read and one 16-byte store per
// erased data shard (rows at out + b*out_bs + r*ss), flat grid, one chunk per lane, nt loads and
// stores; the present mask reaches the lane as:
//   RMODE 0  a per-lane vector load of the block's mask (the library twin, fec_probe.hip)
//   RMODE 1  wave-uniform scalar loads of the wave's <= 2 masks
//   RMODE 2  a kernel argument (one pattern for every block: addresses known at launch)
//   RMODE 3  the wave's <= 2 records (160 bytes each, the mask in the first dword) vector-loaded into
//            LDS, then read back (the rebuild's plan-record staging, fec_rebuild.hip)
struct RebuildProbeArgs {
    const uint8_t* data;
    const uint8_t* parity;
    uint8_t* out;
    const uint32_t* masks;
    const uint8_t* recs;
    uint64_t dbs, pbs, ss, out_bs;
    uint32_t len, cps, total, nblocks, cmask;
    FastDiv div_cps;
};

template <int RMODE>
__global__ __launch_bounds__(256) void rebuild_probe_kernel(RebuildProbeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int K = 16, M = 8, REC = 160;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t i0 = xcd_order() * 256 + (wave << 6);
    if (i0 >= a.total) return;
    const uint32_t item = i0 + lane;
    const bool inr = item < a.total;
    const uint32_t bfirst = fdiv(i0, a.div_cps);
    const uint32_t blk = inr ? fdiv(item, a.div_cps) : bfirst;
    const uint32_t c = item - blk * a.cps;
    uint32_t mask;
    if constexpr (RMODE == 0) {
        mask = a.masks[blk];
    } else if constexpr (RMODE == 1) {
        typedef __attribute__((address_space(4))) const uint32_t CU32;
        CU32* cm = (CU32*)a.masks;
        const uint32_t bf = (uint32_t)__builtin_amdgcn_readfirstlane((int)bfirst);
        const uint32_t m0 = cm[bf];
        const uint32_t m1 = cm[(uint32_t)__builtin_amdgcn_readfirstlane((int)min(bf + 1, a.nblocks - 1))];
        mask = blk == bfirst ? m0 : m1;
    } else if constexpr (RMODE == 2) {
        mask = a.cmask;
    } else {
        uint8_t* slice = smem + (size_t)wave * 2 * REC;
        const uint32_t nb = fdiv(min(i0 + 63u, a.total - 1u), a.div_cps) - bfirst + 1;   // <= 2
        const uint32_t nw = nb * REC / 16;
        if (lane < nw) reinterpret_cast<uint4*>(slice)[lane] = reinterpret_cast<const uint4*>(a.recs + (uint64_t)bfirst * REC)[lane];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        mask = *reinterpret_cast<const uint32_t*>(slice + (blk - bfirst) * REC);
    }
    if (!inr) return;
    mask &= (1u << (K + M)) - 1u;
    const uint32_t e = K - __popc(mask & 0xFFFFu);
    if (e == 0 || (uint32_t)__popc(mask) < K) return;
    const uint8_t* d0 = a.data + (uint64_t)blk * a.dbs + (uint64_t)c * kChunk;
    const uint8_t* p0 = a.parity + (uint64_t)blk * a.pbs + (uint64_t)c * kChunk;
    uint32_t rest = mask;
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint32_t s = __ffs(rest) - 1;
        rest &= rest - 1;
        const uint4 x = ld16<true>(s < (uint32_t)K ? d0 + (uint64_t)s * a.ss : p0 + (uint64_t)(s - K) * a.ss);
        acc.x ^= x.x;
        acc.y ^= x.y;
        acc.z ^= x.z;
        acc.w ^= x.w;
    }
    const uint32_t nbytes = min(a.len - c * kChunk, (uint32_t)kChunk);
    uint8_t* o = a.out + (uint64_t)blk * a.out_bs + (uint64_t)c * kChunk;
#pragma unroll
    for (int r = 0; r < M; ++r)
        if ((uint32_t)r < e) st16<true>(o + (uint64_t)r * a.ss, keep_bytes(acc, nbytes));
    if (a.cmask == 0x5A5A5A5Au) smem[0] = 1;   // never: keeps the LDS allocation
}

extern "C" int rebuild_probe(int mode, int wpc, const void* data, const void* parity, void* out, const uint32_t* masks,
                             const void* recs, uint32_t cmask, size_t dbs, size_t pbs, size_t ss, size_t out_bs,
                             unsigned len, unsigned nblocks, void* stream) {
    RebuildProbeArgs a{};
    a.data = (const uint8_t*)data;
    a.parity = (const uint8_t*)parity;
    a.out = (uint8_t*)out;
    a.masks = masks;
    a.recs = (const uint8_t*)recs;
    a.cmask = cmask;
    a.dbs = dbs;
    a.pbs = pbs;
    a.ss = ss;
    a.out_bs = out_bs;
    a.len = len;
    a.cps = (len + 15) / 16;
    a.total = a.cps * nblocks;
    a.nblocks = nblocks;
    a.div_cps = host_fastdiv(a.cps);
    const int grid = (int)((a.total + 255) / 256);
    const size_t lds = occupancy_lds(wpc, 4 * 2 * 160);
    hipStream_t s = (hipStream_t)stream;
    if (mode == 0) hipLaunchKernelGGL((rebuild_probe_kernel<0>), dim3(grid), dim3(256), lds, s, a);
    else if (mode == 1) hipLaunchKernelGGL((rebuild_probe_kernel<1>), dim3(grid), dim3(256), lds, s, a);
    else if (mode == 2) hipLaunchKernelGGL((rebuild_probe_kernel<2>), dim3(grid), dim3(256), lds, s, a);
    else if (mode == 3) hipLaunchKernelGGL((rebuild_probe_kernel<3>), dim3(grid), dim3(256), lds, s, a);
    else return -1;
    return (int)hipGetLastError();
}
