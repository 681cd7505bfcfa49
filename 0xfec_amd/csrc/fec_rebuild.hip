// fec_rebuild.hip — multi-erasure rebuild with the data shard count known at compile time, for the
// codes whose decode is VALU-bound: RS(16,24) (BASELINE config #4) and RS(20,30), the reference's
// own sender/receiver code (manager.go:58-59,81-82; ReconstructData, reed_solomon.go:124).
//
// Same work split as rs_reconstruct_wave_kernel's compile-time-k form (fec_decode.hip): lane = one
// 16-byte chunk, a wave's 64 items span at most two blocks (shards of 64+ chunks), the wave stages
// its blocks' sorted plan records and PermTab rows in a wave-private LDS slice, then folds the k
// inputs through a rolling window of W loads. What changes is the per-wave overhead around the
// field arithmetic (the products themselves are the same 3 v_perm + 1.5 v_bitop3 per coefficient
// and dword):
//   * PermTab rows are copied from a workgroup-shared table of all 256 coefficients' PermTabs
//     (20 bytes each, loaded from a compile-time device table once per workgroup), instead of
//     being computed per coefficient (a doubling chain and byte permutes, ~63 VALU a round);
//   * the k input addresses of each block are 64-bit offsets from the block's data chunk, computed
//     once per (block, input) by the wave's lanes into LDS, so an input load costs one 64-bit add
//     instead of a slot extract, two selects and a 32x32+64 multiply-add (~6 VALU);
//   * the PermTab words are stored split (16-byte T0|T1 word, 4-byte T2 word): 20 instead of 32
//     bytes of LDS per coefficient;
//   * the wave index is made wave-uniform, so the staging arithmetic runs on the scalar unit.
#include "fec_recon.hpp"

namespace fk {

namespace {

// PermTabs of all 256 coefficients, split: t01[c] = {t0lo, t0hi, t1lo, t1hi}, t2[c].
struct PermTabSplit {
    uint32_t t01[256][4];
    uint32_t t2[256];
};

constexpr uint8_t dbl8(uint32_t x) { return (uint8_t)(((x << 1) ^ ((x & 0x80u) ? 0x11Du : 0u)) & 0xFFu); }

constexpr PermTabSplit make_split_tables() {
    PermTabSplit t{};
    for (uint32_t c = 0; c < 256; ++c) {
        uint8_t p[8] = {};
        p[0] = (uint8_t)c;
        for (int b = 1; b < 8; ++b) p[b] = dbl8(p[b - 1]);
        uint32_t w[5] = {};
        for (int i = 0; i < 8; ++i) {
            const uint32_t t0 = ((i & 1) ? p[0] : 0) ^ ((i & 2) ? p[1] : 0) ^ ((i & 4) ? p[2] : 0);
            const uint32_t t1 = ((i & 1) ? p[3] : 0) ^ ((i & 2) ? p[4] : 0) ^ ((i & 4) ? p[5] : 0);
            w[i >> 2] |= t0 << (8 * (i & 3));
            w[2 + (i >> 2)] |= t1 << (8 * (i & 3));
        }
        for (int i = 0; i < 4; ++i) w[4] |= (uint32_t)(((i & 1) ? p[6] : 0) ^ ((i & 2) ? p[7] : 0)) << (8 * i);
        for (int q = 0; q < 4; ++q) t.t01[c][q] = w[q];
        t.t2[c] = w[4];
    }
    return t;
}

__device__ const PermTabSplit kPermTabSplit = make_split_tables();

// Known answers (c * {0..7}, c * {0, 8, .., 56}, c * {0, 64, 128, 192} over 0x11D): c = 1 is the
// identity; c = 0x80 and 0xFF exercise the reduction.
constexpr PermTabSplit kSplitCheck = make_split_tables();
static_assert(kSplitCheck.t01[1][0] == 0x03020100u && kSplitCheck.t01[1][1] == 0x07060504u &&
                  kSplitCheck.t01[1][2] == 0x18100800u && kSplitCheck.t01[1][3] == 0x38302820u &&
                  kSplitCheck.t2[1] == 0xC0804000u,
              "PermTab of 1");
static_assert(kSplitCheck.t01[0x80][0] == 0x9D1D8000u && kSplitCheck.t01[0x80][1] == 0xA727BA3Au &&
                  kSplitCheck.t01[0x80][2] == 0x9CE87400u && kSplitCheck.t01[0x80][3] == 0x5125B9CDu &&
                  kSplitCheck.t2[0x80] == 0x94138700u,
              "PermTab of 0x80");
static_assert(kSplitCheck.t01[0xFF][0] == 0x1CE3FF00u && kSplitCheck.t01[0xFF][3] == 0x76DD3D96u &&
                  kSplitCheck.t2[0xFF] == 0x53623100u && kSplitCheck.t2[0] == 0u,
              "PermTab of 0xFF");

constexpr uint32_t kTabLds = 256 * 16 + 256 * 4;   // the workgroup's copy of kPermTabSplit

// A wave's LDS slice: PermTab words of R rows x K inputs for each of its WB blocks, the blocks'
// input offsets, their plan records. (RS(16,24)'s 2048-byte T0|T1 and 512-byte T2 block strides put
// the two blocks' rows on the same banks, 24 % of its LDS cycles in conflicts; padding them 32 banks
// apart measured +0.1 % for RS(16,24) and -1.2 % for RS(20,30), r04c, and 4 banks apart -0.03 % and
// -0.1 %, r06d (profiles/r06/lpad_*_r06d.log): not on the critical path.)
template <int K, int R>
struct Slice {
    static constexpr uint32_t WB = 2;
    static constexpr uint32_t bs01 = R * K * 16;   // bytes per block
    static constexpr uint32_t bs2 = R * K * 4;
    static constexpr uint32_t t01 = 0;                        // uint4    [WB][R][K], blocks bs01 apart
    static constexpr uint32_t t2 = t01 + WB * bs01;           // uint32_t [WB][R][K], blocks bs2 apart
    static constexpr uint32_t offs = t2 + WB * bs2;           // uint64_t [WB][K]
    static constexpr uint32_t plans = offs + WB * K * 8;      // [WB][stride]
    static_assert(bs01 % 16 == 0 && t2 % 16 == 0 && offs % 16 == 0 && plans % 16 == 0, "16-byte aligned parts");
    __host__ __device__ static size_t bytes(uint32_t stride) { return plans + (size_t)WB * stride; }
};

// acc ^= c_a x_a ^ c_b x_b (one 16-byte chunk), c by its split PermTab words.
__device__ __forceinline__ void mac2s(uint32_t (&acc)[4], const Idx (&ia)[4], const Idx (&ib)[4], const uint4& la,
                                      uint32_t a2, const uint4& lb, uint32_t b2) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const Prod3 p = gprod(ia[d], la, a2);
        const Prod3 q = gprod(ib[d], lb, b2);
        acc[d] = xor3(xor3(xor3(acc[d], p.p0, p.p1), p.p2, q.p0), q.p1, q.p2);
    }
}

// The ROWS rows' products of one input pair. RP: each row's table words read one row ahead of
// their use under scheduling barriers (2 rows' words live instead of all of them: RS(20,30)'s
// 10-row body otherwise holds 100 VGPRs of table words).
template <int K, int ROWS, bool RP>
__device__ __forceinline__ void pair_rows(uint32_t (&acc)[ROWS][4], const Idx (&ia)[4], const Idx (&ib)[4],
                                          const uint4* T01, const uint32_t* T2, int j) {
    // the pair's two T2 words in one 8-byte read (j even, K even: aligned), which takes an
    // immediate offset where two 4-byte reads would need an address add
    auto t2pair = [&](int r) { return *reinterpret_cast<const uint2*>(T2 + r * K + j); };
    if constexpr (RP) {
        uint4 la = T01[j], lb = T01[j + 1];
        uint2 w2 = t2pair(0);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            uint4 na = la, nb = lb;
            uint2 n2 = w2;
            if (r + 1 < ROWS) {
                na = T01[(r + 1) * K + j];
                nb = T01[(r + 1) * K + j + 1];
                n2 = t2pair(r + 1);
            }
            __builtin_amdgcn_sched_barrier(0);
            mac2s(acc[r], ia, ib, la, w2.x, lb, w2.y);
            __builtin_amdgcn_sched_barrier(0);
            la = na, lb = nb, w2 = n2;
        }
    } else {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const uint2 w2 = t2pair(r);
            mac2s(acc[r], ia, ib, T01[r * K + j], w2.x, T01[r * K + j + 1], w2.y);
        }
    }
}

// One item's ROWS rebuilt chunks: the K inputs at dbase + offs[j] through a rolling window of W
// loads (each folded pair's registers take the loads of the pair W inputs ahead).
template <int K, int ROWS, int W, bool RP>
__device__ __forceinline__ void rebuild_rows(const ReconArgs& a, const uint8_t* out_idx, const uint4* T01,
                                             const uint32_t* T2, const uint64_t* offs, uint8_t* dbase,
                                             uint8_t* obase, uint32_t c, uint32_t nout) {
    static_assert(K % 2 == 0 && W % 2 == 0 && W <= K, "inputs are folded and loaded in pairs");
    // a body that opens like no other (the compiler would hoist an opening the row bodies share
    // in front of the switch, where it is live across all of them)
    asm volatile("; rows %0" ::"n"(ROWS));
    // two inputs' offsets per 16-byte read (immediate LDS offsets)
    auto load2 = [&](int j, uint4& xa, uint4& xb) {
        const ulonglong2 o = *reinterpret_cast<const ulonglong2*>(offs + j);
        xa = ld16<kNT>(dbase + o.x);
        xb = ld16<kNT>(dbase + o.y);
    };
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < W; j += 2) load2(j, x[j], x[j + 1]);
    uint32_t acc[ROWS][4];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0;
#pragma unroll
    for (int j = 0; j < K; j += 2) {
        // opaque zero per input pair: keeps each pair's table reads next to their use
        uint32_t toff = 0;
        asm volatile("" : "+s"(toff));
        const uint4* t01 = T01 + toff;
        const uint32_t* t2 = T2 + toff;
        const uint4 xa = x[j], xb = x[j + 1];
        __builtin_amdgcn_sched_barrier(0);
        // (splits by 64-bit shifts, 64 fewer VALU per body, measured +0.2 %, r03m)
        Idx ia[4], ib[4];
        split4(ia, xa);
        split4(ib, xb);
        if (j + W < K) load2(j + W, x[j + W], x[j + W + 1]);
        pair_rows<K, ROWS, RP>(acc, ia, ib, t01, t2, j);
    }
    const uint32_t nb = a.len - c * kChunk;
#pragma unroll
    for (int r = 0; r < ROWS; ++r)
        if (r < (int)nout)
            store_chunk<kNT>(obase ? obase + (uint64_t)r * a.ss : dbase + (uint64_t)out_idx[r] * a.ss, as_uint4(acc[r]),
                             nb);
}

// Flat grid, one wave per 64 consecutive items of the (sorted) plan order; R: the code's largest
// rebuilt row count (min(k, m)); W: loads in flight per lane; RP: row-pipelined table reads.
template <int K, int R, int W, bool RP>
__global__ __launch_bounds__(kThreads) void rs_rebuild_k_kernel(ReconArgs a) {
    using S = Slice<K, R>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint4* g01 = reinterpret_cast<uint4*>(smem);
    uint32_t* g2 = reinterpret_cast<uint32_t*>(smem + 256 * 16);
    // the workgroup's PermTab table: one coefficient per thread (kThreads == 256)
    g01[threadIdx.x] = *reinterpret_cast<const uint4*>(kPermTabSplit.t01[threadIdx.x]);
    g2[threadIdx.x] = kPermTabSplit.t2[threadIdx.x];
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t lane = threadIdx.x & 63;
    const PlanLayout lay = a.lay;
    uint8_t* slice = smem + kTabLds + (size_t)wave * S::bytes(lay.stride);
    uint64_t* offs = reinterpret_cast<uint64_t*>(slice + S::offs);
    uint8_t* plans = slice + S::plans;
    const uint32_t total = a.nblocks * a.cps;
    const uint32_t i0 = xcd_order() * kThreads + (wave << 6);
    const bool live = i0 < total;   // wave-uniform
    uint32_t bfirst = 0, nb = 0;
    if (live) {
        // the wave's <= 2 plan records, loaded under the table copy
        bfirst = fdiv(i0, a.div_cps);
        nb = fdiv(min(i0 + 63u, total - 1u), a.div_cps) - bfirst + 1;
        const uint32_t nw = nb * lay.stride / 16;
        const uint4* src = reinterpret_cast<const uint4*>(a.plans + (uint64_t)bfirst * lay.stride);
        if (lane < nw) reinterpret_cast<uint4*>(plans)[lane] = src[lane];
    }
    __syncthreads();   // the table and the wave's records
    if (!live) return;
    const uint32_t n0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)plans[lay.nout_off]);
    const uint32_t n1 =
        nb > 1 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)plans[lay.stride + lay.nout_off]) : 0u;
    {
        // PermTab rows of the rows each block rebuilds: entry i of n0*K + n1*K; the coefficient area
        // is row-major with row stride K, so an entry's index within its block is its coefficient's
        const uint32_t c0 = n0 * K, cn = c0 + n1 * K;
        for (uint32_t i = lane; i < cn; i += 64) {
            const uint32_t g = i >= c0 ? 1u : 0u;
            const uint32_t rem = i - (g ? c0 : 0u);
            const uint32_t coef = plans[g * lay.stride + lay.coef_off + rem];
            reinterpret_cast<uint4*>(slice + S::t01 + g * S::bs01)[rem] = g01[coef];
            reinterpret_cast<uint32_t*>(slice + S::t2 + g * S::bs2)[rem] = g2[coef];
        }
        // input j of block g at its data chunk + offs[g][j] (64-bit, wrapping)
        if (lane < nb * K) {
            const uint32_t g = lane >= (uint32_t)K ? 1u : 0u;
            const uint32_t j = lane - g * K;
            const uint8_t* P = plans + g * lay.stride;
            const uint32_t slot = P[lay.in_off + j];
            const uint64_t blk = a.sorted ? *reinterpret_cast<const uint32_t*>(P + lay.blk_off) : bfirst + g;
            uint64_t off = (uint64_t)slot * a.ss;
            if (slot >= (uint32_t)K)
                off = ((uint64_t)(uintptr_t)a.parity - (uint64_t)(uintptr_t)a.data) + blk * a.pbs - blk * a.dbs +
                      (uint64_t)(slot - K) * a.pss;
            offs[g * K + j] = off;
        }
    }
    wave_sync();
    const uint32_t item = i0 + lane;
    const bool inr = item < total;
    const uint32_t blk = inr ? fdiv(item, a.div_cps) : bfirst;
    const uint32_t g = blk - bfirst;
    const uint32_t c = item - blk * a.cps;
    const uint8_t* P = plans + g * lay.stride;
    const uint32_t nout = inr ? P[lay.nout_off] : 0;
    const uint32_t rows = wave_rows<R>(nout);
    if (nout == 0) return;
    const uint32_t rb = a.sorted ? *reinterpret_cast<const uint32_t*>(P + lay.blk_off) : blk;
    uint8_t* dbase = a.data + (uint64_t)rb * a.dbs + (uint64_t)c * kChunk;
    uint8_t* obase = a.out ? a.out + (uint64_t)rb * a.out_bs + (uint64_t)c * kChunk : nullptr;
    const uint4* T01 = reinterpret_cast<const uint4*>(slice + S::t01 + g * S::bs01);
    const uint32_t* T2 = reinterpret_cast<const uint32_t*>(slice + S::t2 + g * S::bs2);
    const uint64_t* O = offs + g * K;
    const uint8_t* oi = P + lay.out_off;
    static_assert(R <= 10, "row bodies 1..10");
#define FEC_RB_ROWS(N) rebuild_rows<K, N, W, RP>(a, oi, T01, T2, O, dbase, obase, c, nout)
    switch (rows) {   // wave-uniform
        case 1: FEC_RB_ROWS(1); break;
        case 2: if constexpr (R >= 2) FEC_RB_ROWS(2); break;
        case 3: if constexpr (R >= 3) FEC_RB_ROWS(3); break;
        case 4: if constexpr (R >= 4) FEC_RB_ROWS(4); break;
        case 5: if constexpr (R >= 5) FEC_RB_ROWS(5); break;
        case 6: if constexpr (R >= 6) FEC_RB_ROWS(6); break;
        case 7: if constexpr (R >= 7) FEC_RB_ROWS(7); break;
        case 8: if constexpr (R >= 8) FEC_RB_ROWS(8); break;
        case 9: if constexpr (R >= 9) FEC_RB_ROWS(9); break;
        default: if constexpr (R >= 10) FEC_RB_ROWS(10); break;
    }
#undef FEC_RB_ROWS
}

template <int K, int R, int W, bool RP>
hipError_t rebuild_launch(const ReconArgs& a, hipStream_t s) {
    const uint64_t total = (uint64_t)a.nblocks * a.cps;
    const int grid = (int)((total + kThreads - 1) / kThreads);
    if (grid == 0) return hipSuccess;
    const size_t lds = occupancy_lds(g_tune.dec_wpc, kTabLds + 4 * Slice<K, R>::bytes(a.lay.stride));
    hipLaunchKernelGGL((rs_rebuild_k_kernel<K, R, W, RP>), dim3(grid), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

}  // namespace

bool rebuild_k_applies(uint32_t k, uint32_t maxe, uint32_t cps) {
    return cps >= 64 && ((k == 16 && maxe == 8) || (k == 20 && maxe == 10));
}

hipError_t launch_rs_rebuild_k(const ReconArgs& a, hipStream_t s) {
    // windows by interleaved A/B (r03k): RS(16,24) 8 -> 4 +0.3 % (4 / 6 / 8 within 0.7 %); RS(20,30)
    // 8 -> 6 +6.7 % (137 -> 125 VGPRs: 4 instead of 3 waves per SIMD)
    if (a.k == 16) return rebuild_launch<16, 8, 4, false>(a, s);
    return rebuild_launch<20, 10, 6, true>(a, s);
}

}  // namespace fk
