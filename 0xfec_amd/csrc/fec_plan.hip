// fec_plan.hip — sorted decode plans for gfx950 (reed_solomon.go:124 ReconstructData: which shards
// to read and with which coefficients to rebuild the erased data shards of each block).
//
// rs_plan_kernel (fec_decode.hip) gives one block to one lane: its k^2 + 3ek table lookups run
// one after another (~0.2 ms for 2^19 RS(16,24) blocks with 1-8 losses). Here a group of
// plan_lanes(k) lanes of one wave shares a block: lane p builds input slot p, the Lagrange
// denominator D_p and coefficient column p; lane r < e the numerator N_r — k-long chains instead
// of k^2.
//
// The records of a window of 64 blocks are then stored ordered by erasure count (descending,
// blocks with nothing to rebuild last), each naming its block. The rebuild kernel walks records
// in storage order, so the <= 3 blocks a rebuild wave touches have (nearly always) the same
// erasure count: its wave-uniform row count is the blocks' own, not the maximum of unrelated
// neighbours (RS(16,24) with 1-8 losses: 3.8 -> 3.1 rows per wave).
//
// Two forms: rs_plan_code_kernel (form 3) compiled for RS(16,24) / RS(20,30), and
// rs_plan_sorted_kernel (form 2) for every other code.
#include <algorithm>

#include "fec_recon.hpp"

namespace fk {

namespace {

constexpr uint32_t kPlanSortThreads = 256;
constexpr uint32_t kGroupScratch = 160;   // per block: S[32] slots, O[32] erased, X[32] others, D|N[64]

struct SortLds {
    size_t prows, dall, scratch, pos, rank, recs, total;
};
// Plan form 2 stages exp over [0, 768) (exp[i mod 255], so a sum of three logs needs no reduction),
// log over [768, 1024), then log of 0..31 in 4 copies (log 0 taken as 0): lane l reads copy l & 3,
// so the 32 lanes of a half-wave that look up log(i ^ j) for shard indices i, j < 32 never meet on
// a bank (32 banks of 4 bytes per half-wave).
constexpr uint32_t kV2Exp = 0, kV2Log = 768, kV2Log32 = 1024, kV2Tables = 1152;
constexpr uint32_t kRankBins = 33;   // erasure counts 0..32
// recs: the records of `win` segments of `groups` blocks, sorted together (sort window)
__host__ __device__ inline SortLds sort_lds(uint32_t m, uint32_t k, uint32_t groups, uint32_t stride,
                                            uint32_t win, uint32_t gscratch = kGroupScratch) {
    SortLds l;
    l.prows = kV2Tables;
    l.dall = l.prows + (size_t)m * k;
    l.scratch = (l.dall + 32 + 15) & ~(size_t)15;
    l.pos = l.scratch + (size_t)groups * gscratch;
    // ranking scratch: per wave of records and bin, a count (then its prefix), and per bin a start
    l.rank = l.pos + (size_t)groups * win * 4;
    l.recs = (l.rank + ((size_t)(groups * win + 63) / 64 + 1) * kRankBins * 4 + 15) & ~(size_t)15;
    l.total = l.recs + (size_t)groups * win * stride;
    return l;
}

// Segments sorted together: as many as make 64 blocks. A rebuild wave spans two neighbouring
// records, and its row count is the larger of their two erasure counts; sorted over one segment
// (16 blocks for RS(16,24), 8 for RS(20,30)) neighbours still differ by about one row. 64 blocks
// against 128 / 256 / 512 (r03y, r04s): the window's records in LDS cost the plan kernel
// residency that the rebuild does not win back.
__host__ __device__ inline uint32_t sort_window(uint32_t groups) { return groups < 64u ? 64u / groups : 1u; }

// The window's nw record slots (first block base0) from LDS to their storage order in a.plans:
// erasure count descending, then block order (stable). Workgroup-wide (barriers inside).
__device__ __forceinline__ void sort_window_out(const PlanArgs& a, uint8_t* smem, const SortLds& L, uint32_t nw,
                                                uint32_t base0) {
    const PlanLayout lay = a.lay;
    uint32_t* s_pos = reinterpret_cast<uint32_t*>(smem + L.pos);
    __syncthreads();   // every record of the window written
    const uint32_t nvalid = min(nw, a.nblocks - base0);
    // counting sort: position = records with a larger count + earlier records with the same
    // count (past-the-batch groups: nothing to rebuild, last indices, so they rank last).
    // Per wave of records and bin, a ballot gives the count and each record's rank in its wave.
    const uint32_t U = a.maxe + 1, nwv = (nw + 63) / 64;
    uint32_t* wc = reinterpret_cast<uint32_t*>(smem + L.rank);   // [nwv][U], then start[U]
    uint32_t* start = wc + nwv * U;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (uint32_t t = threadIdx.x; t < nwv * 64; t += kPlanSortThreads) {   // wave-uniform bound
        const uint32_t v = t < nw ? smem[L.recs + (size_t)t * lay.stride + lay.nout_off] : kRankBins;
        uint32_t rin = 0;
        for (uint32_t u = 0; u < U; ++u) {
            const uint64_t bm = __ballot(v == u);
            if (v == u) rin = (uint32_t)__popcll(bm & lt);
            if (lane == 0) wc[(t >> 6) * U + u] = (uint32_t)__popcll(bm);
        }
        if (t < nw) s_pos[t] = rin;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        // bins in descending order; within a bin, waves in order: wc becomes each wave's offset
        uint32_t acc = 0;
        for (uint32_t u = U; u-- > 0;) {
            start[u] = acc;
            for (uint32_t w = 0; w < nwv; ++w) {
                const uint32_t c = wc[w * U + u];
                wc[w * U + u] = acc;
                acc += c;
            }
        }
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < nw; t += kPlanSortThreads) {
        const uint32_t v = smem[L.recs + (size_t)t * lay.stride + lay.nout_off];
        s_pos[t] += wc[(t >> 6) * U + v];
    }
    __syncthreads();
    const uint32_t per = lay.stride / 16;
    const uint4* src = reinterpret_cast<const uint4*>(smem + L.recs);
    uint4* dst = reinterpret_cast<uint4*>(a.plans + (uint64_t)base0 * lay.stride);
    for (uint32_t i = threadIdx.x; i < nvalid * per; i += kPlanSortThreads) {
        const uint32_t r = i / per, q = i - r * per;
        dst[(size_t)s_pos[r] * per + q] = src[(size_t)r * per + q];
    }
}

// The routed in-place form's word (fec_recover.hip): zero, no block needs a plan (workgroup-uniform).
__device__ __forceinline__ bool route_skips(const PlanArgs& a) {
    typedef __attribute__((address_space(4))) const uint32_t ConstU32;
    return a.route && *(ConstU32*)a.route == 0;
}

template <uint32_t LPB>
__global__ __launch_bounds__(kPlanSortThreads) void rs_plan_sorted_kernel(PlanArgs a, uint32_t segs, uint32_t win) {
    constexpr uint32_t G = kPlanSortThreads / LPB;   // blocks per workgroup segment
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (route_skips(a)) return;
    const PlanLayout lay = a.lay;
    const SortLds L = sort_lds(a.m, a.k, G, lay.stride, win);
    uint8_t* s_exp = smem + kV2Exp;
    uint8_t* s_log = smem + kV2Log;
    // this lane's copy of log(0..31)
    const uint8_t* s_l32 = smem + kV2Log32 + (threadIdx.x & 3u) * 32u;
    uint8_t* s_prows = smem + L.prows;
    const uint32_t k = a.k, m = a.m, n = k + m;
    const uint32_t gb = threadIdx.x / LPB, gl = threadIdx.x % LPB;   // block group, lane in group
    // the tables (the layout above), the parity rows and dall: staged once per workgroup, which
    // then plans `segs` consecutive segments of G blocks
    for (uint32_t i = threadIdx.x; i < kV2Tables; i += kPlanSortThreads) {
        const uint32_t j = i - kV2Log32;
        smem[i] = i < kV2Log ? gf::kTables.exp[i % 255u]
                : i < kV2Log32 ? gf::kTables.log[i - kV2Log]
                : (j & 31u) ? gf::kTables.log[j & 31u] : (uint8_t)0;
    }
    for (uint32_t i = threadIdx.x; i < m * k; i += kPlanSortThreads) s_prows[i] = a.prows[i];
    uint8_t* s_dall = smem + L.dall;
    if (threadIdx.x < n) s_dall[threadIdx.x] = a.dall[threadIdx.x];
    uint8_t* S = smem + L.scratch + gb * kGroupScratch;   // first k present shards
    uint8_t* O = S + 32;                                  // erased data shards, ascending
    uint8_t* X = S + 64;                                  // the other n - k shard indices
    uint8_t* Dt = S + 96;                                 // D_p (k bytes), then N_r (maxe bytes)
    uint8_t* Nt = Dt + k;
    const uint32_t all = low_mask(n), kmask = low_mask(k);
    const uint32_t seg0 = blockIdx.x * segs;
    // the first segment's masks in flight while the tables stage
    uint32_t mask_next = seg0 * G + gb < a.nblocks ? a.masks[seg0 * G + gb] : 0u;
    for (uint32_t sg = 0; sg < segs; ++sg) {
        const uint32_t base = (seg0 + sg) * G;
        if (base >= a.nblocks) break;   // workgroup-uniform
        const uint32_t b = base + gb;
        const bool valid = b < a.nblocks;
        const uint32_t mask_in = mask_next;
        // the next segment's mask loads before this segment's work
        const uint32_t bn = b + G;
        mask_next = (sg + 1 < segs && bn < a.nblocks) ? a.masks[bn] : 0u;
        const uint32_t wl = sg % win;   // segment within the sort window
        // a window's first segment: tables staged (first pass), the previous window's records
        // copied out; within a window a block group's scratch is its own lanes' (wave-local)
        if (wl == 0) __syncthreads();
        else wave_sync();
        uint8_t* P = smem + L.recs + ((size_t)wl * G + gb) * lay.stride;
        const uint32_t mask = valid ? mask_in & all : all;   // past the batch: nothing to rebuild
        const uint32_t e = k - __popc(mask & kmask);
        int32_t st = a.max_out ? (int32_t)e : 0;
        uint32_t nout = 0;
        if (e != 0) {
            if ((uint32_t)__popc(mask) < k) {
                st = -4;   // FEC_ERR_TOO_FEW_SHARDS
                if (gl == 0) wave_flag(a.err, 1);
            } else if (a.max_out && e > a.max_out) {
                st = -1;   // FEC_ERR_INVALID_ARG: more erasures than output slots
                if (gl == 0) wave_flag(a.err, 2);
            } else {
                nout = e;
            }
        }
        if (gl == 0) {
            P[lay.nout_off] = (uint8_t)nout;
            *reinterpret_cast<uint32_t*>(P + lay.blk_off) = b;
            if (valid && a.status) a.status[b] = st;
        }
        if (nout) {
            for (uint32_t t = gl; t < n; t += LPB) {
                const uint32_t pos = __popc(mask & low_mask(t));
                if (((mask >> t) & 1u) && pos < k) {
                    S[pos] = (uint8_t)t;
                } else {
                    X[t - min(pos, k)] = (uint8_t)t;   // not an input: erased, or present past the first k
                    if (t < k && !((mask >> t) & 1u)) O[__popc(~mask & kmask & low_mask(t))] = (uint8_t)t;
                }
            }
        }
        wave_sync();
        uint8_t* C = P + lay.coef_off;
        if (nout) {
            if (gl < k) P[lay.in_off + gl] = S[gl];
            if (gl < nout) P[lay.out_off + gl] = O[gl];
            if (e == 1) {
                // one erasure: x_E = inv(A[R0][E]) * (p_R0 ^ sum_j A[R0][j] x_j)
                const uint32_t E0 = O[0];
                const uint32_t R0 = __ffs(mask >> k) - 1;   // e = 1 with k present shards: a parity, k < 32
                const uint8_t* row = s_prows + R0 * k;
                const uint32_t inv = s_exp[255 - s_log[row[E0]]];
                if (gl < k) {
                    const uint32_t sj = S[gl];
                    C[gl] = (uint8_t)(sj < k ? (row[sj] ? s_exp[s_log[inv] + s_log[row[sj]]] : 0u) : inv);
                }
            } else {
                // D_p and N_r are the same sum for the shard t = s_p or i_r, over the set Y = the
                // others X (complement form, n - k < k: sum over all n indices, dall, minus the n - k
                // others) or the inputs S; log32(0) = 0 drops the t = y term. Lane q of the group
                // takes t = S[q] (q < k) or O[q - k]: RS(20,30) both sets in one pass over 30 lanes;
                // Nt = Dt + k. coef[r][p] = exp(N_r - log(i_r ^ s_p) - D_p) (Lagrange over the shard
                // indices, rs_plan_kernel).
                const bool comp = n - k < k;
                const uint32_t ny = comp ? n - k : k;
                const uint8_t* Y = comp ? X : S;
                for (uint32_t q = gl; q < k + e; q += LPB) {
                    const uint32_t t = q < k ? S[q] : O[q - k];
                    uint32_t s = 0;
                    for (uint32_t u = 0; u < ny; ++u) s += s_l32[t ^ Y[u]];
                    if (comp) s = s_dall[t] + 255u * 32u - s;
                    Dt[q] = (uint8_t)(s % 255u);
                }
            }
        }
        wave_sync();
        if (nout >= 2 && gl < k) {
            const uint32_t sp = S[gl], dp = Dt[gl];
            for (uint32_t r = 0; r < nout; ++r) {
                // < 765: exp needs no reduction
                const uint32_t v = Nt[r] + 2u * 255u - s_l32[O[r] ^ sp] - dp;
                C[r * k + gl] = s_exp[v];
            }
        }
        // at the end of a sort window (or of the work): storage order of the window's records,
        // erasure count descending, then block order (stable)
        const bool last = sg + 1 == segs || base + G >= a.nblocks;
        if (wl + 1 < win && !last) continue;   // workgroup-uniform
        sort_window_out(a, smem, L, (wl + 1) * G, base - wl * G);
    }
}

// Form 3: the same plans for one code known at compile time, K data and M parity shards with
// M < K (the complement sums: RS(16,24), RS(20,30)), so every loop is unrolled and the sums are built
// for the fewest instructions (r04d/e: VALU per plan wave 3171 -> 2064 for RS(20,30), 2176 -> 1380
// for RS(16,24), decode +0.8-0.9 % over form 2):
//   * tables: exp over [0, 768), then 255 - log j for j < 32 in 4 copies (j = 0: 255, i.e. log 0 = 0),
//     then log; lane l reads copy l & 3, and its table address t ^ y ^ (copy << 5) is one XOR of
//     a shard index y with the lane's t ^ (copy << 5);
//   * with nl(j) = 255 - log j the complement sum D = dall[t] + 255*32 - sum_y log(t ^ y) is
//     dall[t] + sum_y nl(t ^ y) mod 255: no compare, no subtraction;
//   * the others X, the erased O and the numerators N sit in dword scratch, read into registers
//     by wide LDS loads, and coef = exp(N_r + nl(O_r ^ s_p) + (255 - D_p)) is one three-input add
//     (the argument < 765: exp needs no reduction).
// (Two segments interleaved per wave, r04i, and a window ranked from the masks first, r04t, left
// the decode within +-0.4 % and 0.8-2 % slower: not kept.)
constexpr uint32_t kV3Exp = 0, kV3NLog32 = 768, kV3Log = 896, kV3Tables = 1152;
typedef const __attribute__((address_space(3))) uint8_t lds_cu8;
// LDS address of a pointer into the kernel's LDS, and a byte load from one: lets the table
// address be formed as one XOR (the compiler, given generic pointers, adds the LDS base per load)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ uint32_t lds_ld8(uint32_t addr) { return *(lds_cu8*)(uintptr_t)addr; }
static_assert(kV3Tables == kV2Tables, "forms 2 and 3 share sort_lds's table area");
// group scratch: S bytes [0, 32), X dwords [32, 80), O dwords [80, 128), N dwords [128, 176), 255 - D_p
// bytes [176, 208)
constexpr uint32_t kV3S = 0, kV3X = 32, kV3O = 80, kV3N = 128, kV3D = 176, kGroupScratch3 = 208;

template <uint32_t K, uint32_t M>
__global__ __launch_bounds__(kPlanSortThreads) void rs_plan_code_kernel(PlanArgs a, uint32_t segs, uint32_t win) {
    constexpr uint32_t N = K + M, LPB = K <= 16 ? 16u : 32u, G = kPlanSortThreads / LPB, MAXE = M;
    static_assert(M < K && M <= 12 && K <= LPB && N <= 32, "complement-sum codes with the scratch above");
    extern __shared__ __attribute__((aligned(128))) uint8_t smem[];
    const PlanLayout lay = a.lay;
    const SortLds L = sort_lds(M, K, G, lay.stride, win, kGroupScratch3);
    const uint8_t* s_exp = smem + kV3Exp;
    const uint8_t* s_log = smem + kV3Log;
    const uint8_t* s_nl = smem + kV3NLog32;
    const uint32_t copy5 = (threadIdx.x & 3u) << 5;
    // nl(t ^ y) of the lane's copy at nlb ^ y, nlb = the table's LDS address + (t ^ copy << 5): one
    // XOR per term, exact while the table starts on a 128-byte boundary: smem is declared 128-byte
    // aligned and the table sits 768 bytes into it (the check below cannot fire; if it ever did,
    // the sticky error fails the call, device and host paths alike)
    const uint32_t nl_base = lds_addr(s_nl);
    if (nl_base & 127u) {
        if (threadIdx.x == 0) atomicOr(a.err, 4);
        return;
    }
    uint8_t* s_prows = smem + L.prows;
    const uint32_t gb = threadIdx.x / LPB, gl = threadIdx.x % LPB;
    for (uint32_t i = threadIdx.x; i < kV3Tables; i += kPlanSortThreads) {
        const uint32_t j = (i - kV3NLog32) & 31u;
        smem[i] = i < kV3NLog32 ? gf::kTables.exp[i % 255u]
                : i < kV3Log ? (uint8_t)(j ? 255u - gf::kTables.log[j] : 255u)
                : gf::kTables.log[i - kV3Log];
    }
    for (uint32_t i = threadIdx.x; i < M * K; i += kPlanSortThreads) s_prows[i] = a.prows[i];
    uint8_t* s_dall = smem + L.dall;
    if (threadIdx.x < N) s_dall[threadIdx.x] = a.dall[threadIdx.x];
    // the group scratch starts zeroed: the coefficient rows below read O and N past a block's own
    // erasure count (stale or zero shard indices and sums, always table-range values)
    for (uint32_t i = threadIdx.x; i < G * kGroupScratch3 / 4; i += kPlanSortThreads)
        reinterpret_cast<uint32_t*>(smem + L.scratch)[i] = 0u;
    uint8_t* grp = smem + L.scratch + gb * kGroupScratch3;
    uint8_t* S = grp + kV3S;
    uint32_t* Xd = reinterpret_cast<uint32_t*>(grp + kV3X);
    uint32_t* Od = reinterpret_cast<uint32_t*>(grp + kV3O);
    uint32_t* Nd = reinterpret_cast<uint32_t*>(grp + kV3N);
    uint8_t* Dn = grp + kV3D;
    constexpr uint32_t all = N >= 32 ? 0xFFFFFFFFu : (1u << N) - 1u, kmask = (1u << K) - 1u;
    const uint32_t seg0 = blockIdx.x * segs;
    // the first segment's masks in flight while the tables stage
    uint32_t mask_next = seg0 * G + gb < a.nblocks ? a.masks[seg0 * G + gb] : 0u;
    for (uint32_t sg = 0; sg < segs; ++sg) {
        const uint32_t base = (seg0 + sg) * G;
        if (base >= a.nblocks) break;   // workgroup-uniform
        const uint32_t wl = sg % win;
        if (wl == 0) __syncthreads();
        else wave_sync();
        const uint32_t b = base + gb;
        const bool valid = b < a.nblocks;
        const uint32_t mask_in = mask_next;
        const uint32_t bn = b + G;
        mask_next = (sg + 1 < segs && bn < a.nblocks) ? a.masks[bn] : 0u;
        uint8_t* P = smem + L.recs + ((size_t)wl * G + gb) * lay.stride;
        const uint32_t mask = valid ? mask_in & all : all;   // past the batch: nothing to rebuild
        const uint32_t e = K - __popc(mask & kmask);
        int32_t st = a.max_out ? (int32_t)e : 0;
        uint32_t nout = 0;
        if (e != 0) {
            if ((uint32_t)__popc(mask) < K) {
                st = -4;   // FEC_ERR_TOO_FEW_SHARDS
                if (gl == 0) wave_flag(a.err, 1);
            } else if (a.max_out && e > a.max_out) {
                st = -1;   // FEC_ERR_INVALID_ARG: more erasures than output slots
                if (gl == 0) wave_flag(a.err, 2);
            } else {
                nout = e;
            }
        }
        if (gl == 0) {
            P[lay.nout_off] = (uint8_t)nout;
            *reinterpret_cast<uint32_t*>(P + lay.blk_off) = b;
            if (valid && a.status) a.status[b] = st;
        }
        if (nout) {
#pragma unroll
            for (uint32_t t0 = 0; t0 < N; t0 += LPB) {
                const uint32_t t = t0 + gl;
                if (t < N) {
                    const uint32_t below = mask & ((1u << t) - 1u);   // t < 32
                    const uint32_t pos = __popc(below);
                    if (((mask >> t) & 1u) && pos < K) {
                        S[pos] = (uint8_t)t;
                    } else {
                        Xd[t - min(pos, K)] = t;   // not an input: erased, or present past the first K
                        if (t < K && !((mask >> t) & 1u)) Od[t - pos] = t;   // erased data shards below t: t - pos
                    }
                }
            }
        }
        wave_sync();
        if (nout) {
            if (gl < K) P[lay.in_off + gl] = S[gl];
            if (gl < nout) P[lay.out_off + gl] = (uint8_t)Od[gl];
            if (e == 1) {
                // one erasure: x_E = inv(A[R0][E]) * (p_R0 ^ sum_j A[R0][j] x_j)
                const uint32_t E0 = Od[0];
                const uint32_t R0 = __ffs(mask >> K) - 1;
                const uint8_t* row = s_prows + R0 * K;
                const uint32_t inv = s_exp[255 - s_log[row[E0]]];
                if (gl < K) {
                    const uint32_t sj = S[gl];
                    P[lay.coef_off + gl] = (uint8_t)(sj < K ? (row[sj] ? s_exp[s_log[inv] + s_log[row[sj]]] : 0u) : inv);
                }
            } else {
                uint32_t x[M];
#pragma unroll
                for (uint32_t u = 0; u < M; ++u) x[u] = Xd[u];
#pragma unroll
                for (uint32_t q0 = 0; q0 < K + MAXE; q0 += LPB) {
                    const uint32_t q = q0 + gl;
                    if (q < K + e) {
                        const uint32_t t = q < K ? (uint32_t)S[q] : Od[q - K];
                        const uint32_t tb = nl_base + (t ^ copy5);
                        uint32_t sum = s_dall[t];
#pragma unroll
                        for (uint32_t u = 0; u < M; ++u) sum += lds_ld8(tb ^ x[u]);
                        sum %= 255u;
                        if (q < K) Dn[q] = (uint8_t)(255u - sum);
                        else Nd[q - K] = sum;
                    }
                }
            }
        }
        wave_sync();
        // coefficient rows in chunks of 4, each chunk computed whole (rows past a block's count read
        // stale but in-range scratch, and are not stored) so its 12 LDS loads are in flight together;
        // a chunk runs while some block of the wave needs it
        uint32_t nw = nout;
#pragma unroll
        for (uint32_t o = LPB; o < 64; o <<= 1) nw = max(nw, (uint32_t)__shfl_xor((int)nw, (int)o));
        nw = (uint32_t)__builtin_amdgcn_readfirstlane((int)nw);
        const uint32_t exp_base = lds_addr(s_exp);
#pragma unroll
        for (uint32_t r0 = 0; r0 < MAXE; r0 += 4) {
            if (r0 >= nw || nw < 2 || gl >= K) continue;   // wave-uniform but for gl
            const uint32_t sb = nl_base + ((uint32_t)S[gl] ^ copy5), dn = Dn[gl];
            uint32_t c[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (r0 + j < MAXE) c[j] = lds_ld8(exp_base + Nd[r0 + j] + lds_ld8(sb ^ Od[r0 + j]) + dn);
            uint8_t* C = P + lay.coef_off + gl;
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (r0 + j < MAXE && r0 + j < nout && nout >= 2) C[(r0 + j) * K] = (uint8_t)c[j];
        }
        const bool last = sg + 1 >= segs || base + G >= a.nblocks;
        if (wl + 1 < win && !last) continue;   // workgroup-uniform
        sort_window_out(a, smem, L, (wl + 1) * G, base - wl * G);
    }
}

// Segments per workgroup: enough workgroups to fill the chip several times over, each staging the
// tables once for all its segments; a sort window never spans two workgroups.
inline uint32_t plan_segments(uint32_t nseg, uint32_t win) {
    uint32_t segs = std::max<uint32_t>(1, nseg / 4096);
    segs = std::min<uint32_t>(segs, std::max<uint32_t>(64, win));
    return (segs + win - 1) / win * win;
}

template <uint32_t K, uint32_t M>
hipError_t code_launch(const PlanArgs& a, hipStream_t s) {
    constexpr uint32_t LPB = K <= 16 ? 16u : 32u, G = kPlanSortThreads / LPB;
    const uint32_t nseg = (a.nblocks + G - 1) / G;
    if (nseg == 0) return hipSuccess;
    const uint32_t win = sort_window(G), segs = plan_segments(nseg, win);
    const uint32_t grid = (nseg + segs - 1) / segs;
    const size_t lds = sort_lds(M, K, G, a.lay.stride, win, kGroupScratch3).total;
    hipLaunchKernelGGL((rs_plan_code_kernel<K, M>), dim3(grid), dim3(kPlanSortThreads), lds, s, a, segs, win);
    return hipGetLastError();
}

template <uint32_t LPB>
hipError_t sorted_launch(const PlanArgs& a, hipStream_t s) {
    constexpr uint32_t G = kPlanSortThreads / LPB;
    const uint32_t nseg = (a.nblocks + G - 1) / G;
    if (nseg == 0) return hipSuccess;
    const uint32_t win = sort_window(G), segs = plan_segments(nseg, win);
    const uint32_t grid = (nseg + segs - 1) / segs;
    const size_t lds = sort_lds(a.m, a.k, G, a.lay.stride, win).total;
    hipLaunchKernelGGL((rs_plan_sorted_kernel<LPB>), dim3(grid), dim3(kPlanSortThreads), lds, s, a, segs, win);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_rs_plan_sorted(const PlanArgs& a, hipStream_t s) {
    if (a.k == 16 && a.m == 8 && a.maxe == 8) return code_launch<16, 8>(a, s);
    if (a.k == 20 && a.m == 10 && a.maxe == 10) return code_launch<20, 10>(a, s);
    switch (plan_lanes(a.k)) {
        case 2: return sorted_launch<2>(a, s);
        case 4: return sorted_launch<4>(a, s);
        case 8: return sorted_launch<8>(a, s);
        case 16: return sorted_launch<16>(a, s);
        default: return sorted_launch<32>(a, s);
    }
}

}  // namespace fk
