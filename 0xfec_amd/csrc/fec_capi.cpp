// fec_capi.cpp — C ABI of the MI355X FEC codec (include/fec_hip.h).
//
// Owns the per-device context: HIP stream, per-(k, m) code cache (systematic matrix,
// device parity rows, encode PermTabs), decode plan workspace, pinned staging for the
// FEC_HOST path. No CPU compute fallback exists: without a HIP device every compute
// entry point fails with FEC_ERR_NO_DEVICE / FEC_ERR_HIP.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <map>
#include <memory>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/fec_hip.h"
#include "fec_kernels.hpp"
#include "gf256.h"
#include "rs_matrix.hpp"

namespace {

struct Code {
    int k = 0, m = 0;
    std::vector<uint8_t> matrix;   // n x k
    uint8_t* d_prows = nullptr;    // m x k
    uint32_t* d_tabs = nullptr;    // m x k PermTabs
    uint32_t* d_dytabs = nullptr;  // dyadic codes: leaf PermTabs of the split-recursive encode
    uint32_t* d_single = nullptr;  // single-erasure decode tables (fk::direct_table_words), when small
    uint32_t* d_single_coef = nullptr;   // their coefficient bytes, (k*m) rows of ceil(k/4) dwords
    std::vector<uint32_t> single_coef;   // host copy
    uint8_t* d_dall = nullptr;     // n bytes: sum_{t != s} log(s ^ t) mod 255 (sorted plans)
};

// Parity row r, column j of a dyadic code is g(r ^ j), g = parity row 0 (fec_kernels.hip,
// "dyadic encode"); k and m powers of two, m <= k. Returns the leaf constants of the recursion
// conv(C, D) = (P ^ Q, R ^ P ^ Q) for each group h of m columns, in the kernel's order (P's
// leaves, Q's, R's), or nothing when the matrix is not dyadic.
std::vector<uint8_t> dyadic_leaves(const std::vector<uint8_t>& matrix, int k, int m) {
    auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
    if (!pow2(k) || !pow2(m) || m > k) return {};
    const uint8_t* g = matrix.data() + (size_t)k * k;
    for (int r = 1; r < m; ++r)
        for (int j = 0; j < k; ++j)
            if (g[(size_t)r * k + j] != g[r ^ j]) return {};
    std::vector<uint8_t> out;
    std::function<void(const std::vector<uint8_t>&)> leaves = [&](const std::vector<uint8_t>& c) {
        if (c.size() == 1) {
            out.push_back(c[0]);
            return;
        }
        const size_t h = c.size() / 2;
        std::vector<uint8_t> lo(c.begin(), c.begin() + h), hi(c.begin() + h, c.end()), sum(h);
        for (size_t i = 0; i < h; ++i) sum[i] = (uint8_t)(lo[i] ^ hi[i]);
        leaves(lo);
        leaves(hi);
        leaves(sum);
    };
    for (int h = 0; h < k / m; ++h) leaves(std::vector<uint8_t>(g + (size_t)h * m, g + (size_t)(h + 1) * m));
    return out;
}


// Bytes of staged shards per FEC_HOST chunk (x2 buffers, in and out).
constexpr size_t kStageBytes = size_t(128) << 20;
// Upper bound on decode plan workspace.
constexpr size_t kPlanBytes = size_t(256) << 20;
// nblocks * chunks-per-shard must stay below 2^31 per launch (32-bit item ids).
constexpr uint64_t kMaxItems = uint64_t(1) << 31;

}  // namespace

// Device scratch of the kernels enqueued on one stream: decode plan records. Each stream the ctx
// launches on (its own / the caller's, and one per host-path staging set) has its own, so
// launches that overlap on different streams never share one (nor free one the other stream
// still reads).
struct Work {
    uint8_t* d_plans = nullptr;
    size_t plans_cap = 0;
    uint32_t* d_wflags = nullptr;   // routed in-place decode: the classify pass's route word
    size_t wflags_cap = 0;
    void release() {
        if (d_plans) (void)hipFree(d_plans);
        if (d_wflags) (void)hipFree(d_wflags);
        *this = Work{};
    }
};

// One staging set of the host-resident path: pinned host and device buffers for one chunk of
// blocks, and the events that carry that chunk through the pipeline's streams (HostPipe).
struct HostSet {
    uint8_t* h_in = nullptr;
    uint8_t* h_out = nullptr;
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    uint32_t* h_masks = nullptr;
    uint32_t* d_masks = nullptr;
    int32_t* h_status = nullptr;
    int32_t* d_status = nullptr;
    uint8_t* d_raw_in = nullptr;    // FEC_HOST_PINNED: the caller's span, copied linearly (fec_pack.hip)
    uint8_t* d_raw_out = nullptr;   // FEC_HOST_PINNED: the packed image of the outputs, copied down linearly
    size_t in_cap = 0, out_cap = 0, blk_cap = 0, raw_in_cap = 0, raw_out_cap = 0;
    hipEvent_t up_done = nullptr;     // its H2D copies have landed
    hipEvent_t k_done = nullptr;      // its kernels are done (the device inputs are free)
    hipEvent_t down_done = nullptr;   // its D2H copies have landed (the set is free)
};

// The host-resident pipeline. Chunk c of a call uses set c % kHostSets and moves through three
// streams in order: H2D copies on `up`, kernels on `comp`, D2H copies on `down`, ordered by the
// set's events alone. PCIe's two directions and the kernels of different chunks therefore overlap,
// and the up direction (the larger one on every path) never waits for the host: the host blocks only
// to reuse a set, on its chunk kHostSets back, and at the end of a call. Measured on one MI355X
// (tools/pcie_duplex_probe.hip, profiles/r04/pcie_duplex_probe_r04b.log): H2D 57.6 GB/s, D2H 57.0,
// both at once 48.6 each way; this shape with 64 MiB chunks moved 53.8 GB/s up.
constexpr int kHostSets = 3;
struct HostPipe {
    hipStream_t up = nullptr, comp = nullptr, down = nullptr;
    Work w;   // scratch of the kernels on comp
    HostSet set[kHostSets];
};

struct fec_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    std::map<std::pair<int, int>, Code> codes;
    Work main;               // scratch of the kernels on `own` / the caller's stream
    Work* work = &main;      // scratch of the kernels on `stream` (on_stream switches both)
    int* d_err = nullptr;    // [0] sticky device-path error, [1] host-path error
    uint8_t* h_stage = nullptr;
    uint8_t* d_stage = nullptr;
    size_t stage_cap = 0;
    uint32_t* d_masks = nullptr;
    int32_t* d_status = nullptr;
    size_t masks_cap = 0;
    HostPipe pipe;           // host-resident path (FEC_HOST / FEC_HOST_PINNED)
    hipEvent_t handoff = nullptr;   // orders a newly set stream after the previous one
};

#define HIP_TRY(expr)                      \
    do {                                   \
        if ((expr) != hipSuccess) {        \
            (void)hipGetLastError();       \
            return FEC_ERR_HIP;            \
        }                                  \
    } while (0)

static int select_device(fec_ctx* ctx) {
    if (!ctx) return FEC_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    return FEC_OK;
}

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

static int get_code(fec_ctx* ctx, int k, int m, Code** out) {
    if (k <= 0 || m < 0) return FEC_ERR_INV_SHARD_NUM;
    if (k + m > 256) return FEC_ERR_MAX_SHARD_NUM;
    auto key = std::make_pair(k, m);
    auto it = ctx->codes.find(key);
    if (it != ctx->codes.end()) {
        *out = &it->second;
        return FEC_OK;
    }
    Code c;
    c.k = k;
    c.m = m;
    c.matrix = rs::build_matrix(k, k + m);
    if (c.matrix.empty()) return FEC_ERR_INV_SHARD_NUM;
    if (m > 0) {
        std::vector<uint32_t> tabs((size_t)m * k * 8);
        for (int r = 0; r < m; ++r)
            for (int j = 0; j < k; ++j) {
                gf::PermTab t = gf::make_permtab(c.matrix[(size_t)(k + r) * k + j]);
                memcpy(&tabs[((size_t)r * k + j) * 8], &t, sizeof(t));
            }
        HIP_TRY(hipMalloc(&c.d_prows, (size_t)m * k));
        HIP_TRY(hipMalloc(&c.d_tabs, tabs.size() * 4));
        HIP_TRY(hipMemcpy(c.d_prows, c.matrix.data() + (size_t)k * k, (size_t)m * k, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c.d_tabs, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice));
        // single-erasure plans: data shard E0 lost, parity R0 the first present one; inputs are
        // the other data shards in order, then parity R0 (the first k present shards):
        // x_E0 = inv(A[R0][E0]) * (p_R0 ^ sum_{j != E0} A[R0][j] x_j)   (reed_solomon.go:124)
        if (k + m <= FEC_MAX_DECODE_SHARDS) {
            // the coefficient bytes of every single-erasure plan (small for every decodable code:
            // RS(20,30) 4 KB): the direct decode reads a wave's rows by scalar loads
            const size_t kw = ((size_t)k + 3) / 4;
            std::vector<uint32_t> sc((size_t)k * m * kw, 0);
            for (int e0 = 0; e0 < k; ++e0)
                for (int r0 = 0; r0 < m; ++r0) {
                    const uint8_t* row = c.matrix.data() + (size_t)(k + r0) * k;
                    const uint8_t inv = gf::inv(row[e0]);
                    uint8_t* dst = reinterpret_cast<uint8_t*>(&sc[((size_t)e0 * m + r0) * kw]);
                    for (int j = 0, pos = 0; j <= k; ++j)
                        if (j != e0) dst[pos++] = j < k ? gf::mul(inv, row[j]) : inv;
                }
            c.single_coef = sc;
            HIP_TRY(hipMalloc(&c.d_single_coef, sc.size() * 4));
            HIP_TRY(hipMemcpy(c.d_single_coef, sc.data(), sc.size() * 4, hipMemcpyHostToDevice));
        }
        if (k + m <= FEC_MAX_DECODE_SHARDS && fk::direct_table_words((uint32_t)k, (uint32_t)m) * 4 <= 16 * 1024) {
            // the same plans expanded to PermTabs (k*m*k*32 bytes; small codes only)
            std::vector<uint32_t> st(fk::direct_table_words((uint32_t)k, (uint32_t)m), 0);
            for (int e0 = 0; e0 < k; ++e0)
                for (int r0 = 0; r0 < m; ++r0) {
                    const uint8_t* row = c.matrix.data() + (size_t)(k + r0) * k;
                    const uint8_t inv = gf::inv(row[e0]);
                    for (int j = 0, pos = 0; j <= k; ++j) {
                        if (j == e0) continue;
                        const uint8_t coef = j < k ? gf::mul(inv, row[j]) : inv;
                        gf::PermTab t = gf::make_permtab(coef);
                        memcpy(&st[(((size_t)e0 * m + r0) * k + pos) * 8], &t, sizeof(t));
                        ++pos;
                    }
                }
            HIP_TRY(hipMalloc(&c.d_single, st.size() * 4));
            HIP_TRY(hipMemcpy(c.d_single, st.data(), st.size() * 4, hipMemcpyHostToDevice));
        }
        if (k + m <= FEC_MAX_DECODE_SHARDS) {
            uint8_t dall[FEC_MAX_DECODE_SHARDS] = {};
            for (int sidx = 0; sidx < k + m; ++sidx) {
                unsigned d = 0;
                for (int t = 0; t < k + m; ++t)
                    if (t != sidx) d += gf::kTables.log[sidx ^ t];
                dall[sidx] = (uint8_t)(d % 255u);
            }
            HIP_TRY(hipMalloc(&c.d_dall, FEC_MAX_DECODE_SHARDS));
            HIP_TRY(hipMemcpy(c.d_dall, dall, FEC_MAX_DECODE_SHARDS, hipMemcpyHostToDevice));
        }
        const std::vector<uint8_t> leaves = dyadic_leaves(c.matrix, k, m);
        if (!leaves.empty() && leaves.size() <= (size_t)m * k) {   // staged like m x k tables
            std::vector<uint32_t> dy((size_t)m * k * 8, 0);
            for (size_t i = 0; i < leaves.size(); ++i) {
                gf::PermTab t = gf::make_permtab(leaves[i]);
                memcpy(&dy[i * 8], &t, sizeof(t));
            }
            HIP_TRY(hipMalloc(&c.d_dytabs, dy.size() * 4));
            HIP_TRY(hipMemcpy(c.d_dytabs, dy.data(), dy.size() * 4, hipMemcpyHostToDevice));
        }
    }
    auto res = ctx->codes.emplace(key, std::move(c));
    *out = &res.first->second;
    // the uploads above are plain hipMemcpy (null stream, and from pageable memory they may return
    // before the DMA lands): finish them before a kernel on a non-blocking ctx stream reads a table
    HIP_TRY(hipDeviceSynchronize());
    return FEC_OK;
}

static int grow_plans(fec_ctx* ctx, size_t bytes) {
    Work& w = *ctx->work;
    if (bytes <= w.plans_cap) return FEC_OK;
    HIP_TRY(hipStreamSynchronize(ctx->stream));   // the only stream that reads this workspace
    if (w.d_plans) HIP_TRY(hipFree(w.d_plans));
    w.d_plans = nullptr;
    w.plans_cap = 0;
    HIP_TRY(hipMalloc(&w.d_plans, bytes));
    w.plans_cap = bytes;
    return FEC_OK;
}

static int grow_wflags(fec_ctx* ctx, size_t n) {
    Work& w = *ctx->work;
    if (n <= w.wflags_cap) return FEC_OK;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (w.d_wflags) HIP_TRY(hipFree(w.d_wflags));
    w.d_wflags = nullptr;
    w.wflags_cap = 0;
    HIP_TRY(hipMalloc(&w.d_wflags, n * 4));
    w.wflags_cap = n;
    return FEC_OK;
}

static int grow_stage(fec_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->stage_cap) return FEC_OK;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (ctx->h_stage) HIP_TRY(hipHostFree(ctx->h_stage));
    if (ctx->d_stage) HIP_TRY(hipFree(ctx->d_stage));
    ctx->h_stage = nullptr;
    ctx->d_stage = nullptr;
    ctx->stage_cap = 0;
    HIP_TRY(hipHostMalloc(&ctx->h_stage, bytes, hipHostMallocDefault));
    HIP_TRY(hipMalloc(&ctx->d_stage, bytes));
    ctx->stage_cap = bytes;
    return FEC_OK;
}

static int grow_masks(fec_ctx* ctx, size_t n) {
    if (n <= ctx->masks_cap) return FEC_OK;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (ctx->d_masks) HIP_TRY(hipFree(ctx->d_masks));
    if (ctx->d_status) HIP_TRY(hipFree(ctx->d_status));
    ctx->d_masks = nullptr;
    ctx->d_status = nullptr;
    ctx->masks_cap = 0;
    HIP_TRY(hipMalloc(&ctx->d_masks, n * 4));
    HIP_TRY(hipMalloc(&ctx->d_status, n * 4));
    ctx->masks_cap = n;
    return FEC_OK;
}

static size_t round16(size_t x) { return (x + 15) & ~size_t(15); }

// Workgroups for a flat (block, chunk) item launch: one item per lane (total < 2^31).
static int flat_grid(uint32_t total) {
    return (int)std::max<uint64_t>(1, ((uint64_t)total + fk::kThreads - 1) / fk::kThreads);
}

// ---------------------------------------------------------------- device-memory cores

static int rs_encode_device(fec_ctx* ctx, Code* code, size_t len, size_t nblocks, const uint8_t* data,
                            size_t dbs, uint8_t* parity, size_t pbs, size_t ss) {
    const uint32_t cps = (uint32_t)((len + fk::kChunk - 1) / fk::kChunk);
    const size_t per_launch = std::max<size_t>(1, (size_t)(kMaxItems / cps));
    const int k = code->k;
    for (size_t b0 = 0; b0 < nblocks; b0 += per_launch) {
        const size_t nb = std::min(per_launch, nblocks - b0);
        for (int r0 = 0; r0 < code->m; r0 += 16) {
            const int mr = std::min(16, code->m - r0);
            fk::EncodeArgs a{};
            a.in = data + b0 * dbs;
            a.out = parity + b0 * pbs + (size_t)r0 * ss;
            a.in_bs = dbs;
            a.out_bs = pbs;
            a.ss = ss;
            a.k = (uint32_t)k;
            a.m = (uint32_t)mr;
            a.len = (uint32_t)len;
            a.cps = cps;
            a.total = (uint32_t)(nb * cps);
            a.div_cps = fk::make_fastdiv(cps);
            a.tabs = code->d_tabs + (size_t)r0 * k * 8;
            a.dytabs = (r0 == 0 && mr == code->m) ? code->d_dytabs : nullptr;
            a.sp = fk::encode_store_policy(fk::g_tune.st_pol, data, dbs, parity, pbs, nblocks);
            if (fk::fixed_encode_applies((uint32_t)k, (uint32_t)mr, a.dytabs != nullptr)) {
                HIP_TRY(fk::launch_rs_encode_fixed(a, ctx->stream));
                continue;
            }
            HIP_TRY(fk::launch_rs_encode(a, flat_grid(a.total), ctx->stream));
        }
    }
    return FEC_OK;
}

static int rs_reconstruct_device(fec_ctx* ctx, Code* code, size_t len, size_t nblocks, uint8_t* data,
                                 size_t dbs, const uint8_t* parity, size_t pbs, size_t ss, const uint32_t* masks,
                                 int32_t* status, int* err, uint8_t* out = nullptr, size_t out_bs = 0,
                                 uint32_t out_slots = 0, size_t pss = 0) {
    if (pss == 0) pss = ss;
    if ((ss | pss) >> 32) return FEC_ERR_INVALID_ARG;   // the rebuild kernels take 32-bit shard strides
    const uint32_t k = (uint32_t)code->k, m = (uint32_t)code->m;
    const uint32_t maxe = std::max<uint32_t>(1, std::min(k, m));
    const uint32_t cps = (uint32_t)((len + fk::kChunk - 1) / fk::kChunk);
    const fk::PlanLayout lay_block = fk::plan_layout(k, maxe), lay_sorted = fk::plan_layout(k, maxe, true);
    // Three forms:
    //  * direct (fec_recover.hip): no plan kernel; single-erasure tables of the code, for calls
    //    where no block can need more (one output slot per block, or m = 1). Small codes (RS(2,3),
    //    RS(8,12)) and RS(16,24) / RS(20,30) (RS(20,30) single erasure +15 % over plan + rebuild,
    //    r03h);
    //  * shards of 32+ chunks: sorted plans (fec_plan.hip), then the wave-form rebuild
    //    (fec_rebuild.hip for RS(16,24) / RS(20,30) with 64+ chunks, else fec_decode.hip);
    //  * short shards: plans in block order, then the workgroup-tile rebuild.
    //  * routed (in-place calls of RS(8,12)): a classify pass reduces the masks to one word; the
    //    sorted plans run only if some block has two or more erased data shards, and one kernel
    //    runs the direct body or the wave rebuild by that word (fec_recover.hip).
    const bool single_slot = out && out_slots == 1;
    const bool direct = code->d_single_coef && fk::direct_recon_applies(k, m, cps, single_slot);
    const bool wave = !direct && fk::wave_recon_applies(cps, k, maxe, lay_sorted.stride);
    const bool routed = wave && !out && code->d_single_coef && !fk::rebuild_k_applies(k, maxe, cps) &&
                        fk::routed_recon_applies(k, m, cps, maxe, lay_sorted.stride);
    const fk::PlanLayout lay = wave ? lay_sorted : lay_block;
    size_t per_launch = std::min<size_t>(direct ? nblocks : kPlanBytes / lay.stride, (size_t)(kMaxItems / cps));
    per_launch = std::max<size_t>(1, std::min(per_launch, nblocks));
    if (!direct) {
        const int rc = grow_plans(ctx, per_launch * lay.stride);
        if (rc) return rc;
    }
    if (routed) {
        const int rc = grow_wflags(ctx, 1);
        if (rc) return rc;
    }
    const uint32_t G = fk::pick_tile_blocks(cps, k, maxe, lay);
    for (size_t b0 = 0; b0 < nblocks; b0 += per_launch) {
        const size_t nb = std::min(per_launch, nblocks - b0);
        fk::PlanArgs p{};
        p.masks = masks + b0;
        p.plans = ctx->work->d_plans;
        p.status = status ? status + b0 : nullptr;
        p.err = err;
        p.prows = code->d_prows;
        p.k = k;
        p.m = m;
        p.nblocks = (uint32_t)nb;
        p.maxe = maxe;
        p.lay = lay;
        p.max_out = out ? out_slots : 0;
        p.dall = code->d_dall;
        fk::ReconArgs a{};
        a.data = data + b0 * dbs;
        a.parity = parity + b0 * pbs;
        a.dbs = dbs;
        a.pbs = pbs;
        a.ss = ss;
        a.pss = pss;
        a.plans = ctx->work->d_plans;
        a.k = k;
        a.len = (uint32_t)len;
        a.cps = cps;
        a.nblocks = (uint32_t)nb;
        a.maxe = maxe;
        a.lay = lay;
        a.g = G;
        a.ntiles = (uint32_t)((nb + G - 1) / G);
        a.div_cps = fk::make_fastdiv(cps);
        a.sorted = wave ? 1u : 0u;
        a.out = out ? out + b0 * out_bs : nullptr;
        a.out_bs = out_bs;
        if (direct || routed) {
            a.masks = p.masks;
            a.status = p.status;
            a.err = p.err;
            a.prows = p.prows;
            a.m = m;
            a.max_out = p.max_out;
            a.single = code->d_single;
            a.single_coef = code->d_single_coef;
            a.single_coef_host = code->single_coef.data();
            a.sp = fk::decode_store_policy(fk::g_tune.dst_pol, data, dbs, parity, pbs, out, out_bs, nblocks);
        }
        if (direct) {
            HIP_TRY(fk::launch_rs_recover_direct(a, ctx->stream));
        } else if (routed) {
            a.route = p.route = ctx->work->d_wflags;
            HIP_TRY(fk::launch_rs_route_classify(a, ctx->work->d_wflags, ctx->stream));
            HIP_TRY(fk::launch_rs_plan_sorted(p, ctx->stream));
            HIP_TRY(fk::launch_rs_reconstruct_routed(a, ctx->stream));
        } else if (wave) {
            HIP_TRY(fk::launch_rs_plan_sorted(p, ctx->stream));
            if (fk::rebuild_k_applies(k, maxe, cps)) HIP_TRY(fk::launch_rs_rebuild_k(a, ctx->stream));
            else HIP_TRY(fk::launch_rs_reconstruct_wave(a, ctx->stream));
        } else {
            HIP_TRY(fk::launch_rs_plan(p, ctx->stream));
            HIP_TRY(fk::launch_rs_reconstruct(a, (int)std::max<uint32_t>(1, a.ntiles), ctx->stream));
        }
    }
    return FEC_OK;
}

static int xor_encode_device(fec_ctx* ctx, int k, size_t len, size_t nblocks, const uint8_t* data, size_t dbs,
                             uint8_t* parity, size_t pbs, size_t ss) {
    const uint32_t cps = (uint32_t)((len + fk::kChunk - 1) / fk::kChunk);
    const size_t per_launch = std::max<size_t>(1, (size_t)(kMaxItems / cps));
    for (size_t b0 = 0; b0 < nblocks; b0 += per_launch) {
        const size_t nb = std::min(per_launch, nblocks - b0);
        fk::XorArgs a{};
        a.in = data + b0 * dbs;
        a.out = parity + b0 * pbs;
        a.in_bs = dbs;
        a.out_bs = pbs;
        a.ss = ss;
        a.k = (uint32_t)k;
        a.len = (uint32_t)len;
        a.cps = cps;
        a.total = (uint32_t)(nb * cps);
        a.div_cps = fk::make_fastdiv(cps);
        HIP_TRY(fk::launch_xor_encode(a, flat_grid(a.total), ctx->stream));
    }
    return FEC_OK;
}

static int xor_reconstruct_device(fec_ctx* ctx, int k, size_t len, size_t nblocks, uint8_t* data, size_t dbs,
                                  const uint8_t* parity, size_t pbs, size_t ss, const uint32_t* masks,
                                  int32_t* status, int* err) {
    const uint32_t cps = (uint32_t)((len + fk::kChunk - 1) / fk::kChunk);
    const size_t per_launch = std::max<size_t>(1, (size_t)(kMaxItems / cps));
    for (size_t b0 = 0; b0 < nblocks; b0 += per_launch) {
        const size_t nb = std::min(per_launch, nblocks - b0);
        fk::XorArgs a{};
        a.in = data + b0 * dbs;
        a.out = data + b0 * dbs;
        a.parity = parity + b0 * pbs;
        a.in_bs = dbs;
        a.out_bs = dbs;
        a.par_bs = pbs;
        a.ss = ss;
        a.masks = masks + b0;
        a.status = status ? status + b0 : nullptr;
        a.err = err;
        a.k = (uint32_t)k;
        a.len = (uint32_t)len;
        a.cps = cps;
        a.total = (uint32_t)(nb * cps);
        a.nblocks = (uint32_t)nb;
        a.div_cps = fk::make_fastdiv(cps);
        HIP_TRY(fk::launch_xor_reconstruct(a, flat_grid(a.total), ctx->stream));
    }
    return FEC_OK;
}

// ---------------------------------------------------------------- validation helpers

// FEC_DEVICE masks and statuses are read and written as 4-byte words (the masks by scalar loads,
// which ignore the low two address bits: a misaligned mask array would be read wrong, silently).
static int check_device_words(const uint32_t* masks, const int32_t* status) {
    return (((uintptr_t)masks | (uintptr_t)status) & 3u) ? FEC_ERR_ALIGNMENT : FEC_OK;
}

static int check_device_layout(const void* p, size_t bs, size_t ss, size_t len) {
    if (!p) return FEC_ERR_INVALID_ARG;
    if (!aligned16(p) || (bs & 15) || (ss & 15)) return FEC_ERR_ALIGNMENT;
    if (ss < len) return FEC_ERR_INVALID_ARG;
    return FEC_OK;
}

// ---------------------------------------------------------------- host-resident path
// FEC_HOST (pageable host memory): each chunk of blocks is staged by the calling thread into a
// pinned buffer, copied up with one hipMemcpyAsync, coded, copied down with one, and its results
// copied out once its set comes round again. FEC_HOST_PINNED (the caller's buffers are pinned or
// registered): no staging copies; the caller's span of a chunk goes up in one linear DMA and is
// repacked into 16-byte slots on the device (or one 2D DMA per shard column when the span is
// sparse), and packed outputs come down the same way. Only what the code needs crosses PCIe:
// encode sends the k data shards and returns the m parity shards; reconstruct sends the data
// shards and the parity planes its blocks read, and returns only the rebuilt shards. Chunks run
// through HostPipe's three streams (up / kernels / down), kHostSets at a time.

// Blocks per chunk of a host-path call of nblocks: at most kStageBytes of staged input (128 MiB:
// larger chunks gain nothing, r04o), and for a call of fewer than kHostSets such chunks, the call
// split over the sets, so its three sets together hold about the call rather than three full
// chunks; never below kMinChunkBlocks (chunks of 3072-4096 RS(8,12) blocks lose 10 % to their
// per-chunk overhead, 6144 and up do not: host_chunk_sweep_r04o.log).
constexpr size_t kMinChunkBlocks = 6144;
static size_t host_chunk_blocks(size_t nblocks, size_t bytes_per_block) {
    if (fk::g_tune.host_chunk > 0) return std::min(nblocks, (size_t)fk::g_tune.host_chunk);   // tests: many small chunks
    const size_t full = std::max<size_t>(1, kStageBytes / std::max<size_t>(1, bytes_per_block));
    const size_t split = std::max(kMinChunkBlocks, (nblocks + kHostSets - 1) / kHostSets);
    return std::max<size_t>(1, std::min({nblocks, full, split}));
}

// Copy workers made once per process for parallel_for: a chunk's staging or scatter copy then
// costs two condition-variable hand-offs instead of creating and joining a thread per part
// (tens of microseconds each, ~40 times per pageable bench step). One call at a time: a caller
// that finds the pool busy (another thread's FEC_HOST call) makes its own threads as before.
class CopyPool {
   public:
    static CopyPool& get() {
        static CopyPool* p = new CopyPool();   // never destroyed: workers may outlive static teardown
        return *p;
    }
    // false: busy, nothing run
    bool run(unsigned parts, size_t n, const std::function<void(size_t, size_t)>& fn) {
        std::unique_lock<std::mutex> call(call_mu_, std::try_to_lock);
        if (!call.owns_lock()) return false;
        std::unique_lock<std::mutex> lk(mu_);
        while (th_.size() + 1 < parts) th_.emplace_back([this] { work(); });
        fn_ = &fn;
        n_ = n;
        per_ = (n + parts - 1) / parts;
        parts_ = (unsigned)((n + per_ - 1) / per_);
        next_ = 1;   // part 0 is the caller's
        left_ = parts_;
        ++gen_;
        lk.unlock();
        cv_.notify_all();
        fn(0, std::min(n, per_));
        lk.lock();
        --left_;
        for (;;) {   // the caller takes parts too while any are unclaimed
            if (next_ >= parts_) break;
            const unsigned i = next_++;
            lk.unlock();
            fn(i * per_, std::min(n, (i + 1) * per_));
            lk.lock();
            --left_;
        }
        done_.wait(lk, [this] { return left_ == 0; });
        fn_ = nullptr;
        return true;
    }

   private:
    void work() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return gen_ != seen; });
            seen = gen_;
            while (fn_ && next_ < parts_) {
                const unsigned i = next_++;
                const auto* fn = fn_;
                const size_t lo = i * per_, hi = std::min(n_, (i + 1) * per_);
                lk.unlock();
                (*fn)(lo, hi);
                lk.lock();
                if (--left_ == 0) done_.notify_all();
            }
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    const std::function<void(size_t, size_t)>* fn_ = nullptr;
    size_t n_ = 0, per_ = 0;
    unsigned parts_ = 0, next_ = 0, left_ = 0;
    uint64_t gen_ = 0;
};

// fn(lo, hi) over [0, n) on up to host_threads threads (knob, 8): the staging and scatter copies
// of FEC_HOST (one core copies ~10 GB/s, a fifth of PCIe), on CopyPool's persistent workers (r04j:
// +0.7 to +1.6 GiB/s pageable over threads made per call); a caller that finds them busy makes
// its own.
template <class F>
static void parallel_for(size_t n, F fn) {
    const unsigned T = std::min<unsigned>((unsigned)std::max(1, (int)fk::g_tune.host_threads),
                                          std::max(1u, std::thread::hardware_concurrency()));
    if (n < 512 || T == 1) {
        fn((size_t)0, n);
        return;
    }
    if (CopyPool::get().run(T, n, std::function<void(size_t, size_t)>(fn))) return;
    std::vector<std::thread> th;
    const size_t per = (n + T - 1) / T;
    for (size_t lo = 0; lo < n; lo += per) th.emplace_back(fn, lo, std::min(n, lo + per));
    for (auto& t : th) t.join();
}

static int grow_dev(uint8_t** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return FEC_OK;
    if (*p) HIP_TRY(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc(p, bytes));
    *cap = bytes;
    return FEC_OK;
}

// Bytes of the caller's span of nb blocks (shards of len bytes, cols per block).
static size_t span_bytes(size_t nb, size_t cols, size_t bs, size_t ss, size_t len) {
    return (nb - 1) * bs + (cols - 1) * ss + len;
}

// A span worth one linear copy: at most a quarter more bytes than the shards themselves.
static bool dense_span(size_t nb, size_t cols, size_t bs, size_t ss, size_t len) {
    return span_bytes(nb, cols, bs, ss, len) * 4 <= nb * cols * len * 5;
}

// Caller's columns [0, cols) of nb blocks toward the device stage [nb][st_bs/st_ss], on stream
// `up`: when the span of all span_cols >= cols columns is dense, one linear DMA of it into `raw`
// (a few unneeded columns ride along: one linear DMA beats narrow 2D rows) and *repack = true (the
// kernel stream then runs pinned_repack); else one 2D DMA per column straight into the stage.
static int pinned_up(hipStream_t up, uint8_t* stage, size_t st_bs, size_t st_ss, const uint8_t* src, size_t bs,
                     size_t ss, size_t nb, size_t cols, size_t len, uint8_t* raw, size_t span_cols, bool* repack) {
    *repack = dense_span(nb, span_cols, bs, ss, len);
    if (*repack) {
        HIP_TRY(hipMemcpyAsync(raw, src, span_bytes(nb, span_cols, bs, ss, len), hipMemcpyHostToDevice, up));
        return FEC_OK;
    }
    for (size_t j = 0; j < cols; ++j)
        HIP_TRY(hipMemcpy2DAsync(stage + j * st_ss, st_bs, src + j * ss, bs, len, nb, hipMemcpyHostToDevice, up));
    return FEC_OK;
}

// The caller layout's outputs are packed (no bytes between shards): the kernel stream packs the
// device stage into one image that goes down in one linear DMA.
static bool packed_out(size_t bs, size_t ss, size_t cols, size_t len) { return ss == len && bs == cols * len; }

// Device stage [nb][st_bs/st_ss] columns back to the caller, on stream `down`: the packed image
// (packed_out) in one linear DMA, else one 2D DMA per column, which writes exactly len bytes per
// shard.
static int pinned_down(hipStream_t down, uint8_t* dst, size_t bs, size_t ss, const uint8_t* stage, size_t st_bs,
                       size_t st_ss, size_t nb, size_t cols, size_t len, const uint8_t* raw) {
    if (packed_out(bs, ss, cols, len)) {
        HIP_TRY(hipMemcpyAsync(dst, raw, nb * cols * len, hipMemcpyDeviceToHost, down));
        return FEC_OK;
    }
    for (size_t j = 0; j < cols; ++j)
        HIP_TRY(hipMemcpy2DAsync(dst + j * ss, bs, stage + j * st_ss, st_bs, len, nb, hipMemcpyDeviceToHost, down));
    return FEC_OK;
}

static int host_pipe_init(HostPipe& p) {
    if (p.up) return FEC_OK;
    for (hipStream_t* q : {&p.up, &p.comp, &p.down}) HIP_TRY(hipStreamCreateWithFlags(q, hipStreamNonBlocking));
    for (HostSet& s : p.set)
        for (hipEvent_t* e : {&s.up_done, &s.k_done, &s.down_done})
            HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return FEC_OK;
}

// Buffers of every set for chunks of in / out staged bytes and `blocks` blocks (a call grows them
// before its first chunk, when no chunk of the pipe is in flight).
static int host_pipe_grow(HostPipe& p, size_t in_bytes, size_t out_bytes, size_t blocks) {
    int rc;
    if ((rc = host_pipe_init(p))) return rc;
    for (HostSet& s : p.set) {
        if (in_bytes > s.in_cap) {
            if (s.h_in) HIP_TRY(hipHostFree(s.h_in));
            if (s.d_in) HIP_TRY(hipFree(s.d_in));
            s.h_in = s.d_in = nullptr;
            s.in_cap = 0;
            HIP_TRY(hipHostMalloc(&s.h_in, in_bytes, hipHostMallocDefault));
            HIP_TRY(hipMalloc(&s.d_in, in_bytes));
            s.in_cap = in_bytes;
        }
        if (out_bytes > s.out_cap) {
            if (s.h_out) HIP_TRY(hipHostFree(s.h_out));
            if (s.d_out) HIP_TRY(hipFree(s.d_out));
            s.h_out = s.d_out = nullptr;
            s.out_cap = 0;
            HIP_TRY(hipHostMalloc(&s.h_out, out_bytes, hipHostMallocDefault));
            HIP_TRY(hipMalloc(&s.d_out, out_bytes));
            s.out_cap = out_bytes;
        }
        if (blocks > s.blk_cap) {
            for (void* q : {(void*)s.h_masks, (void*)s.h_status})
                if (q) HIP_TRY(hipHostFree(q));
            for (void* q : {(void*)s.d_masks, (void*)s.d_status})
                if (q) HIP_TRY(hipFree(q));
            s.h_masks = s.d_masks = nullptr;
            s.h_status = s.d_status = nullptr;
            s.blk_cap = 0;
            HIP_TRY(hipHostMalloc(&s.h_masks, blocks * 4, hipHostMallocDefault));
            HIP_TRY(hipHostMalloc(&s.h_status, blocks * 4, hipHostMallocDefault));
            HIP_TRY(hipMalloc(&s.d_masks, blocks * 4));
            HIP_TRY(hipMalloc(&s.d_status, blocks * 4));
            s.blk_cap = blocks;
        }
    }
    return FEC_OK;
}

// Run `fn` with the ctx's kernels enqueued on the pipe's kernel stream, with its scratch.
template <class F>
static int on_pipe(fec_ctx* ctx, F fn) {
    hipStream_t keep = ctx->stream;
    Work* keep_w = ctx->work;
    ctx->stream = ctx->pipe.comp;
    ctx->work = &ctx->pipe.w;
    const int rc = fn();
    ctx->stream = keep;
    ctx->work = keep_w;
    return rc;
}

// One chunk of a host-path call: blocks [b0, b0 + nb) and what its stages decided.
struct HostChunk {
    size_t b0 = 0, nb = 0;
    bool live = false;
    bool repack = false;      // pinned: the data span came up raw, the kernel stream repacks it
    size_t planes = 0;        // reconstruct: parity planes [0, planes) reach the device
    uint32_t gather = 0;      // reconstruct, pinned: planes the device pulls itself (bit r)
    size_t slots = 1;         // reconstruct: output slots per block
};

// Chunks of `chunk` blocks through the pipe. up(s, ch): host staging, then the H2D copies on
// p.up; kern(s, ch): kernels on p.comp; down(s, ch): D2H copies on p.down; finish(s, ch) on the
// host once the chunk's copies have landed. On any failure every stream is drained before the
// error returns, so no set is left in flight.
template <class Up, class Kern, class Down, class Finish>
static int host_pipeline(fec_ctx* ctx, size_t nblocks, size_t chunk, Up up, Kern kern, Down down, Finish finish) {
    HostPipe& p = ctx->pipe;
    HostChunk pend[kHostSets];
    auto run = [&]() -> int {
        int rc;
        size_t c = 0;
        for (size_t b0 = 0; b0 < nblocks; b0 += chunk, ++c) {
            const int i = (int)(c % kHostSets);
            HostSet& s = p.set[i];
            if (pend[i].live) {   // the set's chunk kHostSets back: all of its buffers are free after this
                HIP_TRY(hipEventSynchronize(s.down_done));
                pend[i].live = false;
                if ((rc = finish(s, pend[i]))) return rc;
            }
            HostChunk ch;
            ch.b0 = b0;
            ch.nb = std::min(chunk, nblocks - b0);
            if ((rc = up(s, ch))) return rc;
            HIP_TRY(hipEventRecord(s.up_done, p.up));
            HIP_TRY(hipStreamWaitEvent(p.comp, s.up_done, 0));
            if ((rc = kern(s, ch))) return rc;
            HIP_TRY(hipEventRecord(s.k_done, p.comp));
            HIP_TRY(hipStreamWaitEvent(p.down, s.k_done, 0));
            if ((rc = down(s, ch))) return rc;
            HIP_TRY(hipEventRecord(s.down_done, p.down));
            ch.live = true;
            pend[i] = ch;
        }
        for (size_t t = 0; t < (size_t)kHostSets; ++t) {   // oldest chunk first
            const int i = (int)((c + t) % kHostSets);
            if (!pend[i].live) continue;
            HIP_TRY(hipEventSynchronize(p.set[i].down_done));
            pend[i].live = false;
            if ((rc = finish(p.set[i], pend[i]))) return rc;
        }
        return FEC_OK;
    };
    const int rc = run();
    if (rc) {
        for (hipStream_t q : {p.up, p.comp, p.down})
            if (q) (void)hipStreamSynchronize(q);
        (void)hipGetLastError();
    }
    return rc;
}

// Encode (RS when code != nullptr, else XOR(k, 1)): host data -> host parity.
static int host_encode(fec_ctx* ctx, Code* code, int k, int m, size_t len, size_t nblocks, const uint8_t* data,
                       size_t dbs, uint8_t* parity, size_t pbs, size_t ss, bool pinned) {
    const size_t ssd = round16(len);
    const size_t chunk = host_chunk_blocks(nblocks, (size_t)k * ssd);
    HostPipe& p = ctx->pipe;
    int rc;
    if ((rc = host_pipe_grow(p, chunk * k * ssd, chunk * m * ssd, 1))) return rc;
    const bool pack = pinned && packed_out(pbs, ss, (size_t)m, len);
    if (pinned)
        for (HostSet& s : p.set) {
            if ((rc = grow_dev(&s.d_raw_in, &s.raw_in_cap, span_bytes(chunk, k, dbs, ss, len) + 16))) return rc;
            if (pack && (rc = grow_dev(&s.d_raw_out, &s.raw_out_cap, chunk * m * len + 16))) return rc;
        }
    auto up = [&](HostSet& s, HostChunk& ch) -> int {
        if (pinned)
            return pinned_up(p.up, s.d_in, (size_t)k * ssd, ssd, data + ch.b0 * dbs, dbs, ss, ch.nb, k, len, s.d_raw_in,
                             k, &ch.repack);
        parallel_for(ch.nb, [&](size_t lo, size_t hi) {
            for (size_t b = lo; b < hi; ++b)
                for (int j = 0; j < k; ++j) memcpy(s.h_in + (b * k + j) * ssd, data + (ch.b0 + b) * dbs + j * ss, len);
        });
        HIP_TRY(hipMemcpyAsync(s.d_in, s.h_in, ch.nb * k * ssd, hipMemcpyHostToDevice, p.up));
        return FEC_OK;
    };
    auto kern = [&](HostSet& s, HostChunk& ch) -> int {
        if (ch.repack)
            HIP_TRY(fk::launch_span_to_stage(s.d_in, (size_t)k * ssd, ssd, s.d_raw_in, dbs, ss, (uint32_t)ch.nb,
                                             (uint32_t)k, (uint32_t)len, p.comp));
        const int r = on_pipe(ctx, [&] {
            return code ? rs_encode_device(ctx, code, len, ch.nb, s.d_in, (size_t)k * ssd, s.d_out, (size_t)m * ssd, ssd)
                        : xor_encode_device(ctx, k, len, ch.nb, s.d_in, (size_t)k * ssd, s.d_out, ssd, ssd);
        });
        if (r) return r;
        if (pack)
            HIP_TRY(fk::launch_stage_to_packed(s.d_raw_out, s.d_out, (size_t)m * ssd, ssd, (uint32_t)ch.nb,
                                               (uint32_t)m, (uint32_t)len, p.comp));
        return FEC_OK;
    };
    auto down = [&](HostSet& s, HostChunk& ch) -> int {
        if (pinned)
            return pinned_down(p.down, parity + ch.b0 * pbs, pbs, ss, s.d_out, (size_t)m * ssd, ssd, ch.nb, m, len,
                               s.d_raw_out);
        HIP_TRY(hipMemcpyAsync(s.h_out, s.d_out, ch.nb * m * ssd, hipMemcpyDeviceToHost, p.down));
        return FEC_OK;
    };
    auto finish = [&](HostSet& s, HostChunk& ch) -> int {
        if (!pinned)
            parallel_for(ch.nb, [&](size_t lo, size_t hi) {
                for (size_t b = lo; b < hi; ++b)
                    for (int r = 0; r < m; ++r)
                        memcpy(parity + (ch.b0 + b) * pbs + r * ss, s.h_out + (b * m + r) * ssd, len);
            });
        return FEC_OK;
    };
    return host_pipeline(ctx, nblocks, chunk, up, kern, down, finish);
}

// RS reconstruct, in place in the caller's data slots: per chunk, the data shards and the parity
// planes its blocks read go up (P = 1 + the highest parity index any block of the chunk reads
// among its first k present shards); the recover kernel rebuilds each block's erased data shards
// into [block][slot] outputs (slots = the chunk's largest erasure count); only those come down
// and are scattered into the erased slots. Pinned callers: a parity plane that at least 3/4 of
// the chunk's blocks read goes up by one 2D DMA (tools/zerocopy_probe.hip: 52 GB/s for a 1202-B
// row of every 4808 B); a sparser one is pulled by the device, plane by plane and block by block,
// straight from the caller's buffer (gather_planes_kernel), which moves only what is read but runs
// slower beside a D2H copy (pcie_duplex_probe: a kernel reading host memory and a D2H DMA at once
// make 29.9 GB/s each way).
static int host_reconstruct_rs(fec_ctx* ctx, Code* code, int k, int m, size_t len, size_t nblocks, uint8_t* data,
                               size_t dbs, const uint8_t* parity, size_t pbs, size_t ss, const uint32_t* masks,
                               int32_t* block_status, bool pinned) {
    const size_t ssd = round16(len);
    const size_t n = (size_t)k + m;
    const uint32_t all = fk::low_mask((uint32_t)n), kmask = fk::low_mask((uint32_t)k);
    const size_t maxe = (size_t)std::max(1, std::min(k, m));
    const size_t chunk = host_chunk_blocks(nblocks, n * ssd);
    HostPipe& p = ctx->pipe;
    int rc;
    if ((rc = host_pipe_grow(p, chunk * n * ssd, chunk * maxe * ssd, chunk))) return rc;
    if (pinned)
        for (HostSet& s : p.set)
            if ((rc = grow_dev(&s.d_raw_in, &s.raw_in_cap, span_bytes(chunk, k, dbs, ss, len) + 16))) return rc;
    // the sticky device word of the host path: statuses report every per-block failure, but a plan
    // kernel that cannot run (fec_plan.hip form 3's LDS-alignment guard, bit 4) writes no statuses
    HIP_TRY(hipMemsetAsync(ctx->d_err + 1, 0, sizeof(int), p.comp));
    bool failed = false;
    auto up = [&](HostSet& s, HostChunk& ch) -> int {
        const size_t nb = ch.nb, b0 = ch.b0;
        // per block: the parity planes its first k present shards reach, its erasure count
        uint32_t needers[32] = {};
        for (size_t b = 0; b < nb; ++b) {
            const uint32_t mask = masks[b0 + b] & all;
            s.h_masks[b] = mask;
            const uint32_t e = (uint32_t)k - (uint32_t)__builtin_popcount(mask & kmask);
            if (e == 0 || (uint32_t)__builtin_popcount(mask) < (uint32_t)k) continue;
            uint32_t need = e;   // parities among the first k present: the first e present ones
            for (int r = 0; r < m && need; ++r)
                if ((mask >> (k + r)) & 1u) {
                    --need;
                    ++needers[r];
                    ch.planes = std::max(ch.planes, (size_t)r + 1);
                }
            ch.slots = std::max(ch.slots, (size_t)e);
        }
        uint8_t* d_par = s.d_in + nb * k * ssd;   // parity planes [P][nb][ssd]
        HIP_TRY(hipMemcpyAsync(s.d_masks, s.h_masks, nb * 4, hipMemcpyHostToDevice, p.up));
        if (pinned) {
            if ((rc = pinned_up(p.up, s.d_in, (size_t)k * ssd, ssd, data + b0 * dbs, dbs, ss, nb, k, len, s.d_raw_in, k,
                                &ch.repack)))
                return rc;
            // the device reads sparse planes straight out of the caller's pinned buffer (needs a
            // device mapping of it; otherwise every plane goes by DMA)
            const uint8_t* dpar = nullptr;
            const bool mapped = ch.planes &&
                                hipHostGetDevicePointer((void**)&dpar, (void*)(parity + b0 * pbs), 0) == hipSuccess &&
                                dpar;
            if (ch.planes && !mapped) (void)hipGetLastError();
            for (size_t r = 0; r < ch.planes; ++r) {
                const bool sparse = needers[r] * 4 < nb * 3;
                if (mapped && sparse) {
                    ch.gather |= 1u << r;
                    continue;
                }
                HIP_TRY(hipMemcpy2DAsync(d_par + r * nb * ssd, ssd, parity + b0 * pbs + r * ss, pbs, len, nb,
                                         hipMemcpyHostToDevice, p.up));
            }
            return FEC_OK;
        }
        const size_t P = ch.planes;
        parallel_for(nb, [&](size_t lo, size_t hi) {
            for (size_t b = lo; b < hi; ++b) {
                const uint32_t mask = s.h_masks[b];
                if ((mask & kmask) == kmask) continue;   // nothing to rebuild: nothing read
                for (int j = 0; j < k; ++j)
                    if ((mask >> j) & 1u) memcpy(s.h_in + (b * k + j) * ssd, data + (b0 + b) * dbs + j * ss, len);
                for (size_t r = 0; r < P; ++r)
                    if ((mask >> (k + r)) & 1u)
                        memcpy(s.h_in + nb * k * ssd + (r * nb + b) * ssd, parity + (b0 + b) * pbs + r * ss, len);
            }
        });
        HIP_TRY(hipMemcpyAsync(s.d_in, s.h_in, (nb * k + P * nb) * ssd, hipMemcpyHostToDevice, p.up));
        return FEC_OK;
    };
    auto kern = [&](HostSet& s, HostChunk& ch) -> int {
        const size_t nb = ch.nb;
        uint8_t* d_par = s.d_in + nb * k * ssd;
        if (ch.repack)
            HIP_TRY(fk::launch_span_to_stage(s.d_in, (size_t)k * ssd, ssd, s.d_raw_in, dbs, ss, (uint32_t)nb,
                                             (uint32_t)k, (uint32_t)len, p.comp));
        if (ch.gather) {
            const uint8_t* dpar = nullptr;
            HIP_TRY(hipHostGetDevicePointer((void**)&dpar, (void*)(parity + ch.b0 * pbs), 0));
            HIP_TRY(fk::launch_gather_planes(dpar, pbs, ss, (uint32_t)len, s.d_masks, (uint32_t)nb, (uint32_t)ch.planes,
                                             ch.gather, (uint32_t)k, d_par, ssd, p.comp));
        }
        return on_pipe(ctx, [&] {
            return rs_reconstruct_device(ctx, code, len, nb, s.d_in, (size_t)k * ssd, d_par, ssd, ssd, s.d_masks,
                                         s.d_status, ctx->d_err + 1, s.d_out, ch.slots * ssd, (uint32_t)ch.slots,
                                         nb * ssd);
        });
    };
    auto down = [&](HostSet& s, HostChunk& ch) -> int {
        HIP_TRY(hipMemcpyAsync(s.h_out, s.d_out, ch.nb * ch.slots * ssd, hipMemcpyDeviceToHost, p.down));
        HIP_TRY(hipMemcpyAsync(s.h_status, s.d_status, ch.nb * 4, hipMemcpyDeviceToHost, p.down));
        return FEC_OK;
    };
    auto finish = [&](HostSet& s, HostChunk& ch) -> int {
        for (size_t b = 0; b < ch.nb; ++b) {
            const int32_t st = s.h_status[b];
            if (block_status) block_status[ch.b0 + b] = st < 0 ? st : 0;
            if (st < 0) failed = true;
        }
        parallel_for(ch.nb, [&](size_t lo, size_t hi) {
            for (size_t b = lo; b < hi; ++b) {
                const int32_t st = s.h_status[b];
                const uint32_t mask = s.h_masks[b];
                for (int j = 0, r = 0; j < k && r < st; ++j)
                    if (!((mask >> j) & 1u))
                        memcpy(data + (ch.b0 + b) * dbs + j * ss, s.h_out + (b * ch.slots + r++) * ssd, len);
            }
        });
        return FEC_OK;
    };
    if ((rc = host_pipeline(ctx, nblocks, chunk, up, kern, down, finish))) return rc;
    int err = 0;
    HIP_TRY(hipMemcpyAsync(&err, ctx->d_err + 1, sizeof(int), hipMemcpyDeviceToHost, p.comp));
    HIP_TRY(hipStreamSynchronize(p.comp));
    if (err & 4) return FEC_ERR_HIP;
    return failed ? FEC_ERR_TOO_FEW_SHARDS : FEC_OK;
}

// FEC_HOST XOR(k,1) reconstruct (the scheme mirror's per-block recovery): the present shards of
// each chunk as [block][k+1][ssd], rebuilt in place on the device, the data slots copied back.
static int host_reconstruct_xor(fec_ctx* ctx, int k, size_t len, size_t nblocks, uint8_t* data, size_t dbs,
                                const uint8_t* parity, size_t pbs, size_t ss, const uint32_t* masks,
                                int32_t* block_status) {
    const size_t ssd = round16(len);
    const size_t n = (size_t)k + 1;
    const uint32_t all = fk::low_mask((uint32_t)n), kmask = fk::low_mask((uint32_t)k);
    const size_t chunk = host_chunk_blocks(nblocks, n * ssd);
    int rc;
    if ((rc = grow_stage(ctx, chunk * n * ssd))) return rc;
    if ((rc = grow_masks(ctx, chunk))) return rc;
    HIP_TRY(hipMemsetAsync(ctx->d_err + 1, 0, sizeof(int), ctx->stream));
    std::vector<int32_t> st;
    for (size_t b0 = 0; b0 < nblocks; b0 += chunk) {
        const size_t nb = std::min(chunk, nblocks - b0);
        for (size_t b = 0; b < nb; ++b) {
            const uint32_t mask = masks[b0 + b] & all;
            if ((mask & kmask) == kmask) continue;
            for (size_t i = 0; i < n; ++i)
                if ((mask >> i) & 1u)
                    memcpy(ctx->h_stage + (b * n + i) * ssd,
                           i < (size_t)k ? data + (b0 + b) * dbs + i * ss : parity + (b0 + b) * pbs, len);
        }
        HIP_TRY(hipMemcpyAsync(ctx->d_masks, masks + b0, nb * 4, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->d_stage, ctx->h_stage, nb * n * ssd, hipMemcpyHostToDevice, ctx->stream));
        if ((rc = xor_reconstruct_device(ctx, k, len, nb, ctx->d_stage, n * ssd, ctx->d_stage + k * ssd, n * ssd, ssd,
                                         ctx->d_masks, ctx->d_status, ctx->d_err + 1)))
            return rc;
        st.resize(nb);
        HIP_TRY(hipMemcpyAsync(st.data(), ctx->d_status, nb * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->h_stage, ctx->d_stage, nb * n * ssd, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        for (size_t b = 0; b < nb; ++b) {
            if (block_status) block_status[b0 + b] = st[b];
            if (st[b] != 0) continue;
            const uint32_t mask = masks[b0 + b] & all;
            for (int i = 0; i < k; ++i)
                if (!((mask >> i) & 1u)) memcpy(data + (b0 + b) * dbs + i * ss, ctx->h_stage + (b * n + i) * ssd, len);
        }
    }
    int err = 0;
    HIP_TRY(hipMemcpy(&err, ctx->d_err + 1, sizeof(int), hipMemcpyDeviceToHost));
    return err ? FEC_ERR_TOO_FEW_SHARDS : FEC_OK;
}

// ---------------------------------------------------------------- C ABI

extern "C" {

const char* fec_version(void) { return "0xfec-mi355x 0.1.0 (gfx950)"; }

const char* fec_strerror(int code) {
    switch (code) {
        case FEC_OK: return "ok";
        case FEC_ERR_INVALID_ARG: return "invalid argument";
        case FEC_ERR_INV_SHARD_NUM: return "cannot create Encoder with less than one data shard or less than zero parity shards";
        case FEC_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
        case FEC_ERR_TOO_FEW_SHARDS: return "too few shards given";
        case FEC_ERR_SHARD_SIZE: return "shard sizes do not match";
        case FEC_ERR_SHARD_NO_DATA: return "no shard data";
        case FEC_ERR_ALIGNMENT: return "device shard layout must be 16-byte aligned";
        case FEC_ERR_HIP: return "HIP runtime error";
        case FEC_ERR_NOMEM: return "out of memory";
        case FEC_ERR_NO_DEVICE: return "no HIP device";
        case -21: return "EOF";   // FEC_ERR_EOF (fec_wire.h): io.EOF
        default: return "unknown error";
    }
}

int fec_device_count(int* count) {
    if (!count) return FEC_ERR_INVALID_ARG;
    *count = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return FEC_ERR_NO_DEVICE;
    }
    *count = n;
    return n > 0 ? FEC_OK : FEC_ERR_NO_DEVICE;
}

int fec_ctx_create(int device, fec_ctx** out) {
    if (!out) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return FEC_ERR_NO_DEVICE;
    }
    if (device < 0 || device >= n) return FEC_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(device));
    fec_ctx* ctx = new fec_ctx();
    ctx->device = device;
    if (hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&ctx->d_err, 2 * sizeof(int)) != hipSuccess ||
        hipMemset(ctx->d_err, 0, 2 * sizeof(int)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {   // null-stream memsets done before any ctx stream runs
        (void)hipGetLastError();
        fec_ctx_destroy(ctx);
        return FEC_ERR_HIP;
    }
    ctx->stream = ctx->own;
    {   // LDS a workgroup may use (160 KiB on gfx950): bounds the wave-form rebuild's slices
        int lds = 0;
        if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && lds > 0)
            fk::g_max_lds = (size_t)lds;
    }
    *out = ctx;
    return FEC_OK;
}

void fec_ctx_destroy(fec_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->codes) {
        if (kv.second.d_prows) (void)hipFree(kv.second.d_prows);
        if (kv.second.d_tabs) (void)hipFree(kv.second.d_tabs);
        if (kv.second.d_dytabs) (void)hipFree(kv.second.d_dytabs);
        if (kv.second.d_single) (void)hipFree(kv.second.d_single);
        if (kv.second.d_single_coef) (void)hipFree(kv.second.d_single_coef);
        if (kv.second.d_dall) (void)hipFree(kv.second.d_dall);
    }
    if (ctx->own) (void)hipStreamSynchronize(ctx->own);
    if (ctx->stream && ctx->stream != ctx->own) (void)hipStreamSynchronize(ctx->stream);
    ctx->main.release();
    if (ctx->d_err) (void)hipFree(ctx->d_err);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    if (ctx->d_masks) (void)hipFree(ctx->d_masks);
    if (ctx->d_status) (void)hipFree(ctx->d_status);
    HostPipe& p = ctx->pipe;
    for (hipStream_t q : {p.up, p.comp, p.down})
        if (q) (void)hipStreamSynchronize(q);
    for (HostSet& s : p.set) {
        for (void* q : {(void*)s.h_in, (void*)s.h_out, (void*)s.h_masks, (void*)s.h_status})
            if (q) (void)hipHostFree(q);
        for (void* q : {(void*)s.d_in, (void*)s.d_out, (void*)s.d_masks, (void*)s.d_status, (void*)s.d_raw_in,
                        (void*)s.d_raw_out})
            if (q) (void)hipFree(q);
        for (hipEvent_t e : {s.up_done, s.k_done, s.down_done})
            if (e) (void)hipEventDestroy(e);
    }
    p.w.release();
    for (hipStream_t q : {p.up, p.comp, p.down})
        if (q) (void)hipStreamDestroy(q);
    if (ctx->handoff) (void)hipEventDestroy(ctx->handoff);
    if (ctx->own) (void)hipStreamDestroy(ctx->own);
    (void)hipGetLastError();
    delete ctx;
}

// Switch the ctx to `next`. The ctx's own / caller's stream share one workspace (`main`: plan
// records), so work already queued on the old
// stream must finish before anything on the new one touches it: the new stream waits on an
// event recorded on the old one (no host wait). grow_* then sync only the current stream,
// which by this wait covers the old one's kernels too.
static int switch_stream(fec_ctx* ctx, hipStream_t next) {
    if (next == ctx->stream) return FEC_OK;
    int rc = select_device(ctx);
    if (rc) return rc;
    if (!ctx->handoff) HIP_TRY(hipEventCreateWithFlags(&ctx->handoff, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ctx->handoff, ctx->stream));
    HIP_TRY(hipStreamWaitEvent(next, ctx->handoff, 0));
    ctx->stream = next;
    return FEC_OK;
}

int fec_ctx_release_staging(fec_ctx* ctx) {
    int rc = select_device(ctx);
    if (rc) return rc;
    HostPipe& p = ctx->pipe;
    for (hipStream_t q : {p.up, p.comp, p.down})
        if (q) HIP_TRY(hipStreamSynchronize(q));
    if (ctx->stream) HIP_TRY(hipStreamSynchronize(ctx->stream));
    // Every buffer is freed and forgotten even when a free fails (the first failure is returned),
    // so the ctx never keeps a pointer it has handed back.
    hipError_t first = hipSuccess;
    auto drop = [&first](hipError_t e) {
        if (e != hipSuccess && first == hipSuccess) first = e;
    };
    for (HostSet& s : p.set) {
        for (void* q : {(void*)s.h_in, (void*)s.h_out, (void*)s.h_masks, (void*)s.h_status})
            if (q) drop(hipHostFree(q));
        for (void* q : {(void*)s.d_in, (void*)s.d_out, (void*)s.d_masks, (void*)s.d_status, (void*)s.d_raw_in,
                        (void*)s.d_raw_out})
            if (q) drop(hipFree(q));
        s.h_in = s.h_out = s.d_in = s.d_out = s.d_raw_in = s.d_raw_out = nullptr;
        s.h_masks = s.d_masks = nullptr;
        s.h_status = s.d_status = nullptr;
        s.in_cap = s.out_cap = s.blk_cap = s.raw_in_cap = s.raw_out_cap = 0;
    }
    if (ctx->h_stage) drop(hipHostFree(ctx->h_stage));
    if (ctx->d_stage) drop(hipFree(ctx->d_stage));
    ctx->h_stage = ctx->d_stage = nullptr;
    ctx->stage_cap = 0;
    if (first != hipSuccess) {
        (void)hipGetLastError();
        return FEC_ERR_HIP;
    }
    return FEC_OK;
}

int fec_ctx_set_stream(fec_ctx* ctx, void* hip_stream) {
    if (!ctx) return FEC_ERR_INVALID_ARG;
    return switch_stream(ctx, (hipStream_t)hip_stream);
}

// Internal, test-only tuning entry point (not part of the public ABI): knob `key` of fk::Tuning
// (fec_kernels.hpp, keys 0..kTuningKeys-1 in declaration order) set to `value`, process-wide, for
// every ctx. Tests and tools set knobs while no other thread submits work. Returns the previous
// value, or FEC_ERR_INVALID_ARG for an unknown key.
int fec__set_tuning(fec_ctx* ctx, int key, int value) {
    if (!ctx) return FEC_ERR_INVALID_ARG;
    fk::Tuning& t = fk::g_tune;
    std::atomic<int>* slots[fk::kTuningKeys] = {&t.enc_wpc,   &t.gen_wpc,    &t.dec_wpc,      &t.dir_wpc,
                                                &t.enc_bwpc,  &t.enc_fixed,  &t.dec_wave,     &t.dec_direct,
                                                &t.host_chunk, &t.host_threads, &t.bat_zc,     &t.dec_route,
                                                &t.st_pol,     &t.dst_pol,    &t.route_wpc,
                                                &t.route_ww,   &t.xor_wpc,
                                                &t.enc_ww};
    if (key < 0 || key >= fk::kTuningKeys) return FEC_ERR_INVALID_ARG;
    return slots[key]->exchange(value);
}

// Internal self-test (not part of the public ABI, no device needed): parallel_for covers [0, n)
// exactly once, for sizes around the part boundaries and part counts 2..16, with four threads
// calling at once (one holds the persistent copy workers, the others find them busy and make
// their own threads). 0 on success, else the failing case.
extern "C" int fec__selftest_copypool(void) {
    const int saved = fk::g_tune.host_threads;
    int fail = 0;
    const size_t sizes[] = {511, 512, 513, 1000, 4097, 65536, 100003};
    for (int T : {2, 3, 8, 16}) {
        fk::g_tune.host_threads = T;
        std::vector<std::thread> callers;
        std::vector<int> bad(4, 0);
        for (int t = 0; t < 4; ++t)
            callers.emplace_back([&, t] {
                for (size_t n : sizes) {
                    std::unique_ptr<std::atomic<uint32_t>[]> hits(new std::atomic<uint32_t>[n]);
                    for (size_t i = 0; i < n; ++i) hits[i].store(0);
                    parallel_for(n, [&](size_t lo, size_t hi) {
                        for (size_t i = lo; i < hi; ++i) hits[i].fetch_add(1);
                    });
                    for (size_t i = 0; i < n; ++i)
                        if (hits[i].load() != 1) bad[t] = 1;
                }
            });
        for (auto& th : callers) th.join();
        for (int b : bad)
            if (b) fail = 100 + T;
        if (fail) break;
    }
    fk::g_tune.host_threads = saved;
    return fail;
}

// Internal self-test (not part of the public ABI, no device needed): the lane-arithmetic PermTab
// builder the kernels use equals the byte-wise one for every coefficient. 0 on success, else
// 1 + the first failing coefficient.
int fec__selftest_permtab(void) {
    for (uint32_t c = 0; c < 256; ++c) {
        const gf::PermTab a = gf::make_permtab((uint8_t)c), b = gf::make_permtab_fast(c);
        if (a.t0lo != b.t0lo || a.t0hi != b.t0hi || a.t1lo != b.t1lo || a.t1hi != b.t1hi || a.t2 != b.t2)
            return 1 + (int)c;
    }
    return 0;
}

int fec_ctx_reset_stream(fec_ctx* ctx) {
    if (!ctx) return FEC_ERR_INVALID_ARG;
    return switch_stream(ctx, ctx->own);
}

void* fec_ctx_stream(fec_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int fec_sync(fec_ctx* ctx) {
    int rc = select_device(ctx);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    int err = 0;
    HIP_TRY(hipMemcpy(&err, ctx->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (err) {
        HIP_TRY(hipMemsetAsync(ctx->d_err, 0, sizeof(int), ctx->stream));
        // 1: a block with too few shards; 2: more erasures than output slots; 4: internal (the
        // form-3 plan kernel's LDS-alignment guard)
        return (err & 1) ? FEC_ERR_TOO_FEW_SHARDS : (err & 4) ? FEC_ERR_HIP : FEC_ERR_INVALID_ARG;
    }
    return FEC_OK;
}

int fec_rs_matrix(int k, int m, uint8_t* out) {
    if (!out) return FEC_ERR_INVALID_ARG;
    if (k <= 0 || m < 0) return FEC_ERR_INV_SHARD_NUM;
    if (k + m > 256) return FEC_ERR_MAX_SHARD_NUM;
    std::vector<uint8_t> mat = rs::build_matrix(k, k + m);
    if (mat.empty()) return FEC_ERR_INV_SHARD_NUM;
    memcpy(out, mat.data(), mat.size());
    return FEC_OK;
}

int fec_rs_prepare(fec_ctx* ctx, int k, int m) {
    int rc = select_device(ctx);
    if (rc) return rc;
    Code* code = nullptr;
    return get_code(ctx, k, m, &code);
}

int fec_rs_encode_batch(fec_ctx* ctx, int k, int m, size_t shard_len, size_t nblocks, const uint8_t* data,
                        size_t data_block_stride, uint8_t* parity, size_t parity_block_stride,
                        size_t shard_stride, int flags) {
    if (k <= 0 || m < 0) return FEC_ERR_INV_SHARD_NUM;
    if (k + m > 256) return FEC_ERR_MAX_SHARD_NUM;
    if (flags != FEC_DEVICE && flags != FEC_HOST && flags != FEC_HOST_PINNED) return FEC_ERR_INVALID_ARG;
    if (shard_len == 0) return FEC_ERR_SHARD_NO_DATA;
    if (shard_len > (size_t(1) << 30)) return FEC_ERR_INVALID_ARG;
    int rc = select_device(ctx);
    if (rc) return rc;
    Code* code = nullptr;
    if ((rc = get_code(ctx, k, m, &code))) return rc;
    if (nblocks == 0 || m == 0) return FEC_OK;
    if (!data || !parity) return FEC_ERR_INVALID_ARG;
    if (flags == FEC_DEVICE) {
        if ((rc = check_device_layout(data, data_block_stride, shard_stride, shard_len))) return rc;
        if ((rc = check_device_layout(parity, parity_block_stride, shard_stride, shard_len))) return rc;
        return rs_encode_device(ctx, code, shard_len, nblocks, data, data_block_stride, parity,
                                parity_block_stride, shard_stride);
    }
    return host_encode(ctx, code, k, m, shard_len, nblocks, data, data_block_stride, parity, parity_block_stride,
                       shard_stride, flags == FEC_HOST_PINNED);
}

int fec_rs_reconstruct_batch(fec_ctx* ctx, int k, int m, size_t shard_len, size_t nblocks, uint8_t* data,
                             size_t data_block_stride, const uint8_t* parity, size_t parity_block_stride,
                             size_t shard_stride, const uint32_t* present_mask, int32_t* block_status, int flags) {
    if (k <= 0 || m < 0) return FEC_ERR_INV_SHARD_NUM;
    if (k + m > FEC_MAX_DECODE_SHARDS) return FEC_ERR_MAX_SHARD_NUM;
    if (flags != FEC_DEVICE && flags != FEC_HOST && flags != FEC_HOST_PINNED) return FEC_ERR_INVALID_ARG;
    if (shard_len == 0) return FEC_ERR_SHARD_NO_DATA;
    if (shard_len > (size_t(1) << 30)) return FEC_ERR_INVALID_ARG;
    int rc = select_device(ctx);
    if (rc) return rc;
    Code* code = nullptr;
    if ((rc = get_code(ctx, k, m, &code))) return rc;
    if (nblocks == 0) return FEC_OK;
    if (!data || !present_mask || (m > 0 && !parity)) return FEC_ERR_INVALID_ARG;
    if (m == 0) parity = data;   // never read: no parity slot exists
    if (flags == FEC_DEVICE) {
        if ((rc = check_device_layout(data, data_block_stride, shard_stride, shard_len))) return rc;
        if ((rc = check_device_layout(parity, parity_block_stride, shard_stride, shard_len))) return rc;
        if ((rc = check_device_words(present_mask, block_status))) return rc;
        return rs_reconstruct_device(ctx, code, shard_len, nblocks, data, data_block_stride, parity,
                                     parity_block_stride, shard_stride, present_mask, block_status, ctx->d_err);
    }
    return host_reconstruct_rs(ctx, code, k, m, shard_len, nblocks, data, data_block_stride, parity,
                               parity_block_stride, shard_stride, present_mask, block_status, flags == FEC_HOST_PINNED);
}

int fec_rs_recover_batch(fec_ctx* ctx, int k, int m, size_t shard_len, size_t nblocks, const uint8_t* data,
                         size_t data_block_stride, const uint8_t* parity, size_t parity_block_stride,
                         size_t shard_stride, const uint32_t* present_mask, uint8_t* out, size_t out_block_stride,
                         int out_slots, int32_t* block_status, int flags) {
    if (k <= 0 || m < 0) return FEC_ERR_INV_SHARD_NUM;
    if (k + m > FEC_MAX_DECODE_SHARDS) return FEC_ERR_MAX_SHARD_NUM;
    if (flags != FEC_DEVICE) return FEC_ERR_INVALID_ARG;
    if (shard_len == 0) return FEC_ERR_SHARD_NO_DATA;
    if (shard_len > (size_t(1) << 30) || out_slots <= 0) return FEC_ERR_INVALID_ARG;
    int rc = select_device(ctx);
    if (rc) return rc;
    Code* code = nullptr;
    if ((rc = get_code(ctx, k, m, &code))) return rc;
    if (nblocks == 0) return FEC_OK;
    if (!data || !present_mask || !out || (m > 0 && !parity)) return FEC_ERR_INVALID_ARG;
    if (m == 0) parity = data;
    if ((rc = check_device_layout(data, data_block_stride, shard_stride, shard_len))) return rc;
    if ((rc = check_device_layout(parity, parity_block_stride, shard_stride, shard_len))) return rc;
    if ((rc = check_device_layout(out, out_block_stride, shard_stride, shard_len))) return rc;
    if ((rc = check_device_words(present_mask, block_status))) return rc;
    return rs_reconstruct_device(ctx, code, shard_len, nblocks, const_cast<uint8_t*>(data), data_block_stride,
                                 parity, parity_block_stride, shard_stride, present_mask, block_status, ctx->d_err,
                                 out, out_block_stride, (uint32_t)out_slots);
}

int fec_xor_encode_batch(fec_ctx* ctx, int k, size_t shard_len, size_t nblocks, const uint8_t* data,
                         size_t data_block_stride, uint8_t* parity, size_t parity_block_stride, size_t shard_stride,
                         int flags) {
    if (k <= 0) return FEC_ERR_INV_SHARD_NUM;
    if (k + 1 > 256) return FEC_ERR_MAX_SHARD_NUM;
    if (flags != FEC_DEVICE && flags != FEC_HOST && flags != FEC_HOST_PINNED) return FEC_ERR_INVALID_ARG;
    if (shard_len == 0) return FEC_ERR_SHARD_NO_DATA;
    if (shard_len > (size_t(1) << 30)) return FEC_ERR_INVALID_ARG;
    int rc = select_device(ctx);
    if (rc) return rc;
    if (nblocks == 0) return FEC_OK;
    if (!data || !parity) return FEC_ERR_INVALID_ARG;
    if (flags == FEC_DEVICE) {
        if ((rc = check_device_layout(data, data_block_stride, shard_stride, shard_len))) return rc;
        if ((rc = check_device_layout(parity, parity_block_stride, shard_stride, shard_len))) return rc;
        return xor_encode_device(ctx, k, shard_len, nblocks, data, data_block_stride, parity, parity_block_stride,
                                 shard_stride);
    }
    return host_encode(ctx, nullptr, k, 1, shard_len, nblocks, data, data_block_stride, parity, parity_block_stride,
                       shard_stride, flags == FEC_HOST_PINNED);
}

int fec_xor_reconstruct_batch(fec_ctx* ctx, int k, size_t shard_len, size_t nblocks, uint8_t* data,
                              size_t data_block_stride, const uint8_t* parity, size_t parity_block_stride,
                              size_t shard_stride, const uint32_t* present_mask, int32_t* block_status, int flags) {
    if (k <= 0) return FEC_ERR_INV_SHARD_NUM;
    if (k + 1 > FEC_MAX_DECODE_SHARDS) return FEC_ERR_MAX_SHARD_NUM;
    if (flags != FEC_DEVICE && flags != FEC_HOST && flags != FEC_HOST_PINNED) return FEC_ERR_INVALID_ARG;
    if (shard_len == 0) return FEC_ERR_SHARD_NO_DATA;
    if (shard_len > (size_t(1) << 30)) return FEC_ERR_INVALID_ARG;
    int rc = select_device(ctx);
    if (rc) return rc;
    if (nblocks == 0) return FEC_OK;
    if (!data || !parity || !present_mask) return FEC_ERR_INVALID_ARG;
    if (flags == FEC_DEVICE) {
        if ((rc = check_device_layout(data, data_block_stride, shard_stride, shard_len))) return rc;
        if ((rc = check_device_layout(parity, parity_block_stride, shard_stride, shard_len))) return rc;
        if ((rc = check_device_words(present_mask, block_status))) return rc;
        return xor_reconstruct_device(ctx, k, shard_len, nblocks, data, data_block_stride, parity,
                                      parity_block_stride, shard_stride, present_mask, block_status, ctx->d_err);
    }
    return host_reconstruct_xor(ctx, k, shard_len, nblocks, data, data_block_stride, parity, parity_block_stride,
                                shard_stride, present_mask, block_status);
}

}  // extern "C"
