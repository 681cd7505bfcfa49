// fec_kernels.hpp — host-side launch interface of the gfx950 FEC kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>

namespace fk {

constexpr int kThreads = 256;       // 4 waves of 64
constexpr int kInGroup = 8;         // input shards loaded back to back per lane
constexpr int kChunk = 16;          // bytes per lane per shard (global_load_dwordx4)
constexpr int kMaxLdsTabs = 2048;   // uniform (encode) tables kept in LDS: 64 KiB

// q = n / d for 32-bit n via a multiply-high (d fixed per launch).
struct FastDiv {
    uint32_t d, magic, shift;
};
FastDiv make_fastdiv(uint32_t d);

// Flat launches (encode, XOR): item = one 16-byte column chunk of one block,
// item -> (block = item / cps, chunk = item % cps).
struct EncodeArgs {
    const uint8_t* in;   // data shard 0 of block 0
    uint8_t* out;        // parity shard 0 of block 0
    uint64_t in_bs, out_bs, ss;
    uint32_t k, m, len, cps;   // cps = chunks per shard = ceil(len / 16)
    uint32_t total;            // nblocks * cps (< 2^31 per launch)
    FastDiv div_cps;
    const uint32_t* tabs;      // m * k PermTabs (8 dwords each), device memory
    const uint32_t* dytabs;    // dyadic codes (nullable): leaf PermTabs of the split-recursive
                               // form (fec_capi.cpp dyadic_leaves), padded to m * k entries
    uint32_t sp;               // store policy of the fixed-shape encodes (fec_device.hpp st16p): 1 sc1
                               // where the parity region is apart from the data region, else 0 nt
};

// The encodes' store policy for a call (knob st_pol): sc1 stores let parity lines leave the XCD's L2
// (-1.4 to -2.1 % RS(8,12) encode time on split buffers), but into parity slots interleaved with the
// data being read ([B][k+m][S]) they cost 26 % (the XOR layout's twin, r06h): so sc1 only when the
// [lo, hi) ranges of the two regions do not meet.
inline bool regions_apart(const void* a, uint64_t abs, const void* b, uint64_t bbs, uint64_t nblocks) {
    const uintptr_t a0 = (uintptr_t)a, a1 = a0 + abs * nblocks, b0 = (uintptr_t)b, b1 = b0 + bbs * nblocks;
    return b1 <= a0 || a1 <= b0;
}
inline uint32_t encode_store_policy(int st_pol, const void* data, uint64_t dbs, const void* parity, uint64_t pbs,
                                    uint64_t nblocks) {
    // (st_pol 2: sc1 whatever the layout, measurement only)
    return st_pol == 2 || (st_pol == 1 && nblocks && regions_apart(data, dbs, parity, pbs, nblocks)) ? 1u : 0u;
}
// The RS(8,12) direct decode's (knob dst_pol): nt sc1 only into an output region apart from the
// shards it reads (recover calls), else nt (in place: the rebuilt shard lands among the data).
inline uint32_t decode_store_policy(int dst_pol, const void* data, uint64_t dbs, const void* parity, uint64_t pbs,
                                    const void* out, uint64_t obs, uint64_t nblocks) {
    return dst_pol == 3 && out && nblocks && regions_apart(data, dbs, out, obs, nblocks) &&
                   regions_apart(parity, pbs, out, obs, nblocks)
               ? 3u
               : 0u;
}

// Bits [0, n) set, for n in [0, 32] (a present mask over n shards; 1u << 32 is undefined).
__host__ __device__ inline uint32_t low_mask(uint32_t n) { return n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u); }

// Decode plan, one record of `stride` bytes per block (offsets from plan_layout()):
//   [in_off,   +rup8(k))  input shard slots = the first k present shards, in index order
//   [out_off,  +maxe)     erased data shard slots (ascending)
//   [nout_off]            number of erased data shards to rebuild (0: nothing / failed)
//   [coef_off, +maxe*k)   GF coefficients, row r = output r, column j = input j
//   [blk_off,  +4)        sorted plans only: the block the record belongs to (uint32)
struct PlanLayout {
    uint32_t in_off, out_off, nout_off, coef_off, stride;
    uint32_t blk_off;          // 0: records are in block order (no block field)
};
PlanLayout plan_layout(uint32_t k, uint32_t maxe, bool sorted = false);

struct PlanArgs {
    const uint32_t* masks;
    uint8_t* plans;            // nblocks * lay.stride bytes
    int32_t* status;           // optional
    int* err;                  // sticky error word
    const uint8_t* prows;      // m x k parity rows of the systematic matrix
    uint32_t k, m, nblocks, maxe;
    PlanLayout lay;
    uint32_t max_out;          // recover: output slots per block (0: in place, unlimited)
    const uint8_t* dall;       // sorted plans: per shard index s < n, sum_{t < n, t != s} log(s ^ t) mod 255
    // routed in-place form (fec_recover.hip): the classify pass's word; zero (no block needs more than
    // the direct body) makes the plan kernel exit at once (null: always plan)
    const uint32_t* route;
};

// Sorted plans (fec_plan.hip): lanes per block and blocks per 256-thread workgroup for k.
inline uint32_t plan_lanes(uint32_t k) {
    uint32_t l = 2;
    while (l < k) l <<= 1;
    return l;
}

struct ReconArgs {
    uint8_t* data;             // data shard 0 of block 0 (rebuilt shards are written here)
    const uint8_t* parity;     // parity shard 0 of block 0
    uint64_t dbs, pbs, ss;
    uint64_t pss;              // parity shard stride (parity i of block b at parity + b*pbs + i*pss; = ss
                               // in the ABI's layouts, parity-major in the host path's staging)
    const uint8_t* plans;
    uint32_t k, len, cps, nblocks, maxe;
    PlanLayout lay;
    uint32_t g;                // blocks per tile
    uint32_t ntiles;
    FastDiv div_cps;
    uint8_t* out;              // recover: rebuilt shard r of block b at out + b*out_bs + r*ss
    uint64_t out_bs;           //          (nullptr: rebuild in place into the data region)
    uint32_t sorted;           // plans from rs_plan_sorted_kernel: the block of a record is its blk field
    // direct form (plans built in the kernel, no plan kernel): as PlanArgs
    const uint32_t* masks;
    int32_t* status;
    int* err;
    const uint8_t* prows;
    uint32_t m, max_out;
    // direct form (rs_recover_direct_kernel): single-erasure coefficient tables, k*m*k PermTabs,
    // entry ((E0*m + R0)*k + j) = coefficient of input j (data shards != E0 in order, then
    // parity R0) when data shard E0 is the only erasure and R0 the first present parity
    const uint32_t* single;
    const uint32_t* single_coef;   // the same plans' coefficient bytes: (k*m) rows of ceil(k/4) dwords
    const uint32_t* single_coef_host;   // host copy of single_coef (passed as a kernel argument when small)
    // routed in-place form (fec_recover.hip rs_reconstruct_routed_kernel): the classify pass's word,
    // zero when no recoverable block has two or more erased data shards (the direct body runs), else
    // nonzero (the wave rebuild of the sorted plans runs)
    const uint32_t* route;
    uint32_t sp;               // store policy of the RS(8,12) direct decode (decode_store_policy)
};


struct XorArgs {
    const uint8_t* in;         // data shard 0 of block 0
    uint8_t* out;              // encode: parity shard 0; reconstruct: == in (rebuilt in place)
    const uint8_t* parity;     // reconstruct: parity shard of block 0
    uint64_t in_bs, out_bs, ss;
    uint64_t par_bs;           // reconstruct: parity block stride
    const uint32_t* masks;     // reconstruct only
    int32_t* status;           // reconstruct only, optional
    int* err;
    uint32_t k, len, cps, total;
    uint32_t nblocks;          // reconstruct: blocks in this launch (total / cps)
    FastDiv div_cps;
};

// Tuning knobs: residency of the shipped kernels, routing among shipped kernels (so the tests can
// run each one on shapes it does not serve by default), and host-path sizes. Every knob's default
// is the measured best; no knob selects a kernel form that is not shipped. Set only through the
// internal, test-only fec__set_tuning() (fec_capi.cpp): process-wide, read without locks by every
// ctx's launches (the fields are atomic, so a concurrent write is not a data race, but the tests
// and tools set knobs only while no other thread submits work).
struct Tuning {
    // resident workgroups per CU (dynamic-LDS caps, occupancy_lds; 0 = as many as fit)
    std::atomic<int> enc_wpc{3};    // RS(8,12) fixed-shape encode (2 / 4 / uncapped slower)
    std::atomic<int> gen_wpc{0};    // generic RS encode and the RS(2,3) encode
    std::atomic<int> dec_wpc{0};    // plan-path rebuilds
    std::atomic<int> dir_wpc{-1};   // direct single-erasure decode; -1: by shape (k >= 8: 3, else 0)
    std::atomic<int> enc_bwpc{0};   // bit-sliced encode (RS(16,24), RS(20,30))
    // routing among shipped kernels (tests)
    std::atomic<int> enc_fixed{1};  // 0: every shape by the generic encode
    std::atomic<int> dec_wave{1};   // 0: the workgroup-tile rebuild for long shards too
    std::atomic<int> dec_direct{1}; // 0: no direct decode (plan path for every code); 1: direct where it
                                    // applies (one output slot, or m = 1), rows from the kernel
                                    // argument where the coefficient words fit it (RS(2,3): its own
                                    // kernel); 2: rows always copied from the PermTab table
    // host paths
    std::atomic<int> host_chunk{0};     // FEC_HOST / FEC_HOST_PINNED: blocks per staging chunk (0: 128 MiB worth)
    std::atomic<int> host_threads{8};   // FEC_HOST (pageable): copy workers for the staging / scatter copies
    std::atomic<int> bat_zc{4 << 20};   // batch encoder / decoder (fec_batch.cpp): sets of at most this many
                                        // input bytes are coded straight from / into their pinned buffers
    // in-place reconstructs of RS(8,12): routed by a classify pass between the direct body and the
    // sorted plans (fec_recover.hip); 0: the sorted-plan route for every batch
    std::atomic<int> dec_route{1};
    // store cache policy of the fixed-shape encodes (st_pol: 1 sc1, 0 nt: RS(2,3), RS(8,12), RS(16,24),
    // RS(20,30)) and of the RS(8,12) direct decode (dst_pol: 3 nt sc1, 0 nt) (fec_device.hpp st16p),
    // and of their traffic twins
    std::atomic<int> st_pol{1};
    std::atomic<int> dst_pol{3};
    // resident workgroups per CU of the routed in-place kernel (0: as many as fit)
    std::atomic<int> route_wpc{4};
    // waves per workgroup that run the routed kernel's direct body (3: the fourth wave of each
    // workgroup exits at once, so the direct route runs 12 of the 16 resident waves per CU, the
    // direct body's best residency, while the plan route keeps 16; 4: all)
    std::atomic<int> route_ww{3};
    std::atomic<int> xor_wpc{6};    // XOR encode and reconstruct (fec_xor.hip)
    // waves per workgroup that take items in the RS(8,12) encode (3: the fourth stages its table
    // words and exits, 9 working waves per CU at 3 workgroups/CU, shard loads before the barrier; 4: all)
    std::atomic<int> enc_ww{3};
};
constexpr int kTuningKeys = 18;   // fec__set_tuning keys 0..17, in the order above

// Dynamic LDS that caps residency at `wpc` workgroups per CU (160 KiB of LDS per CU on gfx950):
// halfway between 160K/(wpc+1) and 160K/wpc, never below what the kernel itself needs.

inline size_t occupancy_lds(int wpc, size_t own) {
    if (wpc <= 0) return own;
    const size_t cu = 160u * 1024u;
    size_t pad = (cu / (size_t)wpc + cu / (size_t)(wpc + 1)) / 2;
    pad &= ~(size_t)255;
    return own > pad ? own : pad;
}

extern Tuning g_tune;
extern size_t g_max_lds;   // LDS per workgroup the device allows (set at ctx creation)

hipError_t launch_rs_encode(const EncodeArgs& a, int grid, hipStream_t s);
// Encodes compiled for one code (flat grid): RS(2,3), RS(8,12) (dyadic: leaf tables given),
// RS(16,24), RS(20,30).
bool fixed_encode_applies(uint32_t k, uint32_t m, bool dyadic);
hipError_t launch_rs_encode_fixed(const EncodeArgs& a, hipStream_t s);
bool rs_encode23_applies(uint32_t k, uint32_t m);            // fec_encode23.hip
hipError_t launch_rs_encode23(const EncodeArgs& a, hipStream_t s);
hipError_t launch_rs_plan(const PlanArgs& a, hipStream_t s);
// Sorted plans (fec_plan.hip): lanes of a wave cooperate on one block's plan; within each
// workgroup's segment of blocks the records are stored ordered by erasure count, each naming
// its block (layout from plan_layout(k, maxe, true)), so a rebuild wave meets blocks of equal
// row counts.
hipError_t launch_rs_plan_sorted(const PlanArgs& a, hipStream_t s);
hipError_t launch_rs_reconstruct(const ReconArgs& a, int grid, hipStream_t s);
bool wave_recon_applies(uint32_t cps, uint32_t k, uint32_t maxe, uint32_t stride);
hipError_t launch_rs_reconstruct_wave(const ReconArgs& a, hipStream_t s);
// Compile-time-k rebuild of RS(16,24) / RS(20,30) with table-copied PermTab rows and per-block input
// offsets (fec_rebuild.hip), for the wave form's shapes with shards of 64+ chunks.
bool rebuild_k_applies(uint32_t k, uint32_t maxe, uint32_t cps);
hipError_t launch_rs_rebuild_k(const ReconArgs& a, hipStream_t s);
// Direct form (fec_recover.hip): applies when the single-erasure tables of (k, m) fit in LDS.
bool direct_recon_applies(uint32_t k, uint32_t m, uint32_t cps, bool single_slot);
// The routed in-place form (fec_recover.hip): RS(8,12)-shaped codes in place, classify pass ->
// route word -> sorted plans (skipped on a zero word) -> one routed kernel (the direct body on a
// zero word, the wave rebuild otherwise).
bool routed_recon_applies(uint32_t k, uint32_t m, uint32_t cps, uint32_t maxe, uint32_t stride);
hipError_t launch_rs_route_classify(const ReconArgs& a, uint32_t* route, hipStream_t s);
hipError_t launch_rs_reconstruct_routed(const ReconArgs& a, hipStream_t s);
size_t direct_table_words(uint32_t k, uint32_t m);
hipError_t launch_rs_recover_direct(const ReconArgs& a, hipStream_t s);
hipError_t launch_xor_encode(const XorArgs& a, int grid, hipStream_t s);
hipError_t launch_xor_reconstruct(const XorArgs& a, int grid, hipStream_t s);

// Host-resident path layout conversion (fec_pack.hip): caller's span -> 16-byte stage slots, and
// stage slots -> packed [nb][cols][len] image (written rounded up to 4 bytes).
hipError_t launch_span_to_stage(uint8_t* stage, uint64_t st_bs, uint64_t st_ss, const uint8_t* span, uint64_t src_bs,
                                uint64_t src_ss, uint32_t nb, uint32_t cols, uint32_t len, hipStream_t s);
hipError_t launch_stage_to_packed(uint8_t* packed, const uint8_t* stage, uint64_t st_bs, uint64_t st_ss, uint32_t nb,
                                  uint32_t cols, uint32_t len, hipStream_t s);

// Device-side gathers out of pinned, device-mapped host memory (fec_pack.hip). A descriptor
// names one payload or framed shard: `len` bytes at `src` (a device-visible address), and
// `frame` = the block's biggest payload length, at which BE16(len) is written
// (reed_solomon.go:77-87), or kNoFrame for bytes copied verbatim. Shard i is written to
// dst + i * slot, all slot bytes (zeros past the content).
constexpr uint32_t kNoFrame = 0xFFFFFFFFu;
struct GatherDesc {
    uint64_t src;
    uint32_t len;
    uint32_t frame;
};
hipError_t launch_gather_desc(const GatherDesc* desc, uint32_t n, uint8_t* dst, uint64_t slot, hipStream_t s);
// The parity planes r < planes with bit r of plane_bits set, of nb blocks (block b, plane r at
// base + b*bs + r*ss), that each block's present mask makes it read, to dst + (r*nb + b)*slot; the
// others are skipped.
hipError_t launch_gather_planes(const uint8_t* base, uint64_t bs, uint64_t ss, uint32_t len, const uint32_t* masks,
                                uint32_t nb, uint32_t planes, uint32_t plane_bits, uint32_t k, uint8_t* dst,
                                uint64_t slot, hipStream_t s);

// Blocks per decode tile for shard chunk count `cps`, bounded by LDS.
uint32_t pick_tile_blocks(uint32_t cps, uint32_t k, uint32_t maxe, const PlanLayout& lay);
size_t recon_lds_bytes(uint32_t g, uint32_t k, uint32_t maxe, const PlanLayout& lay);

}  // namespace fk
