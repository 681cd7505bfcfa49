// fec_kernels.hpp — host-side launch interface of the gfx950 FEC kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

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
    uint32_t pad_zero;         // tail chunk: full 16-B store, bytes past len zeroed
    uint32_t rot;              // chunk rotation inside a block (line_rotation())
    uint32_t swz;              // XCD-contiguous workgroup order (xcd_order())
    uint32_t* ctr;             // queue kernel: 8 ticket counters kCtrStride words apart, then the
                               // arrival counter; all zero at launch, rewound by the last workgroup
    uint32_t per_xcd;          // queue kernel: items per XCD range
    const uint32_t* dytabs;    // dyadic codes (nullable): leaf PermTabs of the split-recursive
                               // form, dyadic_leaf_tables(), padded to m * k entries
};

// Bits [0, n) set, for n in [0, 32] (a present mask over n shards; 1u << 32 is undefined).
__host__ __device__ inline uint32_t low_mask(uint32_t n) { return n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u); }

constexpr int kCtrStride = 32;      // one 128-byte line per ticket counter
constexpr int kCtrWords = 9 * kCtrStride;

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
    const uint32_t* gate;      // nullable: run only when gate[0] == gate_want
    uint32_t gate_want;
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
    uint32_t pad_zero;
    uint32_t rot;
    uint8_t* out;              // recover: rebuilt shard r of block b at out + b*out_bs + r*ss
    uint64_t out_bs;           //          (nullptr: rebuild in place into the data region)
    uint32_t swz;
    uint32_t diag;             // diagnostics (knob dec_diag): every wave stages block 0's plan (wrong output)
    uint32_t sorted;           // plans from rs_plan_sorted_kernel: the block of a record is its blk field
    // fused form (plans built in the reconstruct kernel, no rs_plan_kernel): as PlanArgs
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
    uint32_t* hard;            // multi-erasure worklist: [0] count, [kHardDone] done, [kHardList..] wave items
    uint32_t hard_cap;         // entries the worklist holds (a count past it is reported, never written)
    uint32_t list_grid;        // workgroups of the persistent worklist kernels (tier B)
    const uint32_t* gate;      // nullable: run only when gate[0] == gate_want (rs_classify_kernel's pick)
    uint32_t gate_want;
    // gated launches: the flat grid's workgroups as virtual ones [0, vgrid) walked by a persistent
    // grid, so the path the classify kernel did not pick exits after one round of workgroups
    // instead of dispatching the whole flat grid (0: flat launch)
    uint32_t vgrid;
    uint32_t persist_ncu;      // host side: nonzero asks the launcher for that persistent form (CUs)
};

// Launch geometry for a flat grid of `flat` workgroups of `kernel` (lds bytes each): the flat grid
// (a->persist_ncu == 0), or the workgroups resident at once on persist_ncu CUs (a multiple of 8, at
// most flat) walking it, with a->vgrid = flat.
int flat_or_persistent(ReconArgs* a, const void* kernel, size_t lds, int flat);

constexpr uint32_t kHardDone = 32, kHardList = 64;   // worklist words (own 128-byte lines)

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
    FastDiv div_cps;
    uint32_t pad_zero;
    uint32_t rot;
    uint32_t swz;
};

// Kernel-selection knobs. Defaults are the measured best (tools/kbench.py A/Bs them through
// the internal fec__set_tuning() entry point; results in DESIGN.md).
struct Tuning {
    int enc_nt = 3;           // encode/XOR cache policy: 0 plain, nonzero non-temporal loads and stores
    int enc_early = 2;        // fixed-shape flat encode: shard loads issued before the table staging, LDS-only
                              // barrier (fec_encode.hip rs_encode_fixed_kernel POL bit 4); 1: every shape, 2:
                              // RS(2,3) only. enc_select r04g: RS(2,3) (65 536 blocks, 40-us launches) +1.7 %,
                              // RS(8,12) +0.03 %, RS(16,24) dyadic -2.9 % (four table dwords held per lane)
    int dec_nt = 3;           // reconstruct cache policy, same values
    int grid_mult = 1;        // persistent grids: workgroups = grid_mult * CUs * resident/CU
    int dec_max_rounds = 8;   // bound on item rounds per decode tile (pick_tile_blocks)
    int pad_zero = 1;         // tail chunks: zero-padded full 16-B stores instead of partial
    int items_per_thread = 1; // >0: flat grids = total / (256 * items_per_thread); 0: persistent
    int tiles_per_wg = 1;     // >0: decode grid = ntiles / tiles_per_wg; 0: persistent
    int rotate = 0;           // rotate chunk order so shard boundaries share a wave (measured: no gain)
    int xcd_swz = 1;          // encode / XOR: workgroups of one XCD take one contiguous range of the grid
    int dec_swz = 1;          // same for reconstruct
    int enc_wpc = 3;          // resident workgroups per CU, fixed-shape encode (0: as many as fit)
    int gen_wpc = 0;          // same for the generic encode and XOR encode
    int dec_wpc = 0;          // same for reconstruct
    int enc_fixed = 1;        // compile-time-shape encode for RS(2,3), RS(8,12), RS(16,24)
    int enc_queue = 0;        // ... as the persistent ticket-queue kernel (0: flat grid, measured faster)
    int enc_qwpc = 2;         // resident workgroups per CU of the queue kernel
    int enc_qdepth = 0;       // chunks the queue kernel loads ahead (0: none, __syncthreads; -1: none, LDS-only barrier)
    int dec_wave = 1;         // reconstruct: wave-private plan staging (shards of 32+ chunks)
    int dec_fused = 0;        // ... with the plans built inside the wave kernel (measured 11 % slower: off)
    int enc_diag = 0;         // diagnostics only: queue kernel without the field arithmetic (wrong output)
    int enc_dyadic = 1;       // fixed-shape encode of dyadic codes (RS(8,12), RS(16,24)) by the
                              // split-recursive product (fewer field multiplications)
    int dec_diag = 0;         // diagnostics only: wave reconstruct with one shared plan (wrong output)
    int dec_direct = 1;       // single-erasure codes with small tables: no plan kernel, per-lane table
                              // lookup (1: rows expanded from scalar-loaded coefficients, 2: PermTab rows
                              // copied by a vector load); multi-erasure waves go to a worklist kernel
    int host_chunk = 0;       // host-resident path: blocks per staging chunk (0: 128 MiB worth)
    int host_threads = 8;     // FEC_HOST (pageable): host threads for the staging / scatter copies
    int host_pool = 1;        // FEC_HOST copies on persistent workers (fec_capi.cpp CopyPool); 0: per call
    int dec_rwin = 4;         // plan form 5 (rank-first, dec_pv 5): sort window in units of 64 blocks (1..8).
                              // r04t: level with form 3 at 64-128 blocks, 0.8-2 % slower at 256-512 (not default)
    int dec_pdiag = 0;        // plan form 3 diagnostics (timing only, wrong plans): bit 0 no coefficient rows,
                              // bit 1 records copied out as their first 48 bytes (fec_plan.hip)
    int xor_fix2 = 0;         // XOR(2,1) reconstruct by its own one-item-per-lane kernel (fec_xor.hip). r04m,
                              // three interleaved rounds: 0.6443 vs 0.6395 ms for the generic kernel (-0.7 %):
                              // the gap to the XOR twin (0.955) is the in-place write, not the loop. Off
    int enc_x23 = 1;          // RS(2,3) fixed-shape encode by its [3 2] parity row, one GF doubling per byte and
                              // no tables (fec_encode23.hip); 0: the table-driven fixed kernel
    int dec_fixk = 4;         // RS(16,24) / RS(20,30) rebuild with k at compile time (1: all k loads in
                              // flight; 2: a rolling window of 8 loaded inputs, shards of 64+ chunks,
                              // RS(20,30) also with the rows' table reads pipelined one row ahead;
                              // 3: both codes pipelined; 4: fec_rebuild.hip, PermTab rows copied from a
                              // workgroup table and input addresses as per-block offsets)
    int dec_sorted = 1;       // multi-erasure codes (plan path, shards of 32+ chunks): sorted parallel plans
    int dec_ipl = 0;          // wave-form reconstruct items per lane: 1; 2 loaded together; 3: 2 one
                              // after the other (one plan stage); 0: 2 for k <= 4, else 1
    int dir_wpc = -1;         // direct decode residency (workgroups per CU, 0 uncapped); -1: by shape,
                              // 4 for k >= 8 (RS(8,12) +3.6 %), uncapped below (RS(2,3): caps cost 10-60 %)
    int dec_pseg = 0;         // sorted plan kernel: segments of blocks per workgroup (0: by batch size)
    int dir_nt = -1;          // direct decode cache policy (3 nt loads + stores, 2 plain loads + nt
                              // stores, 0 plain); -1: by shape, 2 for k <= 4 (RS(2,3) +8 %), else 3
    int enc_bits = 9;         // bit-sliced XOR-network encode (gen_bitslice.py): bit 0 RS(16,24), bit 1
                              // RS(8,12), bit 2 loads streamed one network group ahead. Measured
                              // (enc_select.py, one box): RS(16,24) 5.35 -> 6.36 TB/s; RS(8,12)
                              // 6.42 vs 6.51 for the dyadic perm body (off); streamed -0.2 % (off)
    int enc_bwpc = 0;         // its residency (workgroups per CU, 0 uncapped)
    int dec_direct_big = 0;   // direct single-erasure decode for RS(16,24) and RS(20,30) too (rows by scalar
                              // loads from the device coefficient table; multi-erasure waves to the worklist)
    int dec_gate = 0;         // with dec_direct_big: a classify kernel picks, on the device, per batch, the
                              // direct path (few multi-erasure blocks) or the plan + rebuild path; the
                              // other path's kernels exit at once
    int dec_gate_pm = 10;     // multi-erasure blocks (per mille) above which the plan path is taken
    int dec_tier = 0;         // RS(16,24) / RS(20,30) rebuild in two tiers: waves of <= dec_tier rows
                              // (1, 2 or 4) in a small-register launch, the rest from a worklist (0: off)
    int dec_win = 0;          // fec_rebuild.hip: loads in flight per lane (4, 6, 8; 0: by code, RS(16,24) 4,
                              // RS(20,30) 6: 125 instead of 137 VGPRs, 4 instead of 3 waves/SIMD)
    int dec_psort = 1;        // sorted plans: records sorted over windows of 64 * dec_psort blocks (0: one
                              // segment of 256 / plan_lanes(k) blocks). 64 / 128 blocks: RS(20,30) -8 / -7 %
                              // decode time, RS(16,24) -3 % (rebuild rows; a cheaper ranking); 256 / 512
                              // cost the plan kernel residency (its LDS) more than the rebuild gains (r03y)
    int dec_s64 = 0;          // fec_rebuild.hip: input splits by 64-bit shifts (two dwords a shift)
    int bat_zc = 4 << 20;     // batch encoder / decoder (fec_batch.cpp): sets of at most this many input bytes are coded
                              // straight from / into their pinned buffers (device-mapped), no copies. Receive
                              // bursts (go_batch_bench burst, r04c), run loop held p50 by a non-blocking poll:
                              // RS(8,12) 1 / 8 / 64 blocks 14.6 / 14.7 / 28.2 -> 4.1 / 5.5 / 20.3 us, RS(20,30)
                              // 15.7 / 15.9 / 48.4 -> 5.0 / 7.8 / 40.1 us; data back 1.3-1.6x sooner
    int dec_lpad = 0;         // fec_rebuild.hip: the two blocks' PermTab rows of a wave slice 32 banks apart
                              // (RS(16,24)'s unpadded rows share banks: 24 % LDS conflict cycles). Measured
                              // (r04c): RS(16,24) +0.1 %, RS(20,30) -1.2 %: the conflicts are not on the
                              // critical path of a VALU-bound wave. Off.
    int dec_povl = 0;         // multi-erasure decode (sorted plans + fec_rebuild.hip): sub-batches per launch
                              // whose plan kernels run on a high-priority side stream beside the rebuild of
                              // the sub-batches before them (0 / 1: one plan launch, then one rebuild).
                              // Measured slower (r04b: RS(20,30) 2 / 4 / 8 sub-batches -0.8 / -1.9 / -3.5 %,
                              // RS(16,24) -0.9 / -2.0 / -4.3 %): the rebuild is VALU-bound, so a plan beside
                              // it takes issue slots, and each sub-batch adds a launch tail. Off.
    int dec_pv = 3;           // sorted plan kernel form: 1, or 2 (log(i ^ j) of shard indices from a 4-copy
                              // table no half-wave meets on a bank; D_p and N_r in one merged pass; exp
                              // over [0, 768) so the coefficient sums need no reduction). Form 2: VALU
                              // per plan wave 4446 -> 3171 (RS(20,30)), plan 211 -> 153 us, decode
                              // U{1..10} 2930 -> 2872 us (+2.0 %); RS(16,24) +0.2 % (r04b). 3: RS(16,24) and
                              // RS(20,30) by a kernel compiled for the code (fec_plan.hip form 3), the rest 2.
                              // Form 3 over form 2 (r04d, r04e): VALU per plan wave 3171 -> 2064 (RS(20,30)),
                              // 2176 -> 1380 (RS(16,24)); decode +0.8-0.9 % on both. 4: form 3 on two
                              // segments at a time (r04i: plan busy cycles unchanged, decode +0.2-0.35 %)
    int host_gather = 1;      // FEC_HOST_PINNED reconstruct: parity planes that few blocks read are pulled by
                              // the device straight from the caller's pinned buffer, the rest by 2D DMA (0:
                              // every plane by DMA; 2: every plane by the device)
};

// Dynamic LDS that caps residency at `wpc` workgroups per CU (160 KiB of LDS per CU on gfx950):
// halfway between 160K/(wpc+1) and 160K/wpc, never below what the kernel itself needs.
// Workgroups of `kernel` (kThreads each, `lds` dynamic LDS) resident on one CU at once, by the
// runtime's occupancy calculator; cached per (kernel, lds). At least 1.
int resident_per_cu(const void* kernel, size_t lds);

inline size_t occupancy_lds(int wpc, size_t own) {
    if (wpc <= 0) return own;
    const size_t cu = 160u * 1024u;
    size_t pad = (cu / (size_t)wpc + cu / (size_t)(wpc + 1)) / 2;
    pad &= ~(size_t)255;
    return own > pad ? own : pad;
}

// Chunks to rotate for shard stride ss: the chunks after the last 128-byte line boundary of a
// line-aligned shard, when they fit in the shard's chunk range.
inline uint32_t line_rotation(uint64_t ss, uint32_t cps) {
    const uint32_t r = (uint32_t)((ss & 127) >> 4);
    return r < cps ? r : 0;
}
extern Tuning g_tune;
extern size_t g_max_lds;   // LDS per workgroup the device allows (set at ctx creation)

hipError_t launch_rs_encode(const EncodeArgs& a, int grid, hipStream_t s);
// Fixed-shape encode (flat grid, one item per lane) for the shapes it is instantiated for.
bool fixed_encode_applies(uint32_t k, uint32_t m);
hipError_t launch_rs_encode_fixed(EncodeArgs a, int ncu, hipStream_t s);
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
// Tiered form of the RS(16,24) / RS(20,30) rebuild (fec_decode.hip): needs a.hard / a.hard_cap /
// a.err / a.list_grid.
bool tier_recon_applies(uint32_t k, uint32_t maxe, uint32_t cps);
hipError_t launch_rs_reconstruct_tiered(const ReconArgs& a, hipStream_t s);
// Compile-time-k rebuild of RS(16,24) / RS(20,30) with table-copied PermTab rows and per-block input
// offsets (fec_rebuild.hip), for the wave form's shapes with shards of 64+ chunks.
bool rebuild_k_applies(uint32_t k, uint32_t maxe, uint32_t cps);
hipError_t launch_rs_rebuild_k(const ReconArgs& a, hipStream_t s);
hipError_t launch_rs_recover_fused(const ReconArgs& a, hipStream_t s);
// Direct form (fec_recover.hip): applies when the single-erasure tables of (k, m) fit in LDS.
bool direct_recon_applies(uint32_t k, uint32_t m, uint32_t cps, uint32_t stride, bool single_slot);
size_t direct_table_words(uint32_t k, uint32_t m);
hipError_t launch_rs_recover_direct(const ReconArgs& a, int ncu, hipStream_t s);
// Pick the decode path of a batch on the device (fec_recover.hip): gate[0] = 1 (direct: at most
// thr_pm per mille of the blocks rebuild two or more data shards) or 2 (plan + rebuild). gate:
// kGateWords zeroed words; the kernel rewinds its counters.
constexpr uint32_t kGateCount = 32, kGateDone = 64, kGateWords = 96;
hipError_t launch_rs_classify(const uint32_t* masks, uint32_t nblocks, uint32_t k, uint32_t m, uint32_t max_out,
                              uint32_t* gate, uint32_t thr_pm, int ncu, hipStream_t s);
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
// Resident workgroups on the device for kernel `which` (0 encode, 1 reconstruct, 2 XOR).
int occupancy_grid(int device, int which, uint32_t m_or_maxe, size_t lds_bytes);
// Host stubs of the kernels occupancy_grid() sizes against (one per translation unit).
const void* encode_occupancy_kernel(uint32_t m);
const void* recon_occupancy_kernel(uint32_t maxe);
const void* xor_occupancy_kernel();

}  // namespace fk
