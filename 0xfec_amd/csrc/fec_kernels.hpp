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

struct EncodeArgs {
    const uint8_t* in;   // data shard 0 of block 0
    uint8_t* out;        // parity shard 0 of block 0
    uint64_t in_bs, out_bs, ss;
    uint32_t k, m, len, cps;   // cps = chunks per shard = ceil(len / 16)
    uint32_t total;            // nblocks * cps (< 2^32 per launch)
    FastDiv div_cps;
    const uint32_t* tabs;      // m * k PermTabs (8 dwords each), device memory
};

struct PlanArgs {
    const uint32_t* masks;
    uint8_t* plans;            // nblocks * plan_stride bytes
    int32_t* status;           // optional
    int* err;                  // sticky error word
    const uint8_t* prows;      // m x k parity rows of the systematic matrix
    uint32_t k, m, nblocks, plan_stride, maxe;
};

struct ReconArgs {
    uint8_t* shards;
    uint64_t bs, ss;
    const uint8_t* plans;
    uint32_t k, len, cps, nblocks, plan_stride, maxe;
    uint32_t g;                // blocks per tile
    uint32_t ntiles;
    FastDiv div_cps;
};

struct XorArgs {
    const uint8_t* in;
    uint8_t* out;
    uint64_t in_bs, out_bs, ss;
    const uint32_t* masks;     // reconstruct only
    int32_t* status;           // reconstruct only, optional
    int* err;
    uint32_t k, len, cps, total;
    FastDiv div_cps;
};

// Plan layout per block (plan_stride bytes, 16-aligned):
//   [0] nout   [4, 4+maxe) out slots   [4+maxe, 4+maxe+k) input slots
//   [4+maxe+k, +maxe*k) coefficients, row r = output r, column = input position
inline uint32_t plan_stride_bytes(uint32_t k, uint32_t maxe) {
    return (4 + maxe + k + maxe * k + 15) & ~15u;
}

hipError_t launch_rs_encode(const EncodeArgs& a, int grid, hipStream_t s);
hipError_t launch_rs_plan(const PlanArgs& a, hipStream_t s);
hipError_t launch_rs_reconstruct(const ReconArgs& a, int grid, hipStream_t s);
hipError_t launch_xor_encode(const XorArgs& a, int grid, hipStream_t s);
hipError_t launch_xor_reconstruct(const XorArgs& a, int grid, hipStream_t s);

// Blocks per decode tile for shard chunk count `cps`, bounded by LDS.
uint32_t pick_tile_blocks(uint32_t cps, uint32_t k, uint32_t maxe);
// Resident workgroups per CU for the encode/reconstruct kernels (occupancy API).
int occupancy_grid(int device, int which, uint32_t m_or_maxe, size_t lds_bytes);

}  // namespace fk
