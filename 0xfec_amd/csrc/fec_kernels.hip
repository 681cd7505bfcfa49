// fec_kernels.hip — gfx950 (MI355X, CDNA4) kernels for block FEC.
//
// Hot path of ddritzenhoff/0xFEC internal/fec (reed_solomon.go:51 Encode, :124
// ReconstructData; xor.go:28-33, :80-86), rebuilt for CDNA4:
//   * byte-wise GF(2^8) work on packed dwords with v_perm_b32 product tables
//     (three lookups per dword per coefficient; no MFMA — this is not a contraction)
//   * every lane owns one 16-byte column chunk of a block and streams the k input
//     shards of that chunk with global_load_dwordx4 (a wave covers 1 KiB contiguous
//     per input shard), accumulating all outputs in VGPRs, so each input byte is read
//     from HBM exactly once and each output byte written once
//   * coefficient tables sit in LDS and are read wave-uniform (broadcast)
//   * decode solves only the e x e system of the erased data shards per block
//     (rs_plan_kernel), which is the same linear solution klauspost computes from the
//     full k x k inverse of the first k present rows.
// Grid shapes, non-temporal access and tail-store form were chosen by measurement (DESIGN.md
// "Kernel tuning").
//
// The kernels live in fec_encode*.hip, fec_decode.hip, fec_plan.hip, fec_rebuild.hip,
// fec_recover.hip and fec_xor.hip (separate translation units, compiled in parallel); this file
// holds the process-wide tuning and the host helpers.
#include <hip/hip_runtime.h>


#include "fec_kernels.hpp"

namespace fk {

Tuning g_tune;
size_t g_max_lds = 65536;

FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{d, 0, 0};
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.shift = l;
    f.magic = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    return f;
}

PlanLayout plan_layout(uint32_t k, uint32_t maxe, bool sorted) {
    PlanLayout l;
    l.in_off = 0;
    l.out_off = (k + 7) & ~7u;                       // in slots, read 8 at a time
    l.nout_off = l.out_off + maxe;
    l.blk_off = sorted ? (l.nout_off + 1 + 3) & ~3u : 0;
    l.coef_off = sorted ? l.blk_off + 4 : (l.nout_off + 1 + 3) & ~3u;
    l.stride = (l.coef_off + maxe * k + 15) & ~15u;
    return l;
}

}  // namespace fk

