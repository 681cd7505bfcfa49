// fec_encode23.hip — RS(2,3) encode (the reference's benchmark config #1 code) from its parity
// row alone.
//
// klauspost's matrix for k = 2, n = 3 (buildMatrix, reference call site reed_solomon.go:16;
// rs_matrix.hpp) has the parity row [3 2], so p = 3*x0 ^ 2*x1 = x0 ^ 2*(x0 ^ x1): one doubling
// in GF(2^8) (polynomial 0x11d) per byte, four bytes of a dword at once,
//   2*v = ((v << 1) & 0xFEFEFEFE) ^ (((v >> 7) & 0x01010101) * 0x1D),
// and no product tables: no LDS staging and no barrier, which are most of the table-driven
// kernel's prologue in a 40-us launch of ~20 000 one-item-per-lane workgroups. The launcher
// checks the row on the host, so any other matrix falls back to the generic kernel. Layout, tail
// handling and workgroup order are rs_encode_fixed_kernel's (fec_encode.hip).
#include <hip/hip_runtime.h>

#include "fec_device.hpp"
#include "fec_kernels.hpp"
#include "rs_matrix.hpp"

namespace fk {
namespace {

__device__ __forceinline__ uint32_t gf_dbl4(uint32_t v) {
    return ((v << 1) & 0xFEFEFEFEu) ^ (((v >> 7) & 0x01010101u) * 0x1Du);
}

__device__ __forceinline__ uint32_t parity23(uint32_t x0, uint32_t x1) { return x0 ^ gf_dbl4(x0 ^ x1); }

// Non-temporal loads (with plain loads back-to-back launches re-read the config's whole batch, 239
// MB, from the 256 MiB Infinity Cache, +11 % that a stream of fresh inputs never sees: DESIGN.md 3,
// r04); stores by policy SP (fec_device.hpp st16p)
template <int SP>
__global__ __launch_bounds__(kThreads) void rs_encode23_kernel(EncodeArgs a) {
    constexpr bool NTL = true;
    const uint32_t it = xcd_order() * kThreads + threadIdx.x;
    if (it >= a.total) return;
    const uint32_t b = fdiv(it, a.div_cps);
    const uint32_t c = it - b * a.cps;
    const uint8_t* src = a.in + (uint64_t)b * a.in_bs + (uint64_t)c * kChunk;
    const uint4 x0 = ld16<NTL>(src), x1 = ld16<NTL>(src + a.ss);
    const uint4 p = make_uint4(parity23(x0.x, x1.x), parity23(x0.y, x1.y), parity23(x0.z, x1.z),
                               parity23(x0.w, x1.w));
    const uint32_t nb = min(a.len - c * kChunk, (uint32_t)kChunk);
    st16p<SP>(a.out + (uint64_t)b * a.out_bs + (uint64_t)c * kChunk, keep_bytes(p, nb));
}

bool row_is_3_2() {
    static const bool yes = [] {
        const std::vector<uint8_t> mx = rs::build_matrix(2, 3);
        return mx.size() == 6 && mx[4] == 3 && mx[5] == 2;
    }();
    return yes;
}

}  // namespace

// The code is RS(2,3) with klauspost's [3 2] parity row.
bool rs_encode23_applies(uint32_t k, uint32_t m) { return k == 2 && m == 1 && row_is_3_2(); }

// RS(2,3) encode with the fixed kernels' argument block (16-byte aligned layout, pad-zero tail);
// the caller has checked rs_encode23_applies.
hipError_t launch_rs_encode23(const EncodeArgs& a, hipStream_t s) {
    const uint32_t chunks = (a.total + kThreads - 1) / kThreads;
    if (chunks == 0) return hipSuccess;
    // stores by the call's policy (a.sp: fec_kernels.hpp encode_store_policy)
    const size_t lds = occupancy_lds(g_tune.gen_wpc, 0);
    if (a.sp == 1) hipLaunchKernelGGL(rs_encode23_kernel<1>, dim3(chunks), dim3(kThreads), lds, s, a);
    else hipLaunchKernelGGL(rs_encode23_kernel<0>, dim3(chunks), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

}  // namespace fk
