// zerocopy_probe.hip — how fast can a kernel pull bytes straight out of pinned host memory
// (no DMA engine), against hipMemcpyAsync of the same bytes? Decides whether the host-resident
// paths gather packet payloads on the device instead of staging them with host memcpy.
//
//   linear DMA     hipMemcpyAsync H2D of the whole span
//   linear kernel  lanes read the span 16 B each (grid-stride) and write it to HBM
//   shard gather   one wave per 1202-B shard, shards `pick` of every `cols` (e.g. 1 of 4: the
//                  single parity plane a single-erasure decode reads out of [B][4][1202])
//   DMA span       hipMemcpyAsync of the whole [B][cols][1202] span (what the path does today)
//
// build: hipcc --offload-arch=gfx950 -O3 -o zerocopy_probe zerocopy_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__global__ void linear_read(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// one wave per picked shard: shard b of the span at src + b*bs (len bytes, 2-byte aligned),
// written to dst + b*1216; dword loads at the aligned-down address, funnel-shifted
__global__ void shard_gather(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t nshards, size_t bs,
                             uint32_t len) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
    if (wave >= nshards) return;
    const uint8_t* s = src + (size_t)wave * bs;
    const uintptr_t a = (uintptr_t)s & ~(uintptr_t)3;
    const uint32_t sh = (uint32_t)((uintptr_t)s & 3);
    const uint32_t* A = reinterpret_cast<const uint32_t*>(a);
    const uint32_t ndw = (len + 3) / 4;
    for (uint32_t w = lane; w < ndw; w += 64) {
        uint32_t lo = A[w];
        uint32_t hi = (sh && 4 * w + 4 - sh < len) ? A[w + 1] : 0u;
        uint32_t v = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
        reinterpret_cast<uint32_t*>(dst + (size_t)wave * 1216)[w] = v;
    }
}

int main(int argc, char** argv) {
    const size_t B = argc > 1 ? strtoull(argv[1], 0, 10) : 131072;
    const uint32_t cols = argc > 2 ? atoi(argv[2]) : 4, L = 1202;
    const size_t span = B * cols * L;
    uint8_t *h, *d, *dd;
    CK(hipHostMalloc(&h, span + 64, hipHostMallocDefault));
    memset(h, 7, span);
    CK(hipMalloc(&d, span + 64));
    CK(hipMalloc(&dd, B * 1216 + 64));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto fn) {
        fn();
        CK(hipStreamSynchronize(st));
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0, st));
            fn();
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        printf("{\"probe\": \"%s\", \"bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.2f}\n", name, bytes, best,
               bytes / (best * 1e-3) / 1e9);
        fflush(stdout);
    };
    timeit("dma_span_h2d", (double)span, [&] { CK(hipMemcpyAsync(d, h, span, hipMemcpyHostToDevice, st)); });
    for (int wpc : {4, 16, 64}) {
        char nm[64];
        snprintf(nm, sizeof nm, "kernel_linear_read_%dwg_per_cu", wpc);
        timeit(nm, (double)(span / 16 * 16), [&] {
            hipLaunchKernelGGL(linear_read, dim3(256 * wpc), dim3(256), 0, st, (const uint4*)h, (uint4*)d, span / 16);
        });
    }
    timeit("kernel_gather_1_of_cols", (double)B * L, [&] {
        hipLaunchKernelGGL(shard_gather, dim3((uint32_t)((B + 3) / 4)), dim3(256), 0, st, h + 2 * L, dd, (uint32_t)B,
                           (size_t)cols * L, L);
    });
    timeit("kernel_gather_all_shards", (double)B * cols * L, [&] {
        for (uint32_t c = 0; c < cols; ++c)
            hipLaunchKernelGGL(shard_gather, dim3((uint32_t)((B + 3) / 4)), dim3(256), 0, st, h + c * L, dd,
                               (uint32_t)B, (size_t)cols * L, L);
    });
    timeit("dma_one_shard_2d", (double)B * L, [&] {
        CK(hipMemcpy2DAsync(dd, 1216, h + 2 * L, (size_t)cols * L, L, B, hipMemcpyHostToDevice, st));
    });
    CK(hipDeviceSynchronize());
    // check the gather
    uint8_t* back = (uint8_t*)malloc(1216);
    for (size_t i = 0; i < span; ++i) h[i] = (uint8_t)(i * 131 + 7);
    hipLaunchKernelGGL(shard_gather, dim3((uint32_t)((B + 3) / 4)), dim3(256), 0, st, h + 2 * L, dd, (uint32_t)B,
                       (size_t)cols * L, L);
    CK(hipStreamSynchronize(st));
    int bad = 0;
    for (size_t b : {(size_t)0, B / 2, B - 1}) {
        CK(hipMemcpy(back, dd + b * 1216, L, hipMemcpyDeviceToHost));
        if (memcmp(back, h + b * cols * L + 2 * L, L)) bad++;
    }
    printf("{\"gather_check\": %s}\n", bad ? "false" : "true");
    (void)hipHostFree(h);
    (void)hipFree(d);
    (void)hipFree(dd);
    return bad;
}
