// pcie_duplex_probe.hip — what the host link of one MI355X can move, per direction and at once.
// Decides the shape of the host-resident pipeline (fec_capi.cpp, FEC_HOST / FEC_HOST_PINNED):
// whether an H2D stream and a D2H stream overlap (full duplex), whether two H2D streams beat one,
// and whether kernels reading / writing pinned host memory directly ("zero-copy") can stand in
// for either DMA direction while the other runs.
//
//   dma_h2d / dma_d2h            one hipMemcpyAsync of `bytes`, one stream
//   dma_h2d_x2                   two H2D copies of bytes/2 on two streams at once
//   dma_duplex                   H2D of `bytes` on one stream, D2H of `bytes` on another, at once
//   zc_read / zc_write           a kernel streaming pinned host memory into HBM / HBM into host
//   zc_read+dma_d2h              kernel pulls from host while a DMA pushes to host
//   dma_h2d+zc_write             DMA pulls while a kernel writes to host
//   zc_read+zc_write             both directions by kernels
//   pipe_<chunk>                 the host path's pipeline shape: chunks of `chunk` bytes go up on
//                                an up stream and (half as many bytes) come down on a down
//                                stream, 3 device buffer sets, ordered by events only (no host
//                                waits inside); reports the up rate
// Each line: {"probe", "bytes_up", "bytes_down", "ms", "up_GBps", "down_GBps", "total_GBps"},
// best of 5 (host wall clock around a full device synchronisation).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/pcie_duplex_probe tools/pcie_duplex_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <functional>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

// grid-stride 16-B copy; either side may be a device-mapped host address
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__global__ void stream_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = __builtin_nontemporal_load(src + i);
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : 1024) << 20;   // MiB per direction
    uint8_t *h_up, *h_down, *d_up, *d_down;
    CK(hipHostMalloc(&h_up, bytes, hipHostMallocDefault));
    CK(hipHostMalloc(&h_down, bytes, hipHostMallocDefault));
    memset(h_up, 7, bytes);
    memset(h_down, 9, bytes);
    CK(hipMalloc(&d_up, bytes));
    CK(hipMalloc(&d_down, bytes));
    CK(hipMemset(d_down, 3, bytes));
    void *m_up = nullptr, *m_down = nullptr;   // device addresses of the pinned buffers
    CK(hipHostGetDevicePointer(&m_up, h_up, 0));
    CK(hipHostGetDevicePointer(&m_down, h_down, 0));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int zc_grid = ncu * 4;   // r03 zerocopy_probe: 4-64 workgroups per CU all read ~55 GB/s

    auto zc = [&](const void* src, void* dst, size_t n, hipStream_t s) {
        hipLaunchKernelGGL(stream_copy, dim3(zc_grid), dim3(256), 0, s, (const v4u*)src, (v4u*)dst, n / 16);
    };
    auto run = [&](const char* name, double up, double down, const std::function<void()>& fn) {
        fn();
        CK(hipDeviceSynchronize());
        double best = 1e30;
        for (int r = 0; r < 5; ++r) {
            const double t0 = now_ms();
            fn();
            CK(hipDeviceSynchronize());
            best = std::min(best, now_ms() - t0);
        }
        printf("{\"probe\": \"%s\", \"bytes_up\": %.0f, \"bytes_down\": %.0f, \"ms\": %.3f, \"up_GBps\": %.2f, "
               "\"down_GBps\": %.2f, \"total_GBps\": %.2f}\n",
               name, up, down, best, up / best / 1e6, down / best / 1e6, (up + down) / best / 1e6);
        fflush(stdout);
    };
    const double B = (double)bytes;
    run("dma_h2d", B, 0, [&] { CK(hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, s1)); });
    run("dma_d2h", 0, B, [&] { CK(hipMemcpyAsync(h_down, d_down, bytes, hipMemcpyDeviceToHost, s1)); });
    run("dma_h2d_x2", B, 0, [&] {
        CK(hipMemcpyAsync(d_up, h_up, bytes / 2, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(d_up + bytes / 2, h_up + bytes / 2, bytes / 2, hipMemcpyHostToDevice, s2));
    });
    run("dma_duplex", B, B, [&] {
        CK(hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(h_down, d_down, bytes, hipMemcpyDeviceToHost, s2));
    });
    run("zc_read", B, 0, [&] { zc(m_up, d_up, bytes, s1); });
    run("zc_write", 0, B, [&] { zc(d_down, m_down, bytes, s1); });
    run("zc_read+dma_d2h", B, B, [&] {
        zc(m_up, d_up, bytes, s1);
        CK(hipMemcpyAsync(h_down, d_down, bytes, hipMemcpyDeviceToHost, s2));
    });
    run("dma_h2d+zc_write", B, B, [&] {
        CK(hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, s1));
        zc(d_down, m_down, bytes, s2);
    });
    run("zc_read+zc_write", B, B, [&] {
        zc(m_up, d_up, bytes, s1);
        zc(d_down, m_down, bytes, s2);
    });
    // the pipeline shape: up chunk c (s1) -> "kernel" (a device copy on s3 standing for the codec)
    // -> down chunk c (s2), 3 buffer sets, events only
    hipStream_t s3;
    CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
    hipEvent_t up_done[3], k_done[3], down_done[3];
    for (int i = 0; i < 3; ++i) {
        CK(hipEventCreateWithFlags(&up_done[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&k_done[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&down_done[i], hipEventDisableTiming));
    }
    uint8_t* d_work;
    CK(hipMalloc(&d_work, bytes));
    for (size_t chunk_mb : {4, 16, 64}) {
        const size_t chunk = chunk_mb << 20, half = chunk / 2;
        const size_t nchunks = bytes / chunk;
        if (nchunks < 3) continue;
        char nm[64];
        snprintf(nm, sizeof nm, "pipe_%zuMiB_down_half", chunk_mb);
        run(nm, (double)(nchunks * chunk), (double)(nchunks * half), [&] {
            for (size_t c = 0; c < nchunks; ++c) {
                const int i = (int)(c % 3);
                uint8_t* din = d_up + (size_t)i * chunk;          // set i's device input
                uint8_t* dout = d_work + (size_t)i * chunk;       // set i's device output
                if (c >= 3) CK(hipStreamWaitEvent(s1, k_done[i], 0));     // kernel c-3 has read din
                CK(hipMemcpyAsync(din, h_up + c * chunk, chunk, hipMemcpyHostToDevice, s1));
                CK(hipEventRecord(up_done[i], s1));
                CK(hipStreamWaitEvent(s3, up_done[i], 0));
                if (c >= 3) CK(hipStreamWaitEvent(s3, down_done[i], 0));  // down c-3 has read dout
                zc(din, dout, half, s3);
                CK(hipEventRecord(k_done[i], s3));
                CK(hipStreamWaitEvent(s2, k_done[i], 0));
                CK(hipMemcpyAsync(h_down + c * half, dout, half, hipMemcpyDeviceToHost, s2));
                CK(hipEventRecord(down_done[i], s2));
            }
        });
    }
    // Hardware queues: HIP maps streams onto at most GPU_MAX_HW_QUEUES (4 on the box) hardware
    // queues per device; two streams that share one run their operations in one FIFO. Duplex again
    // with other streams busy in the process first (a stream gets its queue on first use), then
    // with the copy streams at the highest priority.
    {
        __global__ void (*nop)(const v4u*, v4u*, size_t) = stream_copy;
        hipStream_t extra[6];
        for (hipStream_t& q : extra) {
            CK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
            hipLaunchKernelGGL(nop, dim3(1), dim3(64), 0, q, (const v4u*)d_down, (v4u*)d_work, (size_t)0);
        }
        CK(hipDeviceSynchronize());
        hipStream_t a, b;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        run("dma_duplex_after_6_streams", B, B, [&] {
            CK(hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, a));
            CK(hipMemcpyAsync(h_down, d_down, bytes, hipMemcpyDeviceToHost, b));
        });
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        hipStream_t pa, pb;
        CK(hipStreamCreateWithPriority(&pa, hipStreamNonBlocking, hi));
        CK(hipStreamCreateWithPriority(&pb, hipStreamNonBlocking, hi));
        run("dma_duplex_after_6_streams_prio_high", B, B, [&] {
            CK(hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, pa));
            CK(hipMemcpyAsync(h_down, d_down, bytes, hipMemcpyDeviceToHost, pb));
        });
        hipStream_t pc;
        CK(hipStreamCreateWithPriority(&pc, hipStreamNonBlocking, hi));
        run("dma_duplex_prio_high_and_normal", B, B, [&] {
            CK(hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, pc));
            CK(hipMemcpyAsync(h_down, d_down, bytes, hipMemcpyDeviceToHost, b));
        });
        run("dma_duplex_same_stream_pair_s1_s2", B, B, [&] {
            CK(hipMemcpyAsync(d_up, h_up, bytes, hipMemcpyHostToDevice, s1));
            CK(hipMemcpyAsync(h_down, d_down, bytes, hipMemcpyDeviceToHost, s2));
        });
        printf("{\"priority_range\": [%d, %d]}\n", lo, hi);
    }
    // check a zero-copy write landed
    memset(h_down, 0, 4096);
    CK(hipMemset(d_down, 0x5a, 4096));
    CK(hipDeviceSynchronize());   // the null-stream memset does not order against s1
    zc(d_down, m_down, 4096, s1);
    CK(hipStreamSynchronize(s1));
    int bad = 0;
    for (int i = 0; i < 4096; ++i) bad += h_down[i] != 0x5a;
    printf("{\"zc_write_check\": %s}\n", bad ? "false" : "true");   // informational
    return 0;
}
