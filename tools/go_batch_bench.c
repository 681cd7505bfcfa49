/*
 * go_batch_bench.c — host-resident throughput of the batched Go ABI (include/fec_go.h), the path
 * a Go sender / receiver would take (go/internal/fec/batch_hip.go): payloads in ordinary host
 * memory, one submit per block, frames / payloads polled back into caller buffers. Times the
 * whole loop (staging copies into pinned memory, H2D, kernels, D2H, delivery) on one host
 * thread, as one connection's run loop would run it.
 *
 *   usage: go_batch_bench rs|xor k m blocks max_blocks [payload_len]
 * prints one JSON line: encode and decode payload GB/s and blocks/s.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "fec_go.h"

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s rs|xor k m blocks max_blocks [len]\n", argv[0]);
        return 2;
    }
    const int xr = !strcmp(argv[1], "xor");
    const int scheme = xr ? FEC_SCHEME_XOR : FEC_SCHEME_REED_SOLOMON;
    const int k = atoi(argv[2]), m = xr ? 1 : atoi(argv[3]), nb = atoi(argv[4]);
    const size_t maxb = (size_t)atoi(argv[5]), len = argc > 6 ? (size_t)atoi(argv[6]) : 1200;
    uint8_t *pay = malloc((size_t)nb * k * len);
    uint64_t x = 0x0FEC;
    for (size_t i = 0; i < (size_t)nb * k * len; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        pay[i] = (uint8_t)(x >> 56);
    }
    uint8_t *reps = malloc((size_t)nb * m * FEC_GO_SLOT);
    uint32_t rlen = 0;
    const uint8_t **ptrs = malloc((size_t)(k + m) * sizeof *ptrs);
    size_t *lens = malloc((size_t)(k + m) * sizeof *lens);
    uint64_t *ids = malloc(maxb * 8), *offs = malloc(maxb * 8);
    uint32_t *rl = malloc(maxb * 4);
    uint8_t *rp = malloc(maxb * (size_t)m * FEC_GO_SLOT);
    int rc = 0;
    double best_e = 1e30, best_d = 1e30;
    for (int rep = 0; rep < 4; ++rep) {
        /* ---- encode */
        fec_go_encoder *e = fec_go_encoder_new(scheme, k, m, maxb, 0, &rc);
        if (!e) {
            fprintf(stderr, "encoder: %d %s\n", rc, fec_last_error());
            return 1;
        }
        int polled = 0;
        double t0 = now();
        for (int b = 0; b < nb; ++b) {
            for (int i = 0; i < k; ++i) {
                ptrs[i] = pay + ((size_t)b * k + i) * len;
                lens[i] = len;
            }
            if ((rc = fec_go_encoder_submit(e, (uint64_t)b, ptrs, lens, k))) {
                fprintf(stderr, "submit: %s\n", fec_last_error());
                return 1;
            }
            if ((b & 255) == 255) {
                size_t got = 0;
                fec_go_encoder_poll(e, 0, ids, rl, rp, maxb, &got);
                for (size_t d = 0; d < got; ++d, ++polled)
                    memcpy(reps + (size_t)polled * m * FEC_GO_SLOT, rp + d * m * FEC_GO_SLOT, (size_t)m * FEC_GO_SLOT);
            }
        }
        while (polled < nb) {
            size_t got = 0;
            fec_go_encoder_poll(e, 1, ids, rl, rp, maxb, &got);
            for (size_t d = 0; d < got; ++d, ++polled) {
                memcpy(reps + (size_t)polled * m * FEC_GO_SLOT, rp + d * m * FEC_GO_SLOT, (size_t)m * FEC_GO_SLOT);
                rlen = rl[d];
            }
        }
        const double te = now() - t0;
        fec_go_encoder_free(e);
        best_e = te < best_e ? te : best_e;

        /* ---- decode: source 0 of every block lost, repair 0 received */
        fec_go_decoder *d = fec_go_decoder_new(scheme, k, m, maxb, 0, &rc);
        const size_t out_cap = maxb * len;
        uint8_t *out = malloc(out_cap);
        size_t done = 0, checked = 0;
        t0 = now();
        for (int b = 0; b < nb; ++b) {
            ptrs[0] = NULL;
            lens[0] = 0;
            for (int i = 1; i < k; ++i) {
                ptrs[i] = pay + ((size_t)b * k + i) * len;
                lens[i] = len;
            }
            for (int p = 0; p < m; ++p) {
                ptrs[k + p] = p == 0 ? reps + (size_t)b * m * FEC_GO_SLOT : NULL;
                lens[k + p] = rlen;
            }
            int st = 0;
            if ((rc = fec_go_decoder_submit(d, (uint64_t)b, (uint64_t)b * k, (uint64_t)b * k + k - 1, (int)len, ptrs,
                                            lens, ptrs + k, lens + k, &st)) || !st) {
                fprintf(stderr, "dsubmit: %s\n", fec_last_error());
                return 1;
            }
            if ((b & 255) == 255 || b == nb - 1) {
                size_t got = 0;
                do {
                    fec_go_decoder_poll(d, b == nb - 1, ids, rl, offs, out, out_cap, maxb, &got);
                    for (size_t q = 0; q < got; ++q, ++done)
                        if (checked < 64 && ++checked && memcmp(out + offs[q], pay + (size_t)ids[q] * k * len, len)) {
                            fprintf(stderr, "mismatch block %llu\n", (unsigned long long)ids[q]);
                            return 1;
                        }
                } while (b == nb - 1 && done < (size_t)nb && got);
            }
        }
        const double td = now() - t0;
        free(out);
        fec_go_decoder_free(d);
        if (done != (size_t)nb) {
            fprintf(stderr, "decoded %zu of %d\n", done, nb);
            return 1;
        }
        best_d = td < best_d ? td : best_d;
    }
    const double bytes = (double)nb * k * len;
    printf("{\"scheme\": \"%s(%d,%d)\", \"host_threads\": 1, \"blocks\": %d, \"max_blocks\": %zu, \"payload_len\": %zu, "
           "\"encode_GBps\": %.3f, \"encode_blocks_per_s\": %.0f, \"decode_GBps\": %.3f, \"decode_blocks_per_s\": %.0f}\n",
           xr ? "XOR" : "RS", k, xr ? 1 : k + m, nb, maxb, len, bytes / best_e / 1e9, nb / best_e, bytes / best_d / 1e9,
           nb / best_d);
    return 0;
}
