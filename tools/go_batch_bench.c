/*
 * go_batch_bench.c — host-resident throughput of the batched Go ABI (include/fec_go.h), the path
 * a Go sender / receiver takes (go/internal/fec/batch_hip.go): payloads in ordinary host memory,
 * one submit per block, frames / payloads polled back into caller buffers. Times the whole loop
 * (staging copies into pinned memory, H2D, kernels, D2H, delivery). T host threads each drive
 * their own encoder and decoder over their own blocks, as T connection run loops would; the
 * rate is all blocks over the wall time of the slowest thread.
 *
 *   usage: go_batch_bench rs|xor k m blocks max_blocks [payload_len] [threads] [copy|ref]
 * prints one JSON line: encode and decode payload GB/s and blocks/s.
 *
 * ref: every source payload sits in a registered packet buffer (fec_go_pool_new, one buffer per
 * payload, written before the timed region as the packer would write the frame into it) and is
 * submitted with fec_go_encoder_submit_ref: the device gathers it, the host copies nothing in.
 * On the receive side (RS) the received sources and repair sit in pool buffers too (as the wire
 * parser would have written them) and go in with fec_go_decoder_submit_ref.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "fec_go.h"
#include "fec_hip.h"

/* the library's internal, test-only tuning entry (not in the public headers; process-wide knobs,
 * keys in fk::Tuning declaration order, fec_kernels.hpp) */
int fec__set_tuning(fec_ctx *ctx, int key, int value);
enum { kTuneBatZc = 10 };

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

typedef struct {
    int scheme, k, m, nb;
    size_t maxb, len;
    const uint8_t *pay;     /* this thread's nb * k payloads */
    int ref;                /* submit by reference from a registered pool */
    uint8_t *reps;          /* nb * m * FEC_GO_SLOT */
    pthread_barrier_t *bar;
    double te, td;
    int fail;
} Job;

static void *run(void *arg) {
    Job *j = (Job *)arg;
    const int k = j->k, m = j->m, nb = j->nb;
    const size_t maxb = j->maxb, len = j->len;
    const uint8_t **ptrs = malloc((size_t)(k + m) * sizeof *ptrs);
    size_t *lens = malloc((size_t)(k + m) * sizeof *lens);
    uint64_t *ids = malloc(maxb * 8), *offs = malloc(maxb * 8);
    uint32_t *rl = malloc(maxb * 4);
    uint8_t *rp = malloc(maxb * (size_t)m * FEC_GO_SLOT);
    uint8_t *out = malloc(maxb * len);
    uint32_t rlen = 0;
    int rc = 0;
    fec_go_encoder *e = fec_go_encoder_new(j->scheme, k, m, maxb, 0, &rc);
    fec_go_decoder *d = fec_go_decoder_new(j->scheme, k, m, maxb, 0, &rc);
    if (!e || !d) {
        fprintf(stderr, "new: %d %s\n", rc, fec_last_error());
        j->fail = 1;
    }
    /* ref: the payloads, one per registered packet buffer */
    fec_go_pool *pool = NULL;
    uint8_t *pbase = NULL;
    if (j->ref && !j->fail) {
        pool = fec_go_pool_new((size_t)nb * (k + 1), &pbase, &rc);
        if (!pool) {
            fprintf(stderr, "pool: %d %s\n", rc, fec_last_error());
            j->fail = 1;
        } else {
            for (size_t i = 0; i < (size_t)nb * k; ++i) memcpy(pbase + i * FEC_GO_POOL_SLOT, j->pay + i * len, len);
        }
    }
    /* warm-up outside the timed region: the first submit of an encoder / decoder allocates its
     * pinned staging sets (tens of ms), which a connection pays once */
    if (!j->fail) {
        size_t got = 0;
        for (int i = 0; i < k; ++i) {
            ptrs[i] = j->pay + (size_t)i * len;
            lens[i] = len;
        }
        if (fec_go_encoder_submit(e, ~0ull, ptrs, lens, k) || fec_go_encoder_poll(e, 1, ids, rl, rp, maxb, &got))
            j->fail = 1;
        rlen = rl[0];
        ptrs[0] = NULL;
        for (int p = 0; p < m; ++p) {
            ptrs[k + p] = p == 0 ? rp : NULL;
            lens[k + p] = rlen;
        }
        int st = 0;
        if (fec_go_decoder_submit(d, ~0ull, 0, (uint64_t)k - 1, (int)len, ptrs, lens, ptrs + k, lens + k, &st) ||
            fec_go_decoder_poll(d, 1, ids, rl, offs, out, maxb * len, maxb, &got))
            j->fail = 1;
    }
    /* ---- encode */
    pthread_barrier_wait(j->bar);
    double t0 = now();
    int polled = 0;
    for (int b = 0; b < nb && !j->fail; ++b) {
        for (int i = 0; i < k; ++i) {
            ptrs[i] = j->ref ? pbase + ((size_t)b * k + i) * FEC_GO_POOL_SLOT : j->pay + ((size_t)b * k + i) * len;
            lens[i] = len;
        }
        if (j->ref ? fec_go_encoder_submit_ref(e, (uint64_t)b, ptrs, lens, k)
                   : fec_go_encoder_submit(e, (uint64_t)b, ptrs, lens, k)) {
            fprintf(stderr, "submit: %s\n", fec_last_error());
            j->fail = 1;
        }
        if ((b & 255) == 255) {
            size_t got = 0;
            fec_go_encoder_poll(e, 0, ids, rl, rp, maxb, &got);
            for (size_t q = 0; q < got; ++q, ++polled)
                memcpy(j->reps + (size_t)polled * m * FEC_GO_SLOT, rp + q * m * FEC_GO_SLOT, (size_t)m * FEC_GO_SLOT);
        }
    }
    while (polled < nb && !j->fail) {
        size_t got = 0;
        fec_go_encoder_poll(e, 1, ids, rl, rp, maxb, &got);
        if (!got) j->fail = 1;
        for (size_t q = 0; q < got; ++q, ++polled) {
            memcpy(j->reps + (size_t)polled * m * FEC_GO_SLOT, rp + q * m * FEC_GO_SLOT, (size_t)m * FEC_GO_SLOT);
            rlen = rl[q];
        }
    }
    j->te = now() - t0;
    /* ref: each block's received repair 0 in a pool buffer (after the sources' nb * k buffers) */
    const int dref = j->ref && !j->fail && j->scheme == FEC_SCHEME_REED_SOLOMON;
    if (dref)
        for (int b = 0; b < nb; ++b)
            memcpy(pbase + ((size_t)nb * k + b) * FEC_GO_POOL_SLOT, j->reps + (size_t)b * m * FEC_GO_SLOT, rlen);
    /* ---- decode: source 0 of every block lost, repair 0 received */
    pthread_barrier_wait(j->bar);
    t0 = now();
    size_t done = 0, checked = 0;
    for (int b = 0; b < nb && !j->fail; ++b) {
        ptrs[0] = NULL;
        lens[0] = 0;
        for (int i = 1; i < k; ++i) {
            ptrs[i] = dref ? pbase + ((size_t)b * k + i) * FEC_GO_POOL_SLOT : j->pay + ((size_t)b * k + i) * len;
            lens[i] = len;
        }
        for (int p = 0; p < m; ++p) {
            ptrs[k + p] = p != 0 ? NULL
                          : dref ? pbase + ((size_t)nb * k + b) * FEC_GO_POOL_SLOT
                                 : j->reps + (size_t)b * m * FEC_GO_SLOT;
            lens[k + p] = rlen;
        }
        int st = 0;
        if ((dref ? fec_go_decoder_submit_ref : fec_go_decoder_submit)(d, (uint64_t)b, (uint64_t)b * k,
                                                                       (uint64_t)b * k + k - 1, (int)len, ptrs, lens,
                                                                       ptrs + k, lens + k, &st) ||
            !st) {
            fprintf(stderr, "dsubmit: %s\n", fec_last_error());
            j->fail = 1;
        }
        if ((b & 255) == 255 || b == nb - 1) {
            size_t got = 0;
            do {
                fec_go_decoder_poll(d, b == nb - 1, ids, rl, offs, out, maxb * len, maxb, &got);
                for (size_t q = 0; q < got; ++q, ++done)
                    if (checked < 64 && ++checked && memcmp(out + offs[q], j->pay + (size_t)ids[q] * k * len, len)) {
                        fprintf(stderr, "mismatch block %llu\n", (unsigned long long)ids[q]);
                        j->fail = 1;
                    }
            } while (b == nb - 1 && done < (size_t)nb && got);
        }
    }
    j->td = now() - t0;
    if (done != (size_t)nb) j->fail = 1;
    /* ref: the encoded repairs must equal the copy path's: spot-check block 0 and nb-1 against a
       fresh copy-mode encode (the encode loop above already checked the decode round trip) */
    if (j->ref && !j->fail) {
        for (int b = 0; b < nb; b += nb - 1 > 0 ? nb - 1 : 1) {
            for (int i = 0; i < k; ++i) {
                ptrs[i] = j->pay + ((size_t)b * k + i) * len;
                lens[i] = len;
            }
            size_t got = 0;
            int same = !fec_go_encoder_submit(e, ~1ull, ptrs, lens, k) && !fec_go_encoder_poll(e, 1, ids, rl, rp, maxb, &got) &&
                       got == 1;
            for (int p = 0; same && p < m; ++p)
                same = !memcmp(rp + (size_t)p * FEC_GO_SLOT, j->reps + ((size_t)b * m + p) * FEC_GO_SLOT, rl[0]);
            if (!same) {
                fprintf(stderr, "ref encode differs from copy encode at block %d\n", b);
                j->fail = 1;
            }
            if (nb == 1) break;
        }
    }
    if (e) fec_go_encoder_free(e);
    if (d) fec_go_decoder_free(d);
    if (pool) fec_go_pool_free(pool);
    free(ptrs), free(lens), free(ids), free(offs), free(rl), free(rp), free(out);
    return NULL;
}

static int cmp_dbl(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static double pct(const double *s, int n, double p) {
    int i = (int)(p * (n - 1) + 0.5);
    return s[i < 0 ? 0 : i >= n ? n - 1 : i];
}

/* Receive-side stall of one run-loop burst (connection.go.diff handleRecoveredFEC): N recoverable
 * blocks (source 0 lost, repair 0 received) are submitted, then
 *   block:  fec_go_decoder_poll(wait=1) until all N are back: the time the run loop is held;
 *   poll:   one fec_go_decoder_poll(wait=0) right after the submits (it launches the staged set),
 *           the time the run loop is held; then non-blocking polls until all N are back: the
 *           completion latency the recovered frames see.
 * Timed per burst over `reps` bursts; prints p50 / p99 / max in microseconds. */
static int zc_bytes = 0;

static int burst(int k, int m, int N, int reps, size_t len, int ref) {
    const int pool_blocks = N * 4 > 256 ? N * 4 : 256;   /* distinct blocks, reused round robin */
    const size_t maxb = (size_t)(N > 64 ? N : 64);
    uint8_t *pay = malloc((size_t)pool_blocks * k * len), *reps_buf = calloc((size_t)pool_blocks * m, FEC_GO_SLOT);
    uint64_t x = 0xB0057;
    for (size_t i = 0; i < (size_t)pool_blocks * k * len; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        pay[i] = (uint8_t)(x >> 56);
    }
    const uint8_t **ptrs = malloc((size_t)(k + m) * sizeof *ptrs);
    size_t *lens = malloc((size_t)(k + m) * sizeof *lens);
    uint64_t *ids = malloc(maxb * 8), *offs = malloc(maxb * 8);
    uint32_t *rl = malloc(maxb * 4);
    uint8_t *rp = malloc(maxb * (size_t)m * FEC_GO_SLOT), *out = malloc(maxb * len);
    int rc = 0;
    fec_go_encoder *e = fec_go_encoder_new(FEC_SCHEME_REED_SOLOMON, k, m, maxb, 0, &rc);
    fec_go_decoder *d = fec_go_decoder_new(FEC_SCHEME_REED_SOLOMON, k, m, maxb, 0, &rc);
    if (!e || !d) {
        fprintf(stderr, "new: %d %s\n", rc, fec_last_error());
        return 1;
    }
    /* repairs of every pool block (outside the timing) */
    uint32_t rlen = 0;
    for (int b = 0, polled = 0; b < pool_blocks; ++b) {
        for (int i = 0; i < k; ++i) {
            ptrs[i] = pay + ((size_t)b * k + i) * len;
            lens[i] = len;
        }
        if (fec_go_encoder_submit(e, (uint64_t)b, ptrs, lens, k)) return 1;
        while (polled <= b) {
            size_t got = 0;
            if (fec_go_encoder_poll(e, 1, ids, rl, rp, maxb, &got)) return 1;
            for (size_t q = 0; q < got; ++q, ++polled) {
                memcpy(reps_buf + (size_t)ids[q] * m * FEC_GO_SLOT, rp + q * m * FEC_GO_SLOT, (size_t)m * FEC_GO_SLOT);
                rlen = rl[q];
            }
        }
    }
    fec_go_pool *pool = NULL;
    uint8_t *pbase = NULL;
    if (ref) {   /* received payloads as the wire parser leaves them: in registered pool buffers */
        pool = fec_go_pool_new((size_t)pool_blocks * (k + 1), &pbase, &rc);
        if (!pool) return 1;
        for (int b = 0; b < pool_blocks; ++b) {
            for (int i = 0; i < k; ++i)
                memcpy(pbase + ((size_t)b * (k + 1) + i) * FEC_GO_POOL_SLOT, pay + ((size_t)b * k + i) * len, len);
            memcpy(pbase + ((size_t)b * (k + 1) + k) * FEC_GO_POOL_SLOT, reps_buf + (size_t)b * m * FEC_GO_SLOT, rlen);
        }
    }
    double *held = malloc((size_t)reps * sizeof(double)), *lat = malloc((size_t)reps * sizeof(double));
    /* send side: N completed blocks submitted, then one non-blocking poll (the packer's
     * PollRepairFrames, which launches the staged set): the hold; then polls until every block's
     * repair frames are back */
    uint64_t sid = (uint64_t)pool_blocks;
    for (int r = -8; r < reps; ++r) {
        const double t0 = now();
        for (int j = 0; j < N; ++j) {
            const int b = (int)(sid % (uint64_t)pool_blocks);
            for (int i = 0; i < k; ++i) {
                ptrs[i] = pay + ((size_t)b * k + i) * len;
                lens[i] = len;
            }
            if (fec_go_encoder_submit(e, sid++, ptrs, lens, k)) return 1;
        }
        size_t done = 0, got = 0;
        if (fec_go_encoder_poll(e, 0, ids, rl, rp, maxb, &got)) return 1;
        done += got;
        const double t_held = now() - t0;
        while (done < (size_t)N) {
            if (fec_go_encoder_poll(e, 0, ids, rl, rp, maxb, &got)) return 1;
            done += got;
        }
        const double t_done = now() - t0;
        const int b = (int)((sid - 1) % (uint64_t)pool_blocks);   /* the last block's frames */
        for (int p = 0; got && p < m; ++p)
            if (memcmp(rp + ((got - 1) * m + p) * FEC_GO_SLOT, reps_buf + ((size_t)b * m + p) * FEC_GO_SLOT, rl[got - 1])) {
                fprintf(stderr, "send mismatch at burst %d\n", r);
                return 1;
            }
        if (r >= 0) held[r] = t_held * 1e6, lat[r] = t_done * 1e6;
    }
    qsort(held, (size_t)reps, sizeof(double), cmp_dbl);
    qsort(lat, (size_t)reps, sizeof(double), cmp_dbl);
    printf("{\"mode\": \"burst\", \"side\": \"send\", \"scheme\": \"RS(%d,%d)\", \"submit\": \"copy\", \"policy\": "
           "\"poll (wait=0), re-poll\", \"burst_blocks\": %d, \"bursts\": %d, \"run_loop_held_us\": {\"p50\": %.1f, "
           "\"p99\": %.1f, \"max\": %.1f}, \"frames_after_us\": {\"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f}, "
           "\"zero_copy_set_bytes\": %d}\n",
           k, k + m, N, reps, pct(held, reps, 0.5), pct(held, reps, 0.99), held[reps - 1], pct(lat, reps, 0.5),
           pct(lat, reps, 0.99), lat[reps - 1], zc_bytes);
    uint64_t next_id = 0;
    for (int policy = 0; policy < 2; ++policy) {
        for (int r = -8; r < reps; ++r) {   /* 8 untimed bursts first */
            const double t0 = now();
            for (int j = 0; j < N; ++j) {
                const int b = (int)(next_id % (uint64_t)pool_blocks);
                const uint8_t *base = ref ? pbase + (size_t)b * (k + 1) * FEC_GO_POOL_SLOT : NULL;
                ptrs[0] = NULL;
                lens[0] = 0;
                for (int i = 1; i < k; ++i) {
                    ptrs[i] = ref ? base + (size_t)i * FEC_GO_POOL_SLOT : pay + ((size_t)b * k + i) * len;
                    lens[i] = len;
                }
                for (int p = 0; p < m; ++p) {
                    ptrs[k + p] = p ? NULL : ref ? base + (size_t)k * FEC_GO_POOL_SLOT : reps_buf + (size_t)b * m * FEC_GO_SLOT;
                    lens[k + p] = p ? 0 : rlen;
                }
                int st = 0;
                if ((ref ? fec_go_decoder_submit_ref : fec_go_decoder_submit)(d, next_id, next_id * k, next_id * k + k - 1,
                                                                              (int)len, ptrs, lens, ptrs + k, lens + k, &st) ||
                    !st) {
                    fprintf(stderr, "dsubmit: %s\n", fec_last_error());
                    return 1;
                }
                ++next_id;
            }
            size_t done = 0, got = 0;
            double t_held = 0;
            if (policy == 0) {
                while (done < (size_t)N) {
                    if (fec_go_decoder_poll(d, 1, ids, rl, offs, out, maxb * len, maxb, &got)) return 1;
                    done += got;
                }
                t_held = now() - t0;
            } else {
                if (fec_go_decoder_poll(d, 0, ids, rl, offs, out, maxb * len, maxb, &got)) return 1;
                done += got;
                t_held = now() - t0;
                while (done < (size_t)N) {
                    if (fec_go_decoder_poll(d, 0, ids, rl, offs, out, maxb * len, maxb, &got)) return 1;
                    done += got;
                }
            }
            const double t_done = now() - t0;
            /* the last recovered payload must be its block's lost source 0 */
            const int b = (int)((next_id - 1) % (uint64_t)pool_blocks);
            if (got && memcmp(out + offs[got - 1], pay + (size_t)b * k * len, len)) {
                fprintf(stderr, "mismatch at burst %d\n", r);
                return 1;
            }
            if (r >= 0) held[r] = t_held * 1e6, lat[r] = t_done * 1e6;
        }
        qsort(held, (size_t)reps, sizeof(double), cmp_dbl);
        qsort(lat, (size_t)reps, sizeof(double), cmp_dbl);
        printf("{\"mode\": \"burst\", \"scheme\": \"RS(%d,%d)\", \"submit\": \"%s\", \"policy\": \"%s\", \"burst_blocks\": %d, "
               "\"bursts\": %d, \"run_loop_held_us\": {\"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f}, "
               "\"recovered_after_us\": {\"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f}, \"held_us_per_block_p50\": %.2f, "
               "\"zero_copy_set_bytes\": %d}\n",
               k, k + m, ref ? "ref" : "copy", policy ? "poll (wait=0), re-poll" : "block (wait=1)", N, reps,
               pct(held, reps, 0.5), pct(held, reps, 0.99), held[reps - 1], pct(lat, reps, 0.5), pct(lat, reps, 0.99),
               lat[reps - 1], pct(held, reps, 0.5) / N, zc_bytes);
        fflush(stdout);
    }
    fec_go_encoder_free(e);
    fec_go_decoder_free(d);
    if (pool) fec_go_pool_free(pool);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 2 && !strcmp(argv[1], "burst")) {
        if (argc < 6) {
            fprintf(stderr, "usage: %s burst k m N reps [len] [copy|ref] [zc=BYTES]\n", argv[0]);
            return 2;
        }
        if (argc > 8 && !strncmp(argv[8], "zc=", 3)) {   /* the decoder's zero-copy set size (knob bat_zc) */
            fec_ctx *c = NULL;
            zc_bytes = atoi(argv[8] + 3);
            if (fec_ctx_create(0, &c) || fec__set_tuning(c, kTuneBatZc, zc_bytes) < 0) {
                fprintf(stderr, "tuning: %s\n", fec_last_error());
                return 1;
            }
            fec_ctx_destroy(c);
        }
        const int rc = burst(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), atoi(argv[5]),
                             argc > 6 ? (size_t)atoi(argv[6]) : 1200, argc > 7 && !strcmp(argv[7], "ref"));
        fflush(stdout);
        _exit(rc);
    }
    if (argc < 6) {
        fprintf(stderr, "usage: %s rs|xor k m blocks max_blocks [len] [threads] [copy|ref]\n"
                        "       %s burst k m N reps [len] [copy|ref]\n", argv[0], argv[0]);
        return 2;
    }
    const int xr = !strcmp(argv[1], "xor");
    const int k = atoi(argv[2]), m = xr ? 1 : atoi(argv[3]), nb = atoi(argv[4]);
    const size_t maxb = (size_t)atoi(argv[5]), len = argc > 6 ? (size_t)atoi(argv[6]) : 1200;
    const int T = argc > 7 ? atoi(argv[7]) : 1;
    const int ref = argc > 8 && !strcmp(argv[8], "ref");
    const int per = nb / T;
    uint8_t *pay = malloc((size_t)T * per * k * len);
    uint64_t x = 0x0FEC;
    for (size_t i = 0; i < (size_t)T * per * k * len; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        pay[i] = (uint8_t)(x >> 56);
    }
    double best_e = 1e30, best_d = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
        pthread_barrier_t bar;
        pthread_barrier_init(&bar, NULL, (unsigned)T);
        Job *jobs = calloc((size_t)T, sizeof *jobs);
        pthread_t *th = malloc((size_t)T * sizeof *th);
        for (int t = 0; t < T; ++t) {
            jobs[t] = (Job){xr ? FEC_SCHEME_XOR : FEC_SCHEME_REED_SOLOMON, k, m, per, maxb, len,
                            pay + (size_t)t * per * k * len, ref, calloc((size_t)per * m, FEC_GO_SLOT), &bar, 0, 0, 0};
            pthread_create(&th[t], NULL, run, &jobs[t]);
        }
        double te = 0, td = 0;
        for (int t = 0; t < T; ++t) {
            pthread_join(th[t], NULL);
            if (jobs[t].fail) {
                fprintf(stderr, "thread %d failed\n", t);
                return 1;
            }
            te = jobs[t].te > te ? jobs[t].te : te;
            td = jobs[t].td > td ? jobs[t].td : td;
            free(jobs[t].reps);
        }
        pthread_barrier_destroy(&bar);
        free(jobs);
        free(th);
        best_e = te < best_e ? te : best_e;
        best_d = td < best_d ? td : best_d;
    }
    const double blocks = (double)T * per, bytes = blocks * k * len;
    printf("{\"scheme\": \"%s(%d,%d)\", \"submit\": \"%s\", \"host_threads\": %d, \"blocks\": %.0f, \"max_blocks\": %zu, "
           "\"payload_len\": %zu, \"encode_GBps\": %.3f, \"encode_blocks_per_s\": %.0f, \"decode_GBps\": %.3f, "
           "\"decode_blocks_per_s\": %.0f}\n",
           xr ? "XOR" : "RS", k, xr ? 1 : k + m, ref ? "ref (registered pool, device gather)" : "copy", T, blocks, maxb, len, bytes / best_e / 1e9, blocks / best_e,
           bytes / best_d / 1e9, blocks / best_d);
    fflush(stdout);
    _exit(0);
}
