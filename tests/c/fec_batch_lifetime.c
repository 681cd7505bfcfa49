/* fec_batch_lifetime.c — a connection's queue freed while the batched codec still owes it blocks.
 *
 * The batch encoder keeps a block's frames in a backlog while the connection's RepairQueue is
 * full (the reference would panic, repair_queue.go:53), and a batch decoder owes a connection its
 * recovered payloads until the batch completes. A connection may close (and free its queue) at
 * any of these moments; the codec must then drop that queue's blocks, as the reference's closed
 * connection drops its frames, without touching the freed queue or its liveness token.
 *
 * Scenarios, each run through poll and drain afterwards (built plain and against the host
 * ASan/UBSan library, tests/test_sanitizers.py):
 *   backlog   frames held for a full queue, queue freed, then drain
 *   inflight  a batch in flight on the device, its queue freed, then poll + drain
 *   mixed     two queues share a batch; one is freed; the other still gets every frame in order
 *   decoder   a RecoveredQueue freed while its blocks are in flight, then drain
 * Prints "ok <scenarios>" and exits 0; on a device-less host the first codec call fails with
 * "no HIP device" (exit 1). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fec_batch.h"
#include "fec_scheme.h"
#include "fec_wire.h"

#define K 8
#define M 4

static int fail(const char *what, int rc) {
    fprintf(stderr, "%s: rc=%d %s\n", what, rc, fec_last_error());
    return 1;
}

static void fill(uint8_t *p, size_t n, uint32_t seed) {
    uint32_t x = seed * 2654435761u + 1;
    for (size_t i = 0; i < n; ++i) {
        x ^= x << 13, x ^= x >> 17, x ^= x << 5;
        p[i] = (uint8_t)x;
    }
}

/* Submits block `id` (K payloads of `len` bytes) to encoder e for queue q. */
static int submit(fec_batch_encoder *e, uint64_t id, size_t len, fec_repair_queue *q) {
    uint8_t buf[K][1200];
    const uint8_t *ptr[K];
    size_t lens[K];
    for (int i = 0; i < K; ++i) {
        fill(buf[i], len, (uint32_t)(id * K + i));
        ptr[i] = buf[i];
        lens[i] = len;
    }
    return fec_batch_encoder_submit_payloads(e, id, ptr, lens, K, q);
}

static int backlog(void) {
    int err = 0;
    fec_batch_encoder *e = fec_batch_encoder_new(FEC_SCHEME_REED_SOLOMON, K, M, 8, 0, &err);
    if (!e) return fail("encoder_new", err);
    fec_repair_queue *q = fec_repair_queue_new(M);   /* room for one block's frames */
    for (uint64_t b = 0; b < 4; ++b)
        if ((err = submit(e, b, 1000, q))) return fail("submit", err);
    size_t n = 0;
    err = fec_batch_encoder_drain(e, &n);
    if (err != FEC_ERR_SCHEME || fec_batch_encoder_backlog(e) != 3 || fec_repair_queue_len(q) != M)
        return fail("drain into a full queue", err);
    fec_repair_queue_free(q);   /* the backlog now holds the only references to q's token */
    if ((err = fec_batch_encoder_poll(e, &n)) || fec_batch_encoder_backlog(e) != 0 || n != 0)
        return fail("poll after free", err);
    if ((err = fec_batch_encoder_drain(e, &n)) || n != 0) return fail("drain after free", err);
    fec_batch_encoder_free(e);
    return 0;
}

static int inflight(void) {
    int err = 0;
    fec_batch_encoder *e = fec_batch_encoder_new(FEC_SCHEME_REED_SOLOMON, K, M, 2, 0, &err);
    if (!e) return fail("encoder_new", err);
    fec_repair_queue *q = fec_repair_queue_new(64);
    for (uint64_t b = 0; b < 3; ++b)   /* the third submit flushes the first batch of two */
        if ((err = submit(e, b, 1200, q))) return fail("submit", err);
    if (fec_batch_encoder_in_flight(e) == 0 && fec_batch_encoder_backlog(e) == 0 && fec_repair_queue_len(q) == 0)
        return fail("no batch went out", 0);
    fec_repair_queue_free(q);
    size_t n = 0;
    if ((err = fec_batch_encoder_poll(e, &n))) return fail("poll after free", err);
    if ((err = fec_batch_encoder_drain(e, &n)) || fec_batch_encoder_backlog(e) != 0)
        return fail("drain after free", err);
    fec_batch_encoder_free(e);
    return 0;
}

static int mixed(void) {
    int err = 0;
    fec_batch_encoder *e = fec_batch_encoder_new(FEC_SCHEME_REED_SOLOMON, K, M, 16, 0, &err);
    if (!e) return fail("encoder_new", err);
    fec_repair_queue *keep = fec_repair_queue_new(2 * M), *gone = fec_repair_queue_new(M);
    for (uint64_t b = 0; b < 6; ++b)
        if ((err = submit(e, b, 700 + b, (b & 1) ? gone : keep))) return fail("submit", err);
    size_t n = 0;
    (void)fec_batch_encoder_drain(e, &n);   /* both queues overflow: frames held */
    fec_repair_queue_free(gone);
    uint64_t want = 0;
    for (int round = 0; round < 8 && want < 6; ++round) {
        uint64_t bid, pid;
        const uint8_t *p;
        size_t len, cap;
        while (fec_repair_queue_peek(keep, &bid, &pid, &p, &len, &cap)) {
            if (bid != want || len != 700 + bid + 2) return fail("kept queue order", (int)bid);
            if (pid == M - 1) want += 2;
            fec_repair_queue_pop(keep);
        }
        err = fec_batch_encoder_drain(e, &n);
        if (err && err != FEC_ERR_SCHEME) return fail("drain", err);
    }
    if (want != 6 || fec_batch_encoder_backlog(e) != 0) return fail("kept queue incomplete", (int)want);
    fec_repair_queue_free(keep);
    fec_batch_encoder_free(e);
    return 0;
}

static int decoder(void) {
    int err = 0;
    fec_scheme *s = fec_scheme_new(FEC_SCHEME_REED_SOLOMON, K, M, 0);
    fec_batch_decoder *d = fec_batch_decoder_new(FEC_SCHEME_REED_SOLOMON, K, M, 2, 0, &err);
    if (!s || !d) return fail("decoder_new", err);
    fec_recovered_queue *q = fec_recovered_queue_new();
    uint8_t pl[K][1200];
    for (uint64_t b = 0; b < 5; ++b) {
        fec_block *full = fec_block_new(b, K, M);
        for (int i = 0; i < K; ++i) {
            fill(pl[i], 1200, (uint32_t)(b * 31 + i));
            if ((err = fec_block_add_source_symbol(full, b * K + i, pl[i], 1200, 1452)))
                return fail("add source", err);
        }
        fec_frames *fr = NULL;
        if ((err = fec_scheme_repair_symbols(s, full, &fr))) return fail("repair_symbols", err);
        fec_block *rx = fec_block_new(b, K, M);
        for (int i = 1; i < K; ++i)   /* source 0 lost */
            if ((err = fec_block_add_source_symbol(rx, b * K + i, pl[i], 1200, 1452))) return fail("rx source", err);
        const uint8_t *rp;
        size_t rl;
        uint64_t bid, pid;
        if ((err = fec_frames_get(fr, 0, &bid, &pid, &rp, &rl))) return fail("frames_get", err);
        if ((err = fec_block_add_repair_symbol(rx, bid, pid, rp, rl))) return fail("rx repair", err);
        int staged = 0;
        if ((err = fec_batch_decoder_submit(d, rx, q, &staged)) || !staged) return fail("decoder submit", err);
        fec_frames_free(fr);
        fec_block_free(full);
        fec_block_free(rx);
    }
    fec_recovered_queue_free(q);   /* blocks 4 staged, 2..3 in flight, 0..1 possibly delivered */
    size_t n = 0;
    if ((err = fec_batch_decoder_poll(d, &n))) return fail("decoder poll after free", err);
    if ((err = fec_batch_decoder_drain(d, &n))) return fail("decoder drain after free", err);
    if (fec_batch_decoder_staged(d) || fec_batch_decoder_in_flight(d)) return fail("decoder not empty", 0);
    fec_batch_decoder_free(d);
    fec_scheme_free(s);
    return 0;
}

int main(void) {
    if (backlog() || inflight() || mixed() || decoder()) return 1;
    printf("ok backlog inflight mixed decoder\n");
    return 0;
}
