/*
 * fec_go_threads.c — the batched Go ABI (include/fec_go.h) driven the way Go drives it: every
 * encoder and decoder is created on ONE thread (NewBatchSender / NewBatchReceiver on whatever
 * OS thread the creating goroutine runs on), then each is driven by its own connection run loop
 * (connection.go:525) whose goroutine runs on a different OS thread, concurrently with the
 * others; halfway through, the run loops swap threads (goroutine migration). Repair payloads
 * are compared with the CPU oracle (oracle/fec_oracle.c: klauspost Encode / the XOR loops over
 * framed shards, reed_solomon.go:26-68, xor.go:14-56); recovered payloads with what was sent
 * (recoverSymbolPayloads: the lost payloads in SSID order, reed_solomon.go:92-136).
 *
 *   usage: fec_go_threads <blocks per run loop> <seed>
 */
#define _DEFAULT_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "fec_go.h"
#include "../../oracle/fec_oracle.h"

#define CHECK(c, ...)                                                    \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);         \
            fprintf(stderr, __VA_ARGS__);                                \
            fprintf(stderr, " [%s]\n", fec_last_error());                \
            fflush(stderr);                                              \
            _exit(1);                                                    \
        }                                                                \
    } while (0)

static uint64_t rnd(uint64_t *s) {   /* splitmix64 */
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* One connection: its code, its encoder and decoder (created on the main thread). */
typedef struct {
    int scheme, k, m;
    size_t maxb;
    fec_go_encoder *enc;
    fec_go_decoder *dec;
    uint64_t next_id;
    int blocks_done;
} Conn;

typedef struct {
    Conn *c;
    int blocks;
    uint64_t seed;
} Job;

/* Framed shard of payload p (len n) at biggest b: p | zeros | BE16(n) (reed_solomon.go:77-87). */
static void frame(uint8_t *dst, const uint8_t *p, size_t n, size_t b) {
    memset(dst, 0, b + 2);
    if (n) memcpy(dst, p, n);
    dst[b] = (uint8_t)(n >> 8);
    dst[b + 1] = (uint8_t)(n & 0xFF);
}

/* One run loop's slice of work on connection c: `blocks` blocks sent (frames checked against
 * the oracle) and then received with losses (payloads checked against what was sent). */
static void *run_loop(void *arg) {
    Job *j = (Job *)arg;
    Conn *c = j->c;
    uint64_t s = j->seed;
    const int k = c->k, m = c->m, nb = j->blocks;
    uint8_t *pay = malloc((size_t)nb * k * 1434);
    size_t *len = malloc((size_t)nb * k * sizeof(size_t));
    uint8_t *rep = malloc((size_t)nb * m * FEC_GO_SLOT);
    uint32_t *rlen = calloc((size_t)nb, 4);
    uint64_t *ids = malloc(c->maxb * 8);
    uint32_t *rl = malloc(c->maxb * 4);
    uint8_t *rp = malloc(c->maxb * (size_t)m * FEC_GO_SLOT);
    const uint8_t **ptrs = malloc((size_t)(k + m) * sizeof *ptrs);
    const uint64_t base = c->next_id;
    int polled = 0;
    /* ---- sender: submit, poll now and then, then wait for the rest */
    for (int b = 0; b < nb; ++b) {
        const int full = (int)(rnd(&s) % 3) == 0;
        for (int i = 0; i < k; ++i) {
            size_t n = full ? 1200 : rnd(&s) % 1435;
            uint8_t *p = pay + ((size_t)b * k + i) * 1434;
            len[(size_t)b * k + i] = n;
            for (size_t t = 0; t < n; ++t) p[t] = (uint8_t)rnd(&s);
            ptrs[i] = p;
        }
        CHECK(fec_go_encoder_submit(c->enc, base + (uint64_t)b, ptrs, len + (size_t)b * k, k) == 0, "submit");
        if (rnd(&s) % 5 == 0) {
            size_t got = 0;
            CHECK(fec_go_encoder_poll(c->enc, 0, ids, rl, rp, c->maxb, &got) == 0, "poll");
            for (size_t d = 0; d < got; ++d, ++polled) {
                CHECK(ids[d] == base + (uint64_t)polled, "encoder order");
                rlen[polled] = rl[d];
                memcpy(rep + (size_t)polled * m * FEC_GO_SLOT, rp + d * (size_t)m * FEC_GO_SLOT,
                       (size_t)m * FEC_GO_SLOT);
            }
        }
    }
    while (polled < nb) {
        size_t got = 0;
        CHECK(fec_go_encoder_poll(c->enc, 1, ids, rl, rp, c->maxb, &got) == 0, "poll wait");
        CHECK(got > 0, "encoder made no progress");
        for (size_t d = 0; d < got; ++d, ++polled) {
            CHECK(ids[d] == base + (uint64_t)polled, "encoder order");
            rlen[polled] = rl[d];
            memcpy(rep + (size_t)polled * m * FEC_GO_SLOT, rp + d * (size_t)m * FEC_GO_SLOT, (size_t)m * FEC_GO_SLOT);
        }
    }
    /* frames against the oracle */
    uint8_t *sh = malloc((size_t)(k + m) * 1436);
    for (int b = 0; b < nb; ++b) {
        size_t big = 0;
        for (int i = 0; i < k; ++i) big = len[(size_t)b * k + i] > big ? len[(size_t)b * k + i] : big;
        const size_t L = big + 2;
        CHECK(rlen[b] == L, "repair length");
        for (int i = 0; i < k; ++i)
            frame(sh + (size_t)i * L, pay + ((size_t)b * k + i) * 1434, len[(size_t)b * k + i], big);
        if (c->scheme == FEC_SCHEME_XOR)
            CHECK(fo_xor_encode_batch(k, L, 1, sh, 0, sh + (size_t)k * L, 0, L, 1) == 0, "oracle");
        else
            CHECK(fo_rs_encode_batch(k, m, L, 1, sh, 0, sh + (size_t)k * L, 0, L, 1) == 0, "oracle");
        for (int i = 0; i < m; ++i)
            CHECK(!memcmp(rep + ((size_t)b * m + i) * FEC_GO_SLOT, sh + (size_t)(k + i) * L, L),
                  "repair %d of block %llu differs from the oracle", i, (unsigned long long)(base + b));
    }
    /* ---- receiver: lose 1..m sources (XOR: 1), keep every repair */
    const size_t out_cap = (size_t)c->maxb * k * 1434;
    uint8_t *out = malloc(out_cap);
    uint64_t *oid = malloc(c->maxb * 8), *off = malloc(c->maxb * 8);
    uint32_t *ol = malloc(c->maxb * 4);
    uint8_t *want = malloc((size_t)k * 1434);
    int *order = malloc((size_t)nb * sizeof(int));
    size_t *sl = malloc((size_t)k * 8), *rpl = malloc((size_t)m * 8);
    const uint8_t **rps = malloc((size_t)m * sizeof *rps);
    int staged = 0, next = 0;
    uint8_t *lost = malloc((size_t)nb * k);
    for (int b = 0; b < nb; ++b) {
        memset(lost + (size_t)b * k, 0, (size_t)k);
        const int nl = 1 + (int)(rnd(&s) % (uint64_t)(m < k ? m : k));
        for (int t = 0; t < nl;) {
            const int i = (int)(rnd(&s) % (uint64_t)k);
            if (!lost[(size_t)b * k + i]) lost[(size_t)b * k + i] = 1, ++t;
        }
        for (int i = 0; i < k; ++i) {
            ptrs[i] = lost[(size_t)b * k + i] ? NULL : pay + ((size_t)b * k + i) * 1434;
            sl[i] = len[(size_t)b * k + i];
        }
        for (int p = 0; p < m; ++p) {
            rps[p] = rep + ((size_t)b * m + p) * FEC_GO_SLOT;
            rpl[p] = rlen[b];
        }
        const uint64_t id = base + (uint64_t)b;
        int st = 0;
        CHECK(fec_go_decoder_submit(c->dec, id, id * (uint64_t)k, id * (uint64_t)k + (uint64_t)k - 1,
                                    (int)rlen[b] - 2, ptrs, sl, rps, rpl, &st) == 0 && st == 1, "decoder submit");
        order[staged++] = b;
        if (rnd(&s) % 4 == 0 || b == nb - 1) {
            const int wait = b == nb - 1;
            do {
                size_t got = 0;
                CHECK(fec_go_decoder_poll(c->dec, wait, oid, ol, off, out, out_cap, c->maxb, &got) == 0, "dpoll");
                for (size_t q = 0; q < got; ++q, ++next) {
                    const int bb = order[next];
                    CHECK(oid[q] == base + (uint64_t)bb, "decoder order");
                    size_t wl = 0;
                    for (int i = 0; i < k; ++i)
                        if (lost[(size_t)bb * k + i]) {
                            memcpy(want + wl, pay + ((size_t)bb * k + i) * 1434, len[(size_t)bb * k + i]);
                            wl += len[(size_t)bb * k + i];
                        }
                    CHECK(ol[q] == wl && !memcmp(out + off[q], want, wl), "payload of block %d", bb);
                }
                if (wait && got == 0 && next < staged) CHECK(0, "decoder made no progress");
            } while (wait && next < staged);
        }
    }
    CHECK(next == nb, "recovered %d of %d", next, nb);
    c->blocks_done += nb;
    free(pay), free(len), free(rep), free(rlen), free(ids), free(rl), free(rp), free(ptrs), free(sh), free(out),
        free(oid), free(off), free(ol), free(want), free(order), free(sl), free(rpl), free(rps), free(lost);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s blocks seed\n", argv[0]);
        return 2;
    }
    const int nb = atoi(argv[1]);
    const uint64_t seed = strtoull(argv[2], NULL, 0);
    /* two connections per shape class, all created here, on this one thread */
    Conn c[4] = {{FEC_SCHEME_REED_SOLOMON, 8, 4, 16, 0, 0, 0, 0},
                 {FEC_SCHEME_REED_SOLOMON, 20, 10, 8, 0, 0, 1u << 20, 0},
                 {FEC_SCHEME_REED_SOLOMON, 8, 4, 5, 0, 0, 2u << 20, 0},
                 {FEC_SCHEME_XOR, 2, 1, 16, 0, 0, 3u << 20, 0}};
    for (int i = 0; i < 4; ++i) {
        int rc = 0;
        c[i].enc = fec_go_encoder_new(c[i].scheme, c[i].k, c[i].m, c[i].maxb, 0, &rc);
        CHECK(c[i].enc, "encoder_new rc=%d", rc);
        c[i].dec = fec_go_decoder_new(c[i].scheme, c[i].k, c[i].m, c[i].maxb, 0, &rc);
        CHECK(c[i].dec, "decoder_new rc=%d", rc);
    }
    /* two phases: run loops on fresh threads each time (a goroutine lands on another OS thread) */
    for (int phase = 0; phase < 2; ++phase) {
        pthread_t th[4];
        Job jobs[4];
        for (int i = 0; i < 4; ++i) {
            const int ci = phase ? 3 - i : i;
            jobs[i] = (Job){&c[ci], nb, seed * 131 + (uint64_t)(phase * 4 + i)};
            CHECK(pthread_create(&th[i], NULL, run_loop, &jobs[i]) == 0, "pthread_create");
        }
        for (int i = 0; i < 4; ++i) pthread_join(th[i], NULL);
        for (int i = 0; i < 4; ++i) c[i].next_id += (uint64_t)nb;
    }
    for (int i = 0; i < 4; ++i) {
        fec_go_encoder_free(c[i].enc);
        fec_go_decoder_free(c[i].dec);
    }
    printf("ok connections=4 blocks=%d\n", c[0].blocks_done + c[1].blocks_done + c[2].blocks_done + c[3].blocks_done);
    fflush(stdout);
    fflush(stderr);
    _exit(0);   /* see fec_go_stress.c: skip the HIP runtime's finalizers under host ASan */
}
