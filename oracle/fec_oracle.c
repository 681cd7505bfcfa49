/*
 * fec_oracle.c — CPU restatement of the reference FEC arithmetic (TEST INFRASTRUCTURE ONLY).
 *
 * Never linked into the product library. See fec_oracle.h for scope and pinning.
 *
 * Sources restated (reference = /root/reference, ddritzenhoff/0xFEC @ 2025-03-07):
 *   internal/fec/reed_solomon.go:16,51,124  call sites of klauspost reedsolomon.New / Encode /
 *                                           ReconstructData (v1.12.4, go.mod:24, not vendored):
 *     - galois field: poly x^8+x^4+x^3+x^2+1 (0x11D), generator 2 (klauspost galois.go)
 *     - buildMatrix: vandermonde(n, k)[r][c] = r^c, times the inverse of its top k x k
 *     - Encode:      parity[i] = XOR_j M[k+i][j] * data[j]   (pure-Go galMulSlice(Xor) form:
 *                                                            one 256-entry row of mulTable per
 *                                                            coefficient)
 *     - ReconstructData: rows of M for the first k present shards -> invert -> rebuild only the
 *                        missing data shards.
 *   internal/fec/xor.go:44-56 (xor), :58-63 (xorRepair): byte-wise XOR.
 */
#include "fec_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static uint8_t g_log[256];
static uint8_t g_exp[512];
static uint8_t g_mul[256][256];
static int g_init = 0;

static void fo_init(void) {
    if (g_init) return;
    /* exp/log tables over 0x11D with generator 2 */
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
        g_exp[i] = (uint8_t)x;
        g_exp[i + 255] = (uint8_t)x;
        g_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    g_exp[510] = g_exp[0];
    g_exp[511] = g_exp[1];
    g_log[0] = 0; /* unused: callers special-case zero */
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            g_mul[a][b] = (a == 0 || b == 0) ? 0 : g_exp[g_log[a] + g_log[b]];
    g_init = 1;
}

__attribute__((constructor)) static void fo_ctor(void) { fo_init(); }

uint8_t fo_gf_mul(uint8_t a, uint8_t b) { return g_mul[a][b]; }

uint8_t fo_gf_div(uint8_t a, uint8_t b) {
    if (a == 0) return 0;
    int d = (int)g_log[a] - (int)g_log[b];
    if (d < 0) d += 255;
    return g_exp[d];
}

/* klauspost galExp: n == 0 -> 1 (even for a == 0), a == 0 -> 0, else exp[(log a * n) mod 255]. */
uint8_t fo_gf_exp(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    int l = ((int)g_log[a] * n) % 255;
    return g_exp[l];
}

/* Gauss-Jordan on [M | I]; the inverse is unique, so pivot order does not affect the result. */
int fo_invert(int n, uint8_t *m) {
    int w = 2 * n;
    uint8_t *a = (uint8_t *)calloc((size_t)n * w, 1);
    if (!a) return -1;
    for (int r = 0; r < n; ++r) {
        memcpy(a + (size_t)r * w, m + (size_t)r * n, n);
        a[(size_t)r * w + n + r] = 1;
    }
    for (int col = 0; col < n; ++col) {
        int piv = -1;
        for (int r = col; r < n; ++r)
            if (a[(size_t)r * w + col]) { piv = r; break; }
        if (piv < 0) { free(a); return -1; }
        if (piv != col)
            for (int c = 0; c < w; ++c) {
                uint8_t t = a[(size_t)piv * w + c];
                a[(size_t)piv * w + c] = a[(size_t)col * w + c];
                a[(size_t)col * w + c] = t;
            }
        uint8_t inv = fo_gf_div(1, a[(size_t)col * w + col]);
        for (int c = 0; c < w; ++c) a[(size_t)col * w + c] = g_mul[inv][a[(size_t)col * w + c]];
        for (int r = 0; r < n; ++r) {
            if (r == col) continue;
            uint8_t f = a[(size_t)r * w + col];
            if (!f) continue;
            for (int c = 0; c < w; ++c) a[(size_t)r * w + c] ^= g_mul[f][a[(size_t)col * w + c]];
        }
    }
    for (int r = 0; r < n; ++r) memcpy(m + (size_t)r * n, a + (size_t)r * w + n, n);
    free(a);
    return 0;
}

int fo_build_matrix(int k, int n, uint8_t *out) {
    if (k <= 0 || n < k || n > 256) return -1;
    uint8_t *vm = (uint8_t *)malloc((size_t)n * k);
    uint8_t *top = (uint8_t *)malloc((size_t)k * k);
    if (!vm || !top) { free(vm); free(top); return -1; }
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) vm[(size_t)r * k + c] = fo_gf_exp((uint8_t)r, c);
    memcpy(top, vm, (size_t)k * k);
    if (fo_invert(k, top) != 0) { free(vm); free(top); return -1; }
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int t = 0; t < k; ++t) acc ^= g_mul[vm[(size_t)r * k + t]][top[(size_t)t * k + c]];
            out[(size_t)r * k + c] = acc;
        }
    free(vm);
    free(top);
    return 0;
}

/* out ^= c * in over len bytes (galMulSliceXor, generic form). */
static void mul_slice_xor(uint8_t c, const uint8_t *in, uint8_t *out, size_t len) {
    const uint8_t *row = g_mul[c];
    for (size_t i = 0; i < len; ++i) out[i] ^= row[in[i]];
}

static void set_threads(int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
}

int fo_rs_encode_batch(int k, int m, size_t len, size_t nblocks,
                       const uint8_t *data, size_t data_bs,
                       uint8_t *parity, size_t parity_bs, size_t ss, int threads) {
    if (k <= 0 || m <= 0 || k + m > 256) return -1;
    uint8_t *mat = (uint8_t *)malloc((size_t)(k + m) * k);
    if (!mat || fo_build_matrix(k, k + m, mat) != 0) { free(mat); return -1; }
    set_threads(threads);
#pragma omp parallel for schedule(static)
    for (long long b = 0; b < (long long)nblocks; ++b) {
        const uint8_t *d = data + (size_t)b * data_bs;
        uint8_t *p = parity + (size_t)b * parity_bs;
        for (int i = 0; i < m; ++i) {
            uint8_t *out = p + (size_t)i * ss;
            memset(out, 0, len);
            for (int j = 0; j < k; ++j) mul_slice_xor(mat[(size_t)(k + i) * k + j], d + (size_t)j * ss, out, len);
        }
    }
    free(mat);
    return 0;
}

int fo_rs_reconstruct_batch(int k, int m, size_t len, size_t nblocks,
                            uint8_t *shards, size_t bs, size_t ss,
                            const uint32_t *present_mask, int32_t *status, int threads) {
    int n = k + m;
    if (k <= 0 || m <= 0 || n > 32) return -1;
    uint8_t *mat = (uint8_t *)malloc((size_t)n * k);
    if (!mat || fo_build_matrix(k, n, mat) != 0) { free(mat); return -1; }
    int failed = 0;
    set_threads(threads);
#pragma omp parallel for schedule(static) reduction(| : failed)
    for (long long b = 0; b < (long long)nblocks; ++b) {
        uint32_t mask = present_mask[b];
        uint8_t *blk = shards + (size_t)b * bs;
        int present = 0, data_present = 0;
        for (int i = 0; i < n; ++i)
            if (mask >> i & 1u) { present++; if (i < k) data_present++; }
        if (status) status[b] = 0;
        if (data_present == k) continue;          /* nothing to rebuild */
        if (present < k) { if (status) status[b] = -1; failed = 1; continue; }
        /* first k present shards, in index order */
        int idx[32];
        int cnt = 0;
        for (int i = 0; i < n && cnt < k; ++i)
            if (mask >> i & 1u) idx[cnt++] = i;
        uint8_t sub[32 * 32];
        for (int r = 0; r < k; ++r) memcpy(sub + r * k, mat + (size_t)idx[r] * k, k);
        if (fo_invert(k, sub) != 0) { if (status) status[b] = -1; failed = 1; continue; }
        for (int i = 0; i < k; ++i) {
            if (mask >> i & 1u) continue;
            /* rebuilt into a scratch buffer first: outputs must not alias inputs */
            uint8_t *tmp = (uint8_t *)calloc(len ? len : 1, 1);
            for (int c = 0; c < k; ++c) mul_slice_xor(sub[i * k + c], blk + (size_t)idx[c] * ss, tmp, len);
            memcpy(blk + (size_t)i * ss, tmp, len);
            free(tmp);
        }
    }
    free(mat);
    return failed ? -1 : 0;
}

int fo_xor_encode_batch(int k, size_t len, size_t nblocks,
                        const uint8_t *data, size_t data_bs,
                        uint8_t *parity, size_t parity_bs, size_t ss, int threads) {
    if (k <= 0) return -1;
    set_threads(threads);
#pragma omp parallel for schedule(static)
    for (long long b = 0; b < (long long)nblocks; ++b) {
        const uint8_t *d = data + (size_t)b * data_bs;
        uint8_t *p = parity + (size_t)b * parity_bs;
        memset(p, 0, len);
        for (int j = 0; j < k; ++j)
            for (size_t i = 0; i < len; ++i) p[i] ^= d[(size_t)j * ss + i];
    }
    return 0;
}

int fo_xor_reconstruct_batch(int k, size_t len, size_t nblocks,
                             uint8_t *shards, size_t bs, size_t ss,
                             const uint32_t *present_mask, int32_t *status, int threads) {
    if (k <= 0 || k + 1 > 32) return -1;
    int n = k + 1, failed = 0;
    set_threads(threads);
#pragma omp parallel for schedule(static) reduction(| : failed)
    for (long long b = 0; b < (long long)nblocks; ++b) {
        uint32_t mask = present_mask[b];
        uint8_t *blk = shards + (size_t)b * bs;
        int missing = -1, nmiss = 0;
        for (int i = 0; i < n; ++i)
            if (!(mask >> i & 1u)) { nmiss++; missing = i; }
        if (status) status[b] = 0;
        if (nmiss == 0 || (nmiss == 1 && missing == k)) continue;
        if (nmiss > 1) { if (status) status[b] = -1; failed = 1; continue; }
        uint8_t *out = blk + (size_t)missing * ss;
        memset(out, 0, len);
        for (int j = 0; j < n; ++j) {
            if (j == missing) continue;
            for (size_t i = 0; i < len; ++i) out[i] ^= blk[(size_t)j * ss + i];
        }
    }
    return failed ? -1 : 0;
}
