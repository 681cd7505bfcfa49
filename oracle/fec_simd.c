/*
 * fec_simd.c — SIMD CPU restatement of klauspost/reedsolomon v1.12.4's Encode / ReconstructData
 * (TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and the CPU tests; never linked into
 * the product library).
 *
 * The reference calls klauspost at internal/fec/reed_solomon.go:51 (Encode) and :124
 * (ReconstructData); on x86 klauspost runs Go-assembly kernels selected by cpuid
 * (klauspost/cpuid/v2 v2.2.8, go.sum:64-65), not the pure-Go mulTable loop the scalar oracle
 * (fec_oracle.c) restates. The module is not vendored here, so this file restates the published
 * method of those kernels, bit-exact against fec_oracle.c (tests/test_cpu_simd.py):
 *
 *   avx2         nibble tables: c*x = PSHUFB(T_lo[c], x & 15) ^ PSHUFB(T_hi[c], x >> 4), 32 bytes
 *                per instruction (klauspost galMulAVX2 / mulAvxTwo_{k}x{m} kernels)
 *   gfni-avx2    multiplication by a constant is GF(2)-linear, so one VGF2P8AFFINEQB with the
 *   gfni-avx512  8x8 bit matrix of c per 32 / 64 bytes (klauspost mulGFNI_{k}x{m}_64 kernels)
 *
 * Both fold every input into all m output accumulators held in registers, one 32- or 64-byte
 * column at a time (the _{k}x{m} kernel shape); the tail of a shard (< one vector) runs the
 * scalar mulTable form. ReconstructData inverts the sub-matrix of the first k present shards
 * (cached per present mask, as klauspost's inversion tree caches per erasure pattern) and
 * rebuilds only the missing data shards with the same kernels.
 */
#include "fec_oracle.h"

#include <immintrin.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { FS_SCALAR = 0, FS_AVX2 = 1, FS_GFNI_AVX2 = 2, FS_GFNI_AVX512 = 3 };

static uint8_t mulc(uint8_t a, uint8_t b) { return fo_gf_mul(a, b); }

int fs_best_isa(void) {
    __builtin_cpu_init();
    if (__builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw"))
        return FS_GFNI_AVX512;
    if (__builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx2")) return FS_GFNI_AVX2;
    if (__builtin_cpu_supports("avx2")) return FS_AVX2;
    return FS_SCALAR;
}

const char *fs_isa_name(int isa) {
    switch (isa) {
        case FS_AVX2: return "avx2 (PSHUFB nibble tables)";
        case FS_GFNI_AVX2: return "gfni-avx2 (VGF2P8AFFINEQB, 32 B)";
        case FS_GFNI_AVX512: return "gfni-avx512 (VGF2P8AFFINEQB, 64 B)";
        default: return "scalar (mulTable)";
    }
}

int fs_isa_supported(int isa) {
    __builtin_cpu_init();
    switch (isa) {
        case FS_SCALAR: return 1;
        case FS_AVX2: return __builtin_cpu_supports("avx2");
        case FS_GFNI_AVX2: return __builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx2");
        case FS_GFNI_AVX512:
            return __builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512f") &&
                   __builtin_cpu_supports("avx512bw");
        default: return 0;
    }
}

/* Per-coefficient constants of one (rows x cols) coefficient matrix. */
typedef struct {
    int rows, cols;
    uint8_t *coef;       /* rows * cols */
    uint8_t *nib;        /* rows * cols * 32: T_lo[16] | T_hi[16] */
    uint64_t *aff;       /* rows * cols: VGF2P8AFFINEQB matrix of c */
} Coefs;

/* 8x8 GF(2) matrix of x -> c*x in VGF2P8AFFINEQB's layout: result bit i = parity(byte[7-i] & x),
 * so byte 7-i holds, at bit j, bit i of c * 2^j. */
static uint64_t affine_of(uint8_t c) {
    uint64_t m = 0;
    for (int i = 0; i < 8; ++i) {
        uint8_t row = 0;
        for (int j = 0; j < 8; ++j)
            if (mulc(c, (uint8_t)(1u << j)) >> i & 1u) row |= (uint8_t)(1u << j);
        m |= (uint64_t)row << (8 * (7 - i));
    }
    return m;
}

static void coefs_init(Coefs *cf, int rows, int cols, const uint8_t *coef) {
    cf->rows = rows;
    cf->cols = cols;
    cf->coef = (uint8_t *)malloc((size_t)rows * cols);
    cf->nib = (uint8_t *)aligned_alloc(64, ((size_t)rows * cols * 32 + 127) & ~(size_t)63);   /* C11: size a multiple of the alignment */
    cf->aff = (uint64_t *)malloc((size_t)rows * cols * 8);
    memcpy(cf->coef, coef, (size_t)rows * cols);
    for (int i = 0; i < rows * cols; ++i) {
        const uint8_t c = coef[i];
        for (int x = 0; x < 16; ++x) {
            cf->nib[i * 32 + x] = mulc(c, (uint8_t)x);
            cf->nib[i * 32 + 16 + x] = mulc(c, (uint8_t)(x << 4));
        }
        cf->aff[i] = affine_of(c);
    }
}

static void coefs_free(Coefs *cf) {
    free(cf->coef);
    free(cf->nib);
    free(cf->aff);
}

/* out[r] (= or ^=) sum_c coef[r][c] * in[c] over bytes [from, len), scalar mulTable form. */
static void code_scalar(const Coefs *cf, const uint8_t *const *in, uint8_t *const *out, size_t from, size_t len) {
    for (int r = 0; r < cf->rows; ++r) {
        uint8_t *o = out[r];
        for (size_t x = from; x < len; ++x) o[x] = 0;
        for (int c = 0; c < cf->cols; ++c) {
            const uint8_t k = cf->coef[r * cf->cols + c];
            const uint8_t *i = in[c];
            for (size_t x = from; x < len; ++x) o[x] ^= mulc(k, i[x]);
        }
    }
}

#define FS_MAXR 32

/* The kernels keep all R output accumulators in registers (klauspost's fixed-shape _{k}x{m}
 * kernels): each body is written once with R a parameter and instantiated for R = 1..8 by
 * always-inlined calls with constant R; other R run the same body with R = FS_MAXR storage. */
#define FS_INLINE static inline __attribute__((always_inline))

__attribute__((target("avx2"))) FS_INLINE size_t body_avx2(const Coefs *cf, const uint8_t *const *in,
                                                           uint8_t *const *out, size_t len, const int R) {
    const __m256i low = _mm256_set1_epi8(0x0F);
    const size_t n = len & ~(size_t)31;
    const int C = cf->cols;
    for (size_t x = 0; x < n; x += 32) {
        __m256i acc[FS_MAXR];
        for (int r = 0; r < R; ++r) acc[r] = _mm256_setzero_si256();
        for (int c = 0; c < C; ++c) {
            const __m256i v = _mm256_loadu_si256((const __m256i *)(in[c] + x));
            const __m256i lo = _mm256_and_si256(v, low);
            const __m256i hi = _mm256_and_si256(_mm256_srli_epi64(v, 4), low);
            for (int r = 0; r < R; ++r) {
                const uint8_t *t = cf->nib + (size_t)(r * C + c) * 32;
                const __m256i tl = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i *)t));
                const __m256i th = _mm256_broadcastsi128_si256(_mm_load_si128((const __m128i *)(t + 16)));
                acc[r] = _mm256_xor_si256(acc[r], _mm256_xor_si256(_mm256_shuffle_epi8(tl, lo), _mm256_shuffle_epi8(th, hi)));
            }
        }
        for (int r = 0; r < R; ++r) _mm256_storeu_si256((__m256i *)(out[r] + x), acc[r]);
    }
    return n;
}

__attribute__((target("avx2,gfni"))) FS_INLINE size_t body_gfni256(const Coefs *cf, const uint8_t *const *in,
                                                                   uint8_t *const *out, size_t len, const int R) {
    const size_t n = len & ~(size_t)31;
    const int C = cf->cols;
    for (size_t x = 0; x < n; x += 32) {
        __m256i acc[FS_MAXR];
        for (int r = 0; r < R; ++r) acc[r] = _mm256_setzero_si256();
        for (int c = 0; c < C; ++c) {
            const __m256i v = _mm256_loadu_si256((const __m256i *)(in[c] + x));
            for (int r = 0; r < R; ++r) {
                const __m256i a = _mm256_set1_epi64x((long long)cf->aff[r * C + c]);
                acc[r] = _mm256_xor_si256(acc[r], _mm256_gf2p8affine_epi64_epi8(v, a, 0));
            }
        }
        for (int r = 0; r < R; ++r) _mm256_storeu_si256((__m256i *)(out[r] + x), acc[r]);
    }
    return n;
}

__attribute__((target("avx512f,avx512bw,gfni"))) FS_INLINE size_t body_gfni512(const Coefs *cf, const uint8_t *const *in,
                                                                               uint8_t *const *out, size_t len,
                                                                               const int R) {
    const size_t n = len & ~(size_t)63;
    const int C = cf->cols;
    for (size_t x = 0; x < n; x += 64) {
        __m512i acc[FS_MAXR];
        for (int r = 0; r < R; ++r) acc[r] = _mm512_setzero_si512();
        for (int c = 0; c < C; ++c) {
            const __m512i v = _mm512_loadu_si512((const void *)(in[c] + x));
            for (int r = 0; r < R; ++r) {
                const __m512i a = _mm512_set1_epi64((long long)cf->aff[r * C + c]);
                acc[r] = _mm512_xor_si512(acc[r], _mm512_gf2p8affine_epi64_epi8(v, a, 0));
            }
        }
        for (int r = 0; r < R; ++r) _mm512_storeu_si512((void *)(out[r] + x), acc[r]);
    }
    return n;
}

#define FS_DISPATCH(NAME, TGT)                                                                               \
    __attribute__((target(TGT))) static size_t NAME(const Coefs *cf, const uint8_t *const *in,              \
                                                    uint8_t *const *out, size_t len) {                       \
        switch (cf->rows) {                                                                                  \
            case 1: return body_##NAME(cf, in, out, len, 1);                                                 \
            case 2: return body_##NAME(cf, in, out, len, 2);                                                 \
            case 3: return body_##NAME(cf, in, out, len, 3);                                                 \
            case 4: return body_##NAME(cf, in, out, len, 4);                                                 \
            case 5: return body_##NAME(cf, in, out, len, 5);                                                 \
            case 6: return body_##NAME(cf, in, out, len, 6);                                                 \
            case 7: return body_##NAME(cf, in, out, len, 7);                                                 \
            case 8: return body_##NAME(cf, in, out, len, 8);                                                 \
            default: return body_##NAME(cf, in, out, len, cf->rows);                                         \
        }                                                                                                    \
    }
FS_DISPATCH(avx2, "avx2")
FS_DISPATCH(gfni256, "avx2,gfni")
FS_DISPATCH(gfni512, "avx512f,avx512bw,gfni")

/* out[r] = sum_c coef[r][c] * in[c] over [0, len): the vector body, then the scalar tail. */
static void code_some(const Coefs *cf, const uint8_t *const *in, uint8_t *const *out, size_t len, int isa) {
    size_t done = 0;
    if (cf->rows <= FS_MAXR) {
        if (isa == FS_GFNI_AVX512) done = gfni512(cf, in, out, len);
        else if (isa == FS_GFNI_AVX2) done = gfni256(cf, in, out, len);
        else if (isa == FS_AVX2) done = avx2(cf, in, out, len);
    }
    code_scalar(cf, in, out, done, len);
}

static void set_threads(int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
}

int fs_rs_encode_batch(int k, int m, size_t len, size_t nblocks, const uint8_t *data, size_t data_bs,
                       uint8_t *parity, size_t parity_bs, size_t ss, int threads, int isa) {
    if (k <= 0 || m <= 0 || k + m > 256 || m > FS_MAXR || !fs_isa_supported(isa)) return -1;
    uint8_t *mat = (uint8_t *)malloc((size_t)(k + m) * k);
    if (!mat || fo_build_matrix(k, k + m, mat) != 0) {
        free(mat);
        return -1;
    }
    Coefs cf;
    coefs_init(&cf, m, k, mat + (size_t)k * k);
    set_threads(threads);
#pragma omp parallel for schedule(static)
    for (long long b = 0; b < (long long)nblocks; ++b) {
        const uint8_t *in[256];
        uint8_t *out[FS_MAXR];
        for (int j = 0; j < k; ++j) in[j] = data + (size_t)b * data_bs + (size_t)j * ss;
        for (int i = 0; i < m; ++i) out[i] = parity + (size_t)b * parity_bs + (size_t)i * ss;
        code_some(&cf, in, out, len, isa);
    }
    coefs_free(&cf);
    free(mat);
    return 0;
}

/* Decode matrices cached per present mask (klauspost's inversion tree caches per erasure
 * pattern): a per-thread direct-mapped cache. */
#define FS_CACHE 64
typedef struct {
    uint32_t mask;
    int valid;
    Coefs cf;          /* rows = missing data shards, cols = k (the first k present shards) */
    int idx[32];       /* the first k present shards */
    int miss[32];      /* the missing data shards */
} DecEntry;

int fs_rs_reconstruct_batch(int k, int m, size_t len, size_t nblocks, uint8_t *shards, size_t bs, size_t ss,
                            const uint32_t *present_mask, int32_t *status, int threads, int isa) {
    const int n = k + m;
    if (k <= 0 || m <= 0 || n > 32 || !fs_isa_supported(isa)) return -1;
    uint8_t *mat = (uint8_t *)malloc((size_t)n * k);
    if (!mat || fo_build_matrix(k, n, mat) != 0) {
        free(mat);
        return -1;
    }
    int failed = 0;
    set_threads(threads);
#pragma omp parallel reduction(| : failed)
    {
        DecEntry *cache = (DecEntry *)calloc(FS_CACHE, sizeof(DecEntry));
        uint8_t *tmp = (uint8_t *)malloc((size_t)FS_MAXR * (len + 64));
#pragma omp for schedule(static)
        for (long long b = 0; b < (long long)nblocks; ++b) {
            const uint32_t mask = present_mask[b] & (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u));
            uint8_t *blk = shards + (size_t)b * bs;
            const int present = __builtin_popcount(mask);
            const int data_present = __builtin_popcount(mask & ((1u << k) - 1u));
            if (status) status[b] = 0;
            if (data_present == k) continue;
            if (present < k) {
                if (status) status[b] = -1;
                failed = 1;
                continue;
            }
            DecEntry *e = &cache[(mask * 2654435761u) >> 26];
            if (!e->valid || e->mask != mask) {
                if (e->valid) coefs_free(&e->cf);
                e->valid = 0;
                int cnt = 0, nm = 0;
                for (int i = 0; i < n && cnt < k; ++i)
                    if (mask >> i & 1u) e->idx[cnt++] = i;
                for (int i = 0; i < k; ++i)
                    if (!(mask >> i & 1u)) e->miss[nm++] = i;
                uint8_t sub[32 * 32], rows[32 * 32];
                for (int r = 0; r < k; ++r) memcpy(sub + r * k, mat + (size_t)e->idx[r] * k, k);
                if (fo_invert(k, sub) != 0) {
                    if (status) status[b] = -1;
                    failed = 1;
                    continue;
                }
                for (int r = 0; r < nm; ++r) memcpy(rows + r * k, sub + (size_t)e->miss[r] * k, k);
                coefs_init(&e->cf, nm, k, rows);
                e->mask = mask;
                e->valid = 1;
            }
            const uint8_t *in[32];
            uint8_t *out[FS_MAXR];
            for (int c = 0; c < k; ++c) in[c] = blk + (size_t)e->idx[c] * ss;
            for (int r = 0; r < e->cf.rows; ++r) out[r] = tmp + (size_t)r * (len + 64);
            code_some(&e->cf, in, out, len, isa);   /* into scratch: outputs must not alias inputs */
            for (int r = 0; r < e->cf.rows; ++r) memcpy(blk + (size_t)e->miss[r] * ss, out[r], len);
        }
        for (int i = 0; i < FS_CACHE; ++i)
            if (cache[i].valid) coefs_free(&cache[i].cf);
        free(cache);
        free(tmp);
    }
    free(mat);
    return failed ? -1 : 0;
}
