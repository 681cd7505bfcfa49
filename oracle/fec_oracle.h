/*
 * fec_oracle.h — CPU restatement of the reference's FEC arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product path (0xfec_amd/) may link,
 * load or call this. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * What it restates:
 *   - github.com/klauspost/reedsolomon v1.12.4 (go.mod:24, go.sum:66-67; NOT vendored in
 *     /root/reference, restated from its published algorithm): GF(2^8) with poly 0x11D and
 *     generator 2, buildMatrix = vandermonde(n,k) * inv(top k x k), Encode, ReconstructData
 *     (first k present shards in index order, invert that k x k sub-matrix, rebuild only the
 *     missing data shards).
 *   - the byte loops of the reference's XOR scheme (internal/fec/xor.go:44-56, :58-63).
 *
 * Parity pinning: checked against the golden vectors held in
 *   internal/fec/reed_solomon_test.go:46-88, :89-201, :267-356, :373-400 and
 *   internal/fec/xor_test.go:20-143, :218-266 (tests/golden/, tests/test_oracle_golden.py).
 */
#ifndef FEC_ORACLE_H
#define FEC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* GF(2^8) primitives (klauspost galois.go semantics). */
uint8_t fo_gf_mul(uint8_t a, uint8_t b);
uint8_t fo_gf_div(uint8_t a, uint8_t b); /* b != 0 */
uint8_t fo_gf_exp(uint8_t a, int n);

/* Invert an n x n GF(2^8) matrix in place (row-major). Returns 0, or -1 if singular. */
int fo_invert(int n, uint8_t *m);

/* klauspost buildMatrix(k, n): writes the n x k systematic encoding matrix (row-major).
 * Returns 0 or -1 on bad shape / singular top. */
int fo_build_matrix(int k, int n, uint8_t *out);

/* Batched Encode over blocks laid out as
 *   data shard j of block b  at data   + b*data_bs   + j*ss
 *   parity shard i of block b at parity + b*parity_bs + i*ss
 * each shard `len` bytes. `threads` <= 0 means "all cores" (OpenMP). Returns 0 or -1. */
int fo_rs_encode_batch(int k, int m, size_t len, size_t nblocks,
                       const uint8_t *data, size_t data_bs,
                       uint8_t *parity, size_t parity_bs, size_t ss, int threads);

/* Batched ReconstructData, in place over shards[b*bs + i*ss] (n = k+m shards per block).
 * present_mask[b] bit i set <=> shard i is present. Missing DATA shards are rebuilt from the
 * first k present shards (klauspost semantics). Missing parity shards are left untouched.
 * Per block status (optional, may be NULL): 0 ok, -1 too few shards.
 * Returns 0 if every block succeeded, -1 otherwise. */
int fo_rs_reconstruct_batch(int k, int m, size_t len, size_t nblocks,
                            uint8_t *shards, size_t bs, size_t ss,
                            const uint32_t *present_mask, int32_t *status, int threads);

/* XOR (k,1): parity = XOR of the k data shards (xor.go:44-56 over framed shards). */
int fo_xor_encode_batch(int k, size_t len, size_t nblocks,
                        const uint8_t *data, size_t data_bs,
                        uint8_t *parity, size_t parity_bs, size_t ss, int threads);

/* XOR (k,1) recovery: the single missing data shard = XOR of the other k present shards
 * (xor.go:66-104). Blocks with no missing data shard are untouched; more than one missing
 * shard, or a missing parity together with a missing data shard -> status -1. */
int fo_xor_reconstruct_batch(int k, size_t len, size_t nblocks,
                             uint8_t *shards, size_t bs, size_t ss,
                             const uint32_t *present_mask, int32_t *status, int threads);

/* fec_simd.c: klauspost's SIMD kernel methods restated (cpu_baseline of bench.py). isa: 0 scalar,
 * 1 avx2 (PSHUFB nibble tables), 2 gfni-avx2, 3 gfni-avx512 (VGF2P8AFFINEQB). Same arguments and
 * results as fo_rs_encode_batch / fo_rs_reconstruct_batch; -1 if the CPU lacks the ISA. */
int fs_best_isa(void);
int fs_isa_supported(int isa);
const char *fs_isa_name(int isa);
int fs_rs_encode_batch(int k, int m, size_t len, size_t nblocks, const uint8_t *data, size_t data_bs,
                       uint8_t *parity, size_t parity_bs, size_t ss, int threads, int isa);
int fs_rs_reconstruct_batch(int k, int m, size_t len, size_t nblocks, uint8_t *shards, size_t bs, size_t ss,
                            const uint32_t *present_mask, int32_t *status, int threads, int isa);

#ifdef __cplusplus
}
#endif
#endif
