/*
 * fec_hip.h — C ABI of the MI355X (gfx950) FEC codec: lib0xfec_hip.so
 *
 * This is the device boundary of the reference's hot path. In ddritzenhoff/0xFEC the
 * block codes live in package internal/fec and their arithmetic is a Go call into
 * github.com/klauspost/reedsolomon v1.12.4 (go.mod:24). This library replaces that
 * arithmetic with hand-written HIP kernels; the Go side keeps its block bookkeeping and
 * binds these entry points through cgo. Signatures use only plain
 * pointers and sizes.
 *
 *   entry point                 replaces (reference file:line)
 *   --------------------------  ---------------------------------------------------------
 *   fec_rs_prepare              reedsolomon.New(k, m)       internal/fec/reed_solomon.go:16,
 *                                                           internal/fec/manager.go:60,83
 *   fec_rs_encode_batch         Encoder.Encode(shards)      internal/fec/reed_solomon.go:51
 *   fec_rs_reconstruct_batch    Encoder.ReconstructData     internal/fec/reed_solomon.go:124
 *   fec_rs_recover_batch        ReconstructData + the copy-out of recoverSymbolPayloads
 *                                                           internal/fec/reed_solomon.go:124-133
 *   fec_xor_encode_batch        xorScheme.xor loop          internal/fec/xor.go:28-33,44-56
 *   fec_xor_reconstruct_batch   xorScheme recover loops     internal/fec/xor.go:80-86
 *
 * Shard layout (all entry points). A batch is `nblocks` independent blocks of k data and m
 * parity shards. Data shard j of block b lives at  data + b*data_block_stride + j*shard_stride,
 * parity shard i at  parity + b*parity_block_stride + i*shard_stride; each is `shard_len`
 * bytes long. One interleaved [block][k+m][shard_stride] array is the special case
 * parity = data + k*shard_stride, parity_block_stride = data_block_stride. Shards are
 * (the reference's shard = payload | zero pad | big-endian uint16 length, i.e.
 * biggest+2 bytes: reed_solomon.go:70-89, xor.go:44-56). Bytes [0, shard_len) of every
 * output shard receive the result; with FEC_DEVICE, bytes [shard_len, round_up(shard_len,
 * 16)) of an output shard slot are also written, as zeros (whole 16-byte stores), and
 * nothing past that is touched. FEC_HOST writes exactly shard_len bytes per output.
 *
 * Memory kinds (`flags`):
 *   FEC_DEVICE  pointers are device memory of the ctx's device; shard_stride, block
 *               strides and base pointers must be multiples of 16, every shard slot
 *               (shard_stride bytes) must be readable; present_mask and block_status must be
 *               4-byte aligned (the kernels read masks by 4-byte scalar loads, which drop the
 *               low two address bits). The call is asynchronous on the
 *               ctx stream; per-block decode failures are reported through `block_status`
 *               (if given) and, sticky, by fec_sync().
 *   FEC_HOST    pointers are host memory with any layout; the ctx stages the batch
 *               through pinned buffers (H2D -> kernel -> D2H) and returns when done. Chunks
 *               of the batch alternate between two staging sets on two streams, so staging,
 *               transfers and kernels of neighbouring chunks overlap; only the shards the code
 *               needs cross PCIe (encode: k up, m down; reconstruct: the data shards and the
 *               parity planes the blocks read up, the rebuilt shards down).
 *   FEC_HOST_PINNED  as FEC_HOST, but the caller's buffers are pinned (hipHostMalloc) or
 *               registered (hipHostRegister): no staging copies, each shard column moves with
 *               one 2D DMA between the caller's layout and the device. fec_rs_recover_batch
 *               is FEC_DEVICE only.
 *
 * Threading: a ctx has one HIP stream and is used by one caller at a time (the
 * reference's manager is per connection and not thread-safe either: manager.go:41-48).
 * Use one ctx per device per host thread.
 */
#ifndef FEC_HIP_H
#define FEC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Return codes: 0 on success, negative on failure. */
#define FEC_OK 0
#define FEC_ERR_INVALID_ARG (-1)     /* null pointer, bad stride/length/flags */
#define FEC_ERR_INV_SHARD_NUM (-2)   /* klauspost ErrInvShardNum: k <= 0 or m < 0 */
#define FEC_ERR_MAX_SHARD_NUM (-3)   /* klauspost ErrMaxShardNum: k + m > 256 (decode: > 32) */
#define FEC_ERR_TOO_FEW_SHARDS (-4)  /* klauspost ErrTooFewShards */
#define FEC_ERR_SHARD_SIZE (-5)      /* klauspost ErrShardSize */
#define FEC_ERR_SHARD_NO_DATA (-6)   /* klauspost ErrShardNoData: shard_len == 0 */
#define FEC_ERR_ALIGNMENT (-7)       /* FEC_DEVICE layout not 16-byte aligned, or a mask / status
                                        array not 4-byte aligned */
#define FEC_ERR_HIP (-8)             /* HIP runtime failure */
#define FEC_ERR_NOMEM (-9)
#define FEC_ERR_NO_DEVICE (-10)

#define FEC_DEVICE 0
#define FEC_HOST 1
#define FEC_HOST_PINNED 2

/* Largest n = k + m the reconstruct path accepts (present masks are uint32). */
#define FEC_MAX_DECODE_SHARDS 32

typedef struct fec_ctx fec_ctx;

/* Library / device. */
const char *fec_version(void);
const char *fec_strerror(int code);
int fec_device_count(int *count);

/* Context: device binding, one HIP stream, cached code matrices, workspace, pinned staging. */
int fec_ctx_create(int device, fec_ctx **out);
void fec_ctx_destroy(fec_ctx *ctx);
/* Run subsequent work on an external hipStream_t (NULL = the device's null stream). Work the
 * ctx already queued on its previous stream is ordered before the new stream's (an event wait,
 * no host sync), since both share the ctx's workspace. */
int fec_ctx_set_stream(fec_ctx *ctx, void *hip_stream);
/* Go back to the ctx-owned stream. */
int fec_ctx_reset_stream(fec_ctx *ctx);
void *fec_ctx_stream(fec_ctx *ctx);
/* Free the host-path staging (FEC_HOST / FEC_HOST_PINNED: kHostSets = 3 sets of pinned host and
 * device buffers, each up to one 128 MiB chunk of input plus its outputs, kept by the ctx between
 * calls so that a stream of calls does not re-register memory) after the ctx's host-path work
 * has finished. The next host-path call allocates them again. No reference counterpart (the
 * reference codes in Go memory); INTEGRATION.md lists the per-ctx footprint. */
int fec_ctx_release_staging(fec_ctx *ctx);
/* Wait for the ctx stream. Returns FEC_ERR_TOO_FEW_SHARDS if any FEC_DEVICE reconstruct
 * since the last fec_sync met a block with fewer than k present shards, or
 * FEC_ERR_INVALID_ARG if a recover met a block with more erasures than output slots
 * (then clears it). */
int fec_sync(fec_ctx *ctx);

/* The n x k systematic matrix of RS(k, m) (n = k + m), row-major, host memory. No device
 * needed. Same matrix as klauspost reedsolomon.New(k, m) with default options. */
int fec_rs_matrix(int k, int m, uint8_t *out);

/* Validate (k, m) and cache the code on the ctx (klauspost New). Optional: the batch calls
 * prepare on first use. */
int fec_rs_prepare(fec_ctx *ctx, int k, int m);

/* RS encode: parity shard i of each block = XOR_j M[k+i][j] * data shard j. */
int fec_rs_encode_batch(fec_ctx *ctx, int k, int m, size_t shard_len, size_t nblocks,
                        const uint8_t *data, size_t data_block_stride,
                        uint8_t *parity, size_t parity_block_stride,
                        size_t shard_stride, int flags);

/* RS ReconstructData, in place. present_mask[b] bit i set <=> shard i of block b present
 * (shards 0..k-1 data, k..k+m-1 parity; n = k + m <= 32). For each block, every missing DATA
 * shard is rebuilt, into its own slot, from the first k present shards in index order;
 * missing parity shards are not touched; a block with no missing data shard is untouched.
 * block_status (optional, same memory kind as the masks) receives 0 or
 * FEC_ERR_TOO_FEW_SHARDS per block. FEC_HOST: returns FEC_ERR_TOO_FEW_SHARDS if any block
 * failed (the other blocks are still rebuilt). */
int fec_rs_reconstruct_batch(fec_ctx *ctx, int k, int m, size_t shard_len, size_t nblocks,
                             uint8_t *data, size_t data_block_stride,
                             const uint8_t *parity, size_t parity_block_stride,
                             size_t shard_stride, const uint32_t *present_mask,
                             int32_t *block_status, int flags);

/* Out-of-place RS recovery: the device form of reedSolomonScheme.recoverSymbolPayloads
 * (internal/fec/reed_solomon.go:92-136), whose result is the erased source payloads in
 * ascending shard order. For block b the e erased data shards are rebuilt (same arithmetic
 * as fec_rs_reconstruct_batch) into  out + b*out_block_stride + r*shard_stride, r = 0..e-1,
 * in ascending shard order; data and parity are only read. out_slots = shard slots per block
 * in `out`. block_status (optional) receives e (>= 0) or FEC_ERR_TOO_FEW_SHARDS, or
 * FEC_ERR_INVALID_ARG when e > out_slots (that block is not written). FEC_DEVICE only;
 * fec_sync() reports any failed block. */
int fec_rs_recover_batch(fec_ctx *ctx, int k, int m, size_t shard_len, size_t nblocks,
                         const uint8_t *data, size_t data_block_stride,
                         const uint8_t *parity, size_t parity_block_stride,
                         size_t shard_stride, const uint32_t *present_mask,
                         uint8_t *out, size_t out_block_stride, int out_slots,
                         int32_t *block_status, int flags);

/* XOR(k, 1) encode: parity = XOR of the k data shards. */
int fec_xor_encode_batch(fec_ctx *ctx, int k, size_t shard_len, size_t nblocks,
                         const uint8_t *data, size_t data_block_stride,
                         uint8_t *parity, size_t parity_block_stride,
                         size_t shard_stride, int flags);

/* XOR(k, 1) recovery, in place (shard k is the parity): a single missing data shard is the
 * XOR of the other k shards. Two or more missing shards with a data shard among them ->
 * FEC_ERR_TOO_FEW_SHARDS for that block. */
int fec_xor_reconstruct_batch(fec_ctx *ctx, int k, size_t shard_len, size_t nblocks,
                              uint8_t *data, size_t data_block_stride,
                              const uint8_t *parity, size_t parity_block_stride,
                              size_t shard_stride, const uint32_t *present_mask,
                              int32_t *block_status, int flags);

#ifdef __cplusplus
}
#endif
#endif /* FEC_HIP_H */
