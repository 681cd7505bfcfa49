/*
 * fec_go.h — the batched C ABI the Go package binds (go/internal/fec/batch_hip.go), exported
 * from lib0xfec_hip.so.
 *
 * The reference encodes one block at a time inside the packet packer (packet_packer.go:1005 ->
 * manager.go:145 -> reed_solomon.go:51) and recovers one block at a time in the receive path
 * (connection.go:1342 -> manager.go:182 -> reed_solomon.go:124). On the GPU the win is in
 * batches, so these entry points take a Go block's payloads one Go pointer per call (a pointer
 * to memory without Go pointers: legal cgo with no pinning), copy them at once and keep
 * nothing; complete / recoverable blocks are coded in batches and handed back into
 * caller-owned buffers. The Go side keeps its own block bookkeeping (block.go, manager.go); no
 * C++ mirror object crosses the boundary.
 *
 *   entry point                 replaces (reference file:line)
 *   --------------------------  ---------------------------------------------------------------
 *   fec_go_encoder_add/_commit  repairSymbols for one complete block    reed_solomon.go:26-68,
 *                                                                       xor.go:14-56
 *   fec_go_encoder_submit       the same with the k payload pointers in one C array (Go 1.21
 *                               runtime.Pinner pins the payloads for the call; the array itself
 *                               must be C memory)
 *   fec_go_encoder_submit_ref   the same by reference, for payloads in a registered pool
 *                               (fec_go_pool_new): the device gathers them, no host copy
 *   fec_go_encoder_poll         the frames repairSymbols returns, for every completed block
 *   fec_go_decoder_add_*        block.addSourceSymbol / addRepairSymbol  block.go:56-85
 *   fec_go_decoder_commit       recoverSymbolPayloads for one recoverable block
 *                                                                       reed_solomon.go:92-136,
 *                                                                       xor.go:66-104
 *   fec_go_decoder_submit       the same straight from the Go block's state and payload
 *                               pointers (runtime.Pinner, as fec_go_encoder_submit): no
 *                               add_* calls, nothing retained after the call
 *   fec_go_decoder_submit_ref   the same by reference, for received payloads in a registered
 *                               pool: the device gathers them, no host copy (RS)
 *   fec_go_decoder_poll         the payload recoverSymbolPayloads returns, per recovered block
 *
 * Errors: 0, FEC_ERR_SCHEME with the reference's text in fec_last_error() (fec_scheme.h), or a
 * fec_hip.h code. An encoder / decoder is used by one goroutine at a time (the reference's
 * manager is per connection and not thread-safe, manager.go:41-48); that goroutine may move
 * between OS threads from call to call. Each encoder / decoder owns its fec_ctx (stream,
 * workspace, sticky device error), so different ones may be driven concurrently from any
 * threads, whichever thread created them.
 */
#ifndef FEC_GO_H
#define FEC_GO_H

#include <stddef.h>
#include <stdint.h>

#include "fec_scheme.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Repair payload slot of the poll buffers: a packet buffer (protocol.MaxPacketBufferSize). */
#define FEC_GO_SLOT 1452

typedef struct fec_go_encoder fec_go_encoder;
typedef struct fec_go_decoder fec_go_decoder;

/* scheme_id FEC_SCHEME_REED_SOLOMON (k, m) or FEC_SCHEME_XOR (k, 1); max_blocks per batch. */
fec_go_encoder *fec_go_encoder_new(int scheme_id, int k, int m, size_t max_blocks, int device, int *err);
void fec_go_encoder_free(fec_go_encoder *e);
/* Source payload `index` (0..k-1, SSID order) of block `block_id`, copied now. */
int fec_go_encoder_add(fec_go_encoder *e, uint64_t block_id, int index, const uint8_t *payload, size_t len);
/* All k payloads added: validate exactly as repairSymbols (completeness, then size) and stage. */
int fec_go_encoder_commit(fec_go_encoder *e, uint64_t block_id);
/* add x k + commit in one call; payloads[i] pinned by the caller for the call's duration. */
int fec_go_encoder_submit(fec_go_encoder *e, uint64_t block_id, const uint8_t *const *payloads, const size_t *lens,
                          int count);
/* Registered packet buffers (opt-in; buffer_pool.go:87 allocates each packet buffer as
 * make([]byte, 0, protocol.MaxPacketBufferSize), and packet_packer.go:984 each source-symbol
 * payload likewise): nbuf buffers of FEC_GO_POOL_SLOT bytes, back to back from *base, in pinned
 * host memory mapped into the GPU's address space. Memory without Go pointers: Go slices it with
 * unsafe.Slice. fec_go_pool_free stops new references at once; the memory is released when the
 * last batch that reads it completes. */
#define FEC_GO_POOL_SLOT 1456
typedef struct fec_go_pool fec_go_pool;
fec_go_pool *fec_go_pool_new(size_t nbuf, uint8_t **base, int *err);
void fec_go_pool_free(fec_go_pool *p);
/* fec_go_encoder_submit by reference: a payload lying in a pool is not copied; the device reads
 * and frames it when the batch is coded, so the caller keeps it unchanged until poll returns
 * block_id. Payloads elsewhere are copied now. Same checks and errors as fec_go_encoder_submit. */
int fec_go_encoder_submit_ref(fec_go_encoder *e, uint64_t block_id, const uint8_t *const *payloads,
                              const size_t *lens, int count);
/* Start coding the staged blocks (asynchronous). */
int fec_go_encoder_flush(fec_go_encoder *e);
/* Completed blocks, in commit order, up to max_blocks: block_ids[d], repair_len[d] (= its
 * biggest + 2), repair payload i of block d at repairs + (d * m + i) * FEC_GO_SLOT. wait != 0:
 * flush and wait for every staged block first; wait == 0: never blocks, and starts coding the
 * staged blocks when no batch is in flight (so a block never waits for a full batch).
 * *nblocks = blocks written; the rest stay for a later poll. */
int fec_go_encoder_poll(fec_go_encoder *e, int wait, uint64_t *block_ids, uint32_t *repair_len, uint8_t *repairs,
                        size_t max_blocks, size_t *nblocks);

fec_go_decoder *fec_go_decoder_new(int scheme_id, int k, int m, size_t max_blocks, int device, int *err);
void fec_go_decoder_free(fec_go_decoder *d);
/* A SOURCE_SYMBOL / REPAIR payload of block `block_id`, copied now, with block.go's rules
 * (range check, duplicates ignored, biggest updated / overwritten by len - 2). */
int fec_go_decoder_add_source(fec_go_decoder *d, uint64_t block_id, uint64_t ssid, const uint8_t *payload,
                              size_t len);
int fec_go_decoder_add_repair(fec_go_decoder *d, uint64_t block_id, uint64_t parity_id, const uint8_t *payload,
                              size_t len);
/* The block is recoverable: validate exactly as recoverSymbolPayloads and stage it, dropping the
 * block's payloads; *staged = 0 when it is already complete (the reference's nil, nil). */
int fec_go_decoder_commit(fec_go_decoder *d, uint64_t block_id, int *staged);
/* add_* + commit in one call from the Go block (block.go:10-20): sources[i] = the payload of
 * SSID smallest_ssid + i or NULL when absent (k entries), repairs[p] = the payload of ParityID p
 * or NULL (m entries), biggest = biggestSourceSymbolLenSoFar. Source payloads are read as
 * packet buffers (capacity FEC_GO_SLOT, fec_source_symbol_frame.go:34). */
int fec_go_decoder_submit(fec_go_decoder *d, uint64_t block_id, uint64_t smallest_ssid, uint64_t largest_ssid,
                          int biggest, const uint8_t *const *sources, const size_t *source_lens,
                          const uint8_t *const *repairs, const size_t *repair_lens, int *staged);
/* fec_go_decoder_submit by reference (RS decoders): a present source (at most `biggest` bytes)
 * or repair payload lying in a registered pool (fec_go_pool_new) is validated now but read by the
 * device when the batch is coded, so the caller keeps it unchanged until poll returns block_id.
 * Payloads elsewhere, and XOR decoders, are copied now. Same checks and errors as
 * fec_go_decoder_submit. */
int fec_go_decoder_submit_ref(fec_go_decoder *d, uint64_t block_id, uint64_t smallest_ssid, uint64_t largest_ssid,
                              int biggest, const uint8_t *const *sources, const size_t *source_lens,
                              const uint8_t *const *repairs, const size_t *repair_lens, int *staged);
/* Forget a block without recovering it (complete, or given up). */
void fec_go_decoder_drop(fec_go_decoder *d, uint64_t block_id);
int fec_go_decoder_flush(fec_go_decoder *d);
/* Recovered blocks, in commit order: block_ids[d], its payload (recoverSymbolPayloads' result)
 * at out + offsets[d], lens[d] bytes; stops before max_blocks or when out_cap would overflow.
 * wait as fec_go_encoder_poll.
 * When the next payload alone is larger than out_cap: FEC_ERR_INVALID_ARG with the needed size
 * in fec_last_error(), nothing is taken (poll again with a larger buffer). */
int fec_go_decoder_poll(fec_go_decoder *d, int wait, uint64_t *block_ids, uint32_t *lens, uint64_t *offsets,
                        uint8_t *out, size_t out_cap, size_t max_blocks, size_t *nblocks);

#ifdef __cplusplus
}
#endif
#endif /* FEC_GO_H */
