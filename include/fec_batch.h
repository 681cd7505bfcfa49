/*
 * fec_batch.h — C ABI of the sender-side batching layer (C++ in include/fec_batch.hpp,
 * exported from lib0xfec_hip.so). Conventions as fec_scheme.h (0 = nil error,
 * FEC_ERR_SCHEME + fec_last_error() for Go-level errors, fec_hip.h codes otherwise).
 *
 *   entry point                                   reference (file:line) / role
 *   --------------------------------------------  ------------------------------------------
 *   fec_repair_queue_new / _free                  newRepairQueue          repair_queue.go:31-37
 *   fec_repair_queue_add                          repairQueue.Add         repair_queue.go:40-69
 *   fec_repair_queue_peek / _pop                  Peek / Pop              repair_queue.go:73-90
 *   fec_repair_queue_close                        CloseWithError          repair_queue.go:92-95
 *   fec_batch_encoder_*                           deferred repairSymbols for many blocks at once
 *                                                 (replaces the per-block call at
 *                                                 packet_packer.go:1005 / manager.go:145)
 *   fec_manager_add_source_symbol_frame_batched   AddSourceSymbolFrame    manager.go:123-158,
 *                                                 encode deferred to a batch encoder
 *   fec_recovered_queue_*                         the payloads HandleRepairFrame returns
 *                                                 (manager.go:182 -> connection.go:1342)
 *   fec_batch_decoder_*                           deferred recoverSymbolPayloads for many blocks
 *   fec_manager_handle_repair_frame_batched       HandleRepairFrame       manager.go:160-198,
 *                                                 recovery deferred to a batch decoder
 *   fec_manager_handle_source_symbol_frame_batched HandleSourceSymbolFrame manager.go:200-227;
 *                                                 with fec_manager_set_recover_on_source on, a
 *                                                 source that makes its block recoverable
 *                                                 stages it into the batch decoder
 */
#ifndef FEC_BATCH_H
#define FEC_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "fec_scheme.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fec_repair_queue fec_repair_queue;
typedef struct fec_batch_encoder fec_batch_encoder;

/* max_len 0 -> maxRepairSendQueueLen (32, repair_queue.go:14). Add on a full queue returns
 * FEC_ERR_SCHEME "repair queue full" (the reference panics). */
fec_repair_queue *fec_repair_queue_new(size_t max_len);
void fec_repair_queue_free(fec_repair_queue *q);
int fec_repair_queue_add(fec_repair_queue *q, uint64_t block_id, uint64_t parity_id, const uint8_t *p,
                         size_t len);
/* 1 and the front frame (valid until the next pop), or 0 when empty. */
int fec_repair_queue_peek(fec_repair_queue *q, uint64_t *block_id, uint64_t *parity_id, const uint8_t **payload,
                          size_t *len, size_t *cap);
void fec_repair_queue_pop(fec_repair_queue *q);
size_t fec_repair_queue_len(fec_repair_queue *q);
/* Calls of the hasData callback so far (the packer's "more data to send" signal). */
uint64_t fec_repair_queue_has_data_calls(fec_repair_queue *q);
void fec_repair_queue_close(fec_repair_queue *q, const char *msg);

/* scheme_id FEC_SCHEME_REED_SOLOMON (k, m) or FEC_SCHEME_XOR (k, 1); max_blocks per batch. */
fec_batch_encoder *fec_batch_encoder_new(int scheme_id, int k, int m, size_t max_blocks, int device, int *err);
void fec_batch_encoder_free(fec_batch_encoder *e);
int fec_batch_encoder_submit(fec_batch_encoder *e, fec_block *b, fec_repair_queue *q);
int fec_batch_encoder_flush(fec_batch_encoder *e);
int fec_batch_encoder_poll(fec_batch_encoder *e, size_t *blocks);
int fec_batch_encoder_drain(fec_batch_encoder *e, size_t *blocks);
size_t fec_batch_encoder_staged(const fec_batch_encoder *e);
size_t fec_batch_encoder_in_flight(const fec_batch_encoder *e);
/* Encoded blocks whose frames wait for room in their repair queue. Poll / drain return
 * FEC_ERR_SCHEME "repair queue full" while this is nonzero; submit never fails for it. */
size_t fec_batch_encoder_backlog(const fec_batch_encoder *e);

int fec_manager_add_source_symbol_frame_batched(fec_manager *m, uint64_t ssid, const uint8_t *p, size_t len,
                                                size_t cap, fec_batch_encoder *e, fec_repair_queue *q);

typedef struct fec_recovered_queue fec_recovered_queue;
typedef struct fec_batch_decoder fec_batch_decoder;

fec_recovered_queue *fec_recovered_queue_new(void);
void fec_recovered_queue_free(fec_recovered_queue *q);
size_t fec_recovered_queue_len(fec_recovered_queue *q);
/* 1 and the oldest recovered payload (caller frees *out with fec_bytes_free), or 0 when empty. */
int fec_recovered_queue_pop(fec_recovered_queue *q, uint64_t *block_id, fec_bytes **out);

fec_batch_decoder *fec_batch_decoder_new(int scheme_id, int k, int m, size_t max_blocks, int device, int *err);
void fec_batch_decoder_free(fec_batch_decoder *d);
/* *staged = 0 when the block was already complete (the reference's nil, nil). */
int fec_batch_decoder_submit(fec_batch_decoder *d, fec_block *b, fec_recovered_queue *q, int *staged);
int fec_batch_decoder_flush(fec_batch_decoder *d);
int fec_batch_decoder_poll(fec_batch_decoder *d, size_t *blocks);
int fec_batch_decoder_drain(fec_batch_decoder *d, size_t *blocks);
size_t fec_batch_decoder_staged(const fec_batch_decoder *d);
size_t fec_batch_decoder_in_flight(const fec_batch_decoder *d);

int fec_manager_handle_repair_frame_batched(fec_manager *m, uint64_t block_id, uint64_t parity_id, const uint8_t *p,
                                            size_t len, fec_batch_decoder *d, fec_recovered_queue *q);
int fec_manager_handle_source_symbol_frame_batched(fec_manager *m, uint64_t ssid, const uint8_t *p, size_t len,
                                                   size_t cap, fec_bytes **out, fec_batch_decoder *d,
                                                   fec_recovered_queue *q);

#ifdef __cplusplus
}
#endif
#endif /* FEC_BATCH_H */
