/*
 * fec_wire.h — the FEC frames' wire codecs (the data formats either side of the codec,
 * SURVEY.md §8a row a11 / §8f row 4), restated from the reference:
 *
 *   entry point                          reference (file:line)
 *   -----------------------------------  -----------------------------------------------------
 *   fec_varint_len / _append / _read     quicvarint.Len / Append / Read    quicvarint/varint.go:25-140
 *   fec_repair_frame_*                   wire.RepairFrame                  internal/wire/fec_repair_frame.go:11-57
 *   fec_source_symbol_frame_*            wire.SourceSymbolFrame            internal/wire/fec_source_symbol_frame.go:11-58
 *   FEC_WIRE_*_FRAME_TYPE                repairFrameType, sourceSymbolFrameType  internal/wire/frame_parser.go:38-39
 *   fec_batch_encoder_submit_payloads    zero-copy staging of a block's source payloads from the
 *                                        packet buffers (packet_packer.go:980-1016) into pinned memory
 *
 * Parse functions start after the frame type, as the frame parser dispatches on the type first
 * (frame_parser.go:151-154); they return FEC_ERR_EOF where the reference returns io.EOF (a
 * varint or the payload runs past the buffer). Payloads are returned as offsets into the
 * caller's buffer (no copy).
 */
#ifndef FEC_WIRE_H
#define FEC_WIRE_H

#include <stddef.h>
#include <stdint.h>

#include "fec_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FEC_WIRE_REPAIR_FRAME_TYPE 0x32a80fecULL
#define FEC_WIRE_SOURCE_SYMBOL_FRAME_TYPE 0x32a80fec55ULL
#define FEC_WIRE_VARINT_MAX 4611686018427387903ULL /* 2^62 - 1 */
#define FEC_ERR_EOF (-21)

/* Encoded length of v (1, 2, 4 or 8); 0 when v > FEC_WIRE_VARINT_MAX (the reference panics). */
size_t fec_varint_len(uint64_t v);
/* Appends v at dst (minimal length); bytes written, 0 when it does not fit or v is too big. */
size_t fec_varint_append(uint8_t *dst, size_t cap, uint64_t v);
/* Reads one varint; FEC_ERR_EOF when the buffer ends first. */
int fec_varint_read(const uint8_t *src, size_t len, uint64_t *v, size_t *consumed);

size_t fec_repair_frame_length(uint64_t block_id, uint64_t parity_id, size_t payload_len);
/* Type, BlockID, ParityID, length, payload; bytes written, 0 when cap is too small. */
size_t fec_repair_frame_append(uint8_t *dst, size_t cap, uint64_t block_id, uint64_t parity_id,
                               const uint8_t *payload, size_t len);
int fec_repair_frame_parse(const uint8_t *src, size_t len, uint64_t *block_id, uint64_t *parity_id,
                           size_t *payload_off, size_t *payload_len, size_t *consumed);

size_t fec_source_symbol_frame_length(uint64_t ssid, size_t payload_len);
size_t fec_source_symbol_frame_header_len(uint64_t ssid, size_t payload_len);
size_t fec_source_symbol_frame_append(uint8_t *dst, size_t cap, uint64_t ssid, const uint8_t *payload, size_t len);
int fec_source_symbol_frame_parse(const uint8_t *src, size_t len, uint64_t *ssid, size_t *payload_off,
                                  size_t *payload_len, size_t *consumed);

/* Stage the `count` (= k) source payloads of block `block_id` (SSID order) straight into the
 * encoder's pinned staging; checks and errors as repairSymbols. */
int fec_batch_encoder_submit_payloads(fec_batch_encoder *e, uint64_t block_id, const uint8_t *const *payloads,
                                      const size_t *lens, int count, fec_repair_queue *q);

#ifdef __cplusplus
}
#endif
#endif /* FEC_WIRE_H */
