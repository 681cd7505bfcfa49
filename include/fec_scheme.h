/*
 * fec_scheme.h — C ABI of the host-side mirror of the reference's internal/fec scheme and
 * manager layer (C++ in include/fec_scheme.hpp, exported from lib0xfec_hip.so).
 *
 * The reference keeps this layer in Go (internal/fec/block.go, reed_solomon.go, xor.go,
 * manager.go); a Go integration keeps that Go code and binds only fec_hip.h. Because the Go
 * toolchain is absent from this build image, the layer is restated in C++ and exposed here
 * so the parity tests (ctypes) can drive the reference's own table-test cases through the
 * GPU path. Conventions follow the Go API:
 *   - return 0 for a nil error; FEC_ERR_SCHEME for a scheme/bookkeeping error whose Go text
 *     is in fec_last_error(); other negative values are fec_hip.h codec codes (klauspost
 *     errors such as "too few shards given", again with the text in fec_last_error());
 *   - a nil result is reported as *out == NULL;
 *   - payloads are copied in; returned frames/bytes are owned by the caller (free them).
 *
 *   entry point                               reference (file:line)
 *   ----------------------------------------  --------------------------------------------
 *   fec_block_new                             newBlock                block.go:36-49
 *   fec_block_add_source_symbol               block.addSourceSymbol   block.go:56-70
 *   fec_block_add_repair_symbol               block.addRepairSymbol   block.go:73-85
 *   fec_block_is_recoverable / _is_complete   block.go:88-95
 *   fec_scheme_new(2, k, m)                   NewReedSolomonScheme    reed_solomon.go:15-23
 *   fec_scheme_new(1, .., ..)                 xorScheme{}             xor.go:10-12
 *   fec_scheme_repair_symbols                 repairSymbols           reed_solomon.go:26-68, xor.go:14-42
 *   fec_scheme_recover_symbol_payloads        recoverSymbolPayloads   reed_solomon.go:92-136, xor.go:66-104
 *   fec_manager_new_sender / _new_receiver    NewSender / NewReceiver manager.go:50-94
 *   fec_manager_new                           NewManager              manager.go:96-109
 *   fec_manager_next_ssid                     NextSSID                manager.go:111-117
 *   fec_manager_add_source_symbol_frame       AddSourceSymbolFrame    manager.go:123-158
 *   fec_manager_handle_repair_frame           HandleRepairFrame       manager.go:160-198
 *   fec_manager_handle_source_symbol_frame    HandleSourceSymbolFrame manager.go:200-227
 *
 * Extension (off by default so the default behaviour is the reference's):
 *   fec_manager_set_recover_on_source         recovery also fires when a SOURCE symbol makes a
 *                                             block recoverable (the reference only recovers on
 *                                             a REPAIR arrival, manager.go:181 vs :221-226)
 *   fec_manager_handle_source_symbol_frame_recover   HandleSourceSymbolFrame + the recovered
 *                                             payloads (NULL unless this call recovered)
 */
#ifndef FEC_SCHEME_H
#define FEC_SCHEME_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FEC_ERR_SCHEME (-20) /* Go-level error; text in fec_last_error() */

/* DecoderFECScheme ids (internal/protocol/fec.go:21-27) */
#define FEC_SCHEME_DISABLED 0
#define FEC_SCHEME_XOR 1
#define FEC_SCHEME_REED_SOLOMON 2

typedef struct fec_block fec_block;
typedef struct fec_scheme fec_scheme;
typedef struct fec_manager fec_manager;
typedef struct fec_frames fec_frames;
typedef struct fec_bytes fec_bytes;

/* Text of the last error on this thread ("" after a successful call). */
const char *fec_last_error(void);

/* Blocks. fec_block_literal builds a block as the reference's table tests write one (every
 * field given); fec_block_put_* insert map entries directly, like those literals. */
fec_block *fec_block_new(uint64_t id, int tot_src, int tot_rep);
fec_block *fec_block_literal(uint64_t id, int tot_src, int tot_rep, int biggest,
                             uint64_t smallest_ssid, uint64_t largest_ssid);
void fec_block_free(fec_block *b);
int fec_block_put_source(fec_block *b, uint64_t ssid, const uint8_t *p, size_t len, size_t cap);
int fec_block_put_repair(fec_block *b, uint64_t parity_id, const uint8_t *p, size_t len);
int fec_block_add_source_symbol(fec_block *b, uint64_t ssid, const uint8_t *p, size_t len, size_t cap);
int fec_block_add_repair_symbol(fec_block *b, uint64_t block_id, uint64_t parity_id,
                                const uint8_t *p, size_t len);
int fec_block_is_recoverable(const fec_block *b);
int fec_block_is_complete(const fec_block *b);
int fec_block_biggest(const fec_block *b);
int fec_block_num_sources(const fec_block *b);
/* Copies up to out_cap bytes of the source payload; returns its length, or -1 if absent. */
long fec_block_get_source(const fec_block *b, uint64_t ssid, uint8_t *out, size_t out_cap);

/* Schemes (the arithmetic runs on GPU `device`; the context is created on first use). */
fec_scheme *fec_scheme_new(int scheme_id, int k, int m, int device);
void fec_scheme_free(fec_scheme *s);
int fec_scheme_repair_symbols(fec_scheme *s, fec_block *b, fec_frames **out);
int fec_scheme_recover_symbol_payloads(fec_scheme *s, fec_block *b, fec_bytes **out);

size_t fec_frames_count(const fec_frames *f);
int fec_frames_get(const fec_frames *f, size_t i, uint64_t *block_id, uint64_t *parity_id,
                   const uint8_t **payload, size_t *len);
void fec_frames_free(fec_frames *f);
const uint8_t *fec_bytes_data(const fec_bytes *b);
size_t fec_bytes_len(const fec_bytes *b);
void fec_bytes_free(fec_bytes *b);

/* Managers. new_sender/new_receiver return NULL with *err == 0 for FEC_SCHEME_DISABLED. */
fec_manager *fec_manager_new_sender(int scheme_id, int device, int *err);
fec_manager *fec_manager_new_receiver(int scheme_id, int device, int *err);
fec_manager *fec_manager_new(int scheme_id, int k, int m, int device, int *err);
void fec_manager_free(fec_manager *m);
uint64_t fec_manager_next_ssid(fec_manager *m);
uint64_t fec_manager_block_id(const fec_manager *m, uint64_t ssid);
int fec_manager_add_source_symbol_frame(fec_manager *m, uint64_t ssid, const uint8_t *p, size_t len,
                                        size_t cap, fec_frames **out);
int fec_manager_handle_repair_frame(fec_manager *m, uint64_t block_id, uint64_t parity_id,
                                    const uint8_t *p, size_t len, fec_bytes **out);
int fec_manager_handle_source_symbol_frame(fec_manager *m, uint64_t ssid, const uint8_t *p,
                                           size_t len, size_t cap, fec_bytes **out);
int fec_manager_set_recover_on_source(fec_manager *m, int on);
int fec_manager_handle_source_symbol_frame_recover(fec_manager *m, uint64_t ssid, const uint8_t *p,
                                                   size_t len, size_t cap, fec_bytes **out,
                                                   fec_bytes **recovered);

#ifdef __cplusplus
}
#endif
#endif /* FEC_SCHEME_H */
