/*
 * fec_synth.h — synthetic workload generator on the device (lib0xfec_hip.so).
 *
 * Not a reference interface: the benchmark's data loader. Payload bytes are
 * splitmix64 keyed by (seed, global block, shard, 8-byte word), so any split of a global batch
 * over ranks generates the same bytes; 0xfec_amd/shard.py restates both functions on the host
 * (synth_payload_blocks, synth_single_erasures) for the oracle checks. Asynchronous on the ctx
 * stream; device memory only.
 */
#ifndef FEC_SYNTH_H
#define FEC_SYNTH_H

#include <stddef.h>
#include <stdint.h>

#include "fec_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Data shard j of block b (global index first_block + b) at data + b*block_stride +
 * j*shard_stride: payload_len splitmix64 bytes, the big-endian uint16 length trailer
 * (reed_solomon.go:77-87), zeros to the end of the slot. shard_stride % 16 == 0. */
int fec_synth_data(fec_ctx *ctx, uint64_t seed, uint64_t first_block, size_t nblocks, int k, size_t payload_len,
                   uint8_t *data, size_t block_stride, size_t shard_stride);

/* One erased data shard per block, e = key(seed, block) % k: masks[b] = all n = k + m bits
 * except e; erased[b] = e (erased may be NULL). */
int fec_synth_single_erasures(fec_ctx *ctx, uint64_t seed, uint64_t first_block, size_t nblocks, int k, int m,
                              uint32_t *masks, int32_t *erased);

#ifdef __cplusplus
}
#endif
#endif /* FEC_SYNTH_H */
