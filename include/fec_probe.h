/* fec_probe.h — traffic twins of the headline codec kernels (measurement only).
 *
 * No reference counterpart: the reference's path (internal/fec) has no device, and these entry
 * points compute nothing it computes. bench.py times them right after the codec kernels, on the
 * same box and buffers, so the bench line carries that box's ceiling for each kernel's access
 * shape (roofline.probe_TBps, frac_of_probe) beside the 8 TB/s spec.
 *
 *   fec_probe_encode_traffic    the bytes and launch shape of fec_rs_encode_batch's fixed-shape
 *                               kernel (k shard loads, m stores per 16-B chunk, XCD-contiguous
 *                               flat grid, its residency, non-temporal), RS(2,3), RS(8,12),
 *                               RS(16,24), RS(20,30); parity receives the XOR of the inputs, not
 *                               parity
 *   fec_probe_recover_traffic   the bytes and launch shape of fec_rs_recover_batch's direct
 *                               single-erasure kernel: per block the k-1 other data shards and the
 *                               first present parity, one store to out; blocks whose mask is not
 *                               a single data erasure move nothing. out == data: the store goes
 *                               into the erased shard's own slot (the in-place reconstruct's)
 *   fec_probe_rebuild_traffic   the bytes of the multi-erasure decode of RS(16,24) / RS(20,30)
 *                               (sorted plans + rebuild): per block the first k present shards
 *                               and one store per erased data shard into out (block b, row r at
 *                               out + b*out_bs + r*ss), in block order, at the rebuild's residency
 *   fec_probe_stream_traffic    shape-independent reference: per block nin consecutive shards
 *                               of `in` read (shard stride ss), one chunk-wise store to out
 *                               (nin 2, 8, 16, 20)
 * Every twin takes wpc, the resident workgroups per CU it runs at: -1 the twinned kernel's own
 * (bench.py's same-shape figure), 0 as many as fit, n > 0 a cap; the best over residency is the
 * box's ceiling for the access shape (probe_best_TBps).
 *   fec_probe_link              the host link as the FEC_HOST paths drive it: hipMemcpyAsync of
 *                               `bytes` between pinned host and device buffers, H2D alone, D2H
 *                               alone and both at once on two streams (best of reps); GB/s into
 *                               out[0], out[1], out[2] (the duplex rate of each direction)
 * The twins take FEC_DEVICE layouts only (16-byte aligned pointers and strides) and are enqueued
 * on the ctx stream; the link probe allocates, synchronises the device and frees.
 */
#ifndef FEC_PROBE_H
#define FEC_PROBE_H

#include <stddef.h>
#include <stdint.h>

#include "fec_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

int fec_probe_encode_traffic(fec_ctx *ctx, int k, int m, size_t shard_len, size_t nblocks, const void *data,
                             size_t dbs, void *parity, size_t pbs, size_t ss, int wpc);
int fec_probe_recover_traffic(fec_ctx *ctx, int k, int m, size_t shard_len, size_t nblocks, const void *data,
                              size_t dbs, const void *parity, size_t pbs, size_t ss, const uint32_t *masks,
                              void *out, size_t out_bs, int wpc);
int fec_probe_rebuild_traffic(fec_ctx *ctx, int k, int m, size_t shard_len, size_t nblocks, const void *data,
                              size_t dbs, const void *parity, size_t pbs, size_t ss, const uint32_t *masks,
                              void *out, size_t out_bs, int wpc);
int fec_probe_stream_traffic(fec_ctx *ctx, int nin, size_t shard_len, size_t nblocks, const void *in, size_t in_bs,
                             void *out, size_t out_bs, size_t ss, int wpc);
int fec_probe_link(fec_ctx *ctx, size_t bytes, int reps, double *out);

#ifdef __cplusplus
}
#endif
#endif /* FEC_PROBE_H */
