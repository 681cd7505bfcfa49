//go:build fechip

package fec

// #include <stdlib.h>
// #include "fec_hip.h"
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"

	"github.com/quic-go/quic-go/internal/protocol"
	"github.com/quic-go/quic-go/internal/wire"
)

// hipReedSolomonScheme implements BlockFECScheme (scheme.go:5-10) with the MI355X kernels:
// reedsolomon.New (reed_solomon.go:16) -> fec_rs_prepare, enc.Encode (:51) ->
// fec_rs_encode_batch, enc.ReconstructData (:124) -> fec_rs_reconstruct_batch. Checks, error
// texts and output framing are reed_solomon.go's. One fec_ctx per scheme: the manager owning it
// runs on one connection's run loop (connection.go:525), the ctx's one-caller rule.
//
// One block per call is for wire parity (bit-identical repair payloads, so a GPU peer talks to
// a CPU peer); throughput comes from the batched types in batch_hip.go.
type hipReedSolomonScheme struct {
	ctx  *C.fec_ctx
	k, m int
}

var _ BlockFECScheme = &hipReedSolomonScheme{}

func newHipReedSolomonScheme(k, m int) (*hipReedSolomonScheme, error) {
	var ctx *C.fec_ctx
	if err := hipErr(C.fec_ctx_create(C.int(hipDevice()), &ctx)); err != nil {
		return nil, err
	}
	if err := hipErr(C.fec_rs_prepare(ctx, C.int(k), C.int(m))); err != nil {
		C.fec_ctx_destroy(ctx)
		return nil, err
	}
	s := &hipReedSolomonScheme{ctx: ctx, k: k, m: m}
	runtime.SetFinalizer(s, func(s *hipReedSolomonScheme) { C.fec_ctx_destroy(s.ctx) })
	return s, nil
}

// cBuf is n bytes of C memory viewed as a Go slice (freed by the caller).
func cBuf(n int) []byte {
	return unsafe.Slice((*byte)(C.malloc(C.size_t(n))), n)
}

// repairSymbols: reed_solomon.go:26-68. The k shards [payload | zeros | BE16(len)] of L =
// biggest+2 bytes go into C memory back to back ([n][L], parity after the data), encoded with
// FEC_HOST (the library stages them through pinned memory), parity i -> RepairFrame ParityID i.
func (s *hipReedSolomonScheme) repairSymbols(b *block) ([]*wire.RepairFrame, error) {
	if !b.isComplete() {
		return nil, fmt.Errorf("block does not have enough source symbols to generate repair symbols")
	}
	if b.biggestSourceSymbolLenSoFar > protocol.MaxFECPacketBufferSize {
		return nil, fmt.Errorf("source symbol payload len is greater is too big for FEC headers. Max %d and got %d", protocol.MaxFECPacketBufferSize, b.biggestSourceSymbolLenSoFar)
	}
	L := protocol.RepairPayloadMetadataLen + b.biggestSourceSymbolLenSoFar
	n := b.totNumSourceSymbols + b.totNumRepairSymbols
	buf := cBuf(n * L)
	defer C.free(unsafe.Pointer(&buf[0]))
	rs := &reedSolomonScheme{}
	for i := 0; i < b.totNumSourceSymbols; i++ {
		shard, err := rs.addLengthToSourceSymbolPayload(b, b.smallestSSID+protocol.SourceSymbolID(i))
		if err != nil {
			return nil, err
		}
		copy(buf[i*L:(i+1)*L], shard)
	}
	rc := C.fec_rs_encode_batch(s.ctx, C.int(b.totNumSourceSymbols), C.int(b.totNumRepairSymbols), C.size_t(L), 1,
		(*C.uint8_t)(&buf[0]), C.size_t(n*L), (*C.uint8_t)(&buf[b.totNumSourceSymbols*L]), C.size_t(n*L),
		C.size_t(L), C.FEC_HOST)
	if err := hipErr(rc); err != nil {
		return nil, fmt.Errorf("unable to make parity shards: %w", err)
	}
	frames := make([]*wire.RepairFrame, b.totNumRepairSymbols)
	for i := range frames {
		p := make([]byte, L, protocol.MaxPacketBufferSize) // make(0, 1452)[:L'], reed_solomon.go:44-49
		copy(p, buf[(b.totNumSourceSymbols+i)*L:])
		frames[i] = &wire.RepairFrame{
			Metadata: protocol.BlockMetadata{BlockID: b.id, ParityID: protocol.ParityID(i)},
			Payload:  p,
		}
	}
	return frames, nil
}

// recoverSymbolPayloads: reed_solomon.go:92-136. Present shards into C memory [n][L] with the
// present mask (bit i = shard i), ReconstructData in place with FEC_HOST, then the rebuilt
// payloads in ascending index order, each cut to its length trailer.
func (s *hipReedSolomonScheme) recoverSymbolPayloads(b *block) ([]byte, error) {
	if !b.isRecoverable() {
		return nil, fmt.Errorf("not enough present symbols to repair the missing ones")
	}
	if b.isComplete() {
		return nil, nil
	}
	L := protocol.RepairPayloadMetadataLen + b.biggestSourceSymbolLenSoFar
	k, n := b.totNumSourceSymbols, b.totNumSourceSymbols+b.totNumRepairSymbols
	if n > C.FEC_MAX_DECODE_SHARDS {
		return nil, errors.New("too many shards for the GPU decoder") // RS(20,10) has 30
	}
	buf := cBuf(n * L)
	defer C.free(unsafe.Pointer(&buf[0]))
	var mask C.uint32_t
	var missing []int
	rs := &reedSolomonScheme{}
	for i := 0; i < k; i++ {
		ssid := b.smallestSSID + protocol.SourceSymbolID(i)
		if _, ok := b.ssidToSourcePayload[ssid]; !ok {
			missing = append(missing, i)
			continue
		}
		shard, err := rs.addLengthToSourceSymbolPayload(b, ssid)
		if err != nil {
			return nil, err
		}
		copy(buf[i*L:(i+1)*L], shard)
		mask |= 1 << uint(i)
	}
	for pid, payload := range b.pidToRepairPayload {
		i := k + int(pid)
		if len(payload) == 0 {
			continue // klauspost treats a zero-length shard as missing (as stageRecoverPayloads does)
		}
		if len(payload) != L {
			return nil, errors.New("shard sizes do not match") // klauspost ErrShardSize
		}
		copy(buf[i*L:(i+1)*L], payload)
		mask |= 1 << uint(i)
	}
	var status C.int32_t
	rc := C.fec_rs_reconstruct_batch(s.ctx, C.int(k), C.int(b.totNumRepairSymbols), C.size_t(L), 1,
		(*C.uint8_t)(&buf[0]), C.size_t(n*L), (*C.uint8_t)(&buf[k*L]), C.size_t(n*L), C.size_t(L),
		&mask, &status, C.FEC_HOST)
	if err := hipErr(rc); err != nil {
		return nil, err
	}
	out := make([]byte, 0, len(missing)*b.biggestSourceSymbolLenSoFar)
	for _, i := range missing {
		sh := buf[i*L : (i+1)*L]
		plen := int(sh[b.biggestSourceSymbolLenSoFar])<<8 | int(sh[b.biggestSourceSymbolLenSoFar+1])
		out = append(out, sh[:plen]...)
	}
	return out, nil
}
