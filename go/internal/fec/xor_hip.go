//go:build fechip

package fec

// #include <stdlib.h>
// #include "fec_hip.h"
import "C"

import (
	"fmt"
	"runtime"
	"unsafe"

	"github.com/quic-go/quic-go/internal/protocol"
	"github.com/quic-go/quic-go/internal/wire"
)

// hipXorScheme implements BlockFECScheme with the MI355X XOR kernels: xorScheme's byte loops
// (xor.go:44-63) -> fec_xor_encode_batch / fec_xor_reconstruct_batch. Every source is framed
// as [payload | zeros | BE16(len)] of L = biggest+2 bytes: the XOR of those framings is exactly
// xor.go's result (payloads zero-extended, lengths XORed at [biggest]).
type hipXorScheme struct {
	ctx *C.fec_ctx
}

var _ BlockFECScheme = &hipXorScheme{}

func newHipXorScheme() (*hipXorScheme, error) {
	var ctx *C.fec_ctx
	if err := hipErr(C.fec_ctx_create(C.int(hipDevice()), &ctx)); err != nil {
		return nil, err
	}
	s := &hipXorScheme{ctx: ctx}
	runtime.SetFinalizer(s, func(s *hipXorScheme) { C.fec_ctx_destroy(s.ctx) })
	return s, nil
}

// frame writes xor.go's framing of one payload into dst (L bytes, zeroed by the caller).
func xorFrame(dst, payload []byte, biggest int) {
	copy(dst, payload)
	dst[biggest] ^= byte(uint16(len(payload)) >> 8)
	dst[biggest+1] ^= byte(uint16(len(payload)) & 0xFF)
}

// repairSymbols: xor.go:14-42 (same checks, same order, same texts).
func (s *hipXorScheme) repairSymbols(b *block) ([]*wire.RepairFrame, error) {
	if !b.isComplete() {
		return nil, fmt.Errorf("block does not have enough source symbols to generate repair symbols")
	}
	if b.totNumRepairSymbols != 1 {
		return nil, fmt.Errorf("xor only supports 1 repair symbol. Expected 1, received %d", b.totNumRepairSymbols)
	}
	if b.biggestSourceSymbolLenSoFar > protocol.MaxFECPacketBufferSize {
		return nil, fmt.Errorf("source symbol payload len is greater is too big for FEC headers. Max %d and got %d", protocol.MaxFECPacketBufferSize, b.biggestSourceSymbolLenSoFar)
	}
	L := protocol.RepairPayloadMetadataLen + b.biggestSourceSymbolLenSoFar
	k := len(b.ssidToSourcePayload)
	buf := cBuf((k + 1) * L)
	defer C.free(unsafe.Pointer(&buf[0]))
	for i := range buf {
		buf[i] = 0
	}
	i := 0
	for _, payload := range b.ssidToSourcePayload { // XOR commutes: map order is irrelevant
		xorFrame(buf[i*L:(i+1)*L], payload, b.biggestSourceSymbolLenSoFar)
		i++
	}
	rc := C.fec_xor_encode_batch(s.ctx, C.int(k), C.size_t(L), 1, (*C.uint8_t)(&buf[0]), C.size_t((k+1)*L),
		(*C.uint8_t)(&buf[k*L]), C.size_t((k+1)*L), C.size_t(L), C.FEC_HOST)
	if err := hipErr(rc); err != nil {
		return nil, err
	}
	repair := make([]byte, L) // make([]byte, repairPayloadLen), xor.go:33
	copy(repair, buf[k*L:])
	return []*wire.RepairFrame{{Metadata: protocol.BlockMetadata{BlockID: b.id, ParityID: 0}, Payload: repair}}, nil
}

// recoverSymbolPayloads: xor.go:66-104. The recovered symbol is the XOR of every repair payload
// and every present source framed (xor.go:78-84, which walks the maps, not an SSID window), so
// the r repairs and p framed sources go into C memory [p+r+1][1452] and one XOR encode over the
// p+r inputs yields it; its trailer names the payload, which is also stored into the block
// (xor.go:91-96).
func (s *hipXorScheme) recoverSymbolPayloads(b *block) ([]byte, error) {
	if !b.isRecoverable() {
		return nil, fmt.Errorf("not enough present symbols to repair the missing ones")
	}
	if b.isComplete() {
		return nil, nil
	}
	big := b.biggestSourceSymbolLenSoFar
	L := protocol.MaxPacketBufferSize // recoveredSymbol := make([]byte, MaxPacketBufferSize), xor.go:78
	k := len(b.pidToRepairPayload) + len(b.ssidToSourcePayload)
	buf := cBuf((k + 1) * L)
	defer C.free(unsafe.Pointer(&buf[0]))
	for i := range buf {
		buf[i] = 0
	}
	i := 0
	for _, data := range b.pidToRepairPayload {
		copy(buf[i*L:(i+1)*L], data)
		i++
	}
	for _, payload := range b.ssidToSourcePayload {
		xorFrame(buf[i*L:(i+1)*L], payload, big)
		i++
	}
	rc := C.fec_xor_encode_batch(s.ctx, C.int(k), C.size_t(L), 1, (*C.uint8_t)(&buf[0]), C.size_t((k+1)*L),
		(*C.uint8_t)(&buf[k*L]), C.size_t((k+1)*L), C.size_t(L), C.FEC_HOST)
	if err := hipErr(rc); err != nil {
		return nil, err
	}
	rec := make([]byte, L)
	copy(rec, buf[k*L:])
	payloadLen := uint16(rec[big])<<8 | uint16(rec[big+1])
	recovered := rec[:payloadLen]
	for ssid := b.smallestSSID; ssid <= b.largestSSID; ssid++ {
		if _, exists := b.ssidToSourcePayload[ssid]; !exists {
			b.ssidToSourcePayload[ssid] = recovered
		}
	}
	if !b.isComplete() {
		return nil, fmt.Errorf("block is not complete after recovery")
	}
	return recovered, nil
}
