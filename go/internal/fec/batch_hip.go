//go:build fechip

package fec

// #include <stdlib.h>
// #include "fec_go.h"
import "C"

import (
	"fmt"
	"runtime"
	"unsafe"

	"github.com/quic-go/quic-go/internal/protocol"
	"github.com/quic-go/quic-go/internal/wire"
)

// Batched forms of manager.go's sender and receiver steps over include/fec_go.h. The manager
// keeps its blocks (block.go) exactly as today; instead of calling scheme.repairSymbols /
// recoverSymbolPayloads per block on the run loop (manager.go:144-154, 181-193), it submits the
// complete / recoverable block here and takes the frames / payloads of finished blocks from Poll,
// so many blocks are coded in one kernel launch while the run loop carries on.
//
// cgo pointer rules (go 1.21, go.mod:3): the payload pointer arrays are C memory; the payloads
// they point to are Go memory without Go pointers in it, pinned with runtime.Pinner for the
// duration of the call. The library copies everything it needs before returning and retains
// no pointer, so the pins end when the call does.

// BatchSender batches repairSymbols over complete blocks.
type BatchSender struct {
	e       *C.fec_go_encoder
	scheme  protocol.DecoderFECScheme
	k, m    int
	ptrs    *C.uintptr_t // k payload pointers (C memory)
	lens    *C.size_t
	ids     []C.uint64_t
	rlen    []C.uint32_t
	repairs []byte // C memory: maxBlocks * m * FEC_GO_SLOT
}

// NewBatchSender: scheme protocol.XORFECScheme (k, 1) or protocol.ReedSolomonFECScheme (k, m);
// maxBlocks blocks per kernel launch.
func NewBatchSender(id protocol.DecoderFECScheme, k, m, maxBlocks int) (*BatchSender, error) {
	var rc C.int
	e := C.fec_go_encoder_new(C.int(id), C.int(k), C.int(m), C.size_t(maxBlocks), C.int(hipDevice()), &rc)
	if e == nil {
		return nil, goErr(rc)
	}
	if id == protocol.XORFECScheme {
		m = 1
	}
	s := &BatchSender{e: e, scheme: id, k: k, m: m,
		ptrs:    (*C.uintptr_t)(C.malloc(C.size_t(k) * 8)),
		lens:    (*C.size_t)(C.malloc(C.size_t(k) * 8)),
		ids:     make([]C.uint64_t, maxBlocks),
		rlen:    make([]C.uint32_t, maxBlocks),
		repairs: cBuf(maxBlocks * m * C.FEC_GO_SLOT),
	}
	runtime.SetFinalizer(s, (*BatchSender).Close)
	return s, nil
}

func (s *BatchSender) Close() {
	if s.e != nil {
		C.fec_go_encoder_free(s.e)
		C.free(unsafe.Pointer(s.ptrs))
		C.free(unsafe.Pointer(s.lens))
		C.free(unsafe.Pointer(&s.repairs[0]))
		s.e = nil
	}
}

// Submit replaces `m.scheme.repairSymbols(bS.block)` (manager.go:145): the same validation and
// error texts, reported now; the frames arrive from Poll.
func (s *BatchSender) Submit(b *block) error { return s.submit(b, false) }

// SubmitRef is Submit by reference (fec_go_encoder_submit_ref): payloads in a PacketPool are read
// by the device when the batch is coded, so the caller keeps them unchanged until Poll returns the
// block; other payloads are copied now, as Submit.
func (s *BatchSender) SubmitRef(b *block) error { return s.submit(b, true) }

func (s *BatchSender) submit(b *block, byRef bool) error {
	defer lockThread()()
	var pin runtime.Pinner
	defer pin.Unpin()
	ptrs := unsafe.Slice(s.ptrs, s.k)
	lens := unsafe.Slice(s.lens, s.k)
	n := 0
	add := func(p []byte) {
		ptrs[n], lens[n] = 0, C.size_t(len(p))
		if len(p) > 0 {
			pin.Pin(&p[0])
			ptrs[n] = C.uintptr_t(uintptr(unsafe.Pointer(&p[0])))
		}
		n++
	}
	// repairSymbols' block-level checks on the Go block, in its order (reed_solomon.go:27-33,
	// xor.go:15-25); the library repeats them on what it is given
	if !b.isComplete() {
		return fmt.Errorf("block does not have enough source symbols to generate repair symbols")
	}
	if s.scheme == protocol.XORFECScheme && b.totNumRepairSymbols != 1 {
		return fmt.Errorf("xor only supports 1 repair symbol. Expected 1, received %d", b.totNumRepairSymbols)
	}
	if b.biggestSourceSymbolLenSoFar > protocol.MaxFECPacketBufferSize {
		return fmt.Errorf("source symbol payload len is greater is too big for FEC headers. Max %d and got %d", protocol.MaxFECPacketBufferSize, b.biggestSourceSymbolLenSoFar)
	}
	if s.scheme == protocol.XORFECScheme {
		for _, p := range b.ssidToSourcePayload { // XOR commutes: map order is irrelevant
			if n < s.k {
				add(p)
			}
		}
	} else {
		// reed_solomon.go:36-42: shard i is SSID smallestSSID + i
		for i := 0; i < b.totNumSourceSymbols && n < s.k; i++ {
			ssid := b.smallestSSID + protocol.SourceSymbolID(i)
			p, ok := b.ssidToSourcePayload[ssid]
			if !ok {
				return fmt.Errorf("block [%d, %d] is complete but SID %d does not exist", b.smallestSSID, b.largestSSID, ssid)
			}
			add(p)
		}
	}
	if byRef {
		return goErr(C.fec_go_encoder_submit_ref(s.e, C.uint64_t(b.id), (**C.uint8_t)(unsafe.Pointer(s.ptrs)), s.lens, C.int(n)))
	}
	return goErr(C.fec_go_encoder_submit(s.e, C.uint64_t(b.id), (**C.uint8_t)(unsafe.Pointer(s.ptrs)), s.lens, C.int(n)))
}

// Poll hands back the repair frames of finished blocks, in submit order, at most maxBlocks
// blocks (< 0 or more than a batch: one batch's worth; 0: none); the rest stay in the library
// for a later Poll. wait: flush and wait for every staged block first; otherwise the staged blocks
// start coding when no batch is in flight. Each payload is a fresh Go slice of cap
// MaxPacketBufferSize, as reed_solomon.go:44.
func (s *BatchSender) Poll(wait bool, maxBlocks int) ([][]*wire.RepairFrame, error) {
	defer lockThread()()
	w := C.int(0)
	if wait {
		w = 1
	}
	if maxBlocks < 0 || maxBlocks > len(s.ids) {
		maxBlocks = len(s.ids)
	}
	var nb C.size_t
	rc := C.fec_go_encoder_poll(s.e, w, &s.ids[0], &s.rlen[0], (*C.uint8_t)(&s.repairs[0]), C.size_t(maxBlocks), &nb)
	if err := goErr(rc); err != nil {
		return nil, err
	}
	out := make([][]*wire.RepairFrame, int(nb))
	for d := range out {
		L := int(s.rlen[d])
		out[d] = make([]*wire.RepairFrame, s.m)
		for i := 0; i < s.m; i++ {
			p := make([]byte, L, protocol.MaxPacketBufferSize)
			copy(p, s.repairs[(d*s.m+i)*C.FEC_GO_SLOT:])
			out[d][i] = &wire.RepairFrame{
				Metadata: protocol.BlockMetadata{BlockID: protocol.BlockID(s.ids[d]), ParityID: protocol.ParityID(i)},
				Payload:  p,
			}
		}
	}
	return out, nil
}

// BatchReceiver batches recoverSymbolPayloads over recoverable blocks.
type BatchReceiver struct {
	d    *C.fec_go_decoder
	k, m int
	src  *C.uintptr_t // k + m payload pointers (C memory)
	lens *C.size_t
	ids  []C.uint64_t
	plen []C.uint32_t
	offs []C.uint64_t
	out  []byte // C memory
}

func NewBatchReceiver(id protocol.DecoderFECScheme, k, m, maxBlocks int) (*BatchReceiver, error) {
	var rc C.int
	d := C.fec_go_decoder_new(C.int(id), C.int(k), C.int(m), C.size_t(maxBlocks), C.int(hipDevice()), &rc)
	if d == nil {
		return nil, goErr(rc)
	}
	if id == protocol.XORFECScheme {
		m = 1
	}
	r := &BatchReceiver{d: d, k: k, m: m,
		src:  (*C.uintptr_t)(C.malloc(C.size_t(k+m) * 8)),
		lens: (*C.size_t)(C.malloc(C.size_t(k+m) * 8)),
		ids:  make([]C.uint64_t, maxBlocks),
		plen: make([]C.uint32_t, maxBlocks),
		offs: make([]C.uint64_t, maxBlocks),
		out:  cBuf(maxBlocks * k * protocol.MaxPacketBufferSize),
	}
	runtime.SetFinalizer(r, (*BatchReceiver).Close)
	return r, nil
}

func (r *BatchReceiver) Close() {
	if r.d != nil {
		C.fec_go_decoder_free(r.d)
		C.free(unsafe.Pointer(r.src))
		C.free(unsafe.Pointer(r.lens))
		C.free(unsafe.Pointer(&r.out[0]))
		r.d = nil
	}
}

// Submit replaces `m.scheme.recoverSymbolPayloads(bS.block)` (manager.go:182) for a
// recoverable block: validation and error texts as the reference, reported now; staged is
// false for a complete block (the reference's nil, nil). The payload arrives from Poll.
func (r *BatchReceiver) Submit(b *block) (staged bool, err error) { return r.submit(b, false) }

// SubmitRef is Submit by reference (RS): received payloads lying in the registered
// PacketPool are read by the device when the batch is coded (fec_go_decoder_submit_ref), so
// the caller keeps those buffers unchanged until Poll returns the block; others are copied now.
func (r *BatchReceiver) SubmitRef(b *block) (staged bool, err error) { return r.submit(b, true) }

func (r *BatchReceiver) submit(b *block, byRef bool) (staged bool, err error) {
	// recoverSymbolPayloads' block-level checks, on the Go block itself (reed_solomon.go:93-100)
	if !b.isRecoverable() {
		return false, fmt.Errorf("not enough present symbols to repair the missing ones")
	}
	if b.isComplete() {
		return false, nil
	}
	defer lockThread()()
	var pin runtime.Pinner
	defer pin.Unpin()
	ptrs := unsafe.Slice(r.src, r.k+r.m)
	lens := unsafe.Slice(r.lens, r.k+r.m)
	put := func(i int, p []byte) {
		ptrs[i], lens[i] = 0, C.size_t(len(p))
		if p != nil {
			q := p[:cap(p)] // a zero-length payload still counts as present
			if len(q) == 0 {
				q = []byte{0}
			}
			pin.Pin(&q[0])
			ptrs[i] = C.uintptr_t(uintptr(unsafe.Pointer(&q[0])))
		}
	}
	for i := 0; i < r.k; i++ {
		p, ok := b.ssidToSourcePayload[b.smallestSSID+protocol.SourceSymbolID(i)]
		if !ok {
			p = nil
		} else if p == nil {
			p = []byte{}
		}
		put(i, p)
	}
	for pid := 0; pid < r.m; pid++ {
		p, ok := b.pidToRepairPayload[protocol.ParityID(pid)]
		if ok && p == nil {
			p = []byte{}
		}
		put(r.k+pid, p)
	}
	var st C.int
	var rc C.int
	if byRef {
		rc = C.fec_go_decoder_submit_ref(r.d, C.uint64_t(b.id), C.uint64_t(b.smallestSSID), C.uint64_t(b.largestSSID),
			C.int(b.biggestSourceSymbolLenSoFar), (**C.uint8_t)(unsafe.Pointer(r.src)), r.lens,
			(**C.uint8_t)(unsafe.Pointer(&ptrs[r.k])), &lens[r.k], &st)
	} else {
		rc = C.fec_go_decoder_submit(r.d, C.uint64_t(b.id), C.uint64_t(b.smallestSSID), C.uint64_t(b.largestSSID),
			C.int(b.biggestSourceSymbolLenSoFar), (**C.uint8_t)(unsafe.Pointer(r.src)), r.lens,
			(**C.uint8_t)(unsafe.Pointer(&ptrs[r.k])), &lens[r.k], &st)
	}
	return st != 0, goErr(rc)
}

// Recovered is one finished block: recoverSymbolPayloads' result for it.
type Recovered struct {
	BlockID  protocol.BlockID
	Payloads []byte
}

// Poll hands back the recovered payloads of finished blocks, in submit order.
func (r *BatchReceiver) Poll(wait bool) ([]Recovered, error) {
	defer lockThread()()
	w := C.int(0)
	if wait {
		w = 1
	}
	var nb C.size_t
	rc := C.fec_go_decoder_poll(r.d, w, &r.ids[0], &r.plen[0], &r.offs[0], (*C.uint8_t)(&r.out[0]),
		C.size_t(len(r.out)), C.size_t(len(r.ids)), &nb)
	if err := goErr(rc); err != nil {
		return nil, err
	}
	res := make([]Recovered, int(nb))
	for d := range res {
		o, n := int(r.offs[d]), int(r.plen[d])
		res[d] = Recovered{BlockID: protocol.BlockID(r.ids[d]), Payloads: append([]byte(nil), r.out[o:o+n]...)}
	}
	return res, nil
}
