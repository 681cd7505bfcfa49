//go:build fechip

package fec

// #include "fec_go.h"
import "C"

import (
	"sync"
	"unsafe"

	"github.com/quic-go/quic-go/internal/protocol"
)

// PacketPool is the opt-in registered packet-buffer pool (include/fec_go.h fec_go_pool_new,
// FEC_HIP_POOL=<buffers>): SOURCE_SYMBOL payloads are built in its buffers instead of in
// make([]byte, 0, MaxPacketBufferSize) (packet_packer.go:984, through the fecSourcePayloadBuffer
// hook of go/patches/packet_packer.go.diff), and BatchSender.SubmitRef hands them to the library
// by address: the GPU gathers them over PCIe when the batch is coded, so the run loop copies
// nothing in. The buffers are C memory without Go pointers, so cgo passes their addresses with
// no pinning. A buffer goes back to the pool when its block's frames have been polled.
type PacketPool struct {
	p    *C.fec_go_pool
	base unsafe.Pointer
	n    int
	mu   sync.Mutex
	free []int32
	used []bool
}

// NewPacketPool makes a pool of nbuf packet buffers.
func NewPacketPool(nbuf int) (*PacketPool, error) {
	var base *C.uint8_t
	var rc C.int
	p := C.fec_go_pool_new(C.size_t(nbuf), &base, &rc)
	if p == nil {
		return nil, hipErr(rc)
	}
	pp := &PacketPool{p: p, base: unsafe.Pointer(base), n: nbuf, free: make([]int32, nbuf), used: make([]bool, nbuf)}
	for i := range pp.free {
		pp.free[i] = int32(nbuf - 1 - i)
	}
	return pp, nil
}

// Get returns an empty buffer of capacity MaxPacketBufferSize, or nil when every buffer is out
// (the caller then makes one on the Go heap, which SubmitRef copies like Submit).
func (pp *PacketPool) Get() []byte {
	pp.mu.Lock()
	defer pp.mu.Unlock()
	if len(pp.free) == 0 {
		return nil
	}
	i := pp.free[len(pp.free)-1]
	pp.free = pp.free[:len(pp.free)-1]
	pp.used[i] = true
	buf := unsafe.Slice((*byte)(unsafe.Add(pp.base, int(i)*C.FEC_GO_POOL_SLOT)), protocol.MaxPacketBufferSize)
	return buf[:0]
}

// Put returns a buffer Get handed out (any reslice of it); other slices are ignored.
func (pp *PacketPool) Put(b []byte) {
	if cap(b) == 0 {
		return
	}
	off := uintptr(unsafe.Pointer(unsafe.SliceData(b))) - uintptr(pp.base)
	if off >= uintptr(pp.n)*C.FEC_GO_POOL_SLOT {
		return
	}
	i := int32(off / C.FEC_GO_POOL_SLOT)
	pp.mu.Lock()
	defer pp.mu.Unlock()
	if pp.used[i] {
		pp.used[i] = false
		pp.free = append(pp.free, i)
	}
}

// Close releases the pool: new SubmitRef calls copy; the memory itself goes when the last batch
// that reads it completes (the library keeps it alive until then).
func (pp *PacketPool) Close() {
	if pp.p != nil {
		C.fec_go_pool_free(pp.p)
		pp.p = nil
	}
}

var (
	sharedPoolOnce sync.Once
	sharedPool     *PacketPool
)

// hipPacketPool is the process-wide pool every batch sender draws from (FEC_HIP_POOL buffers),
// or nil when the option is off or the pool cannot be made (the copying path then runs).
func hipPacketPool() *PacketPool {
	sharedPoolOnce.Do(func() {
		if n := hipPoolBuffers(); n > 0 {
			sharedPool, _ = NewPacketPool(n)
		}
	})
	return sharedPool
}
