//go:build fechip

package fec

import (
	"sync"
	"unsafe"

	"github.com/quic-go/quic-go/internal/protocol"
	"github.com/quic-go/quic-go/internal/wire"
)

// hipBatchBlocks is the most blocks one kernel launch codes (per staging set of the library).
const hipBatchBlocks = 1024

// hipCode: the (k, m) the reference's factories use for a scheme (manager.go:54-67, 77-90).
func hipCode(id protocol.DecoderFECScheme) (k, m int, ok bool) {
	switch id {
	case protocol.XORFECScheme:
		return 2, 1, true
	case protocol.ReedSolomonFECScheme:
		return 20, 10, true
	}
	return 0, 0, false
}

// newHIPBlockScheme: the per-block GPU schemes (FEC_HIP=block).
func newHIPBlockScheme(id protocol.DecoderFECScheme, k, m int) (BlockFECScheme, error) {
	if id == protocol.XORFECScheme {
		return newHipXorScheme()
	}
	return newHipReedSolomonScheme(k, m)
}

// newHIPSender is the hook go/patches/manager.go.diff puts at the top of NewSender
// (manager.go:50): (sender, true, err) when FEC_HIP selects the GPU for scheme id, else
// (nil, false, nil) and the reference's switch runs. FECDisabled and unknown ids always fall
// through, so their results and errors stay the reference's.
func newHIPSender(id protocol.DecoderFECScheme) (Sender, bool, error) {
	k, m, ok := hipCode(id)
	if !ok || !useHIP() {
		return nil, false, nil
	}
	if hipMode() == "block" {
		s, err := newHIPBlockScheme(id, k, m)
		if err != nil {
			return nil, true, err
		}
		mgr, err := NewManager(s, k, m)
		if err != nil {
			return nil, true, err
		}
		return mgr, true, nil
	}
	bm, err := newBatchManager(id, k, m, true)
	if err != nil {
		return nil, true, err
	}
	return bm, true, nil
}

// newHIPReceiver is the same hook for NewReceiver (manager.go:73).
func newHIPReceiver(id protocol.DecoderFECScheme) (Receiver, bool, error) {
	k, m, ok := hipCode(id)
	if !ok || !useHIP() {
		return nil, false, nil
	}
	if hipMode() == "block" {
		s, err := newHIPBlockScheme(id, k, m)
		if err != nil {
			return nil, true, err
		}
		mgr, err := NewManager(s, k, m)
		if err != nil {
			return nil, true, err
		}
		return mgr, true, nil
	}
	bm, err := newBatchManager(id, k, m, false)
	if err != nil {
		return nil, true, err
	}
	return bm, true, nil
}

// batchManager is manager.go's sender / receiver with its two scheme calls deferred to the GPU
// batch path: the block bookkeeping is the embedded reference manager's own (blockStatuses,
// newBlock, addSourceSymbol / addRepairSymbol, isComplete / isRecoverable, NextSSID,
// HandleSourceSymbolFrame, all unchanged); only `m.scheme.repairSymbols(bS.block)`
// (manager.go:145) becomes BatchSender.Submit and `m.scheme.recoverSymbolPayloads(bS.block)`
// (manager.go:182) becomes BatchReceiver.Submit. Results come back through RepairPoller /
// RecoveredPoller (fec_poll.go), which the packer and connection hooks poll
// (go/patches/packet_packer.go.diff, connection.go.diff). One per connection, driven by its run
// loop only (connection.go:525), like the reference manager; it owns its library encoder /
// decoder, so different connections never share a device context.
type batchManager struct {
	*manager
	tx      *BatchSender
	rx      *BatchReceiver
	pending int // receiver: blocks staged whose data has not been handed out yet
	// sender with a registered packet-buffer pool (FEC_HIP_POOL): payloads of blocks submitted by
	// reference, held until their frames are polled, then returned to the pool
	pool *PacketPool
	held map[protocol.BlockID][][]byte
	// receiver with the pool: received payloads are read into its buffers (wire.FECPayloadBuffer,
	// go/patches/fec_source_symbol_frame.go.diff) and recoverable blocks go in by reference
	// (BatchReceiver.SubmitRef). A staged block's buffers go back once its data has been polled
	// (rxHeld); buffers no block keeps go back at the next PollRecovered (release), because the
	// connection parses a SOURCE_SYMBOL payload after HandleSourceSymbolFrame returns it
	// (connection.go:1653), copying what it keeps (stream_frame.go:56-76).
	rxHeld  map[protocol.BlockID][][]byte
	release [][]byte
	// receiver: the destination connection ID of the packet whose REPAIR frame is being handled
	// (SetRepairDestConnID), and that of each staged block, handed out with its data
	repairDest protocol.ConnectionID
	dest       map[protocol.BlockID]protocol.ConnectionID
}

var (
	_ Sender           = &batchManager{}
	_ Receiver         = &batchManager{}
	_ RepairPoller     = &batchManager{}
	_ RecoveredPoller  = &batchManager{}
	_ PayloadAllocator = &batchManager{}
	_ Closer           = &batchManager{}
)

func newBatchManager(id protocol.DecoderFECScheme, k, m int, send bool) (*batchManager, error) {
	mgr, err := NewManager(nil, k, m) // no scheme: its two calls are the ones replaced below
	if err != nil {
		return nil, err
	}
	bm := &batchManager{manager: mgr}
	if send {
		bm.tx, err = NewBatchSender(id, k, m, hipBatchBlocks)
		if bm.pool = hipPacketPool(); bm.pool != nil {
			bm.held = make(map[protocol.BlockID][][]byte)
		}
	} else {
		bm.rx, err = NewBatchReceiver(id, k, m, hipBatchBlocks)
		bm.dest = make(map[protocol.BlockID]protocol.ConnectionID)
		if bm.pool = hipPacketPool(); bm.pool != nil {
			bm.rxHeld = make(map[protocol.BlockID][][]byte)
			hookWirePayloads(bm.pool)
		}
	}
	if err != nil {
		return nil, err
	}
	return bm, nil
}

// AddSourceSymbolFrame is manager.go:123-158 with repairSymbols (:145) replaced by a Submit of
// the complete block; it returns no frames (they come from PollRepairFrames).
func (m *batchManager) AddSourceSymbolFrame(f *wire.SourceSymbolFrame) ([]*wire.RepairFrame, error) {
	blockID := m.sidToBlockID(f.SSID)
	if _, exists := m.blockStatuses[blockID]; !exists {
		m.blockStatuses[blockID] = blockStatus{
			block:       newBlock(blockID, m.numTotSourceSymbols, m.numTotRepairSymbols),
			isProcessed: false}
	}
	bS := m.blockStatuses[blockID]
	if bS.isProcessed {
		return nil, nil
	}
	if err := bS.block.addSourceSymbol(f); err != nil {
		return nil, err
	}
	if bS.block.isComplete() {
		if m.pool == nil {
			if err := m.tx.Submit(bS.block); err != nil {
				return nil, err
			}
		} else {
			// by reference: the device reads the pool buffers when the batch is coded, so they
			// stay out of the pool until PollRepairFrames returns this block
			if err := m.tx.SubmitRef(bS.block); err != nil {
				return nil, err
			}
			ps := make([][]byte, 0, len(bS.block.ssidToSourcePayload))
			for _, p := range bS.block.ssidToSourcePayload {
				ps = append(ps, p)
			}
			m.held[blockID] = ps
		}
		// the library holds what it needs: drop the block as manager.go:150-153 does
		bS.block = nil
		bS.isProcessed = true
	}
	m.blockStatuses[blockID] = bS
	return nil, nil
}

// PollRepairFrames hands over the repair frames of finished blocks, whole blocks only, at most
// maxFrames frames; the rest wait in the library. Also starts coding the staged blocks when no
// batch is in flight (fec_go_encoder_poll), so a block is never left waiting for a full batch.
func (m *batchManager) PollRepairFrames(maxFrames int) ([]*wire.RepairFrame, error) {
	maxBlocks := 0
	if maxFrames > 0 {
		maxBlocks = maxFrames / m.tx.m
	}
	blocks, err := m.tx.Poll(false, maxBlocks)
	if err != nil {
		return nil, err
	}
	var out []*wire.RepairFrame
	for _, fs := range blocks {
		out = append(out, fs...)
		if m.pool != nil && len(fs) > 0 {
			id := fs[0].Metadata.BlockID
			for _, p := range m.held[id] {
				m.pool.Put(p)
			}
			delete(m.held, id)
		}
	}
	return out, nil
}

// SourcePayloadBuffer is the packer's buffer for the next SOURCE_SYMBOL payload: a registered
// packet buffer when this sender has a pool (nil otherwise, or when the pool is exhausted: the
// packer then makes one as the reference does and SubmitRef copies it).
func (m *batchManager) SourcePayloadBuffer() []byte {
	if m.pool == nil {
		return nil
	}
	return m.pool.Get()
}

var wireHookOnce sync.Once

// hookWirePayloads points the wire parser's payload allocation at the pool (process-wide, as the
// pool is). The bytes past the payload are zeroed, as make's are: addLengthToSourceSymbolPayload
// reslices a source payload into its capacity (reed_solomon.go:77-87).
func hookWirePayloads(pp *PacketPool) {
	wireHookOnce.Do(func() {
		wire.FECPayloadBuffer = func(n int) []byte {
			if n > protocol.MaxPacketBufferSize {
				return nil
			}
			b := pp.Get()
			if b == nil {
				return nil // pool exhausted: the parser makes one on the heap
			}
			b = b[:cap(b)]
			clear(b[n:])
			return b[:0]
		}
	})
}

// sameBuf: a and b are slices of one buffer (block.go:63,80 ignore a duplicate SSID / ParityID,
// whose payload the block then does not keep).
func sameBuf(a, b []byte) bool {
	return cap(a) > 0 && cap(b) > 0 && unsafe.SliceData(a) == unsafe.SliceData(b)
}

// blockPayloads: every payload a block keeps.
func blockPayloads(b *block) [][]byte {
	ps := make([][]byte, 0, len(b.ssidToSourcePayload)+len(b.pidToRepairPayload))
	for _, p := range b.ssidToSourcePayload {
		ps = append(ps, p)
	}
	for _, p := range b.pidToRepairPayload {
		ps = append(ps, p)
	}
	return ps
}

// HandleSourceSymbolFrame is the reference's (manager.go:200-227); with the pool it also notes
// which received buffers no block keeps any longer, to go back at the next PollRecovered.
func (m *batchManager) HandleSourceSymbolFrame(f *wire.SourceSymbolFrame) ([]byte, error) {
	if m.rxHeld == nil {
		return m.manager.HandleSourceSymbolFrame(f)
	}
	blockID := m.sidToBlockID(f.SSID)
	prev := m.blockStatuses[blockID].block // nil: a new block, or one already processed
	payload, err := m.manager.HandleSourceSymbolFrame(f)
	if cur := m.blockStatuses[blockID].block; cur != nil {
		if kept, ok := cur.ssidToSourcePayload[f.SSID]; !ok || !sameBuf(kept, f.Payload) {
			m.release = append(m.release, f.Payload)
		}
	} else if prev != nil { // completed by this symbol: the block is dropped (manager.go:221-224)
		if kept, ok := prev.ssidToSourcePayload[f.SSID]; !ok || !sameBuf(kept, f.Payload) {
			m.release = append(m.release, f.Payload)
		}
		m.release = append(m.release, blockPayloads(prev)...)
	} else {
		m.release = append(m.release, f.Payload)
	}
	return payload, err
}

// HandleRepairFrame is manager.go:160-198 with recoverSymbolPayloads (:182) replaced by a
// Submit of the recoverable block (SubmitRef with the pool); it returns no data (it comes from
// PollRecovered). A block that is already complete is the reference's nil, nil: nothing is
// staged.
func (m *batchManager) HandleRepairFrame(f *wire.RepairFrame) ([]byte, error) {
	if _, exists := m.blockStatuses[f.Metadata.BlockID]; !exists {
		m.blockStatuses[f.Metadata.BlockID] = blockStatus{
			block:       newBlock(f.Metadata.BlockID, m.numTotSourceSymbols, m.numTotRepairSymbols),
			isProcessed: false,
		}
	}
	bS := m.blockStatuses[f.Metadata.BlockID]
	pooled := m.rxHeld != nil
	if bS.isProcessed {
		if pooled {
			m.release = append(m.release, f.Payload)
		}
		return nil, nil
	}
	if err := bS.block.addRepairSymbol(f); err != nil {
		if pooled {
			m.release = append(m.release, f.Payload)
		}
		return nil, err
	}
	if kept := bS.block.pidToRepairPayload[f.Metadata.ParityID]; pooled && !sameBuf(kept, f.Payload) {
		m.release = append(m.release, f.Payload)
	}
	if bS.block.isRecoverable() {
		var staged bool
		var err error
		if pooled {
			staged, err = m.rx.SubmitRef(bS.block)
		} else {
			staged, err = m.rx.Submit(bS.block)
		}
		if err != nil {
			return nil, err
		}
		if staged {
			m.pending++
			m.dest[f.Metadata.BlockID] = m.repairDest
			if pooled { // the device reads these when the batch is coded
				m.rxHeld[f.Metadata.BlockID] = blockPayloads(bS.block)
			}
		} else if pooled {
			m.release = append(m.release, blockPayloads(bS.block)...)
		}
		bS.block = nil
		bS.isProcessed = true
	}
	m.blockStatuses[f.Metadata.BlockID] = bS
	return nil, nil
}

// SetRepairDestConnID: the destination connection ID of the packet whose REPAIR frame the next
// HandleRepairFrame handles (go/patches/connection.go.diff, before handleRepairFrame).
func (m *batchManager) SetRepairDestConnID(id protocol.ConnectionID) { m.repairDest = id }

// PollRecovered hands over the block data of finished recoveries in staging order (wait: every
// staged block), each with the destination connection ID of the packet that staged it. Also
// starts decoding the staged blocks when no batch is in flight.
func (m *batchManager) PollRecovered(wait bool) ([]RecoveredBlock, error) {
	var out []RecoveredBlock
	if m.rxHeld != nil { // the receive burst that used these buffers has been handled
		for _, p := range m.release {
			m.pool.Put(p)
		}
		m.release = m.release[:0]
	}
	for m.pending > 0 {
		rec, err := m.rx.Poll(wait)
		if err != nil {
			return out, err
		}
		for _, r := range rec {
			// a copy (BatchReceiver.Poll): the pool buffers can go back
			out = append(out, RecoveredBlock{Data: r.Payloads, DestConnID: m.dest[r.BlockID]})
			delete(m.dest, r.BlockID)
			if m.rxHeld != nil {
				for _, p := range m.rxHeld[r.BlockID] {
					m.pool.Put(p)
				}
				delete(m.rxHeld, r.BlockID)
			}
		}
		m.pending -= len(rec)
		if !wait || len(rec) == 0 {
			break
		}
	}
	return out, nil
}

// RecoveryPending: staged blocks whose data has not been handed out, or received pool buffers
// waiting to go back (PollRecovered returns them even when nothing is staged, so a lossless
// stream does not drain the pool).
func (m *batchManager) RecoveryPending() bool { return m.pending > 0 || len(m.release) > 0 }

// RecoveriesInFlight: staged blocks whose data has not been handed out (the connection re-polls
// while there are any).
func (m *batchManager) RecoveriesInFlight() bool { return m.pending > 0 }

// Close is the connection's teardown (go/patches/connection.go.diff, after the run loop ends):
// the library encoder / decoder is freed first, which waits for a batch still in flight (the
// device may be reading pool buffers by reference), then every pool buffer this manager still
// holds goes back: blocks submitted but not polled (held, rxHeld), buffers awaiting release, and
// the payloads of blocks that never completed. Buffers from the heap are ignored by Put.
func (m *batchManager) Close() {
	if m.tx != nil {
		m.tx.Close()
	}
	if m.rx != nil {
		m.rx.Close()
		clear(m.dest)
	}
	if m.pool == nil {
		return
	}
	for id, ps := range m.held {
		for _, p := range ps {
			m.pool.Put(p)
		}
		delete(m.held, id)
	}
	for id, ps := range m.rxHeld {
		for _, p := range ps {
			m.pool.Put(p)
		}
		delete(m.rxHeld, id)
	}
	for _, p := range m.release {
		m.pool.Put(p)
	}
	m.release = nil
	for id, bS := range m.blockStatuses {
		if bS.block != nil {
			for _, p := range blockPayloads(bS.block) {
				m.pool.Put(p)
			}
		}
		delete(m.blockStatuses, id)
	}
	m.pending = 0
}
