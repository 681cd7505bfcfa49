package fec

import (
	"github.com/quic-go/quic-go/internal/protocol"
	"github.com/quic-go/quic-go/internal/wire"
)

// The asynchronous faces of Sender and Receiver (manager.go:13-22). No build tag: the packer
// and connection hooks (go/patches/) type-assert these on every build, and only the GPU batch
// managers (batch_manager_hip.go, build tag fechip) implement them, so on the default build the
// assertions fail and the reference's synchronous path runs unchanged.

// RepairPoller is a Sender whose repair frames are produced asynchronously: its
// AddSourceSymbolFrame stages a block that becomes complete and returns no frames
// (manager.go:144-154 returns them at once), and the frames of finished blocks come from
// PollRepairFrames, whole blocks only, in submit order, at most maxFrames frames (the room
// left in the connection's repair queue, which panics when full: repair_queue.go:46-53).
type RepairPoller interface {
	PollRepairFrames(maxFrames int) ([]*wire.RepairFrame, error)
}

// RecoveredBlock is one block's recovered data (recoverSymbolPayloads' result,
// reed_solomon.go:128-133) with the destination connection ID of the 1-RTT packet whose REPAIR
// frame made the block recoverable. The reference handles those frames inside that packet
// (connection.go:1341-1376) with its destConnID (:1370), which handleRetireConnectionIDFrame checks
// the retired sequence number against (:1444, :1605-1606); the batch receiver hands them over
// later, so it carries the ID with the block.
type RecoveredBlock struct {
	Data       []byte
	DestConnID protocol.ConnectionID
}

// RecoveredPoller is a Receiver whose recoveries are produced asynchronously: its
// HandleRepairFrame stages a block that becomes recoverable and returns no data
// (manager.go:181-193 returns it at once), and the data of finished blocks comes from
// PollRecovered in staging order. SetRepairDestConnID names the destination connection ID of the
// packet whose REPAIR frame the next HandleRepairFrame call handles; a block that call stages is
// returned with it. wait: start and wait for every staged block; else hand over what has finished
// and start what is staged. RecoveryPending reports staged blocks whose data has not been handed
// out yet (or received buffers to give back); RecoveriesInFlight only the former, for which the
// connection schedules a re-poll (go/patches/connection.go.diff, maybeResetTimer).
type RecoveredPoller interface {
	SetRepairDestConnID(id protocol.ConnectionID)
	PollRecovered(wait bool) ([]RecoveredBlock, error)
	RecoveryPending() bool
	RecoveriesInFlight() bool
}

// PayloadAllocator is a Sender that wants SOURCE_SYMBOL payloads built in buffers of its own (the
// GPU batch sender's registered packet-buffer pool, read by the device in place). The packer's
// hook (go/patches/packet_packer.go.diff, at packet_packer.go:984) asks it first; nil means
// "make one as the reference does".
type PayloadAllocator interface {
	SourcePayloadBuffer() []byte
}

// Closer is a Sender or Receiver that holds device state and buffers of the process-wide packet
// pool (the GPU batch managers). The connection calls Close once its run loop has ended
// (go/patches/connection.go.diff); the reference managers hold only Go memory and do not
// implement it.
type Closer interface {
	Close()
}
