//go:build !fechip

package fec

import "github.com/quic-go/quic-go/internal/protocol"

// Default build (no -tags fechip): the GPU engine is not linked. The selection hooks that
// go/patches/manager.go.diff adds to NewSender / NewReceiver (manager.go:50-94) find nothing
// here and fall through to the reference's own schemes, so this build behaves, links and
// tests exactly as the reference.

func useHIP() bool { return false }

// newHIPSender / newHIPReceiver: (manager, true, err) when the GPU path takes scheme id;
// (nil, false, nil) to fall through to the reference's switch.
func newHIPSender(id protocol.DecoderFECScheme) (Sender, bool, error) { return nil, false, nil }

func newHIPReceiver(id protocol.DecoderFECScheme) (Receiver, bool, error) { return nil, false, nil }
