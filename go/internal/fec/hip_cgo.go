//go:build fechip

// Package fec additions that bind the MI355X engine (lib0xfec_hip.so). These files are dropped
// into the reference's internal/fec directory (INTEGRATION.md); they use its unexported
// block type and helpers, and build only with `-tags fechip`, so the default build is unchanged.
//
// cgo pointer rules, as applied throughout:
//   - A Go pointer passed to C may point only to memory without Go pointers ([]byte payloads
//     qualify); C must not keep it after the call. Every entry point of fec_hip.h / fec_go.h
//     copies its inputs before returning (FEC_HOST stages through the library's pinned
//     memory; fec_go_*_add copies the payload).
//   - An array of Go pointers (fec_go_encoder_submit) must itself be C memory, and the Go
//     memory it points to must be pinned (runtime.Pinner, Go 1.21 — go.mod:3) until the call
//     returns.
package fec

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/0xfec/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/0xfec/lib -l0xfec_hip -Wl,-rpath,${SRCDIR}/../../third_party/0xfec/lib
#include <stdlib.h>
#include "fec_hip.h"
#include "fec_scheme.h"
#include "fec_go.h"
*/
import "C"

import (
	"errors"
	"os"
	"runtime"
	"strconv"
)

// hipDevice is the GPU the schemes bind (FEC_HIP_DEVICE, default 0).
func hipDevice() int {
	if v, err := strconv.Atoi(os.Getenv("FEC_HIP_DEVICE")); err == nil {
		return v
	}
	return 0
}

// hipMode selects the GPU path in NewSender / NewReceiver (manager.go:50-94, through the hooks
// of go/patches/manager.go.diff):
//   - FEC_HIP=1 or FEC_HIP=batch: the batched managers (batch_manager_hip.go), the path that pays
//     off: blocks of a connection are coded many per kernel launch while the run loop carries on;
//   - FEC_HIP=block: the per-block schemes (reed_solomon_hip.go, xor_hip.go), one synchronous
//     FEC_HOST round trip per block; for wire-parity checks only, slower than the CPU per block;
//   - unset: "", the reference's CPU path.
func hipMode() string {
	switch os.Getenv("FEC_HIP") {
	case "1", "batch":
		return "batch"
	case "block":
		return "block"
	}
	return ""
}

func useHIP() bool { return hipMode() != "" }

// hipPoolBuffers is the size of the registered packet-buffer pool the batch senders build
// SOURCE_SYMBOL payloads in (FEC_HIP_POOL, packet_pool_hip.go); 0 (unset): no pool, payloads are
// copied into the library's pinned staging at submit.
func hipPoolBuffers() int {
	if v, err := strconv.Atoi(os.Getenv("FEC_HIP_POOL")); err == nil && v > 0 {
		return v
	}
	return 0
}

// hipErr turns a fec_hip.h return code into an error (nil for 0).
func hipErr(rc C.int) error {
	if rc == 0 {
		return nil
	}
	return errors.New(C.GoString(C.fec_strerror(rc)))
}

// lockThread keeps the goroutine on its OS thread from a C call to the fec_last_error read in
// goErr (the message is thread-local): `defer lockThread()()`.
func lockThread() func() {
	runtime.LockOSThread()
	return runtime.UnlockOSThread
}

// goErr turns a fec_go.h / fec_scheme.h return code into an error: FEC_ERR_SCHEME carries the
// reference's own error text (fec_last_error, thread-local: the caller holds lockThread).
func goErr(rc C.int) error {
	if rc == 0 {
		return nil
	}
	if msg := C.GoString(C.fec_last_error()); msg != "" {
		return errors.New(msg)
	}
	return hipErr(rc)
}
