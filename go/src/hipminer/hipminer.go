// Package hipminer is the cgo binding of libhipminer.so (include/hipminer.h):
// the MI355X backend for the min-hash scan of the reference miner
// (cmu440/bitcoin/miner/miner.go:46-59, bitcoin.Hash at
// cmu440/bitcoin/hash.go:13-17).
//
// GOPATH layout: this repo's go/ directory is a GOPATH entry (go/src/hipminer),
// next to the reference's p1/ (github.com/cmu440/...).  Go 1.10 (the staff
// binaries' go1.10.3) or newer; with Go >= 1.11 build with GO111MODULE=off.
// Built only where a Go toolchain exists (none in the build image):
// tests/test_cgo_surface.py checks every C.* name used here against
// include/hipminer.h and compiles and runs the same C calls with gcc.
package hipminer

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../distributed_bitcoinminer_amd -lhipminer -Wl,-rpath,${SRCDIR}/../../../distributed_bitcoinminer_amd
#include <stdlib.h>
#include "hipminer.h"
*/
import "C"

import (
	"fmt"
	"unsafe"
)

const maxUint64 = ^uint64(0)

// cbytes copies s into C memory for one call (nil for ""; s may hold any
// byte, NUL included).  The caller frees it with C.free.  Messages are short,
// so the copy costs nothing next to a scan.
func cbytes(s string) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(C.CBytes([]byte(s)))
}

// Return codes of include/hipminer.h that callers branch on.
const (
	ErrInvalid  = int(C.HM_ERR_INVALID)
	ErrNoDevice = int(C.HM_ERR_NO_DEVICE)
	// ErrTimeout (ABI 1.8): the scan missed its deadline (SetDeadline); the
	// context is abandoned -- Close it (no device wait) and answer elsewhere.
	ErrTimeout = int(C.HM_ERR_TIMEOUT)
)

// DeadlineAuto makes SetDeadline use the library's modelled deadline: 2 s +
// 8x the call's modelled kernel time.
const DeadlineAuto = -1

// Error carries an hm_* return code.
type Error struct{ Code int }

func (e Error) Error() string {
	return fmt.Sprintf("hipminer: %s (rc=%d)", C.GoString(C.hm_strerror(C.int(e.Code))), e.Code)
}

// Miner owns one hm_ctx (device buffers, streams).  Safe for concurrent use:
// the library serialises calls per context and re-binds the device on every
// call, so Go may run them on any OS thread.
type Miner struct{ ctx *C.hm_ctx }

// Open binds the given HIP device ordinals; none means every visible device.
func Open(devices ...int) (*Miner, error) {
	var ctx *C.hm_ctx
	var rc C.int
	if len(devices) == 0 {
		rc = C.hm_open(nil, 0, &ctx)
	} else {
		ds := make([]C.int, len(devices))
		for i, d := range devices {
			ds[i] = C.int(d)
		}
		rc = C.hm_open(&ds[0], C.int(len(ds)), &ctx)
	}
	if rc != 0 {
		return nil, Error{int(rc)}
	}
	return &Miner{ctx: ctx}, nil
}

// SetDeadline bounds every later scan on m (HM_OPT_DEADLINE_MS): ms > 0 that
// many milliseconds per call, DeadlineAuto the modelled deadline, 0 none.  A
// scan past its deadline returns Error{ErrTimeout} instead of blocking, so a
// hung GPU cannot keep a heartbeating miner from answering (SURVEY §8(b)).
func (m *Miner) SetDeadline(ms int64) error {
	if rc := C.hm_set_option(m.ctx, C.HM_OPT_DEADLINE_MS, C.int64_t(ms)); rc != 0 {
		return Error{int(rc)}
	}
	return nil
}

// ScanInclusive returns the lexicographic min of (Hash(data, n), n) over the
// inclusive range [lo, hi]; (MaxUint64, 0) when lo > hi.
func (m *Miner) ScanInclusive(data string, lo, hi uint64) (hash, nonce uint64, err error) {
	var out C.hm_result
	p := cbytes(data)
	defer C.free(unsafe.Pointer(p))
	rc := C.hm_scan(m.ctx, p, C.size_t(len(data)), C.uint64_t(lo), C.uint64_t(hi), &out)
	if rc != 0 {
		return 0, 0, Error{int(rc)}
	}
	return uint64(out.hash), uint64(out.nonce), nil
}

// Request is one (data, lo, hi) job of a batch; lo and hi are inclusive.
type Request struct {
	Data   string
	Lo, Hi uint64
}

// ScanChecked is ScanInclusive plus the coverage checksum of
// hm_scan_checked: the sum of every key in [lo, hi] mod 2^64 and the number
// of nonces hashed.  For verification runs; slower than ScanInclusive.
func (m *Miner) ScanChecked(data string, lo, hi uint64) (hash, nonce, sum, count uint64, err error) {
	var out C.hm_result
	var s, c C.uint64_t
	p := cbytes(data)
	defer C.free(unsafe.Pointer(p))
	rc := C.hm_scan_checked(m.ctx, p, C.size_t(len(data)), C.uint64_t(lo), C.uint64_t(hi), &out, &s, &c)
	if rc != 0 {
		return 0, 0, 0, 0, Error{int(rc)}
	}
	return uint64(out.hash), uint64(out.nonce), uint64(s), uint64(c), nil
}

// ScanMany runs hm_scan_many: every request's GPU work is queued before one
// synchronisation.  Results are in request order.
func (m *Miner) ScanMany(reqs []Request) ([][2]uint64, error) {
	if len(reqs) == 0 {
		return nil, nil
	}
	// C memory for the request array: it holds pointers (to the message bytes),
	// which the cgo rules do not allow in Go memory passed to C.
	creqs := (*[1 << 20]C.hm_request)(C.malloc(C.size_t(len(reqs)) * C.size_t(unsafe.Sizeof(C.hm_request{}))))[:len(reqs):len(reqs)]
	defer C.free(unsafe.Pointer(&creqs[0]))
	cbufs := make([]unsafe.Pointer, 0, len(reqs))
	defer func() {
		for _, b := range cbufs {
			C.free(b)
		}
	}()
	for i, r := range reqs {
		p := cbytes(r.Data)
		cbufs = append(cbufs, unsafe.Pointer(p))
		creqs[i] = C.hm_request{msg: p, len: C.size_t(len(r.Data)), lo: C.uint64_t(r.Lo), hi: C.uint64_t(r.Hi)}
	}
	outs := make([]C.hm_result, len(reqs))
	if rc := C.hm_scan_many(m.ctx, &creqs[0], C.int(len(reqs)), &outs[0]); rc != 0 {
		return nil, Error{int(rc)}
	}
	res := make([][2]uint64, len(reqs))
	for i, o := range outs {
		res[i] = [2]uint64{uint64(o.hash), uint64(o.nonce)}
	}
	return res, nil
}

// EvalRequest is the drop-in for miner.go:46-59: it keeps the reference's
// `upper := Upper + 1` uint64 wrap (Upper == MaxUint64 scans nothing) and
// its initial (MaxUint64, 0).
func (m *Miner) EvalRequest(data string, lower, upper uint64) (hash, nonce uint64, err error) {
	end := upper + 1 // wraps exactly like miner.go:52
	if !(lower < end) {
		return maxUint64, 0, nil
	}
	return m.ScanInclusive(data, lower, end-1)
}

// ScanCPU is hm_scan_cpu: the same scan as ScanInclusive, bit-identical, on
// the host's cores (threads <= 0: one thread per CPU in this process's
// affinity mask, at most 1024 -- not every hardware thread of the machine).
// For a miner whose GPU is missing or failed, so that a Result is still
// written (SURVEY §8(b)); orders of magnitude slower than the GPU.
func ScanCPU(data string, lo, hi uint64, threads int) (hash, nonce uint64, err error) {
	var out C.hm_result
	p := cbytes(data)
	defer C.free(unsafe.Pointer(p))
	rc := C.hm_scan_cpu(p, C.size_t(len(data)), C.uint64_t(lo), C.uint64_t(hi), C.int(threads), &out)
	if rc != 0 {
		return 0, 0, Error{int(rc)}
	}
	return uint64(out.hash), uint64(out.nonce), nil
}

// EvalRequestCPU is EvalRequest on the host (ScanCPU), with the same
// `upper := Upper + 1` wrap and initial (MaxUint64, 0).
func EvalRequestCPU(data string, lower, upper uint64, threads int) (hash, nonce uint64, err error) {
	end := upper + 1 // wraps exactly like miner.go:52
	if !(lower < end) {
		return maxUint64, 0, nil
	}
	return ScanCPU(data, lower, end-1, threads)
}

// Close releases the context (an abandoned one after ErrTimeout: host
// memory only, without waiting on the device).
func (m *Miner) Close() {
	if m.ctx != nil {
		C.hm_close(m.ctx)
		m.ctx = nil
	}
}

// Hash is bitcoin.Hash(msg, nonce) computed by the library on the host.
func Hash(msg string, nonce uint64) uint64 {
	p := cbytes(msg)
	defer C.free(unsafe.Pointer(p))
	return uint64(C.hm_hash(p, C.size_t(len(msg)), C.uint64_t(nonce)))
}

// Partition splits the inclusive range [lo, hi] into n contiguous shards of
// near-equal modelled GPU cost for data (hm_partition; host-only).  Shard i
// is [out[i][0], out[i][1]]; an empty shard has out[i][0] > out[i][1].  A
// process-per-GPU launcher gives shard i to the miner on GPU i.
func Partition(data string, lo, hi uint64, n int) ([][2]uint64, error) {
	if n <= 0 {
		return nil, Error{int(C.HM_ERR_INVALID)}
	}
	p := cbytes(data)
	defer C.free(unsafe.Pointer(p))
	bounds := make([]C.uint64_t, 2*n)
	if rc := C.hm_partition(p, C.size_t(len(data)), C.uint64_t(lo), C.uint64_t(hi),
		C.int(n), &bounds[0]); rc != C.HM_OK {
		return nil, Error{int(rc)}
	}
	out := make([][2]uint64, n)
	for i := range out {
		out[i] = [2]uint64{uint64(bounds[2*i]), uint64(bounds[2*i+1])}
	}
	return out, nil
}

// BuildID is hm_build_id(): the digest of the sources libhipminer.so was built
// from (distributed_bitcoinminer_amd/build_id.py), for start-up logs and
// deployment checks.
func BuildID() string {
	return C.GoString(C.hm_build_id())
}
