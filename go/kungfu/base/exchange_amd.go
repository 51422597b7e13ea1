//go:build kungfu_amd

// The multi-GPU exchange (kungfu_amd.h, kf_exchange_*) for the Go runtime:
// what srcs/cpp/src/nccl/gpu_collective.cpp gives the reference's C++ side,
// reachable from Go. The id is created on rank 0 and broadcast by the
// caller's own KungFu session (gpu_collective.cpp:190-200 does it with
// Peer::Broadcast):
//
//	var id [ExchangeIDBytes]byte
//	if rank == 0 { id, _ = ExchangeUniqueID() }
//	w := base.Workspace{SendBuf: idVec, RecvBuf: idVec, Name: "nccl id"}
//	sess.Broadcast(w)                       // session/session.go:164-167
//	ex, _ := NewExchange(id, rank, size, device)
//	ex.AllReduceBatch(bufs, counts, F32, SUM, true, AlgoAuto, stream)
package base

// #include <stdlib.h>
// #include "kungfu_amd.h"
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

const ExchangeIDBytes = C.KF_UNIQUE_ID_BYTES

// Exchange algorithms (enum KF_ExchangeAlgo).
const (
	AlgoAuto             = int(C.KF_ALGO_AUTO)
	AlgoReduceScatter    = int(C.KF_ALGO_REDUCE_SCATTER)
	AlgoAllToAll         = int(C.KF_ALGO_ALL_TO_ALL)
	AlgoReduceScatterAvg = int(C.KF_ALGO_REDUCE_SCATTER_AVG)
)

type Exchange struct {
	h *C.kf_exchange_t
}

func exStatus(fn string, rc C.int) error {
	if rc == C.KF_OK {
		return nil
	}
	return fmt.Errorf("%s: status %d: %s", fn, int(rc), C.GoString(C.kf_exchange_last_error()))
}

// ExchangeUniqueID: ncclGetUniqueId, on rank 0 only.
func ExchangeUniqueID() ([ExchangeIDBytes]byte, error) {
	var id [ExchangeIDBytes]byte
	p := C.malloc(C.size_t(ExchangeIDBytes))
	defer C.free(p)
	if err := exStatus("kf_exchange_unique_id", C.kf_exchange_unique_id(p)); err != nil {
		return id, err
	}
	copy(id[:], unsafe.Slice((*byte)(p), ExchangeIDBytes))
	return id, nil
}

// NewExchange: the communicator of `size` ranks on HIP device `device`.
func NewExchange(id [ExchangeIDBytes]byte, rank, size, device int) (*Exchange, error) {
	return NewExchangeTimeout(id, rank, size, device, -1)
}

// NewExchangeTimeout: NewExchange that gives up after timeoutMs (< 0: no
// limit) if not every rank joined the communicator's init.
func NewExchangeTimeout(id [ExchangeIDBytes]byte, rank, size, device, timeoutMs int) (*Exchange, error) {
	p := C.malloc(C.size_t(ExchangeIDBytes))
	defer C.free(p)
	copy(unsafe.Slice((*byte)(p), ExchangeIDBytes), id[:])
	h := C.kf_exchange_create_timeout(p, C.int(rank), C.int(size), C.int(device), C.int(timeoutMs))
	if h == nil {
		return nil, errors.New("kf_exchange_create: " + C.GoString(C.kf_exchange_last_error()))
	}
	return &Exchange{h: h}, nil
}

// AllReduceBatch: every bucket all-reduced in place (average: SUM then / np),
// queued on s; one grouped RCCL launch per phase for all of them.
func (e *Exchange) AllReduceBatch(bufs []DevicePtr, counts []int, t DataType, op OP,
	average bool, algo int, s Stream) error {
	if len(bufs) != len(counts) {
		return errors.New("kungfu_amd: one count per bucket")
	}
	nb := len(bufs)
	if nb == 0 {
		return nil
	}
	word := C.size_t(unsafe.Sizeof(uintptr(0)))
	ps := C.malloc(C.size_t(nb) * word)
	cs := C.malloc(C.size_t(nb) * C.size_t(unsafe.Sizeof(C.size_t(0))))
	defer C.free(ps)
	defer C.free(cs)
	pv := unsafe.Slice((*uintptr)(ps), nb)
	cv := unsafe.Slice((*C.size_t)(cs), nb)
	for i := range bufs {
		pv[i] = uintptr(bufs[i])
		cv[i] = C.size_t(counts[i])
	}
	avg := C.int(0)
	if average {
		avg = 1
	}
	rc := C.kf_exchange_all_reduce_batch(e.h, (*unsafe.Pointer)(ps), (*unsafe.Pointer)(ps),
		(*C.size_t)(cs), C.int(nb), C.KungFu_Datatype(t), C.KungFu_Op(op), avg, C.int(algo),
		unsafe.Pointer(uintptr(s)))
	return exStatus("kf_exchange_all_reduce_batch", rc)
}

// Check reports an asynchronous RCCL failure.
func (e *Exchange) Check() error { return exStatus("kf_exchange_check", C.kf_exchange_check(e.h)) }

// TransportInfo is what RCCL itself reports (kf_exchange_transport_info):
// the communicator's rank count (ncclCommCount) and RCCL's version code
// (ncclGetVersion); -1 and 0 over a host-provided transport.
func (e *Exchange) TransportInfo() (commCount int, version int, err error) {
	var c, v C.int
	if err := exStatus("kf_exchange_transport_info",
		C.kf_exchange_transport_info(e.h, &c, &v)); err != nil {
		return 0, 0, err
	}
	return int(c), int(v), nil
}

// SetPipeline splits every batch call into groups whose HIP work overlaps the
// next group's RCCL phases (kf_exchange_set_pipeline; 1 = off). Same results.
func (e *Exchange) SetPipeline(groups int) error {
	return exStatus("kf_exchange_set_pipeline", C.kf_exchange_set_pipeline(e.h, C.int(groups)))
}

func (e *Exchange) Close() {
	if e.h != nil {
		C.kf_exchange_destroy(e.h)
		e.h = nil
	}
}
