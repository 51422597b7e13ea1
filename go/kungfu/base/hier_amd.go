//go:build kungfu_amd

// Name-keyed all-reduce, sub-communicators and the hierarchical all-reduce
// (kungfu_amd.h) for the Go runtime.
//
//   - AllReduceNamed is GoKungfuAllReduce with a done callback
//     (srcs/go/libkungfu-comm/collective.go:34-45) on the multi-GPU exchange:
//     ranks may start their names in any order; tensors pair by name, as
//     rchannel/handler/collective.go:48-64 pairs messages.
//   - NewLocalExchange / Split are gpu_collective::new_local / new_group
//     (srcs/cpp/src/nccl/gpu_collective.cpp:202-243).
//   - HierAllReduce is ScheduledHierarchicalNcclAllReduce
//     (srcs/cpp/src/tensorflow/ops/gpu/collective.cpp:108-162): host
//     reduce-scatter, the shard across hosts over the device-mode session,
//     / np, host all-gather.
//
//	sess, _ := base.NewSession(peers, self, "/tmp", token, true)
//	local, _ := base.NewLocalExchange(sess, device)
//	base.HierAllReduce(local, sess, grad, n, F32, SUM, true, AlgoAuto, "grad/0", stream)
package base

/*
#include <stdlib.h>
#include "kungfu_amd.h"
extern void kfGoNamedDone(int status, void *arg);
static int kf_go_named(kf_exchange_t *ex, const char *name, void *buf, size_t count,
                       KungFu_Datatype dt, KungFu_Op op, int average, int algo, void *stream,
                       uintptr_t h)
{
	return kf_exchange_all_reduce_named(ex, name, buf, buf, count, dt, op, average, algo,
	                                    stream, kfGoNamedDone, (void *)h);
}
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime/cgo"
	"unsafe"
)

// Session is the native session engine (kf_session_*): the reference's
// Peer over rchannel, with device-mode buffers in HBM.
type Session struct {
	h *C.kf_session_t
}

func sessStatus(fn string, rc C.int) error {
	if rc == C.KF_OK {
		return nil
	}
	return fmt.Errorf("%s: status %d: %s", fn, int(rc), C.GoString(C.kf_session_last_error()))
}

// NewSession: peer `self` of the KUNGFU_INIT_PEERS-style list `peers`.
func NewSession(peers, self, sockDir string, token uint32, deviceMode bool) (*Session, error) {
	cp, cs, cd := C.CString(peers), C.CString(self), C.CString(sockDir)
	defer C.free(unsafe.Pointer(cp))
	defer C.free(unsafe.Pointer(cs))
	defer C.free(unsafe.Pointer(cd))
	dm := C.int(0)
	if deviceMode {
		dm = 1
	}
	h := C.kf_session_create_peers(cp, cs, cd, C.uint32_t(token), dm)
	if h == nil {
		return nil, errors.New("kf_session_create_peers: " + C.GoString(C.kf_session_last_error()))
	}
	return &Session{h: h}, nil
}

// Info: Rank, Size, LocalRank, LocalSize, HostCount (peer.hpp).
func (s *Session) Info() (rank, size, localRank, localSize, hosts int, err error) {
	var r, n, lr, ls, hc C.int
	err = sessStatus("kf_session_info", C.kf_session_info(s.h, &r, &n, &lr, &ls, &hc))
	return int(r), int(n), int(lr), int(ls), int(hc), err
}

func (s *Session) Close() {
	if s.h != nil {
		C.kf_session_destroy(s.h)
		s.h = nil
	}
}

// NewLocalExchange: an exchange over this host's ranks of the session.
func NewLocalExchange(s *Session, device int) (*Exchange, error) {
	h := C.kf_exchange_create_local(s.h, C.int(device))
	if h == nil {
		return nil, errors.New("kf_exchange_create_local: " + C.GoString(C.kf_exchange_last_error()))
	}
	return &Exchange{h: h}, nil
}

// Split: the ranks passing the same color, ordered by key; nil for color < 0.
func (e *Exchange) Split(color, key int) (*Exchange, error) {
	var st C.int
	h := C.kf_exchange_split(e.h, C.int(color), C.int(key), &st)
	if err := exStatus("kf_exchange_split", st); err != nil {
		return nil, err
	}
	if h == nil {
		return nil, nil
	}
	return &Exchange{h: h}, nil
}

//export kfGoNamedDone
func kfGoNamedDone(status C.int, arg unsafe.Pointer) {
	h := cgo.Handle(uintptr(arg))
	done := h.Value().(func(error))
	h.Delete()
	var err error
	if status != C.KF_OK {
		err = fmt.Errorf("named all-reduce: status %d: %s", int(status),
			C.GoString(C.kf_exchange_last_error()))
	}
	done(err)
}

// AllReduceNamed starts the in-place all-reduce of buf keyed by name; done
// runs on the exchange's completion thread once it finished on the device.
func (e *Exchange) AllReduceNamed(name string, buf DevicePtr, count int, t DataType, op OP,
	average bool, algo int, s Stream, done func(error)) error {
	cn := C.CString(name)
	defer C.free(unsafe.Pointer(cn))
	avg := C.int(0)
	if average {
		avg = 1
	}
	h := cgo.NewHandle(done)
	rc := C.kf_go_named(e.h, cn, unsafe.Pointer(uintptr(buf)), C.size_t(count),
		C.KungFu_Datatype(t), C.KungFu_Op(op), avg, C.int(algo), unsafe.Pointer(uintptr(s)),
		C.uintptr_t(h))
	if rc != C.KF_OK {
		h.Delete()
	}
	return exStatus("kf_exchange_all_reduce_named", rc)
}

// WaitNamed blocks until every name started so far completed.
func (e *Exchange) WaitNamed() error {
	return exStatus("kf_exchange_wait_named", C.kf_exchange_wait_named(e.h))
}

// HierAllReduce: kf_hier_all_reduce of one HBM bucket, in place.
func HierAllReduce(local *Exchange, cross *Session, buf DevicePtr, count int, t DataType, op OP,
	average bool, algo int, name string, s Stream) error {
	cn := C.CString(name)
	defer C.free(unsafe.Pointer(cn))
	avg := C.int(0)
	if average {
		avg = 1
	}
	p := unsafe.Pointer(uintptr(buf))
	rc := C.kf_hier_all_reduce(local.h, cross.h, p, p, C.size_t(count), C.KungFu_Datatype(t),
		C.KungFu_Op(op), avg, C.int(algo), cn, unsafe.Pointer(uintptr(s)))
	return exStatus("kf_hier_all_reduce", rc)
}
