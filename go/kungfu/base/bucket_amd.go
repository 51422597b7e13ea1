//go:build kungfu_amd

// The bucket-level device API (kungfu_amd.h B2) for a Go caller that owns
// HBM buffers: k-input folds, the S-SGD 1/np epilogue and the SMA blend on a
// HIP stream, with status codes instead of exit(1).
package base

// #include <stdlib.h>
// #include "kungfu_amd.h"
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

// DevicePtr is an address in HBM (or page-locked host memory mapped for the
// device); Go never dereferences it.
type DevicePtr uintptr

// Stream is a hipStream_t; 0 is the null stream.
type Stream uintptr

func status(fn string, rc C.int) error {
	if rc == C.KF_OK {
		return nil
	}
	return fmt.Errorf("%s: status %d: %s", fn, int(rc), C.GoString(C.kf_last_error()))
}

// the k input addresses go to C memory: cgo forbids passing Go memory that
// holds pointers, and these are device addresses anyway
func cPtrs(inputs []DevicePtr) (unsafe.Pointer, error) {
	if len(inputs) < 1 || len(inputs) > C.KF_MAX_INPUTS {
		return nil, errors.New("kungfu_amd: 1..KF_MAX_INPUTS inputs")
	}
	arr := C.malloc(C.size_t(len(inputs)) * C.size_t(unsafe.Sizeof(uintptr(0))))
	ps := unsafe.Slice((*uintptr)(arr), len(inputs))
	for i, p := range inputs {
		ps[i] = uintptr(p)
	}
	return arr, nil
}

// BucketReduce: out = ((in[0] op in[1]) op in[2]) ... (left fold, the
// reference chain of Transform2 hops), queued on s, no sync.
func BucketReduce(inputs []DevicePtr, out DevicePtr, n int, t DataType, op OP, s Stream) error {
	arr, err := cPtrs(inputs)
	if err != nil {
		return err
	}
	defer C.free(arr)
	rc := C.kf_bucket_reduce((*unsafe.Pointer)(arr), C.int(len(inputs)),
		unsafe.Pointer(uintptr(out)), C.size_t(n), C.KungFu_Datatype(t),
		C.KungFu_Op(op), unsafe.Pointer(uintptr(s)))
	return status("kf_bucket_reduce", rc)
}

// BucketReduceAvg: out = sum(inputs) / np (sync_sgd.py:103-104, fused).
func BucketReduceAvg(inputs []DevicePtr, out DevicePtr, n int, t DataType, np int, s Stream) error {
	arr, err := cPtrs(inputs)
	if err != nil {
		return err
	}
	defer C.free(arr)
	rc := C.kf_bucket_reduce_avg((*unsafe.Pointer)(arr), C.int(len(inputs)),
		unsafe.Pointer(uintptr(out)), C.size_t(n), C.KungFu_Datatype(t), C.int(np),
		unsafe.Pointer(uintptr(s)))
	return status("kf_bucket_reduce_avg", rc)
}

// BucketDiv: x /= np in place (the shard epilogue between reduce-scatter
// and all-gather).
func BucketDiv(x DevicePtr, n int, t DataType, np int, s Stream) error {
	rc := C.kf_bucket_div(unsafe.Pointer(uintptr(x)), C.size_t(n), C.KungFu_Datatype(t),
		C.int(np), unsafe.Pointer(uintptr(s)))
	return status("kf_bucket_div", rc)
}

// SMABlend: v = (1-alpha) v + alpha (sum / np) (sma_sgd.py:60-65).
func SMABlend(v, sum DevicePtr, n int, t DataType, np int, alpha float64, s Stream) error {
	rc := C.kf_sma_blend(unsafe.Pointer(uintptr(v)), unsafe.Pointer(uintptr(sum)),
		C.size_t(n), C.KungFu_Datatype(t), C.int(np), C.double(alpha),
		unsafe.Pointer(uintptr(s)))
	return status("kf_sma_blend", rc)
}

// SMABlendBatch: SMABlend over many buckets in one launch per 16 of them
// (kf_sma_blend_batch); vs[i] is blended with sums[i], counts[i] elements.
func SMABlendBatch(vs, sums []DevicePtr, counts []int, t DataType, np int, alpha float64,
	s Stream) error {
	if len(vs) != len(sums) || len(vs) != len(counts) {
		return errors.New("SMABlendBatch: vs, sums and counts differ in length")
	}
	if len(vs) == 0 {
		return nil
	}
	pv := C.malloc(C.size_t(len(vs)) * C.size_t(unsafe.Sizeof(uintptr(0))))
	ps := C.malloc(C.size_t(len(vs)) * C.size_t(unsafe.Sizeof(uintptr(0))))
	pc := C.malloc(C.size_t(len(vs)) * C.size_t(unsafe.Sizeof(C.size_t(0))))
	defer C.free(pv)
	defer C.free(ps)
	defer C.free(pc)
	av := (*[1 << 20]unsafe.Pointer)(pv)[:len(vs):len(vs)]
	as := (*[1 << 20]unsafe.Pointer)(ps)[:len(vs):len(vs)]
	ac := (*[1 << 20]C.size_t)(pc)[:len(vs):len(vs)]
	for i := range vs {
		av[i] = unsafe.Pointer(uintptr(vs[i]))
		as[i] = unsafe.Pointer(uintptr(sums[i]))
		ac[i] = C.size_t(counts[i])
	}
	rc := C.kf_sma_blend_batch((*unsafe.Pointer)(pv), (*unsafe.Pointer)(ps), (*C.size_t)(pc),
		C.int(len(vs)), C.KungFu_Datatype(t), C.int(np), C.double(alpha),
		unsafe.Pointer(uintptr(s)))
	return status("kf_sma_blend_batch", rc)
}

// HostRegister page-locks a C-allocated host buffer so Transform2 reduces it
// in place over PCIe (zero copy). Go heap memory must not be registered: the
// collector may move or free it.
func HostRegister(p unsafe.Pointer, bytes int) error {
	return status("kf_host_register", C.kf_host_register(p, C.size_t(bytes)))
}

func HostUnregister(p unsafe.Pointer) error {
	return status("kf_host_unregister", C.kf_host_unregister(p))
}
