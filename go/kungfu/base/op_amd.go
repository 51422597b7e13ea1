//go:build kungfu_amd

// Drop-in for srcs/go/kungfu/base/op.go (reference op.go:1-36): the same
// package API, with std_transform_2 served by libkungfu_amd.so (the gfx950
// HIP reduce) instead of op.cpp/f16.c/dtype.c compiled into the package.
//
// Build (Go is not in this image, so this file is compiled nowhere here):
//
//	CGO_CFLAGS="-I<repo>/include" \
//	CGO_LDFLAGS="-L<repo>/kungfu_amd -Wl,-rpath,<repo>/kungfu_amd" \
//	go build -tags kungfu_amd ./srcs/go/...
//
// with `//go:build !kungfu_amd` added to the reference's op.go, dtype.go,
// op.cpp, f16.c and dtype.c (INTEGRATION.md §1).
package base

// #cgo LDFLAGS: -lkungfu_amd
// #include "kungfu_amd.h"
import "C"

import (
	"fmt"
	"unsafe"
)

type OP C.KungFu_Op

const (
	SUM  OP = C.KungFu_SUM
	MIN  OP = C.KungFu_MIN
	MAX  OP = C.KungFu_MAX
	PROD OP = C.KungFu_PROD
)

// Transform performs y[i] = y[i] op x[i] (reference op.go:17-22).
func Transform(y, x *Vector, op OP) {
	Transform2(y, x, y, op)
}

// Transform2 performs z[i] = x[i] op y[i] (reference op.go:24-36). The
// library reads x and y and writes z before it returns, so no Go pointer is
// kept after the call (the cgo rule the reference works around,
// lsds/KungFu#149). Page-locked buffers (HostRegister) are reduced in place
// over PCIe; pageable ones are staged through HBM. As in the reference, an
// unsupported dtype/op ends the process with exit(1).
func Transform2(z, x, y *Vector, op OP) {
	if z.Count == 0 {
		return
	}
	C.std_transform_2(
		unsafe.Pointer(&x.Data[0]),
		unsafe.Pointer(&y.Data[0]),
		unsafe.Pointer(&z.Data[0]),
		C.int(z.Count), C.KungFu_Datatype(z.Type), C.KungFu_Op(op))
}

// Shutdown gives the library's HIP resources (the scratch and streams that
// Transform2 borrows per call) back while the HIP runtime is still up; call
// it once no Transform2 is running, e.g. before main returns. No library
// destructor calls HIP at exit, so a program that never calls it leaves them
// to the OS (include/kungfu_amd.h kf_shutdown).
func Shutdown() error {
	if rc := C.kf_shutdown(); rc != C.KF_OK {
		return fmt.Errorf("kf_shutdown: %s", C.GoString(C.kf_last_error()))
	}
	return nil
}
