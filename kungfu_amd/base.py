"""Host-side mirror of KungFu's ``srcs/go/kungfu/base`` package.

Same names and argument meaning as the reference, so a caller of the Go base
package finds the same surface:

* ``DataType`` codes            — srcs/go/kungfu/base/dtype.go, dtype.h:21-39
* ``OP`` codes                  — srcs/go/kungfu/base/op.go:10-15, op.h:8-13
* ``Vector`` / ``Slice``        — srcs/go/kungfu/base/vector.go:11-33
* ``Workspace`` / ``Split``     — srcs/go/kungfu/base/workspace.go:10-50
* ``Transform`` / ``Transform2`` — srcs/go/kungfu/base/op.go:17-36

``Transform2`` calls the C-ABI ``std_transform_2`` of libkungfu_amd.so, which
runs the reduce on the GPU (host buffers -> HBM -> HIP kernel -> host). There
is no CPU implementation here: without the library or a GPU it fails loudly.
"""
import ctypes
import enum

import numpy as np

from . import _lib


class DataType(enum.IntEnum):
    U8 = 0x00108
    U16 = 0x00208
    U32 = 0x00408
    U64 = 0x00808
    I8 = 0x10108
    I16 = 0x10208
    I32 = 0x10408
    I64 = 0x10808
    F16 = 0x20208
    F32 = 0x20408
    F64 = 0x20808
    BOOL = 0x30108
    BF16 = 0x20209  # extension: not in the reference

    def size(self):
        return (int(self) >> 8) & 0xFF


class OP(enum.IntEnum):
    SUM = 0
    MIN = 1
    MAX = 2
    PROD = 3


# KungFu op names as the framework ops spell them
# (tensorflow/ops/cpu/collective.cpp:58-63, torch/common.cpp:41-46).
OP_NAMES = {"sum": OP.SUM, "min": OP.MIN, "max": OP.MAX, "prod": OP.PROD}

_NUMPY = {
    DataType.U8: np.uint8, DataType.U16: np.uint16, DataType.U32: np.uint32,
    DataType.U64: np.uint64, DataType.I8: np.int8, DataType.I16: np.int16,
    DataType.I32: np.int32, DataType.I64: np.int64, DataType.F16: np.float16,
    DataType.F32: np.float32, DataType.F64: np.float64, DataType.BOOL: np.bool_,
    DataType.BF16: np.uint16,  # raw bits
}


def numpy_dtype(dt):
    return _NUMPY[DataType(dt)]


def dtype_of(arr):
    """KungFu DataType of a numpy array (bf16 must be passed explicitly)."""
    for k, v in _NUMPY.items():
        if k is DataType.BF16:
            continue
        if np.dtype(v) == arr.dtype:
            return k
    raise TypeError("unsupported dtype %s" % arr.dtype)


class Vector:
    """Typed view over a contiguous byte buffer (vector.go:11-33)."""

    def __init__(self, data, count, dtype):
        self.Data = data  # 1-D numpy array of the element type (a view)
        self.Count = int(count)
        self.Type = DataType(dtype)

    @classmethod
    def new(cls, count, dtype):
        dt = DataType(dtype)
        return cls(np.zeros(count, dtype=numpy_dtype(dt)), count, dt)

    @classmethod
    def of(cls, arr, dtype=None):
        arr = np.ascontiguousarray(arr).reshape(-1)
        return cls(arr, arr.size, dtype if dtype is not None else dtype_of(arr))

    def Slice(self, begin, end):
        return Vector(self.Data[begin:end], end - begin, self.Type)

    def CopyFrom(self, other):
        np.copyto(self.Data, other.Data)

    def ptr(self):
        return self.Data.ctypes.data


class Workspace:
    """SendBuf/RecvBuf/OP/Name (workspace.go:10-16)."""

    def __init__(self, SendBuf, RecvBuf, OP, Name):
        self.SendBuf = SendBuf
        self.RecvBuf = RecvBuf
        self.OP = OP
        self.Name = Name

    def slice(self, begin, end):
        # chunk names are part of the wire protocol and feed the strategy hash
        # (workspace.go:18-25, shard.go:17-23)
        return Workspace(self.SendBuf.Slice(begin, end),
                         self.RecvBuf.Slice(begin, end), self.OP,
                         "part::%s[%d:%d]" % (self.Name, begin, end))

    def Split(self, partition, k):
        return [self.slice(b, e) for b, e in partition(0, self.SendBuf.Count, k)]

    def IsEmpty(self):
        return self.SendBuf.Count == 0 or self.SendBuf.Data.nbytes == 0

    def IsInplace(self):
        return self.SendBuf.ptr() == self.RecvBuf.ptr()

    def Forward(self):
        if not self.IsInplace():
            self.RecvBuf.CopyFrom(self.SendBuf)


def EvenPartition(begin, end, k):
    """k intervals whose lengths differ by at most one; the first ``rem`` get
    the extra element (srcs/go/plan/interval.go:12-27)."""
    n = end - begin
    quo, rem = n // k, n % k
    parts, off = [], begin
    for i in range(k):
        c = quo + 1 if i < rem else quo
        parts.append((off, off + c))
        off += c
    return parts


def Transform2(z, x, y, op):
    """z[i] = op(x[i], y[i]) through std_transform_2 (op.go:25-36)."""
    lib = _lib.load()
    lib.std_transform_2(x.ptr(), y.ptr(), z.ptr(), ctypes.c_int(z.Count),
                        int(z.Type), int(op))


def Transform(y, x, op):
    """y[i] = op(x[i], y[i]) (op.go:17-22: Transform2(y, x, y, op))."""
    Transform2(y, x, y, op)
