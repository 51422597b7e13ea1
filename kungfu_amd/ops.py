"""Device bucket-reduce ops on torch tensors (C-ABI B2, include/kungfu_amd.h).

Every op launches a hand-written gfx950 HIP kernel from libkungfu_amd.so on
the caller's current HIP stream (or the stream given). Tensors must be
contiguous and on the GPU; there is no CPU path — a CPU tensor or a missing
library raises.
"""
import ctypes

import torch

from . import _lib
from .base import OP, OP_NAMES, DataType

_TORCH_DTYPES = {
    torch.uint8: DataType.U8,
    torch.int8: DataType.I8,
    torch.int16: DataType.I16,
    torch.int32: DataType.I32,
    torch.int64: DataType.I64,
    torch.float16: DataType.F16,
    torch.bfloat16: DataType.BF16,
    torch.float32: DataType.F32,
    torch.float64: DataType.F64,
}
for _name, _dt in (("uint16", DataType.U16), ("uint32", DataType.U32),
                   ("uint64", DataType.U64)):
    if hasattr(torch, _name):
        _TORCH_DTYPES[getattr(torch, _name)] = _dt


def kungfu_dtype(t):
    try:
        return _TORCH_DTYPES[t.dtype]
    except KeyError:
        raise TypeError("kungfu_amd: unsupported dtype %s" % t.dtype)


# The reference's TF dtype map, as it is (tensorflow/ops.h:14-33): no fp16,
# and DT_BFLOAT16 -> KungFu_FLOAT16, so a bf16 tensor's bit patterns are
# reduced as fp16 numbers. The build's own map (kungfu_dtype) gives bf16 its
# own code and fp32-accumulated semantics; this one exists so that a caller
# that wants the reference's exact bits can ask for them (pass the code as
# `dtype` to the device ops).
TF_DTYPES = {
    "int32": DataType.I32,
    "int64": DataType.I64,
    "bfloat16": DataType.F16,
    "float32": DataType.F32,
    "float64": DataType.F64,
    "bool": DataType.BOOL,
}


def to_kungfu_type(tf_dtype):
    """ops.h:14-33 to_kungfu_type: a TF dtype name ("float32", "bfloat16", ...
    or anything with such a `name`) -> KungFu code; anything else raises, as
    the reference's `throw std::invalid_argument("unsupported dtype")`."""
    name = getattr(tf_dtype, "name", tf_dtype)
    try:
        return TF_DTYPES[name]
    except KeyError:
        raise ValueError("unsupported dtype")


def _dtype_for(t, dtype):
    """The KungFu code a device op runs with: the tensor's own, or an explicit
    one of the same element size (e.g. to_kungfu_type("bfloat16") on a bf16
    tensor, the reference's TF semantics)."""
    if dtype is None:
        return kungfu_dtype(t)
    dt = DataType(int(dtype))
    if dt.size() != t.element_size():
        raise ValueError("dtype %s does not match the tensor's %d-byte elements"
                         % (dt.name, t.element_size()))
    return dt


def _op(op):
    if op is None:
        return OP.SUM
    if isinstance(op, str):
        return OP_NAMES[op]
    return OP(op)


def _check_dev(ts):
    for t in ts:
        if not t.is_cuda:
            raise ValueError("kungfu_amd device ops need GPU tensors (got %s)"
                             % t.device)
        if not t.is_contiguous():
            raise ValueError("kungfu_amd device ops need contiguous tensors")


def _stream(stream, dev):
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    return s.cuda_stream


def bucket_reduce(inputs, out=None, op="sum", stream=None, dtype=None):
    """out = inputs[0] op inputs[1] op ... (left fold, in the given order).
    `dtype`: a KungFu code to reduce with instead of the tensors' own
    (same element size)."""
    inputs = list(inputs)
    if out is None:
        out = torch.empty_like(inputs[0])
    _check_dev(inputs + [out])
    n = out.numel()
    for t in inputs:
        if t.numel() != n or t.dtype != out.dtype:
            raise ValueError("bucket_reduce: shape/dtype mismatch")
    lib = _lib.load()
    rc = lib.kf_bucket_reduce(_lib.ptr_array([t.data_ptr() for t in inputs]),
                              len(inputs), out.data_ptr(), n,
                              int(_dtype_for(out, dtype)), int(_op(op)),
                              _stream(stream, out.device))
    _lib.check(rc, "kf_bucket_reduce")
    return out


def bucket_reduce_avg(inputs, np_, out=None, stream=None):
    """out = sum(inputs) / np_ with a true division (TF's g / np)."""
    inputs = list(inputs)
    if out is None:
        out = torch.empty_like(inputs[0])
    _check_dev(inputs + [out])
    lib = _lib.load()
    rc = lib.kf_bucket_reduce_avg(
        _lib.ptr_array([t.data_ptr() for t in inputs]), len(inputs),
        out.data_ptr(), out.numel(), int(kungfu_dtype(out)), int(np_),
        _stream(stream, out.device))
    _lib.check(rc, "kf_bucket_reduce_avg")
    return out


def bucket_div_(x, np_, stream=None):
    """x /= np_ in place (the step between reduce-scatter and all-gather)."""
    _check_dev([x])
    lib = _lib.load()
    rc = lib.kf_bucket_div(x.data_ptr(), x.numel(), int(kungfu_dtype(x)),
                           int(np_), _stream(stream, x.device))
    _lib.check(rc, "kf_bucket_div")
    return x


def sma_blend_(v, summed, np_, alpha, stream=None):
    """v = (1 - alpha) * v + alpha * (summed / np_) in place (sma_sgd.py:60-65)."""
    _check_dev([v, summed])
    if v.numel() != summed.numel() or v.dtype != summed.dtype:
        raise ValueError("sma_blend_: shape/dtype mismatch")
    lib = _lib.load()
    rc = lib.kf_sma_blend(v.data_ptr(), summed.data_ptr(), v.numel(),
                          int(kungfu_dtype(v)), int(np_), float(alpha),
                          _stream(stream, v.device))
    _lib.check(rc, "kf_sma_blend")
    return v


def sma_blend_batch_(vs, sums, np_, alpha, stream=None):
    """sma_blend_ over many buckets (one dtype) in one launch per 16 of them
    (kf_sma_blend_batch); the same bits as one sma_blend_ per bucket."""
    vs, sums = list(vs), list(sums)
    if len(vs) != len(sums):
        raise ValueError("sma_blend_batch_: one sum per variable bucket")
    if not vs:
        return vs
    _check_dev(vs + sums)
    for v, s in zip(vs, sums):
        if v.numel() != s.numel() or v.dtype != vs[0].dtype or s.dtype != v.dtype:
            raise ValueError("sma_blend_batch_: shape/dtype mismatch")
    lib = _lib.load()
    cnt = (ctypes.c_size_t * len(vs))(*[v.numel() for v in vs])
    rc = lib.kf_sma_blend_batch(_lib.ptr_array([v.data_ptr() for v in vs]),
                                _lib.ptr_array([s.data_ptr() for s in sums]), cnt, len(vs),
                                int(kungfu_dtype(vs[0])), int(np_), float(alpha),
                                _stream(stream, vs[0].device))
    _lib.check(rc, "kf_sma_blend_batch")
    return vs
