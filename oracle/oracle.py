"""TEST INFRASTRUCTURE ONLY — ctypes wrapper over oracle/libkf_oracle.so.

The CPU restatement of KungFu's host reduce (see kf_oracle.c for the
file:line map). Imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / baseline, never as the product.

Pinned: tests/test_oracle.py checks every function here against the golden
vectors in tests/golden/ that were produced by the reference's own
std_transform_2 compiled from its sources (tests/golden/gen_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libkf_oracle.so")

DT = {
    "u8": 0x00108, "u16": 0x00208, "u32": 0x00408, "u64": 0x00808,
    "i8": 0x10108, "i16": 0x10208, "i32": 0x10408, "i64": 0x10808,
    "f16": 0x20208, "f32": 0x20408, "f64": 0x20808, "bool": 0x30108,
    "bf16": 0x20209,
}
NP = {
    "u8": np.uint8, "u16": np.uint16, "u32": np.uint32, "u64": np.uint64,
    "i8": np.int8, "i16": np.int16, "i32": np.int32, "i64": np.int64,
    "f16": np.float16, "f32": np.float32, "f64": np.float64,
    "bf16": np.uint16,
}
OPS = {"sum": 0, "min": 1, "max": 2, "prod": 3}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        l = ctypes.CDLL(LIB_PATH)
        vp, i64, i = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        l.oracle_type_size.argtypes = [i]
        l.oracle_type_size.restype = ctypes.c_uint32
        l.oracle_transform2.argtypes = [vp, vp, vp, i64, i, i]
        l.oracle_transform2.restype = i
        l.oracle_f16_sum.argtypes = [vp, vp, vp, i64]
        l.oracle_f16_sum.restype = None
        l.oracle_reduce_k.argtypes = [ctypes.POINTER(vp), i, vp, i64, i, i]
        l.oracle_reduce_k.restype = i
        l.oracle_reduce_avg.argtypes = [ctypes.POINTER(vp), i, vp, i64, i, i]
        l.oracle_reduce_avg.restype = i
        l.oracle_sma_blend.argtypes = [vp, vp, i64, i, i, ctypes.c_double]
        l.oracle_sma_blend.restype = i
        l.oracle_bench_transform2.argtypes = [vp, vp, vp, i64, i, i, i, i, i64]
        l.oracle_bench_transform2.restype = ctypes.c_double
        l.oracle_bench_fn.argtypes = [vp, vp, vp, vp, i64, i, i, i, i, i64]
        l.oracle_bench_fn.restype = ctypes.c_double
        _lib = l
    return _lib


def _code(dt):
    return DT[dt] if isinstance(dt, str) else int(dt)


def _ptrs(arrs):
    a = (ctypes.c_void_p * len(arrs))()
    for j, x in enumerate(arrs):
        a[j] = x.ctypes.data
    return a


def type_size(dt):
    return int(lib().oracle_type_size(_code(dt)))


def transform2(x, y, dt, op, out=None):
    """std_transform_2 restated (op.cpp:57-93). Raises where the reference
    would exit(1)."""
    z = np.empty_like(x) if out is None else out
    rc = lib().oracle_transform2(x.ctypes.data, y.ctypes.data, z.ctypes.data,
                                 x.size, _code(dt), OPS.get(op, op))
    if rc != 0:
        raise ValueError("reference rejects dtype=%s op=%s (exit(1))" % (dt, op))
    return z


def reduce_k(inputs, dt, op="sum"):
    """Left fold in the given order, one Transform2 per hop (session.go:255-264)."""
    out = np.empty_like(inputs[0])
    rc = lib().oracle_reduce_k(_ptrs(inputs), len(inputs), out.ctypes.data,
                               out.size, _code(dt), OPS.get(op, op))
    if rc != 0:
        raise ValueError("reference rejects dtype=%s op=%s" % (dt, op))
    return out


def reduce_avg(inputs, dt, np_):
    """sum then g / np (sync_sgd.py:103-104)."""
    out = np.empty_like(inputs[0])
    rc = lib().oracle_reduce_avg(_ptrs(inputs), len(inputs), out.ctypes.data,
                                 out.size, _code(dt), int(np_))
    if rc != 0:
        raise ValueError("unsupported dtype %s" % dt)
    return out


def sma_blend(v, summed, dt, np_, alpha):
    """v' = (1-a) v + a (sum / np) (sma_sgd.py:60-65); returns a new array."""
    out = np.array(v, copy=True)
    rc = lib().oracle_sma_blend(out.ctypes.data, summed.ctypes.data, out.size,
                                _code(dt), int(np_), float(alpha))
    if rc != 0:
        raise ValueError("unsupported dtype %s" % dt)
    return out


REF_LIB = os.path.join(HERE, "_ref", "libkfbase_ref.so")


def ref_transform2_addr():
    """Address of std_transform_2 in the reference's own build
    (oracle/_ref, compiled from /root/reference by `make ref`), or None."""
    if not os.path.exists(REF_LIB):
        return None
    ref = ctypes.CDLL(REF_LIB)
    return ctypes.cast(ref.std_transform_2, ctypes.c_void_p).value


def bench_ref(fn_addr, x, y, z, dt, op, reps, threads=1, chunk_bytes=1 << 20):
    """bench_transform2 around the reference's compiled std_transform_2."""
    return float(lib().oracle_bench_fn(
        fn_addr, x.ctypes.data, y.ctypes.data, z.ctypes.data, x.size, _code(dt),
        OPS.get(op, op), int(reps), int(threads), int(chunk_bytes)))


def bench_transform2(x, y, z, dt, op, reps, threads=1, chunk_bytes=1 << 20):
    """Seconds for `reps` reductions (threads>1: 1 MiB chunk work queue)."""
    return float(lib().oracle_bench_transform2(
        x.ctypes.data, y.ctypes.data, z.ctypes.data, x.size, _code(dt),
        OPS.get(op, op), int(reps), int(threads), int(chunk_bytes)))


# ---- bf16 helpers (build-defined semantics, parity unpinned) --------------

def f32_to_bf16_bits(a):
    u = np.asarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    q = ((u >> 16) | 0x40).astype(np.uint16)
    return np.where(nan, q, r).astype(np.uint16)


def bf16_bits_to_f32(b):
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)
