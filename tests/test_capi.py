"""The C-ABI library loads and exports every symbol include/kungfu_amd.h
declares; host-only entry points behave like the reference (no GPU needed)."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "kungfu_amd.h")
LIB = os.path.join(ROOT, "kungfu_amd", "libkungfu_amd.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"^typedef[^;]*;", "", src, flags=re.M | re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "kungfu_amd", "csrc")],
                       check=True)
    from kungfu_amd import _lib
    return _lib.load()


def test_header_declares_reference_boundary():
    fns = declared_functions()
    for f in ("std_transform_2", "kungfu_type_size", "float16_sum",
              "kf_bucket_reduce", "kf_bucket_reduce_avg", "kf_sma_blend"):
        assert f in fns


def test_all_declared_symbols_exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True,
                         text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    from kungfu_amd import _lib
    for f in declared_functions():
        assert f in exported, f
        assert f in _lib.EXPORTED, f
        assert getattr(lib, f) is not None
    # nothing but the declared C ABI leaks out (no C++ internals)
    assert exported == set(declared_functions()), exported ^ set(declared_functions())


def test_enum_values_bit_identical():
    # srcs/cpp/include/kungfu/dtype.h:21-39, op.h:8-13
    from kungfu_amd.base import OP, DataType
    tc = lambda c, b: (c << 16) | (b << 8) | 8  # noqa: E731
    assert DataType.U8 == tc(0, 1) and DataType.U64 == tc(0, 8)
    assert DataType.I32 == tc(1, 4) and DataType.I64 == tc(1, 8)
    assert DataType.F16 == tc(2, 2) and DataType.F32 == tc(2, 4)
    assert DataType.F64 == tc(2, 8) and DataType.BOOL == tc(3, 1)
    assert (OP.SUM, OP.MIN, OP.MAX, OP.PROD) == (0, 1, 2, 3)
    hdr = open(HEADER).read()
    for name, val in (("KungFu_FLOAT", 0x20408), ("KungFu_FLOAT16", 0x20208),
                      ("KungFu_INT32", 0x10408), ("KungFu_BOOL", 0x30108)):
        assert re.search(r"\b%s\s*=\s*0x%05x\b" % (name, val), hdr, re.I), name


def test_type_size_matches_reference_fixture(lib):
    import golden_io
    codes = {"u8": 0x00108, "u16": 0x00208, "u32": 0x00408, "u64": 0x00808,
             "i8": 0x10108, "i16": 0x10208, "i32": 0x10408, "i64": 0x10808,
             "f16": 0x20208, "f32": 0x20408, "f64": 0x20808, "bool": 0x30108}
    for name, size in golden_io.load_json("type_size.json").items():
        assert lib.kungfu_type_size(codes[name]) == size


def _run(code):
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


def test_type_size_unknown_exits():
    # dtype.c:31-33: unknown dtype -> message + exit(1)
    r = _run("from kungfu_amd import _lib; _lib.load().kungfu_type_size(0x12345)")
    assert r.returncode == 1
    assert "unknown dtype" in r.stderr


@pytest.mark.parametrize("code,op", [(0x20208, 1), (0x20208, 3), (0x30108, 0),
                                     (0x12345, 0), (0x20408, 7)])
def test_rejected_combinations_exit_1(code, op):
    # op.cpp:41,52,89 — the reference exits(1); so does the drop-in
    r = _run("import numpy as np; from kungfu_amd import _lib;"
             "a=np.zeros(64,np.uint8); l=_lib.load();"
             "l.std_transform_2(a.ctypes.data,a.ctypes.data,a.ctypes.data,4,%d,%d)"
             % (code, op))
    assert r.returncode == 1, r.stderr


def test_no_cpu_fallback_without_gpu(lib):
    # with no device the product must fail loudly, never compute on the host
    if lib.kf_device_count() > 0:
        pytest.skip("GPU present")
    r = _run("import numpy as np; from kungfu_amd import _lib;"
             "a=np.ones(8,np.float32); l=_lib.load();"
             "l.std_transform_2(a.ctypes.data,a.ctypes.data,a.ctypes.data,8,0x20408,0)")
    assert r.returncode == 1
    assert "kungfu_amd" in r.stderr


def test_empty_is_noop(lib):
    # std::transform over an empty range does nothing (no device touched)
    lib.std_transform_2(None, None, None, 0, 0x20408, 0)
    assert lib.kf_bucket_reduce(None, 2, None, 0, 0x20408, 0, None) == 0


def test_device_api_arg_errors(lib):
    from kungfu_amd import _lib
    arr = _lib.ptr_array([0, 0])
    assert lib.kf_bucket_reduce(arr, 0, None, 16, 0x20408, 0, None) == 3
    assert lib.kf_bucket_reduce(arr, 17, None, 16, 0x20408, 0, None) == 3
    assert lib.kf_bucket_reduce(arr, 2, None, 16, 0x20408, 0, None) == 3
    assert lib.kf_bucket_reduce_avg(_lib.ptr_array([8, 8]), 2, 8, 16, 0x10408, 2,
                                    None) == 1  # ints have no /np epilogue
    assert lib.kf_bucket_div(8, 16, 0x20408, 0, None) == 3


def test_peers_fold_arg_errors(lib):
    # kf_bucket_reduce_peers: B2 contract (status codes, no device touched)
    from kungfu_amd import _lib
    arr = _lib.ptr_array([8, 8])
    assert lib.kf_bucket_reduce_peers(arr, 2, 8, 0, 0x20408, 0, 0, None) == 0  # n = 0
    assert lib.kf_bucket_reduce_peers(arr, 0, 8, 16, 0x20408, 0, 0, None) == 3
    assert lib.kf_bucket_reduce_peers(arr, 17, 8, 16, 0x20408, 0, 0, None) == 3
    assert lib.kf_bucket_reduce_peers(arr, 2, 8, 16, 0x10408, 0, 2, None) == 1  # int avg
    assert lib.kf_bucket_reduce_peers(arr, 2, 8, 16, 0x20408, 1, 2, None) == 2  # avg needs SUM
    assert lib.kf_bucket_reduce_peers(arr, 2, 8, 16, 0x20208, 1, 0, None) == 2  # f16 MIN
    assert lib.kf_bucket_reduce_peers(arr, 2, 8, 16, 0x30108, 0, 0, None) == 1  # BOOL
    assert lib.kf_bucket_reduce_peers(arr, 2, 8, 16, 0x20408, 0, -1, None) == 3


def test_peer_barrier_arg_errors(lib):
    # kf_peer_barrier / kf_signal_alloc: argument checks before any HIP call
    import ctypes
    from kungfu_amd import _lib
    sigs = _lib.ptr_array([8, 16])
    st = ctypes.c_void_p(8)
    assert lib.kf_peer_barrier(sigs, 1, 0, 1, 1000, st, None) == 0  # world 1: nothing
    assert lib.kf_peer_barrier(sigs, 0, 0, 1, 1000, st, None) == 3
    assert lib.kf_peer_barrier(sigs, 65, 0, 1, 1000, st, None) == 3
    assert lib.kf_peer_barrier(sigs, 2, 2, 1, 1000, st, None) == 3  # rank out of range
    assert lib.kf_peer_barrier(sigs, 2, 0, 1, 1000, None, None) == 3  # no status word
    assert lib.kf_peer_barrier(_lib.ptr_array([8, 0]), 2, 0, 1, 1000, st, None) == 3
    assert lib.kf_peer_barrier(_lib.ptr_array([8, 12]), 2, 0, 1, 1000, st, None) == 3
    assert lib.kf_signal_alloc(0, 0, ctypes.byref(ctypes.c_void_p())) == 3
    assert lib.kf_signal_alloc(4, 0, None) == 3
    assert lib.kf_signal_free(None, 0) == 3


def test_go_overlay_binds_declared_symbols():
    # go/kungfu/base/*.go (the cgo drop-in, compiled nowhere here: no Go
    # toolchain) may only call C names the header declares
    import glob
    import re
    with open(os.path.join(ROOT, "include", "kungfu_amd.h")) as f:
        header = f.read()
    libc = {"malloc", "free", "GoString", "CString", "int", "size_t", "double", "KungFu_Op",
            "KungFu_Datatype", "uint32_t", "uintptr_t"}
    files = glob.glob(os.path.join(ROOT, "go", "kungfu", "base", "*.go"))
    assert files
    for path in files:
        with open(path) as f:
            src = f.read()
        assert src.startswith("//go:build kungfu_amd"), path
        # names the file's own cgo preamble defines (a C trampoline, an
        # exported Go callback) are not the library's
        preamble = src.split('import "C"')[0]
        own = set(re.findall(r"\b([A-Za-z_]\w*)\s*\(", preamble))
        for name in set(re.findall(r"\bC\.([A-Za-z_][A-Za-z0-9_]*)", src)):
            if name in libc or name in own:
                continue
            assert re.search(r"\b%s\b" % re.escape(name), header), (path, name)


def test_tf_dtype_map_is_the_reference_one():
    """kungfu_amd.ops.TF_DTYPES / to_kungfu_type restate tensorflow/ops.h:14-33
    (bf16 -> KungFu_FLOAT16 included); the fixture was read from the
    reference's headers by tests/golden/gen_tf_dtype_map.py."""
    import json
    from kungfu_amd import ops
    with open(os.path.join(ROOT, "tests", "golden", "tf_dtype_map.json")) as f:
        ref = json.load(f)["map"]
    assert {k: int(v) for k, v in ops.TF_DTYPES.items()} == {k: v["code"] for k, v in ref.items()}
    for name, v in ref.items():
        assert int(ops.to_kungfu_type(name)) == v["code"]

    class TfLike:  # anything with a `name`, as a tf.DType
        name = "bfloat16"
    assert int(ops.to_kungfu_type(TfLike())) == 0x20208
    for bad in ("float16", "uint8", "complex64"):  # ops.h: no DT_HALF, throws
        with pytest.raises(ValueError, match="unsupported dtype"):
            ops.to_kungfu_type(bad)


def test_no_test_transport_in_the_product(lib):
    """The loopback transport and its host fold live in the TEST library
    (tests/c/libkf_testing.so), plugged in through the product's
    kf_exchange_create_transport; the shipped library exports none of it and
    has no switch that changes what a one-rank exchange does."""
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True,
                         text=True, check=True).stdout
    names = [l.split()[-1] for l in out.splitlines()]
    assert not [n for n in names if "loopback" in n or "rccl1" in n or "kf_testing" in n]
    strings = subprocess.run(["strings", LIB], capture_output=True, text=True,
                             check=True).stdout
    assert "KUNGFU_AMD_EXCHANGE_W1_COLLECTIVES" not in strings
    assert "loopback" not in strings
    tl = os.path.join(ROOT, "tests", "c")
    subprocess.run(["make", "-s", "-C", tl], check=True)
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(tl, "libkf_testing.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    assert {"kf_loopback_create", "kf_loopback_destroy", "kf_exchange_create_loopback",
            "kf_exchange_create_rccl1"} <= exported
    # no kernel and no copy of the product in the test library: it calls it
    undefined = subprocess.run(["nm", "-D", "--undefined-only",
                                os.path.join(tl, "libkf_testing.so")],
                               capture_output=True, text=True, check=True).stdout
    assert "kf_exchange_create_transport" in undefined
