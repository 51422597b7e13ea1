#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REFERENCE itself.

Run in the build container (needs /root/reference):
    make -C oracle ref && python tests/golden/gen_golden.py

Outputs (data only — inputs and expected outputs):
  transform2.npz + transform2.json
      std_transform_2 of the reference, compiled from its own sources
      (srcs/go/kungfu/base/{op.cpp,f16.c,dtype.c}, see oracle/Makefile `ref`),
      over dtype x op x n x input kind. Small cases are stored whole; large
      cases store the seed plus sha256 of inputs and output.
  rejects.json
      dtype/op combinations for which the reference calls exit(1)
      (op.cpp:41,52,89; dtype.c:31-33), observed by running it in a subprocess.
  type_size.json
      kungfu_type_size for every dtype code (dtype.c:7-35).
  models.json
      gradient-size lists parsed from tests/go/fakemodel/*.go (ResNet-50,
      BERT, VGG16) — the bucket shapes of BASELINE.json configs C4/C5.
"""
import ctypes
import hashlib
import json
import os
import re
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libkfbase_ref.so")
REF = "/root/reference"

DTYPES = {
    "u8": (0x00108, np.uint8), "u16": (0x00208, np.uint16),
    "u32": (0x00408, np.uint32), "u64": (0x00808, np.uint64),
    "i8": (0x10108, np.int8), "i16": (0x10208, np.int16),
    "i32": (0x10408, np.int32), "i64": (0x10808, np.int64),
    "f16": (0x20208, np.float16), "f32": (0x20408, np.float32),
    "f64": (0x20808, np.float64),
}
OPS = {"sum": 0, "min": 1, "max": 2, "prod": 3}
SMALL_N = [1, 7, 8, 9, 31, 1027]
LARGE_N = [262144, 262147]  # one full 1 MiB fp32 chunk, and ragged


def gen_inputs(name, n, seed, kind):
    """Deterministic inputs. kind: 'rand' | 'big' | 'special'."""
    _, dt = DTYPES[name]
    rng = np.random.default_rng(seed)
    if kind == "special":
        return special_inputs(name, n, rng)
    if np.issubdtype(dt, np.integer):
        info = np.iinfo(dt)
        lo, hi = int(info.min), int(info.max)
        if kind == "rand":  # full range: exercises wrap-around
            x = rng.integers(lo, hi, size=n, dtype=dt, endpoint=True)
            y = rng.integers(lo, hi, size=n, dtype=dt, endpoint=True)
        else:  # small magnitudes
            x = rng.integers(-100 if lo < 0 else 0, 100, size=n).astype(dt)
            y = rng.integers(-100 if lo < 0 else 0, 100, size=n).astype(dt)
        return x, y
    if dt is np.float16:
        scale = 1.0 if kind == "rand" else 100.0
        x = (rng.standard_normal(n) * scale).astype(np.float16)
        y = (rng.standard_normal(n) * scale).astype(np.float16)
        return x, y
    scale = 1.0 if kind == "rand" else 1e30
    x = (rng.standard_normal(n) * scale).astype(dt)
    y = (rng.standard_normal(n) * scale).astype(dt)
    return x, y


def special_inputs(name, n, rng):
    _, dt = DTYPES[name]
    if np.issubdtype(dt, np.integer):
        info = np.iinfo(dt)
        pool = np.array([info.min, info.max, 0, 1, -1 if info.min < 0 else 2,
                         info.max // 2, info.min // 2 if info.min < 0 else 3],
                        dtype=dt)
    else:
        fi = np.finfo(dt)
        pool = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0,
                         fi.tiny, -fi.tiny, fi.tiny / 4, -fi.tiny / 8,
                         fi.max, -fi.max, fi.max / 2, fi.eps], dtype=dt)
    x = pool[rng.integers(0, pool.size, size=n)]
    y = pool[rng.integers(0, pool.size, size=n)]
    # all ordered pairs of the pool at the front
    m = min(n, pool.size * pool.size)
    ii, jj = np.meshgrid(np.arange(pool.size), np.arange(pool.size), indexing="ij")
    x[:m] = pool[ii.reshape(-1)[:m]]
    y[:m] = pool[jj.reshape(-1)[:m]]
    return x, y


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def ref_lib():
    lib = ctypes.CDLL(REF_SO)
    lib.std_transform_2.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3
    lib.std_transform_2.restype = None
    lib.kungfu_type_size.argtypes = [ctypes.c_int]
    lib.kungfu_type_size.restype = ctypes.c_uint32
    return lib


def ref_transform(lib, x, y, code, op):
    z = np.empty_like(x)
    lib.std_transform_2(x.ctypes.data, y.ctypes.data, z.ctypes.data, x.size,
                        code, op)
    return z


def ref_exits(code, op):
    """Run the reference op in a child process; return its exit code."""
    prog = ("import ctypes;l=ctypes.CDLL(%r);import numpy as np;"
            "a=np.zeros(16,np.uint8);"
            "l.std_transform_2(ctypes.c_void_p(a.ctypes.data),"
            "ctypes.c_void_p(a.ctypes.data),ctypes.c_void_p(a.ctypes.data),"
            "ctypes.c_int(2),ctypes.c_int(%d),ctypes.c_int(%d))" % (REF_SO, code, op))
    return subprocess.run([sys.executable, "-c", prog]).returncode


def parse_go_sizes(path, var):
    src = open(path).read()
    m = re.search(r"var\s+%s\s*=\s*\[\]int\{(.*?)\}" % var, src, re.S)
    return [int(v) for v in re.findall(r"\d+", m.group(1))]


def main():
    lib = ref_lib()
    arrays, index = {}, []
    cid = 0
    for name, (code, dt) in DTYPES.items():
        for opname, op in OPS.items():
            if name == "f16" and opname != "sum":
                continue  # reference exits: recorded in rejects.json
            kinds = ["rand", "big", "special"]
            for kind in kinds:
                for n in SMALL_N:
                    seed = 1000 * cid + n
                    x, y = gen_inputs(name, n, seed, kind)
                    z = ref_transform(lib, x, y, code, op)
                    key = "c%04d" % cid
                    arrays[key + "_x"], arrays[key + "_y"], arrays[key + "_z"] = x, y, z
                    index.append(dict(id=key, dtype=name, code=code, op=opname,
                                      opcode=op, n=n, seed=seed, kind=kind,
                                      stored=True))
                    cid += 1
            for n in LARGE_N:
                if name not in ("f32", "i32", "f16", "f64") or opname not in ("sum", "max"):
                    continue
                seed = 1000 * cid + 7
                x, y = gen_inputs(name, n, seed, "rand")
                z = ref_transform(lib, x, y, code, op)
                index.append(dict(id="c%04d" % cid, dtype=name, code=code,
                                  op=opname, opcode=op, n=n, seed=seed,
                                  kind="rand", stored=False, sha_x=sha(x),
                                  sha_y=sha(y), sha_z=sha(z)))
                cid += 1
    # in-place aliasing: out == input1 and out == input2 (op.cpp on aliased ptrs)
    for alias in ("x", "y"):
        x, y = gen_inputs("f32", 1023, 77, "rand")
        z_expected = ref_transform(lib, x, y, 0x20408, 0)
        key = "c%04d" % cid
        arrays[key + "_x"], arrays[key + "_y"], arrays[key + "_z"] = x, y, z_expected
        index.append(dict(id=key, dtype="f32", code=0x20408, op="sum", opcode=0,
                          n=1023, seed=77, kind="alias_" + alias, stored=True))
        cid += 1
    np.savez_compressed(os.path.join(HERE, "transform2.npz"), **arrays)
    with open(os.path.join(HERE, "transform2.json"), "w") as f:
        json.dump(index, f, indent=0)

    rejects = []
    for name, code in (("f16", 0x20208),):
        for opname in ("min", "max", "prod"):
            rejects.append(dict(dtype=name, code=code, op=opname,
                                exit=ref_exits(code, OPS[opname])))
    for opname in OPS:
        rejects.append(dict(dtype="bool", code=0x30108, op=opname,
                            exit=ref_exits(0x30108, OPS[opname])))
    rejects.append(dict(dtype="unknown", code=0x12345, op="sum",
                        exit=ref_exits(0x12345, 0)))
    rejects.append(dict(dtype="f32", code=0x20408, op="bad_op_7",
                        exit=ref_exits(0x20408, 7)))
    with open(os.path.join(HERE, "rejects.json"), "w") as f:
        json.dump(rejects, f, indent=1)

    sizes = {name: int(lib.kungfu_type_size(code)) for name, (code, _) in DTYPES.items()}
    sizes["bool"] = int(lib.kungfu_type_size(0x30108))
    with open(os.path.join(HERE, "type_size.json"), "w") as f:
        json.dump(sizes, f, indent=1)

    fm = os.path.join(REF, "tests", "go", "fakemodel")
    models = {
        "resnet50-imagenet": parse_go_sizes(os.path.join(fm, "resnet50-imagenet.go"), "resnet50Imagenet"),
        "bert": parse_go_sizes(os.path.join(fm, "bert.go"), "bert"),
        "vgg16-imagenet": parse_go_sizes(os.path.join(fm, "vgg16-imagenet.go"), "vgg16Imagenet"),
    }
    with open(os.path.join(HERE, "models.json"), "w") as f:
        json.dump(models, f)
    print("cases", cid, "stored arrays", len(arrays), "rejects", len(rejects))
    print({k: (len(v), sum(v)) for k, v in models.items()})


if __name__ == "__main__":
    main()
