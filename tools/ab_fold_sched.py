#!/usr/bin/env python3
"""The runtime-k fold's load schedule (kf_reduce_kernels.hpp KF_FOLD_SCHED),
A/B in ONE process on the same buffers, after the two-input reduce gained
from a scheduling barrier after its loads (tools/ab_reduce_sched.py).

  f0  the compiler's order after inputs 0 and 1's loads
  f1  a scheduling barrier there

Cases (3 rotating sets, 15 interleaved rounds, median), bits compared:
  fold_k3_f32 / fold_k4_f32 / fold_k8_f32   kf_bucket_reduce, k inputs of
                    256 MiB (k = 8 in the one-vector-in-flight schedule)
  fold_k4_bf16      the same in bf16
  a2a_fold_n8_bf16  kf_bucket_reduce_batch k = 8, /8: C5's all-to-all fold
                    (bench.py kernels.c5_a2a_fold_n8_bf16)

    python tools/ab_fold_sched.py build
    python tools/ab_fold_sched.py run > profiles/r06/ab_fold_sched.jsonl

Result (profiles/r06/ab_fold_sched_r06x.jsonl): every case within 0.3 %,
same bits; the product keeps KF_FOLD_SCHED 0.
"""
import ctypes
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "ab_lib")
VARIANTS = ("f0", "f1")
DT = {"f32": 0x20408, "bf16": 0x20209, "f16": 0x20208, "i32": 0x10408}
SUM, MIN, MAX = 0, 1, 2


def lib_path(name):
    return os.path.join(OUT, "libkf_ab_fold_sched_%s.so" % name)


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, "kungfu_amd", "csrc", "kf_capi.hip")
    for name in VARIANTS:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-fPIC", "-shared", "-ffp-contract=off", "-fvisibility=hidden",
                        "-DKF_FOLD_SCHED=%s" % name[1:],
                        "-I" + os.path.join(ROOT, "include"), "-o", lib_path(name), src],
                       check=True)
        print("built", lib_path(name), flush=True)


def run():
    import torch
    from kungfu_amd import _lib
    vp = ctypes.c_void_p
    libs = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(lib_path(name), mode=ctypes.RTLD_LOCAL)
        lib.kf_bucket_reduce.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp, ctypes.c_size_t,
                                         ctypes.c_int, ctypes.c_int, vp]
        lib.kf_bucket_reduce_avg.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp,
                                             ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp]
        lib.kf_bucket_reduce_batch.argtypes = [ctypes.POINTER(vp), ctypes.c_int,
                                               ctypes.POINTER(vp),
                                               ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
        libs[name] = lib
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(17)
    sp = torch.cuda.current_stream().cuda_stream
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16,
           "i32": torch.int32}

    cases = {}
    for name, dt, k in (("fold_k3_f32", "f32", 3), ("fold_k4_f32", "f32", 4),
                        ("fold_k8_f32", "f32", 8), ("fold_k4_bf16", "bf16", 4)):
        t = tdt[dt]
        n = (256 << 20) // torch.empty((), dtype=t).element_size()
        sets = []
        for _ in range(3):
            xs = [torch.randn(n, device=dev, generator=g).to(t) for _ in range(k)]
            z = torch.empty_like(xs[0])
            sets.append((_lib.ptr_array([x.data_ptr() for x in xs]), z, xs))
        cases[name] = (lambda lib, i, sets=sets, dt=dt, k=k, n=n: lib.kf_bucket_reduce(
            sets[i][0], k, sets[i][1].data_ptr(), n, DT[dt], SUM, sp),
            (k + 1) * 256 << 20, lambda sets=sets: sets[0][1].clone())
    import bench
    from kungfu_amd.collective import GradBuckets
    world = 8
    gb = GradBuckets(bench._models()["bert"][:201], torch.bfloat16, dev, world,
                     bucket_bytes=16 << 20)
    qs = [b.numel() // world for b in gb.buckets]
    del gb
    fsets = []
    for _ in range(3):
        ws = [torch.randn(world * q, device=dev, generator=g).bfloat16() for q in qs]
        outs = [torch.empty(q, device=dev, dtype=torch.bfloat16) for q in qs]
        ins = _lib.ptr_array([w.data_ptr() + j * q * 2 for w, q in zip(ws, qs) for j in range(world)])
        fsets.append((ins, _lib.ptr_array([o.data_ptr() for o in outs]),
                      (ctypes.c_size_t * len(qs))(*qs), ws, outs))
    cases["a2a_fold_n8_bf16"] = (lambda lib, i: lib.kf_bucket_reduce_batch(
        fsets[i][0], world, fsets[i][1], fsets[i][2], len(qs), DT["bf16"], SUM, world, sp),
        sum((world + 1) * q * 2 for q in qs), lambda: torch.cat(fsets[0][4]).clone())

    same = {}
    for name, (launch, _, snap) in cases.items():
        outs = {}
        for v, lib in libs.items():
            _lib.check(launch(lib, 0), name + " " + v)
            torch.cuda.synchronize()
            outs[v] = snap()
        same[name] = bool(torch.equal(outs["f0"], outs["f1"]))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = {(c, v): [] for c in cases for v in libs}
    for r in range(15):
        for name, (launch, _, _) in cases.items():
            order = list(libs.items())
            if r % 2:
                order.reverse()
            for v, lib in order:
                for i in range(3):
                    launch(lib, i)
                e0.record()
                for i in range(24):
                    launch(lib, i % 3)
                e1.record()
                torch.cuda.synchronize()
                ts[(name, v)].append(e0.elapsed_time(e1) * 1e3 / 24)
    for (name, v), t in ts.items():
        us = statistics.median(t)
        print(json.dumps({"case": name, "variant": v, "us": round(us, 2),
                          "min_us": round(min(t), 2),
                          "frac": round(cases[name][1] / us / 8e6, 4),
                          "same_bits": same[name]}), flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build()
    elif sys.argv[1:2] == ["run"]:
        run()
    else:
        raise SystemExit(__doc__)
