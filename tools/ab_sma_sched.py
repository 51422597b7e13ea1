#!/usr/bin/env python3
"""The SMA blend's full-tile load schedule (kf_reduce_kernels.hpp
KF_SMA_SCHED), A/B in ONE process on the same buffers.

Held to 64 VGPRs (8 waves per SIMD), the compiler issues the bf16 blend's
eight 16-B loads as three, a wait for the first two, then five, so a wave has
fewer loads in flight than the add/xor kernels of the same bytes, which issue
all eight first. One box (profiles/r06/same_box_probe_r06o.jsonl) put the
blend at 0.792 of 8 TB/s against 0.814 for an in-place xor.

  s0  the compiler's order (round 6 as shipped before this A/B)
  s1  a scheduling barrier after the loads: all eight in flight, then one
      wait for the first seven
  s2  the loads interleaved (v0, s0, v1, s1, ...) and the barrier: all eight
      in flight, each vector's blend waiting for its own two loads

`build` compiles kf_capi.hip once per variant into tools/ab_lib/
(-DKF_SMA_SCHED=n) on the CPU, before the GPU call. `run` loads all of them
(RTLD_LOCAL) and times, interleaved over 15 rounds (median), C5's batch
(bench.py kernels.sma_batch_c5_bf16) and kf_sma_blend over 256 MiB in bf16,
fp16, fp32 and fp64. Every variant's bits are compared with s0's.

    python tools/ab_sma_sched.py build
    python tools/ab_sma_sched.py run > profiles/r06/ab_sma_sched.jsonl
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
VARIANTS = ("s0", "s1", "s2")
BF16, F16, F32, F64 = 0x20209, 0x20208, 0x20408, 0x20808


def lib_path(name):
    return os.path.join(OUT, "libkf_ab_sma_sched_%s.so" % name)


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, "kungfu_amd", "csrc", "kf_capi.hip")
    for name in VARIANTS:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-fPIC", "-shared", "-ffp-contract=off", "-fvisibility=hidden",
                        "-DKF_SMA_SCHED=%s" % name[1:],
                        "-I" + os.path.join(ROOT, "include"), "-o", lib_path(name), src],
                       check=True)
        print("built", lib_path(name), flush=True)


def run():
    import torch
    import bench
    from kungfu_amd import _lib
    from kungfu_amd.collective import GradBuckets, workspace_like
    vp = ctypes.c_void_p
    libs = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(lib_path(name), mode=ctypes.RTLD_LOCAL)
        lib.kf_sma_blend_batch.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp),
                                           ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_double, vp]
        lib.kf_sma_blend_batch.restype = ctypes.c_int
        lib.kf_sma_blend.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_double, vp]
        lib.kf_sma_blend.restype = ctypes.c_int
        libs[name] = lib
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(11)
    sp = torch.cuda.current_stream().cuda_stream
    cases = {}

    bert = bench._models()["bert"][:201]
    sets = []
    for _ in range(3):
        gb = GradBuckets(bert, torch.bfloat16, dev, 8, bucket_bytes=16 << 20)
        for b in gb.buckets:
            b.copy_(torch.randn(b.numel(), device=dev, generator=g).bfloat16())
        sums = workspace_like(gb.buckets)  # as the exchange lays them out
        for t in sums:
            t.copy_(torch.randn(t.numel(), device=dev, generator=g).bfloat16())
        sets.append((_lib.ptr_array([b.data_ptr() for b in gb.buckets]),
                     _lib.ptr_array([t.data_ptr() for t in sums]),
                     (ctypes.c_size_t * len(sums))(*[t.numel() for t in sums]), gb, sums,
                     [b.clone() for b in gb.buckets]))
    nb = len(sets[0][4])
    cases["sma_batch_c5_bf16"] = (
        3, lambda lib, i: lib.kf_sma_blend_batch(sets[i][0], sets[i][1], sets[i][2], nb, BF16, 8,
                                                 0.1, sp),
        3 * 2 * sum(t.numel() for t in sets[0][4]),
        lambda: torch.cat(sets[0][3].buckets).clone(),
        lambda: [b.copy_(o) for b, o in zip(sets[0][3].buckets, sets[0][5])])
    for dt, code, tdt in (("bf16", BF16, torch.bfloat16), ("f16", F16, torch.float16),
                          ("f32", F32, torch.float32), ("f64", F64, torch.float64)):
        n = (256 << 20) // torch.empty((), dtype=tdt).element_size()
        vs = [torch.randn(n, device=dev, generator=g).to(tdt) for _ in range(3)]
        ss = [torch.randn(n, device=dev, generator=g).to(tdt) for _ in range(3)]
        v0 = vs[0].clone()
        cases["sma_blend_%s" % dt] = (
            3, lambda lib, i, vs=vs, ss=ss, n=n, code=code: lib.kf_sma_blend(
                vs[i].data_ptr(), ss[i].data_ptr(), n, code, 8, 0.1, sp),
            3 * 256 << 20, lambda vs=vs: vs[0].clone(), lambda vs=vs, v0=v0: vs[0].copy_(v0))
    same = {}
    for name, (_, launch, _, snap, restore) in cases.items():
        outs = {}
        for v, lib in libs.items():
            restore()
            _lib.check(launch(lib, 0), name + " " + v)
            torch.cuda.synchronize()
            outs[v] = snap()
        same[name] = {v: bool(torch.equal(outs["s0"], o)) for v, o in outs.items()}
        restore()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = {(c, v): [] for c in cases for v in libs}
    for r in range(15):
        for name, (ns, launch, _, _, _) in cases.items():
            order = list(libs.items())
            order = order[r % len(order):] + order[:r % len(order)]
            for v, lib in order:
                for i in range(ns):
                    launch(lib, i)
                e0.record()
                for i in range(8 * ns):
                    launch(lib, i % ns)
                e1.record()
                torch.cuda.synchronize()
                ts[(name, v)].append(e0.elapsed_time(e1) * 1e3 / (8 * ns))
    for (name, v), t in ts.items():
        us = statistics.median(t)
        print(json.dumps({"case": name, "variant": v, "us": round(us, 2),
                          "min_us": round(min(t), 2),
                          "frac": round(cases[name][2] / us / 8e6, 4),
                          "same_bits_as_s0": same[name][v]}), flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build()
    elif sys.argv[1:2] == ["run"]:
        run()
    else:
        raise SystemExit(__doc__)
