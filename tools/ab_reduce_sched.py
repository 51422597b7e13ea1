#!/usr/bin/env python3
"""The compile-time-k reduce's full-tile load schedule
(kf_reduce_kernels.hpp KF_REDUCE_SCHED), A/B in ONE process on the same
buffers — the question the SMA blend raised (tools/ab_sma_sched.py): several
k = 2 instantiations issue their eight 16-B loads as 7 + 1, 6 + 2 or 4 + 4
around a wait (fp16 and integer sums, bf16 min/max, the 2-input average
batch), and even where all eight go first (C2) the waits are spread over the
adds, which for the SMA blend measured slower than one wait.

  r0  the compiler's order
  r1  a scheduling barrier after the loads
  p0  r1 (the shipped schedule since r06s), loads kept as raw 16-B words
  p1  p0 with an empty asm on each word after the barrier (KF_REDUCE_PIN),
      which keeps the 8-bit min/max unpacking behind it
  (AB_VARIANTS=p0,p1 selects a pair)

Cases (3 rotating sets, 15 interleaved rounds, median), bits compared:
  c2_f32            kf_bucket_reduce f32 SUM, 256 MiB (the headline kernel)
  sum_bf16 / sum_f16 / sum_i32 / max_bf16 / min_f32 / max_u8 / min_i8
                    the same shape
  avg_np3_f32       kf_bucket_reduce_avg (x + y) / 3 (IEEE division)
  avg_np8_bf16      (x + y) / 8 in bf16 (multiply by 1/8)
  batch16_f32       kf_bucket_reduce_batch k = 2 SUM, 16 x 4 MiB

    python tools/ab_reduce_sched.py build
    python tools/ab_reduce_sched.py run > profiles/r06/ab_reduce_sched.jsonl
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
# r0 / r1: KF_REDUCE_SCHED 0 / 1 (r06s); p0 / p1: KF_REDUCE_PIN 0 / 1 with the
# barrier on (r06z5)
VARIANTS = tuple(os.environ.get("AB_VARIANTS", "r0,r1").split(","))
FLAGS = {"r0": ["-DKF_REDUCE_SCHED=0"], "r1": ["-DKF_REDUCE_SCHED=1"],
         "p0": ["-DKF_REDUCE_SCHED=1", "-DKF_REDUCE_PIN=0"],
         "p1": ["-DKF_REDUCE_SCHED=1", "-DKF_REDUCE_PIN=1"]}
DT = {"f32": 0x20408, "bf16": 0x20209, "f16": 0x20208, "i32": 0x10408, "u8": 0x00108,
      "i8": 0x10108}
SUM, MIN, MAX = 0, 1, 2


def lib_path(name):
    return os.path.join(OUT, "libkf_ab_reduce_sched_%s.so" % name)


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, "kungfu_amd", "csrc", "kf_capi.hip")
    for name in VARIANTS:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-fPIC", "-shared", "-ffp-contract=off", "-fvisibility=hidden",
                        *FLAGS[name],
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
           "i32": torch.int32, "u8": torch.uint8, "i8": torch.int8}
    lims = {"i32": (-1 << 20, 1 << 20), "u8": (0, 256), "i8": (-128, 128)}

    def bufs(dt, nbytes):
        t = tdt[dt]
        n = nbytes // torch.empty((), dtype=t).element_size()
        out = []
        for _ in range(3):
            if dt in lims:
                x = torch.randint(*lims[dt], (n,), device=dev, generator=g, dtype=t)
                y = torch.randint(*lims[dt], (n,), device=dev, generator=g, dtype=t)
            else:
                x = torch.randn(n, device=dev, generator=g).to(t)
                y = torch.randn(n, device=dev, generator=g).to(t)
            z = torch.empty_like(x)
            out.append((_lib.ptr_array([x.data_ptr(), y.data_ptr()]), z, x, y, n))
        return out

    cases = {}
    for name, dt, op in (("c2_f32", "f32", SUM), ("sum_bf16", "bf16", SUM),
                         ("sum_f16", "f16", SUM), ("sum_i32", "i32", SUM),
                         ("max_bf16", "bf16", MAX), ("min_f32", "f32", MIN),
                         ("max_u8", "u8", MAX), ("min_i8", "i8", MIN)):
        sets = bufs(dt, 256 << 20)
        cases[name] = (lambda lib, i, sets=sets, dt=dt, op=op: lib.kf_bucket_reduce(
            sets[i][0], 2, sets[i][1].data_ptr(), sets[i][4], DT[dt], op, sp),
            3 * 256 << 20, lambda sets=sets: sets[0][1].clone())
    for name, dt, np_ in (("avg_np3_f32", "f32", 3), ("avg_np8_bf16", "bf16", 8)):
        sets = bufs(dt, 256 << 20)
        cases[name] = (lambda lib, i, sets=sets, dt=dt, np_=np_: lib.kf_bucket_reduce_avg(
            sets[i][0], 2, sets[i][1].data_ptr(), sets[i][4], DT[dt], np_, sp),
            3 * 256 << 20, lambda sets=sets: sets[0][1].clone())
    nbk, per = 16, (4 << 20) // 4
    bsets = []
    for _ in range(3):
        xs = [torch.randn(per, device=dev, generator=g) for _ in range(nbk)]
        ys = [torch.randn(per, device=dev, generator=g) for _ in range(nbk)]
        zs = [torch.empty(per, device=dev) for _ in range(nbk)]
        bsets.append((_lib.ptr_array([t.data_ptr() for x, y in zip(xs, ys) for t in (x, y)]),
                      _lib.ptr_array([z.data_ptr() for z in zs]),
                      (ctypes.c_size_t * nbk)(*([per] * nbk)), xs, ys, zs))
    cases["batch16_f32"] = (lambda lib, i: lib.kf_bucket_reduce_batch(
        bsets[i][0], 2, bsets[i][1], bsets[i][2], nbk, DT["f32"], SUM, 0, sp),
        3 * 4 * per * nbk, lambda: torch.cat(bsets[0][5]).clone())

    same = {}
    for name, (launch, _, snap) in cases.items():
        outs = {}
        for v, lib in libs.items():
            _lib.check(launch(lib, 0), name + " " + v)
            torch.cuda.synchronize()
            outs[v] = snap()
        same[name] = bool(torch.equal(outs[VARIANTS[0]], outs[VARIANTS[1]]))
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
