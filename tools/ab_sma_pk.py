#!/usr/bin/env python3
"""The SMA blend's arithmetic, round 5 against round 6, in ONE process on the
same buffers: r05 blends lane by lane in scalar fp32
(63 VGPRs, 8 waves per SIMD); r06 blends pairs of lanes in packed fp32
(v_pk_mul_f32 / v_pk_add_f32, 60 VGPRs, 8 waves). Same IEEE operations, so
the bits must be equal; only the VALU count differs.

`build` compiles kf_capi.hip twice into tools/ab_lib/ — once beside round
5's kf_reduce_kernels.hpp (git show <rev>:...), once beside the working
tree's — on the CPU, before the GPU call. `run` loads both (RTLD_LOCAL) and
times, interleaved over 15 rounds (median):

  sma_batch_c5_bf16  kf_sma_blend_batch, C5's 13 BERT-base buckets in bf16
                     (bench.py kernels.sma_batch_c5_bf16), 3 rotating sets
  sma_blend_bf16     kf_sma_blend over 256 MiB bf16 (kernels.sma_blend_bf16)
  sma_blend_f32      kf_sma_blend over 256 MiB fp32

    python tools/ab_sma_pk.py build [rev]     (default rev: 3146635, round 5's end)
    python tools/ab_sma_pk.py run > profiles/r06/ab_sma_pk.jsonl
"""
import ctypes
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "ab_lib")
VARIANTS = ("r05", "r06")
BF16, F32 = 0x20209, 0x20408


def lib_path(name):
    return os.path.join(OUT, "libkf_ab_sma_%s.so" % name)


def build(rev="3146635"):
    os.makedirs(OUT, exist_ok=True)
    csrc = os.path.join(ROOT, "kungfu_amd", "csrc")
    for name in VARIANTS:
        with tempfile.TemporaryDirectory() as d:
            shutil.copy(os.path.join(csrc, "kf_capi.hip"), d)
            hdr = os.path.join(d, "kf_reduce_kernels.hpp")
            if name == "r05":
                with open(hdr, "w") as f:
                    f.write(subprocess.run(["git", "-C", ROOT, "show",
                                            "%s:kungfu_amd/csrc/kf_reduce_kernels.hpp" % rev],
                                           check=True, capture_output=True, text=True).stdout)
            else:
                shutil.copy(os.path.join(csrc, "kf_reduce_kernels.hpp"), hdr)
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                            "-fPIC", "-shared", "-ffp-contract=off", "-fvisibility=hidden",
                            "-I" + os.path.join(ROOT, "include"), "-o", lib_path(name),
                            os.path.join(d, "kf_capi.hip")], check=True)
        print("built", lib_path(name), flush=True)


def run():
    import torch
    import bench
    from kungfu_amd import _lib
    from kungfu_amd.collective import GradBuckets
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
        sums = [torch.randn(b.numel(), device=dev, generator=g).bfloat16() for b in gb.buckets]
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
    for dt, code, tdt in (("bf16", BF16, torch.bfloat16), ("f32", F32, torch.float32)):
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
        same[name] = bool(torch.equal(outs["r05"], outs["r06"]))
        restore()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = {(c, v): [] for c in cases for v in libs}
    for r in range(15):
        for name, (ns, launch, _, _, _) in cases.items():
            order = list(libs.items())
            if r % 2:
                order.reverse()
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
                          "same_bits_r05_r06": same[name]}), flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build(*sys.argv[2:3])
    elif sys.argv[1:2] == ["run"]:
        run()
    else:
        raise SystemExit(__doc__)
