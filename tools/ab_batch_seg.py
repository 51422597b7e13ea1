#!/usr/bin/env python3
"""The batched launches' bucket lookup, A/B in ONE process on the same
buffers. Up to 16 buckets, a block found its bucket by a linear scan of the
kernarg block table, one dependent scalar load per step before its first
vector load (`scan`, kf_reduce_kernels.hpp at e4f5194); `count` counts the
table's entries <= the block index over the whole table, whose words load
together (segment_count). Cases, 3 rotating sets each, 15 interleaved
rounds (median), bits compared between the variants:

  sma_batch_c5_bf16    kf_sma_blend_batch, C5's 13 BERT-base bf16 buckets
                       (bench.py kernels.sma_batch_c5_bf16)
  c5_a2a_fold_n8_bf16  kf_bucket_reduce_batch k = 8 over the 13 buckets'
                       received shards, /8 (bench.py kernels.c5_a2a_fold_n8_bf16)
  ragged16_sum_f32     kf_bucket_reduce_batch k = 2 SUM over 16 fp32 buckets
                       of 1-4 MiB (unequal, so no 2-D grid)

    python tools/ab_batch_seg.py build
    python tools/ab_batch_seg.py run > profiles/r06/ab_batch_seg.jsonl

Result (profiles/r06/ab_batch_seg_r06q.jsonl): no difference in any case (within
0.1-0.9 %, same bits), so the product keeps the scan; `count` needs the
working-tree header of that A/B (segment_count), which was not kept.
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
VARIANTS = ("scan", "count")
SCAN_REV = "e4f5194"
BF16, F32 = 0x20209, 0x20408
SUM = 0


def lib_path(name):
    return os.path.join(OUT, "libkf_ab_seg_%s.so" % name)


def build():
    os.makedirs(OUT, exist_ok=True)
    csrc = os.path.join(ROOT, "kungfu_amd", "csrc")
    for name in VARIANTS:
        with tempfile.TemporaryDirectory() as d:
            shutil.copy(os.path.join(csrc, "kf_capi.hip"), d)
            hdr = os.path.join(d, "kf_reduce_kernels.hpp")
            if name == "scan":
                with open(hdr, "w") as f:
                    f.write(subprocess.run(["git", "-C", ROOT, "show",
                                            "%s:kungfu_amd/csrc/kf_reduce_kernels.hpp" % SCAN_REV],
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
    from kungfu_amd.collective import GradBuckets, workspace_like
    vp = ctypes.c_void_p
    libs = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(lib_path(name), mode=ctypes.RTLD_LOCAL)
        lib.kf_sma_blend_batch.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp),
                                           ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_double, vp]
        lib.kf_bucket_reduce_batch.argtypes = [ctypes.POINTER(vp), ctypes.c_int,
                                               ctypes.POINTER(vp),
                                               ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
        libs[name] = lib
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(13)
    sp = torch.cuda.current_stream().cuda_stream
    cases = {}

    bert = bench._models()["bert"][:201]
    sets = []
    for _ in range(3):
        gb = GradBuckets(bert, torch.bfloat16, dev, 8, bucket_bytes=16 << 20)
        for b in gb.buckets:
            b.copy_(torch.randn(b.numel(), device=dev, generator=g).bfloat16())
        sums = workspace_like(gb.buckets)
        for t in sums:
            t.copy_(torch.randn(t.numel(), device=dev, generator=g).bfloat16())
        sets.append((_lib.ptr_array([b.data_ptr() for b in gb.buckets]),
                     _lib.ptr_array([t.data_ptr() for t in sums]),
                     (ctypes.c_size_t * len(sums))(*[t.numel() for t in sums]), gb, sums,
                     [b.clone() for b in gb.buckets]))
    nb = len(sets[0][4])
    cases["sma_batch_c5_bf16"] = (
        lambda lib, i: lib.kf_sma_blend_batch(sets[i][0], sets[i][1], sets[i][2], nb, BF16, 8,
                                              0.1, sp),
        3 * 2 * sum(t.numel() for t in sets[0][4]),
        lambda: torch.cat(sets[0][3].buckets).clone(),
        lambda: [b.copy_(o) for b, o in zip(sets[0][3].buckets, sets[0][5])])

    world = 8
    qs = [b.numel() // world for b in sets[0][3].buckets]
    fsets = []
    for _ in range(3):
        ws = [torch.randn(world * q, device=dev, generator=g).bfloat16() for q in qs]
        outs = [torch.empty(q, device=dev, dtype=torch.bfloat16) for q in qs]
        ins = _lib.ptr_array([w.data_ptr() + j * q * 2 for w, q in zip(ws, qs) for j in range(world)])
        fsets.append((ins, _lib.ptr_array([o.data_ptr() for o in outs]),
                      (ctypes.c_size_t * len(qs))(*qs), ws, outs))
    cases["c5_a2a_fold_n8_bf16"] = (
        lambda lib, i: lib.kf_bucket_reduce_batch(fsets[i][0], world, fsets[i][1], fsets[i][2],
                                                  len(qs), BF16, SUM, world, sp),
        sum((world + 1) * q * 2 for q in qs),
        lambda: torch.cat(fsets[0][4]).clone(), lambda: None)

    mib = [1, 3, 2, 4, 1, 2, 3, 4, 2, 1, 4, 3, 2, 2, 1, 3]
    counts = [(m << 20) // 4 + 64 * j for j, m in enumerate(mib)]
    rsets = []
    for _ in range(3):
        xs = [torch.randn(c, device=dev, generator=g) for c in counts]
        ys = [torch.randn(c, device=dev, generator=g) for c in counts]
        zs = [torch.empty(c, device=dev) for c in counts]
        ins = _lib.ptr_array([t.data_ptr() for x, y in zip(xs, ys) for t in (x, y)])
        rsets.append((ins, _lib.ptr_array([z.data_ptr() for z in zs]),
                      (ctypes.c_size_t * len(counts))(*counts), xs, ys, zs))
    cases["ragged16_sum_f32"] = (
        lambda lib, i: lib.kf_bucket_reduce_batch(rsets[i][0], 2, rsets[i][1], rsets[i][2],
                                                  len(counts), F32, SUM, 0, sp),
        3 * 4 * sum(counts),
        lambda: torch.cat(rsets[0][5]).clone(), lambda: None)

    same = {}
    for name, (launch, _, snap, restore) in cases.items():
        outs = {}
        for v, lib in libs.items():
            restore()
            _lib.check(launch(lib, 0), name + " " + v)
            torch.cuda.synchronize()
            outs[v] = snap()
        same[name] = bool(torch.equal(outs["scan"], outs["count"]))
        restore()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = {(c, v): [] for c in cases for v in libs}
    for r in range(15):
        for name, (launch, _, _, _) in cases.items():
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
