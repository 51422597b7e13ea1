#!/usr/bin/env python3
"""Tile shape of the batched launch (kf_bucket_reduce_batch) at the native
exchange's phase-2 shapes (bench.py exchange_phase2: C5's k = 8 all-to-all
fold, C4's and C3's k = 1 shard /np at N = 8) and at C3's 16 x 4 MiB k = 2.

The shape is compile-time (KF_BATCH_UNROLL[_K1] x KF_BATCH_BLOCK in kf_capi.hip),
so `build` compiles kf_capi.hip once per shape into tools/ab_lib/ (on the
CPU, before the GPU call); `run` loads every variant into one process
(RTLD_LOCAL) and times them interleaved on the same buffers, cycling over
>= 0.75 GiB of sets, 15 rounds, median per variant; every variant's result
is checked against the shipped library's bits.

    python tools/ab_batch_shape.py build
    python tools/ab_batch_shape.py run > profiles/r03/ab_batch_shape.jsonl
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
# variant name -> compile-time flags (kf_capi.hip / kf_reduce_kernels.hpp)
VARIANTS = {"u%d_b%d" % (u, b): {"KF_BATCH_UNROLL": u, "KF_BATCH_UNROLL_K1": u, "KF_BATCH_BLOCK": b}
            for u, b in [(4, 256), (2, 256), (1, 256), (2, 512), (1, 512), (1, 1024)]}
# round 5: the k >= 3 batched fold's one-in-flight threshold (blocks per
# launch, KF_BATCH_SERIAL_MIN_BLOCKS; C5's a2a fold is ~1670 blocks at four
# vectors per lane, so it runs four-together by default) and two vectors per
# lane, where the same bytes make ~3340 blocks and the schedule turns on
#   AB_SET=serial python tools/ab_batch_shape.py build|run
if os.environ.get("AB_SET") == "serial":
    VARIANTS = {"u%d_s%d" % (u, t): {"KF_BATCH_UNROLL": u, "KF_BATCH_SERIAL_MIN_BLOCKS": t}
                for u, t in [(4, 2048), (4, 1024), (4, 256), (2, 2048), (2, 1 << 30), (8, 1 << 30)]}
# (round 5 also timed 1-D batched launches with the blocks handed out XCD by
# XCD, each XCD a contiguous eighth, through a temporary KF_BATCH_XCD1D
# variant: C5's fold 42.04 vs 41.93 us, profiles/r05/ab_batch_xcd1d_r05ao.jsonl;
# not kept)
CASES = os.environ.get("AB_CASES")  # comma list; all when unset
# (round 3 also built a KF_FOLD_ALLIN variant of the runtime-k fold here —
# every input's vectors in flight before the first add on resident grids —
# equal within noise at every shape, profiles/r03/ab_fold_allin_r03u.jsonl;
# the variant was not kept)
F32, BF16, SUM = 0x20408, 0x20209, 0


def lib_path(name):
    return os.path.join(OUT, "libkf_ab_%s.so" % name)


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, "kungfu_amd", "csrc", "kf_capi.hip")
    for name, flags in VARIANTS.items():
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "-shared", "-ffp-contract=off", "-fvisibility=hidden",
               "-I" + os.path.join(ROOT, "include")]
        cmd += ["-D%s=%d" % kv for kv in flags.items()]
        cmd += ["-o", lib_path(name), src]
        subprocess.run(cmd, check=True)
        print("built", lib_path(name), flush=True)


def run():
    import torch
    import bench
    from kungfu_amd import _lib
    from kungfu_amd.collective import GradBuckets
    ship = _lib.load()
    vp = ctypes.c_void_p
    argt = [ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t),
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
    libs = {}
    for name in VARIANTS:
        lib = ctypes.CDLL(lib_path(name), mode=ctypes.RTLD_LOCAL)
        lib.kf_bucket_reduce_batch.argtypes = argt
        lib.kf_bucket_reduce_batch.restype = ctypes.c_int
        lib.kf_bucket_reduce.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp, ctypes.c_size_t,
                                         ctypes.c_int, ctypes.c_int, vp]
        lib.kf_bucket_reduce.restype = ctypes.c_int
        libs[name] = lib
    libs["shipped"] = ship
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    sp = torch.cuda.current_stream().cuda_stream
    models = bench._models()
    W = 8

    cases = {}  # name -> (nsets, launch(lib, i), bytes, snapshot(i), restore(i))

    # C5 at N = 8: k = 8 bf16 shards per bucket, rank-order fold, / 8
    bert = models["bert"][:201]
    counts = [c.numel() for c in GradBuckets(bert, torch.bfloat16, dev, W,
                                             bucket_bytes=16 << 20).buckets]
    qs = [c // W for c in counts]
    per = sum((W + 1) * q * 2 for q in qs)
    n5 = max(2, -(-(768 << 20) // per))
    s5 = []
    for _ in range(n5):
        ws = [torch.randn(W * q, device=dev, generator=g).bfloat16() for q in qs]
        outs = [torch.empty(q, device=dev, dtype=torch.bfloat16) for q in qs]
        ins = _lib.ptr_array([w.data_ptr() + j * q * 2 for w, q in zip(ws, qs) for j in range(W)])
        s5.append((ins, _lib.ptr_array([o.data_ptr() for o in outs]),
                   (ctypes.c_size_t * len(qs))(*qs), ws, outs))
    cases["c5_a2a_fold_n8_bf16"] = (
        n5, lambda lib, i: lib.kf_bucket_reduce_batch(s5[i][0], W, s5[i][1], s5[i][2], len(qs),
                                                      BF16, SUM, W, sp), per,
        lambda i: torch.cat(s5[i][4]).clone(), None)

    def shard_div(name, counts):
        q = [c // W for c in counts]
        per = sum(2 * x * 4 for x in q)
        ns = max(2, -(-(768 << 20) // per))
        sets = []
        for _ in range(ns):
            bs = [torch.randn(c, device=dev, generator=g) for c in counts]
            sh = [bb[x * 3:x * 4] for bb, x in zip(bs, q)]
            sets.append((_lib.ptr_array([t.data_ptr() for t in sh]),
                         (ctypes.c_size_t * len(q))(*q), bs, sh, [t.clone() for t in sh]))

        def restore(i):
            for t, r in zip(sets[i][3], sets[i][4]):
                t.copy_(r)
        cases[name] = (ns, lambda lib, i: lib.kf_bucket_reduce_batch(
            sets[i][0], 1, sets[i][0], sets[i][1], len(q), F32, SUM, W, sp), per,
            lambda i: torch.cat(sets[i][3]).clone(), restore)

    rn = GradBuckets(models["resnet50-imagenet"], torch.float32, dev, W, n_buckets=16)
    shard_div("c4_shard_div_n8_f32", [b.numel() for b in rn.buckets])
    del rn
    shard_div("c3_shard_div_n8_f32", [1 << 20] * 64)

    # C3's 16 x 4 MiB k = 2 (bench.py kernels batch_16x4MiB_f32)
    n = 1 << 20
    nb = 16
    nsb = 3
    sb = []
    for _ in range(nsb):
        xs = [torch.randn(n, device=dev, generator=g) for _ in range(2 * nb)]
        zs = [torch.empty(n, device=dev) for _ in range(nb)]
        sb.append((_lib.ptr_array([x.data_ptr() for x in xs]),
                   _lib.ptr_array([z.data_ptr() for z in zs]),
                   (ctypes.c_size_t * nb)(*([n] * nb)), xs, zs))
    cases["batch_16x4MiB_f32"] = (
        nsb, lambda lib, i: lib.kf_bucket_reduce_batch(sb[i][0], 2, sb[i][1], sb[i][2], nb, F32,
                                                       SUM, 0, sp), 12 * n * nb,
        lambda i: torch.cat(sb[i][4]).clone(), None)

    # the star root's k-input fold of 1 MiB chunks and of 4 MiB buckets
    # (kf_bucket_reduce, resident grids), k = 4 and 8
    for k, n in ((4, 1 << 18), (8, 1 << 18), (8, 1 << 20)):
        ns = max(2, -(-(768 << 20) // ((k + 1) * n * 4)))
        fs = []
        for _ in range(ns):
            xs = [torch.randn(n, device=dev, generator=g) for _ in range(k)]
            z = torch.empty(n, device=dev)
            fs.append((_lib.ptr_array([x.data_ptr() for x in xs]), z, xs))
        cases["fold_k%d_%dKiB_f32" % (k, n * 4 >> 10)] = (
            ns, lambda lib, i, fs=fs, k=k, n=n: lib.kf_bucket_reduce(fs[i][0], k, fs[i][1].data_ptr(),
                                                                     n, F32, SUM, sp),
            (k + 1) * n * 4, lambda i, fs=fs: fs[i][1].clone(), None)

    if CASES:
        cases = {c: v for c, v in cases.items() if c in CASES.split(",")}
    # bits: every variant equals the shipped library on set 0
    ok = {}
    for name, (ns, launch, _, snap, restore) in cases.items():
        if restore:
            restore(0)
        _lib.check(launch(ship, 0), name)
        want = snap(0)
        for v, lib in libs.items():
            if restore:
                restore(0)
            _lib.check(launch(lib, 0), name + " " + v)
            ok[(name, v)] = bool(torch.equal(snap(0), want))
    torch.cuda.synchronize()

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
                for i in range(4 * ns):
                    launch(lib, i % ns)
                e1.record()
                torch.cuda.synchronize()
                ts[(name, v)].append(e0.elapsed_time(e1) * 1e3 / (4 * ns))
    for (name, v), t in ts.items():
        us = statistics.median(t)
        print(json.dumps({"case": name, "shape": v, "us": round(us, 2), "min_us": round(min(t), 2),
                          "frac": round(cases[name][2] / us / 8e6, 4), "same_bits": ok[(name, v)],
                          "rounds": len(t)}), flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
