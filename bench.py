#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: "GiB/s device-resident fp32 bucket reduce
per GPU; % of HBM3E peak".

  python bench.py [--gpus N --steps K --warmup W]
  (N > 1: one rank per GPU under torch.distributed.run; without a launcher
  around it, bench.py starts that launcher itself as a child)

N = 1 (BASELINE.json configs[1], C2): one step = one launch of the HIP bucket
reduce z = x + y over a device-resident 256 MiB fp32 bucket (67,108,864
elements; the reference's recvOnto step, session.go:255-264, at bucket
granularity). value = bucket GiB/s = S / t.

N > 1 (configs[2], C3 geometry): one step = the S-SGD all-reduce of 64 x 4 MiB
fp32 gradient buckets (256 MiB) per rank: per bucket RCCL reduce-scatter(sum)
-> HIP /np epilogue on the shard -> RCCL all-gather over xGMI, all 64 in one
native call (kf_exchange_all_reduce_batch). Per-GPU work is fixed (scaling
"weak"); value = S / t, the bucket GiB/s each GPU reduces (the metric is "per
GPU"), with the whole job's N * S / t beside it as value_aggregate. The
local-reduce kernel is also timed on every rank so the roofline object always
describes the HIP reduce kernel.

Roofline: algorithmic bytes per launch = 3 * S (read x, read y, write z)
(SURVEY.md §8d), achieved = 3S / (average launch duration from HIP events on
the launch stream), peak = 8.0 TB/s HBM3E (MI355X_MICROARCH.md). `traffic` is
the PMC-measured HBM bytes per launch from profiles/ (rocprofv3 FETCH_SIZE x2
+ WRITE_SIZE, gfx950 correction), null if not recorded.

cpu_baseline: KungFu's own std_transform_2 compiled from the reference's
sources by `make -C oracle ref` (kind "reference"; built by __graft_entry__
.build() where /root/reference exists, shipped as oracle/_ref/*.so), or the
oracle's bit-exact restatement with the same -O2 -mavx -mf16c flags (kind
"port") when that build is absent; 1 thread on the same 256 MiB sum repeated
for about --cpu-seconds, plus 1 MiB chunks on every core of the GPU's
NUMA node (GOMAXPROCS); rank 0 at
N = 1 only.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident fp32 bucket reduce per GPU; % of HBM3E peak"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md
BUCKET_ELEMS = 64 << 20  # 256 MiB of fp32
KF_FLOAT = 0x20408
KF_SUM = 0
REDUCE_KERNEL = "reduce_kernel<float, SUM, NONE, 2>"
XGMI_LINK_GBPS = 153.0  # per link per direction
PIPE_GROUPS = 4  # kf_exchange_set_pipeline groups of the *_pipe sub-benchmarks


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--elems", type=int, default=BUCKET_ELEMS)
    ap.add_argument("--buckets", type=int, default=64,
                    help="N>1: the 256 MiB gradient set as this many pipelined "
                         "buckets (64 x 4 MiB = BASELINE.json configs[2], C3)")
    ap.add_argument("--rotate", type=int, default=3,
                    help="independent bucket sets cycled by the timed launches, so "
                         "no launch finds its 256 MiB output still in the 256 MiB "
                         "Infinity Cache (cold steady state; DESIGN.md)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-staged", action="store_true")
    ap.add_argument("--no-kernels", action="store_true",
                    help="N=1: skip the other kernel families' rates")
    ap.add_argument("--dist-backend", default="nccl",
                    help="rehearsal only: gloo lets N ranks share one GPU")
    ap.add_argument("--device-index", type=int, default=None,
                    help="rehearsal only: put every rank on this GPU")
    ap.add_argument("--no-extra", action="store_true",
                    help="N>1: skip the C4/C5/P2P sub-benchmarks")
    ap.add_argument("--extras", default="c4,c5,c5_pipe,c5_overlap,c4_overlap,c4_pipe,c4_rs_avg,c4_named,c3_pipe,c3_a2a,c3_fused,c3_torch_fused,c3_per_bucket,c4_torch,"
                                        "c5_torch,c3_ar,c3_p2p,c3_p2p_push,c3_p2p_hostbar,"
                                        "c4_p2p,c5_p2p",
                    help="N>1: which sub-benchmarks to run (comma list)")
    ap.add_argument("--extras-timeout", type=float, default=240.0,
                    help="N>1: seconds for all sub-benchmarks together; past it the "
                         "line is printed with what finished and the ranks exit")
    ap.add_argument("--native-timeout", type=float, default=120.0,
                    help="N>1: seconds for the native exchange's communicator to come up "
                         "before the torch.distributed path is used instead")
    ap.add_argument("--c3-schedule", default="auto",
                    choices=["auto", "grouped", "fused", "a2a", "pipelined"],
                    help="N>1, native exchange: the C3 schedule timed as `value` (auto: "
                         "the fastest of a short parity-checked trial of all five)")
    ap.add_argument("--no-c1", action="store_true",
                    help="N=1: skip the C1 (np=2 localhost) sub-object")
    ap.add_argument("--config", default="default", choices=["default", "c1"],
                    help="c1: BASELINE configs[0], np=2 localhost all-reduce of "
                         "one 4 MiB fp32 bucket over the rchannel wire format")
    ap.add_argument("--c1-np", type=int, default=2,
                    help="peers for --config c1 (BASELINE configs[0] is np=2)")
    ap.add_argument("--c1-modes", default="",
                    help="--config c1: comma list of modes (default: all)")
    ap.add_argument("--c1-repeats", type=int, default=1,
                    help="--config c1: interleaved repeats of the mode list")
    ap.add_argument("--c1-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--c1-cpus", default="", help=argparse.SUPPRESS)
    ap.add_argument("--c1-rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--c1-mode", default="device", help=argparse.SUPPRESS)
    ap.add_argument("--c1-dir", default="", help=argparse.SUPPRESS)
    ap.add_argument("--p2p-child", default="", help=argparse.SUPPRESS)
    ap.add_argument("--p2p-out", default="", help=argparse.SUPPRESS)
    ap.add_argument("--p2p-timeout", type=float, default=150.0, help=argparse.SUPPRESS)
    ap.add_argument("--test-transport", default="none", choices=["none", "ipc"],
                    help="testing: with --dist-backend gloo and every rank on one GPU, run "
                         "the native exchange (primary, sub-benchmarks, c4_named) over the "
                         "TEST-ONLY cross-process IPC transport of tests/c/libkf_testing.so "
                         "instead of falling back to torch.distributed (RCCL refuses two "
                         "ranks per GPU); the line says exchange_kind 'native (test "
                         "transport)' and its rates are not xGMI rates")
    ap.add_argument("--rehearse-exchange", action="store_true",
                    help="testing: run the N > 1 branch (native exchange over RCCL, "
                         "sub-benchmarks, line) with a single rank")
    ap.add_argument("--profile-only", action="store_true",
                    help="only the timed kernel loop (for rocprofv3 runs)")
    return ap.parse_args()


def load_traffic():
    """PMC HBM bytes per launch of the reduce kernel, if profiled (profiles/)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), d.get("source")


def time_local_reduce(lib, sets, steps, warmup, world):
    """Average duration of one reduce launch over `steps` back-to-back launches,
    from HIP events on the launch stream; plus wall time per step. Launch i
    reduces bucket set i % len(sets)."""
    from kungfu_amd import _lib
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    args = [(_lib.ptr_array([x.data_ptr(), y.data_ptr()]), z.data_ptr(), z.numel())
            for x, y, z in sets]
    fn = lib.kf_bucket_reduce
    rc = 0
    for i in range(warmup):
        ptrs, zp, n = args[i % len(args)]
        rc = fn(ptrs, 2, zp, n, KF_FLOAT, KF_SUM, sp)
    if warmup:
        _lib.check(rc, "kf_bucket_reduce")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(steps):
        ptrs, zp, n = args[i % len(args)]
        fn(ptrs, 2, zp, n, KF_FLOAT, KF_SUM, sp)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    err = lib.kf_last_error()
    kernel_s = ev0.elapsed_time(ev1) / 1e3 / steps
    return kernel_s, wall, err


def kernel_families(lib, dev):
    """Every other kernel family behind the C ABI, timed in the driver's own
    run the way the headline is (HIP events on the launch stream, launches
    cycling over independent buffer sets, median of 5 x 20), each against the
    8 TB/s roofline in algorithmic bytes and checked once against a torch
    restatement on the same buffers (bit-exact: these are the same IEEE
    operations). The placement of each allocation moves these rates by up to
    5 %."""
    from kungfu_amd import _lib, ops
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    mib = 1 << 20
    out = {}

    def timed(launch, nsets):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(nsets):
            _lib.check(launch(i), "launch")
        ts = []
        for _ in range(5):
            ev0.record(s)
            for i in range(20):
                launch(i % nsets)
            ev1.record(s)
            torch.cuda.synchronize()
            ts.append(ev0.elapsed_time(ev1) * 1e3 / 20)
        ts.sort()
        return ts[2]

    def report(name, algo_bytes, us, ok, what):
        out[name] = {"us": round(us, 2), "algorithmic_bytes": algo_bytes,
                     "frac": round(algo_bytes / us / 1e3 / HBM_PEAK_GBPS, 4),
                     "correct": bool(ok), "what": what}

    n = 256 * mib // 4
    g = torch.Generator(device=dev).manual_seed(7)
    for k in (4, 8):  # the k-input fold (star root, all-to-all fold)
        sets = []
        for _ in range(3):
            ins = [torch.randn(n, device=dev, generator=g) for _ in range(k)]
            sets.append((_lib.ptr_array([t.data_ptr() for t in ins]), torch.empty(n, device=dev), ins))
        us = timed(lambda i: lib.kf_bucket_reduce(sets[i][0], k, sets[i][1].data_ptr(), n,
                                                  KF_FLOAT, KF_SUM, sp), 3)
        want = sets[0][2][0].clone()
        for t in sets[0][2][1:]:
            want += t
        report("fold_k%d_f32" % k, (k + 1) * 256 * mib, us, torch.equal(sets[0][1], want),
               "kf_bucket_reduce, %d inputs of 256 MiB, left fold" % k)
        del sets, want
        torch.cuda.empty_cache()
    sets = [tuple(torch.randn(n, device=dev, generator=g) for _ in range(3)) for _ in range(3)]
    us = timed(lambda i: lib.kf_bucket_reduce_avg(
        _lib.ptr_array([sets[i][0].data_ptr(), sets[i][1].data_ptr()]), 2, sets[i][2].data_ptr(),
        n, KF_FLOAT, 3, sp), 3)
    x, y, z = sets[0]
    report("avg_k2_np3_f32", 3 * 256 * mib, us,
           torch.equal(z, (x + y) / torch.full_like(x, 3.0)),
           "kf_bucket_reduce_avg, S-SGD fused (x + y) / 3, IEEE division")
    xs = [t[0] for t in sets]
    ref = xs[0].clone()
    _lib.check(lib.kf_bucket_div(xs[0].data_ptr(), n, KF_FLOAT, 8, sp), "kf_bucket_div")
    ok = torch.equal(xs[0], ref / torch.full_like(ref, 8.0))
    us = timed(lambda i: lib.kf_bucket_div(xs[i].data_ptr(), n, KF_FLOAT, 8, sp), 3)
    report("div_shard_np8_f32", 2 * 256 * mib, us, ok,
           "kf_bucket_div in place, the shard /np between reduce-scatter and all-gather")
    del sets, xs, ref
    torch.cuda.empty_cache()
    nb = 128 * mib  # bf16 elements in 256 MiB
    vs = [torch.randn(nb, device=dev, generator=g).bfloat16() for _ in range(3)]
    sm = [torch.randn(nb, device=dev, generator=g).bfloat16() for _ in range(3)]
    v0 = vs[0].clone()
    _lib.check(lib.kf_sma_blend(v0.data_ptr(), sm[0].data_ptr(), nb, 0x20209, 8, 0.1, sp), "sma")
    want = ((1 - 0.1) * vs[0].float() + 0.1 * (sm[0].float() / 8))  # fp32 restatement
    ok = bool(((v0.float() - want).abs() <= want.abs() * 2 ** -7 + 1e-30).all())
    us = timed(lambda i: lib.kf_sma_blend(vs[i].data_ptr(), sm[i].data_ptr(), nb, 0x20209, 8,
                                          0.1, sp), 3)
    report("sma_blend_bf16", 3 * 256 * mib, us, ok,
           "kf_sma_blend in place, v = 0.9 v + 0.1 (s / 8), bf16 (within one bf16 rounding "
           "of the fp32 value; bit-exact checks in tests/)")
    del vs, sm, v0, want
    torch.cuda.empty_cache()
    nbk, bk = 16, 4 * mib // 4  # 16 buckets of 4 MiB fp32 per launch
    sets = []
    for _ in range(6):
        xs = [torch.randn(bk, device=dev, generator=g) for _ in range(nbk)]
        ys = [torch.randn(bk, device=dev, generator=g) for _ in range(nbk)]
        zs = [torch.empty(bk, device=dev) for _ in range(nbk)]
        ins = _lib.ptr_array([p for a, b in zip(xs, ys) for p in (a.data_ptr(), b.data_ptr())])
        sets.append((ins, _lib.ptr_array([t.data_ptr() for t in zs]),
                     (ctypes.c_size_t * nbk)(*[bk] * nbk), xs, ys, zs))
    us = timed(lambda i: lib.kf_bucket_reduce_batch(sets[i][0], 2, sets[i][1], sets[i][2], nbk,
                                                    KF_FLOAT, KF_SUM, 0, sp), 6)
    ok = all(torch.equal(z, x + y) for x, y, z in zip(*sets[0][3:]))
    report("batch_16x4MiB_f32", nbk * 3 * 4 * mib, us, ok,
           "kf_bucket_reduce_batch: 16 buckets of 4 MiB (C3's size), z = x + y, one launch")
    del sets
    torch.cuda.empty_cache()
    # C5's blend step: BERT-base bf16 in the bench's buckets, one batched
    # launch; the sum workspaces laid out as the exchange lays them out
    # (collective.workspace_like). In this 16 MiB-bucket layout every bucket
    # is its own allocation, so the launch blends 13 ranges (buckets of one
    # flat buffer, C4's layout, would merge into one)
    from kungfu_amd.collective import GradBuckets, workspace_like
    bert = _models()["bert"][:201]
    sets = []
    for _ in range(3):
        gbv = GradBuckets(bert, torch.bfloat16, dev, 8, bucket_bytes=16 << 20)
        for b in gbv.buckets:
            b.copy_(torch.randn(b.numel(), device=dev, generator=g).bfloat16())
        sums = workspace_like(gbv.buckets)
        for t in sums:
            t.copy_(torch.randn(t.numel(), device=dev, generator=g).bfloat16())
        sets.append((_lib.ptr_array([b.data_ptr() for b in gbv.buckets]),
                     _lib.ptr_array([t.data_ptr() for t in sums]),
                     (ctypes.c_size_t * len(sums))(*[t.numel() for t in sums]), gbv, sums))
    nbs = len(sets[0][4])
    v0 = [b.clone() for b in sets[0][3].buckets]
    _lib.check(lib.kf_sma_blend_batch(sets[0][0], sets[0][1], sets[0][2], nbs, 0x20209, 8, 0.1,
                                      sp), "sma batch")
    for b, a in zip(v0, sets[0][4]):
        ops.sma_blend_(b, a, 8, 0.1)  # the per-bucket kernel: the same bits
    ok = all(torch.equal(a, b) for a, b in zip(sets[0][3].buckets, v0))
    us = timed(lambda i: lib.kf_sma_blend_batch(sets[i][0], sets[i][1], sets[i][2], nbs, 0x20209,
                                                8, 0.1, sp), 3)
    report("sma_batch_c5_bf16", 3 * 2 * sum(t.numel() for t in sets[0][4]), us, ok,
           "kf_sma_blend_batch: C5's SMA blend step, BERT-base bf16 in %d buckets, one launch "
           "(the exchange's 16 MiB-bucket layout, every bucket its own allocation; "
           "bit-identical to one kf_sma_blend per bucket)"
           % nbs)
    del sets, v0
    torch.cuda.empty_cache()
    out.update(exchange_phase2(lib, dev, g))
    return out


def exchange_phase2(lib, dev, g, world=8):
    """The element-wise step the native exchange launches between its two
    collectives, at the shapes it has on BASELINE's 8-GPU configs (phase 2 of
    kf_exchange.hip's batch): C5's rank-order fold of the 8 received bf16
    shards per bucket with /8 fused (all-to-all algo), and the in-place shard
    /np of C4 (ResNet-50, 16 buckets) and C3 (64 x 4 MiB) after their
    reduce-scatters — each ONE kf_bucket_reduce_batch call on the exact
    pointers and counts the exchange passes. Launches cycle over enough
    independent sets (>= 0.75 GiB) that none is served from the Infinity
    Cache; each checked against the oracle-equivalent torch restatement."""
    from kungfu_amd import _lib
    from kungfu_amd.collective import GradBuckets
    # every launch below goes to this stream, so it can be captured
    cap = torch.cuda.Stream(device=dev)
    sp = cap.cuda_stream
    out = {}
    models = _models()

    def timed(launch, nsets):
        """(GPU us per launch, eager us per launch). The exchange issues
        these launches from C++ between its collectives, so what they cost is
        GPU time: 4 * nsets launches are captured into one HIP graph and the
        graph's replay is timed with events on the capture stream (a graph's
        kernel boundaries cost what a stream's do, MI355X_MICROARCH.md,
        launch costs). The eager figure times the same launches called one by
        one from Python through ctypes: for the short shard /np launches
        (about 6 us) that loop is host-bound (its ~8 us per call was r04's
        figure)."""
        torch.cuda.synchronize()  # inputs were made on the default stream
        with torch.cuda.stream(cap):
            for i in range(nsets):
                _lib.check(launch(i), "launch")
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eager = []
        with torch.cuda.stream(cap):
            for _ in range(5):
                ev0.record(cap)
                for i in range(4 * nsets):
                    _lib.check(launch(i % nsets), "launch")
                ev1.record(cap)
                torch.cuda.synchronize()
                eager.append(ev0.elapsed_time(ev1) * 1e3 / (4 * nsets))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=cap):
            for i in range(4 * nsets):
                # a launch refused during capture would leave the graph short
                # and its replay fast for nothing: fail instead
                _lib.check(launch(i % nsets), "launch during capture")
        torch.cuda.synchronize()
        ts = []
        with torch.cuda.stream(cap):
            for _ in range(5):
                ev0.record(cap)
                graph.replay()
                ev1.record(cap)
                torch.cuda.synchronize()
                ts.append(ev0.elapsed_time(ev1) * 1e3 / (4 * nsets))
        del graph
        ts.sort()
        eager.sort()
        return ts[2], eager[2]

    def report(name, algo_bytes, uss, ok, what, nb):
        us, eager = uss
        out[name] = {"us": round(us, 2), "algorithmic_bytes": algo_bytes,
                     "frac": round(algo_bytes / us / 1e3 / HBM_PEAK_GBPS, 4),
                     "eager_python_us": round(eager, 2),
                     "timing": "HIP graph replay of the launches on one stream",
                     "correct": bool(ok), "buckets": nb, "what": what}

    # C5 at N = 8: per bucket, the workspace holds the 8 received shards back to
    # back (q elements each) and the fold writes shard `rank` of the bucket
    bert = models["bert"][:201]
    counts = [b.numel() for b in GradBuckets(bert, torch.bfloat16, dev, world,
                                             bucket_bytes=16 << 20).buckets]
    qs = [c // world for c in counts]
    per_set = sum((world + 1) * q * 2 for q in qs)
    nsets = max(2, -(-(768 << 20) // per_set))
    sets = []
    for _ in range(nsets):
        ws = [torch.randn(world * q, device=dev, generator=g).bfloat16() for q in qs]
        outs = [torch.empty(q, device=dev, dtype=torch.bfloat16) for q in qs]
        ins = _lib.ptr_array([w.data_ptr() + j * q * 2 for w, q in zip(ws, qs)
                              for j in range(world)])
        sets.append((ins, _lib.ptr_array([o.data_ptr() for o in outs]),
                     (ctypes.c_size_t * len(qs))(*qs), ws, outs))
    us = timed(lambda i: lib.kf_bucket_reduce_batch(sets[i][0], world, sets[i][1], sets[i][2],
                                                    len(qs), 0x20209, KF_SUM, world, sp), nsets)
    ok = True
    for w, o, q in zip(sets[0][3], sets[0][4], qs):
        acc = w[:q].float()
        for j in range(1, world):
            acc = acc + w[j * q:(j + 1) * q].float()  # fp32 accumulation, rank order
        ok = ok and torch.equal(o, (acc / world).bfloat16())
    report("c5_a2a_fold_n8_bf16", per_set, us, ok,
           "C5 at N=8: kf_bucket_reduce_batch, k=8 received bf16 shards per bucket "
           "(%d buckets, shards of %.2f-%.2f MiB), rank-order fold, /8 fused" %
           (len(qs), min(qs) * 2 / 2**20, max(qs) * 2 / 2**20), len(qs))
    del sets
    torch.cuda.empty_cache()

    def shard_div(name, counts, what):
        qs = [c // world for c in counts]
        per_set = sum(2 * q * 4 for q in qs)
        nsets = max(2, -(-(768 << 20) // per_set))
        sets = []
        for _ in range(nsets):
            # the buckets back to back in ONE flat buffer, as GradBuckets lays
            # them out for the exchange: one shard every bucket's length
            flat = torch.randn(sum(counts), device=dev, generator=g)
            offs = [sum(counts[:i]) for i in range(len(counts))]
            bs = [flat[o:o + c] for o, c in zip(offs, counts)]
            shard = [b[q * 3:q * 4] for b, q in zip(bs, qs)]  # rank 3's shard
            ptrs = _lib.ptr_array([s.data_ptr() for s in shard])
            sets.append((ptrs, (ctypes.c_size_t * len(qs))(*qs), bs, shard))
        ref = [s.clone() for s in sets[0][3]]
        torch.cuda.synchronize()
        _lib.check(lib.kf_bucket_reduce_batch(sets[0][0], 1, sets[0][0], sets[0][1], len(qs),
                                              KF_FLOAT, KF_SUM, world, sp), name)
        torch.cuda.synchronize()
        ok = all(torch.equal(s, r / torch.full_like(r, float(world)))
                 for s, r in zip(sets[0][3], ref))
        us = timed(lambda i: lib.kf_bucket_reduce_batch(sets[i][0], 1, sets[i][0], sets[i][1],
                                                        len(qs), KF_FLOAT, KF_SUM, world, sp),
                   nsets)
        report(name, per_set, us, ok, what % (len(qs), qs[0] * 4 / 2**20), len(qs))
        del sets, ref
        torch.cuda.empty_cache()

    rn = GradBuckets(models["resnet50-imagenet"], torch.float32, dev, world, n_buckets=16)
    shard_div("c4_shard_div_n8_f32", [b.numel() for b in rn.buckets],
              "C4 at N=8: kf_bucket_reduce_batch k=1, in-place /8 of each bucket's shard "
              "after the reduce-scatter (%d shards of %.2f MiB)")
    del rn
    shard_div("c3_shard_div_n8_f32", [1 << 20] * 64,
              "C3 at N=8: kf_bucket_reduce_batch k=1, in-place /8 of each 4 MiB bucket's "
              "shard after the reduce-scatter (%d shards of %.2f MiB)")
    return out


def cpu_baseline(x, y, seconds):
    """KungFu's own CPU reduce timed on this host: the reference's
    std_transform_2 compiled from its sources (oracle/_ref, kind "reference")
    when that build is present, else the oracle's bit-exact restatement built
    with the same flags (kind "port"). 1 thread over the whole bucket, plus the
    reference's goroutine-per-1 MiB-chunk fan-out (session.go:317-323) over
    the box's CPU share."""
    from oracle import oracle
    oracle.build()
    xh = x.cpu().numpy()
    yh = y.cpu().numpy()
    zh = np.empty_like(xh)
    ref = oracle.ref_transform2_addr()
    if ref is not None:
        kind, what = "reference", ("KungFu's std_transform_2 built from its sources "
                                   "(op.cpp/f16.c/dtype.c, -O2 -mavx -mf16c)")
        run = lambda reps, threads: oracle.bench_ref(ref, xh, yh, zh, "f32", "sum",  # noqa: E731
                                                     reps, threads=threads)
    else:
        kind, what = "port", "oracle restatement built -O2 -mavx -mf16c"
        run = lambda reps, threads: oracle.bench_transform2(xh, yh, zh, "f32", "sum",  # noqa: E731
                                                            reps, threads=threads)
    run(1, 1)  # page in
    ok = bool(np.array_equal(zh, xh + yh))
    t1 = run(2, 1) / 2
    reps = max(1, min(1000, int(seconds / max(t1, 1e-6))))
    t = run(reps, 1)
    s_bytes = xh.nbytes
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    # the reference's fan-out: one goroutine per 1 MiB chunk, run by
    # GOMAXPROCS threads, which Go sets to the CPUs the process may use
    # (runtime.NumCPU = the affinity mask); also at the GPU's NUMA node and
    # at 16 threads (the box's nominal CPU share), so the curve is visible
    gomaxprocs = len(os.sched_getaffinity(0))
    numa = gpu_local_cpus()
    legs = {"gomaxprocs": gomaxprocs, "numa_node": len(numa) if numa else None,
            "16": min(16, gomaxprocs)}
    by_threads = {}
    for key, nt in legs.items():
        if nt is None or nt < 2:
            continue
        nt = min(nt, 1024)  # the harness's pool limit (oracle/kf_oracle.c MAX_POOL)
        tm1 = run(2, nt) / 2
        target = seconds / 3
        mreps = max(2, min(1000, int(target / max(tm1, 1e-6))))
        tm = run(mreps, nt)
        if tm < target / 2 and mreps < 1000:  # the 2-rep calibration ran slow (thread start)
            mreps = max(2, min(1000, int(mreps * target / max(tm, 1e-6))))
            tm = run(mreps, nt)
        by_threads[key] = {"threads": nt, "value": round(mreps * s_bytes / tm / 2**30, 3),
                           "seconds": round(tm, 2), "reps": mreps}
    # reported: the reference's best fan-out on this box (the conservative
    # baseline); GOMAXPROCS, the reference's own setting, is in by_threads
    top = max(by_threads.values(), key=lambda r: r["value"]) if by_threads else None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            quota = None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    multi = None
    if top is not None:
        multi = {"value": top["value"], "unit": "GiB/s", "cores": top["threads"],
                 "sample": "%d x 256 MiB in 1 MiB chunks, one pool of %d threads taking the "
                           "chunks of every rep in turn, %.1f s: the fastest of the legs in "
                           "by_threads (GOMAXPROCS, the reference's own setting, = the %d "
                           "CPUs of the affinity mask; cgroup quota %s CPUs)"
                           % (top["reps"], top["threads"], top["seconds"], gomaxprocs, quota),
                 "by_threads": by_threads, "cgroup_cpu_quota": quota}
    return {
        "value": round(reps * s_bytes / t / 2**30, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": kind,
        "correct": ok,
        "multi_thread": multi,
        "sample": "%d x std_transform_2(f32, SUM) over the same 256 MiB bucket, 1 thread, "
                  "%s, %.1f s, %s" % (reps, what, t, cpu_model),
    }


def host_staged(lib, x, y):
    """Copy-inclusive rate of the drop-in (std_transform_2's path): pageable
    host buffers (copied to HBM and back through the runtime's staging) and
    page-locked ones (zero copy: the kernel reads x, y and writes z in host
    memory over PCIe); plus the latency of one 1 MiB chunk, the reference's
    unit of work (session.go:301-304), next to the CPU restatement's.
    Never `value`."""
    res = {}
    for kind in ("pageable", "pinned"):
        xh, yh = x.cpu(), y.cpu()
        zh = torch.empty_like(xh)
        if kind == "pinned":
            xh, yh, zh = xh.pin_memory(), yh.pin_memory(), zh.pin_memory()
        n = xh.numel()
        args = (xh.data_ptr(), yh.data_ptr(), zh.data_ptr(), n, KF_FLOAT, KF_SUM)
        rc = lib.kf_transform2_host(*args)
        if rc != 0:
            res[kind] = {"error": lib.kf_last_error().decode()}
            continue
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            lib.kf_transform2_host(*args)
        t = (time.perf_counter() - t0) / reps
        ok = bool(torch.equal(zh, xh + yh))
        res[kind] = {"value": round(xh.numel() * 4 / t / 2**30, 3), "unit": "GiB/s",
                     "ms_per_call": round(t * 1e3, 3), "correct": ok}
    res["path"] = ("host x,y -> HIP kernel -> host z (PCIe incl.), 256 MiB fp32; "
                   "pageable: staged through HBM; pinned: zero copy")
    res["chunk_1MiB"] = chunk_latency(lib, x)
    res["chunk_sweep"] = chunk_sweep(lib, x)
    return res


def chunk_latency(lib, x, reps=2000, chunk_bytes=1 << 20):
    """One fp32 chunk (1 MiB: the reference's unit, session.go:301-304)
    through std_transform_2 with page-locked buffers, and through the
    reference's own compiled reduce (1 thread; the restatement if that build
    is absent)."""
    from oracle import oracle
    n = chunk_bytes // 4
    xh = x[:n].cpu().pin_memory()
    yh = x[n:2 * n].cpu().pin_memory()
    zh = torch.empty_like(xh).pin_memory()
    args = (xh.data_ptr(), yh.data_ptr(), zh.data_ptr(), n, KF_FLOAT, KF_SUM)
    for _ in range(5):
        lib.std_transform_2(*args)
    t0 = time.perf_counter()
    for _ in range(reps):
        lib.std_transform_2(*args)
    gpu_s = (time.perf_counter() - t0) / reps
    ok = bool(torch.equal(zh, xh + yh))
    xa, ya = xh.numpy().copy(), yh.numpy().copy()
    za = np.empty_like(xa)
    # the same chunk in ordinary (malloc'd) host memory page-locked through
    # kf_host_register, as a Go host would register its receive pool
    # (byte_slice_pool.go:28-60): the library finds it in its registry
    # instead of asking HIP for six pointer attributes per call
    rx, ry, rz = (np.empty(n + 1024, np.float32) for _ in range(3))
    off = lambda a: (-a.ctypes.data % 4096) // 4  # noqa: E731  page-aligned views
    rx, ry, rz = (a[off(a):off(a) + n] for a in (rx, ry, rz))
    rx[:], ry[:] = xa, ya
    regd = [a for a in (rx, ry, rz) if lib.kf_host_register(a.ctypes.data, a.nbytes) == 0]
    reg_us = None
    if len(regd) == 3:
        rargs = (rx.ctypes.data, ry.ctypes.data, rz.ctypes.data, n, KF_FLOAT, KF_SUM)
        for _ in range(5):
            lib.std_transform_2(*rargs)
        t0 = time.perf_counter()
        for _ in range(reps):
            lib.std_transform_2(*rargs)
        reg_us = (time.perf_counter() - t0) / reps * 1e6
        ok = ok and bool(np.array_equal(rz, rx + ry))
    for a in regd:
        lib.kf_host_unregister(a.ctypes.data)
    ref = oracle.ref_transform2_addr()
    if ref is not None:
        run = lambda r: oracle.bench_ref(ref, xa, ya, za, "f32", "sum", r)  # noqa: E731
    else:
        run = lambda r: oracle.bench_transform2(xa, ya, za, "f32", "sum", r)  # noqa: E731
    run(5)
    cpu_s = run(reps) / reps
    return {"gpu_pinned_us": round(gpu_s * 1e6, 2),
            "gpu_registered_us": None if reg_us is None else round(reg_us, 2),
            "cpu_us": round(cpu_s * 1e6, 2),
            "cpu_kind": "reference" if ref is not None else "port",
            "correct": ok, "reps": reps}


def chunk_sweep(lib, x):
    """Where the drop-in (zero copy over PCIe) overtakes the reference's
    1-thread CPU reduce: one chunk of 64 KiB .. 64 MiB each way."""
    out = []
    for kib in (64, 256, 1024, 4096, 16384, 65536):
        reps = max(5, min(2000, (256 << 10) // kib))
        r = chunk_latency(lib, x, reps=reps, chunk_bytes=kib << 10)
        r["chunk_KiB"] = kib
        r["gpu_over_cpu"] = round(r["cpu_us"] / r["gpu_pinned_us"], 3)
        if r["gpu_registered_us"]:
            r["gpu_registered_over_cpu"] = round(r["cpu_us"] / r["gpu_registered_us"], 3)
        out.append(r)
    return out


# ---- C1: np = 2 plumbing over the rchannel wire format ----------------------

C1_ELEMS = 1 << 20  # one 4 MiB fp32 bucket


def c1_child(args):
    """One peer of the C1 run. Rank 0 (the star root) reduces with:
    device   — page-locked ingest + HIP fold, bucket resident in HBM;
    dropin   — host buffers, std_transform_2 of libkungfu_amd.so per chunk;
    cpu      — host buffers, the reference's own reduce (oracle/_ref) or the
               oracle's restatement of it (this is bench.py's CPU-baseline leg);
    cpu_dev  — the bucket resident in HBM as in `device`, reduced the way the
               reference does for GPU tensors (KungfuAllReduce is registered
               for DEVICE_CPU only, tensorflow/ops/cpu/collective.cpp:103, so
               the framework copies the tensor to the host and back): D2H into
               a page-locked buffer, the `cpu` all-reduce, H2D, all inside the
               timed step."""
    from kungfu_amd.session import Session
    r, npeers = args.c1_rank, args.c1_np
    if args.c1_cpus:  # the GPU's NUMA node (gpu_local_cpus), every mode alike
        os.sched_setaffinity(0, [int(c) for c in args.c1_cpus.split(",")])
    x = ((r + 1) * (np.arange(C1_ELEMS) % 1024) / 1024).astype(np.float32)
    # sum_r (r+1) * (i mod 1024) / 1024: every partial sum is exact in fp32
    want = (npeers * (npeers + 1) // 2 * (np.arange(C1_ELEMS) % 1024) / 1024).astype(np.float32)
    if args.c1_mode.startswith("device"):
        if args.c1_mode == "device_batched":  # A/B: the k-input fold at the root
            os.environ["KUNGFU_AMD_BATCH_FOLD"] = "1"
        if args.c1_mode == "device_nomirror":  # A/B: the root's result via D2H again
            os.environ["KUNGFU_AMD_ROOT_MIRROR"] = "0"
        dev = torch.device("cuda", 0)
        xs, ys = torch.from_numpy(x).to(dev), torch.zeros(C1_ELEMS, device=dev)
        sess = Session(r, npeers, args.c1_dir, mode="device")
        result = lambda: ys.cpu().numpy()  # noqa: E731
    else:
        xs, ys = x, np.zeros_like(x)
        fn = None
        cpu_kind = None
        if args.c1_mode in ("cpu", "cpu_dev"):
            # the reference's own std_transform_2 (oracle/_ref) when built,
            # else the oracle's restatement of it
            from oracle import oracle
            ref = oracle.ref_transform2_addr()
            if ref is not None:
                oracle.lib().oracle_set_fold_fn(ctypes.c_void_p(ref))
                fn = ctypes.cast(oracle.lib().oracle_fold_via_fn, ctypes.c_void_p)
                cpu_kind = "reference"
            else:
                fn = ctypes.cast(oracle.lib().oracle_transform2, ctypes.c_void_p)
                cpu_kind = "port"
        sess = Session(r, npeers, args.c1_dir, mode="host", host_reduce_fn=fn)
        result = lambda: ys  # noqa: E731
    name = "NegotiatedGrad_0/AllReduce"
    step = lambda: sess.all_reduce(xs, ys, name)  # noqa: E731
    if args.c1_mode == "cpu_dev":
        dev = torch.device("cuda", 0)
        xd, yd = torch.from_numpy(x).to(dev), torch.zeros(C1_ELEMS, device=dev)
        xh = torch.empty(C1_ELEMS, dtype=torch.float32).pin_memory()
        yh = torch.empty(C1_ELEMS, dtype=torch.float32).pin_memory()
        xs, ys = xh.numpy(), yh.numpy()

        def step():
            xh.copy_(xd, non_blocking=True)
            torch.cuda.synchronize()
            sess.all_reduce(xs, ys, name)
            yd.copy_(yh, non_blocking=True)
            torch.cuda.synchronize()
        result = lambda: yd.cpu().numpy()  # noqa: E731
    for _ in range(args.warmup):
        step()
    ok = bool(np.array_equal(result(), want))
    ts = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    ok = ok and bool(np.array_equal(result(), want))
    sess.close()
    if r == 0:
        ts.sort()
        med = ts[len(ts) // 2]
        nbytes = C1_ELEMS * 4
        rec = {"mode": args.c1_mode, "correct": ok,
               "latency_ms_median": round(med * 1e3, 4),
               "latency_ms_min": round(ts[0] * 1e3, 4),
               "rate_GiBps": round(4 * (npeers - 1) * nbytes / med / 2**30, 3)}
        if args.c1_mode in ("cpu", "cpu_dev"):
            rec["kind"] = cpu_kind
        print(json.dumps(rec), flush=True)


def gpu_local_cpus(index=0):
    """The CPUs this process may use that sit on the GPU's own NUMA node
    (sysfs local_cpulist of its PCI function), or None: the C1 peers of every
    mode run there, so no mode's run lands on a far socket by chance (a
    device-mode chunk crosses PCIe up to three times; the CPU fold's buffers
    live in host memory)."""
    try:
        pr = torch.cuda.get_device_properties(index)
        bdf = "%04x:%02x:%02x.0" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
        with open("/sys/bus/pci/devices/%s/local_cpulist" % bdf) as f:
            spec = f.read().strip()
    except Exception:
        return None
    cpus = set()
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    cpus &= os.sched_getaffinity(0)
    return sorted(cpus) or None


# C1's peers are np processes sharing ONE GPU. Each HIP process maps its
# streams onto up to GPU_MAX_HW_QUEUES hardware queues (4 by default); past
# what the GPU schedules at once the queues are time-sliced and every hop
# waits for its process's turn (np = 8: 12.4 ms per all-reduce at 4 queues
# per peer, 3.3 ms at 2; np = 4: 1.60 -> 1.39 ms; np = 2: 0.65 -> 0.61 ms;
# profiles/r04/c1_ab_np{2,4,8}_hwq_r04z.json). Two per peer (KUNGFU_AMD_C1_HW_QUEUES
# overrides it: the box itself exports GPU_MAX_HW_QUEUES=4, HIP's default, so
# an inherited value says nothing). The same applies to any deployment that
# puts several peers on one GPU.
C1_HW_QUEUES = "2"


def c1_run(npeers, modes, steps, warmup, timeout=600, cpus=None):
    """Launch the np peers per mode (subprocesses, one unix socket each);
    {mode: rank 0's record}."""
    import subprocess
    import tempfile
    env = dict(os.environ)
    env["GPU_MAX_HW_QUEUES"] = os.environ.get("KUNGFU_AMD_C1_HW_QUEUES", C1_HW_QUEUES)
    res = {}
    for mode in modes:
        with tempfile.TemporaryDirectory() as d:
            cmd = [sys.executable, os.path.abspath(__file__), "--c1-child",
                   "--c1-mode", mode, "--c1-dir", d, "--steps", str(steps),
                   "--warmup", str(warmup), "--c1-np", str(npeers)]
            if cpus:
                cmd += ["--c1-cpus", ",".join(map(str, cpus))]
            procs = [subprocess.Popen(cmd + ["--c1-rank", str(r)], stdout=subprocess.PIPE,
                                      text=True, cwd=ROOT, env=env) for r in range(npeers)]
            try:
                outs = [p.communicate(timeout=timeout)[0] for p in procs]
            except subprocess.TimeoutExpired:
                for p in procs:
                    p.kill()
                res[mode] = {"error": "not finished within %d s" % timeout}
                continue
            if any(p.returncode for p in procs):
                res[mode] = {"error": "peer exit codes %s" % [p.returncode for p in procs]}
                continue
            res[mode] = json.loads(outs[0].strip().splitlines()[-1])
    return res


def c1_summary(steps=100, warmup=10, repeats=5):
    """BASELINE configs[0] beside the N = 1 line: np = 2 peers on this host,
    one 4 MiB fp32 bucket, median latency and 4(np-1)*bytes/t
    (kungfu-bench-allreduce.go:73-80); the device session against the
    reference's own CPU fold (oracle/_ref) in the same session engine. The
    modes run `repeats` times, interleaved: the CPU fold's median moves by 2x
    between back-to-back runs of the same command on one box
    (profiles/r02/c1_variants.jsonl), so each mode reports the median of its
    runs' medians and every run's median beside it."""
    cpus = gpu_local_cpus()
    runs = [c1_run(2, ("device", "cpu", "cpu_dev"), steps, warmup, timeout=180, cpus=cpus)
            for _ in range(repeats)]
    res = {}
    for mode in ("device", "cpu", "cpu_dev"):
        recs = [r[mode] for r in runs]
        ok = [x for x in recs if "error" not in x]
        if not ok:
            res[mode] = recs[0]
            continue
        meds = sorted(x["latency_ms_median"] for x in ok)
        rec = dict(ok[0])
        rec["latency_ms_median"] = meds[len(meds) // 2]
        rec["latency_ms_min"] = min(x["latency_ms_min"] for x in ok)
        rec["rate_GiBps"] = round(4 * (2 - 1) * C1_ELEMS * 4 / (rec["latency_ms_median"] / 1e3)
                                  / 2**30, 3)
        rec["correct"] = all(x.get("correct") is True for x in recs)
        rec["run_medians_ms"] = [x["latency_ms_median"] for x in ok]
        res[mode] = rec
    out = {"workload": "C1: np=2 localhost, one 4 MiB fp32 bucket, 4 x 1 MiB chunks, STAR "
                       "at rank 0, rchannel framing over unix sockets",
           "np": 2, "steps": steps, "repeats": repeats,
           "unit": "GiB/s (4(np-1)*bytes/t, median of the runs' medians)",
           "modes": "device: bucket in HBM, HIP fold; cpu: bucket in host memory, the "
                    "reference's CPU fold; cpu_dev: bucket in HBM reduced the reference's "
                    "way for GPU tensors (D2H, the cpu all-reduce, H2D)",
           "cpus": ("the GPU's NUMA node: %d CPUs" % len(cpus)) if cpus else "not pinned",
           "hw_queues_per_peer": os.environ.get("KUNGFU_AMD_C1_HW_QUEUES", C1_HW_QUEUES)}
    out.update(res)
    out["correct"] = all(r.get("correct") is True for r in res.values())
    return out


def c1_parent(args):
    modes = ("device", "device_batched", "dropin", "cpu", "cpu_dev") if args.c1_np > 2 else \
        ("device", "device_nomirror", "dropin", "cpu", "cpu_dev")
    if args.c1_modes:
        modes = tuple(args.c1_modes.split(","))
    cpus = gpu_local_cpus()
    runs = [c1_run(args.c1_np, modes, args.steps, args.warmup, cpus=cpus)
            for _ in range(args.c1_repeats)]
    res = runs[0]
    if args.c1_repeats > 1:  # each mode: the median of its runs' medians, every run beside
        for m in modes:
            ok = [r[m] for r in runs if "error" not in r[m]]
            if ok:
                meds = sorted(x["latency_ms_median"] for x in ok)
                res[m] = dict(ok[0], latency_ms_median=meds[len(meds) // 2],
                              run_medians_ms=[x["latency_ms_median"] for x in ok],
                              correct=all(x.get("correct") is True for x in ok))
    line = {
        "metric": "C1 all-reduce rate 4(np-1)*bytes/t (kungfu-bench-allreduce.go:73-80)",
        "unit": "GiB/s",
        "config": {"workload": "C1: np=%d localhost, one 4 MiB fp32 bucket, 4 x 1 MiB "
                               "chunks, STAR at rank 0, rchannel framing over unix "
                               "sockets" % args.c1_np, "elements": C1_ELEMS,
                   "np": args.c1_np},
        "steps": args.steps, "warmup": args.warmup,
        "modes": res,
    }
    print(json.dumps(line), flush=True)


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) with no launcher around it: start the N
    ranks as ONE child, `torch.distributed.run --nproc-per-node N` on
    127.0.0.1, the way the reference's `kungfu-run -np N`
    (srcs/go/kungfu/runner/flags.go:73) starts its benchmark
    (tests/go/cmd/kungfu-bench-allreduce). The child inherits stdout, so
    rank 0's JSON line is this process's line; its exit status is ours. Runs
    before anything in this process touches the GPU (no exec)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.stdout.flush()
    rc = subprocess.call(cmd, env=env)
    if rc != 0:
        print("bench.py: the %d ranks ended with status %d" % (args.gpus, rc), file=sys.stderr)
    return rc


def main():
    args = parse()
    _OPTS["test_transport"] = args.test_transport
    if args.c1_child:
        return c1_child(args)
    if args.config == "c1":
        return c1_parent(args)
    if args.p2p_child:
        return p2p_child(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # nothing has touched the GPU yet: the ranks are children
        return launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (args.rehearse_exchange and world == 1):
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d (launch with --nproc-per-node "
                         "%d, or leave WORLD_SIZE unset and bench.py starts its own ranks)"
                         % (args.gpus, world, args.gpus))
    dev_index = local_rank if args.device_index is None else args.device_index
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    multi = world > 1 or args.rehearse_exchange
    if multi:
        if args.dist_backend == "nccl":
            _quiet(dist.init_process_group, "nccl", device_id=dev)
        else:
            _quiet(dist.init_process_group, args.dist_backend)

    from kungfu_amd import _lib
    lib = _lib.load()
    if lib.kf_device_count() < 1:
        raise SystemExit("kungfu_amd: no HIP device visible")

    n = args.elems
    sets = []
    for j in range(max(1, args.rotate)):
        g0 = torch.Generator(device=dev).manual_seed(1000 * j + 2 * rank)
        g1 = torch.Generator(device=dev).manual_seed(1000 * j + 2 * rank + 1)
        sets.append((torch.randn(n, device=dev, generator=g0),
                     torch.randn(n, device=dev, generator=g1),
                     torch.empty(n, device=dev)))
    x, y, z = sets[0]
    s_bytes = x.numel() * x.element_size()

    kernel_s, wall_local, _ = time_local_reduce(lib, sets, args.steps,
                                                args.warmup, world)
    if args.profile_only:
        if rank == 0:
            print(json.dumps({"kernel_us": kernel_s * 1e6}))
        return
    # same buffers every launch: the 256 MiB output can stay in the Infinity
    # Cache between launches; reported beside, never as `value`
    hot_s, _, _ = time_local_reduce(lib, sets[:1], args.steps, args.warmup, world)

    out = {}
    if not multi:
        step_s = wall_local / args.steps
        value = s_bytes / kernel_s / 2**30
        # parity check of every timed output (full oracle check: tests/)
        for xs, ys, zs in sets:
            assert torch.equal(zs, xs + ys)
        workload = "C2: device-resident z = x + y, one 256 MiB fp32 bucket"
        parallelism = "single GPU"
    else:
        _progress(rank, "C3 all-reduce, %d ranks" % world)
        # the primary exchange: the native C-ABI path (kf_exchange_*: RCCL
        # reduce-scatter -> HIP /np -> RCCL all-gather), every bucket its own
        # shards, all 64 in one call (grouped RCCL launches, one batched HIP
        # epilogue); the torch.distributed path if it cannot be set up
        prim_ex, how, fallback = _primary_exchange(args, rank, world, dev)
        from kungfu_amd.collective import GradBuckets
        gb = GradBuckets([n], torch.float32, dev, world, n_buckets=args.buckets)
        pieces = gb.buckets
        gb.views[0].copy_(x)
        coalesce = fallback is not None  # the torch path fuses contiguous buckets
        # correctness of the timed path before timing it: every rank's x is
        # regenerated from its seed and reduced locally by the HIP k-input
        # fold (rank order) -> must match (bit-exact at N=2, bound beyond)
        from kungfu_amd import ops
        allx = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(2 * r))
                for r in range(world)]
        want = ops.bucket_reduce_avg(allx, world)
        absum = sum(a.abs() for a in allx) if world > 2 else None
        del allx

        def parity():
            try:
                prim_ex.all_reduce_(pieces, average=True, coalesce=coalesce)
                got = gb.views[0]
                ok = (bool(torch.equal(got, want)) if world <= 2 else
                      _within(got, want, absum, world))
            except Exception as e:
                print("[bench] rank %d: primary exchange failed: %r" % (rank, e), file=sys.stderr,
                      flush=True)
                ok = False
            return _agree(ok, dev)

        ok = parity()
        if not ok and fallback is None:
            # the native exchange runs for the first time on a multi-GPU node
            # here: a wrong result must cost the native path, not the line
            from kungfu_amd.collective import Exchange
            _NATIVE.pop("ex", None).close()
            prim_ex, coalesce = Exchange(), True
            how = "torch.distributed RCCL RS -> HIP /np -> AG, contiguous buckets fused into one"
            fallback = "native exchange failed the C3 parity check; torch path used"
            gb.views[0].copy_(x)
            ok = parity()
        trial = None
        if ok and fallback is None and args.c3_schedule != "grouped":
            # the native exchange's schedules for the same S-SGD step, each
            # parity-checked, timed briefly on every rank (max over ranks, so
            # every rank picks the same), the fastest kept for the timed
            # region; all of them are in the line (collective.schedule_trial_ms)
            cands = {
                "grouped": (prim_ex, False, how),
                "fused": (prim_ex, True, "native C-ABI exchange: the %d contiguous buckets as ONE "
                          "RCCL reduce-scatter -> HIP /np -> RCCL all-gather (the reference's "
                          "nccl_fusion, sync_sgd.py:87-92)" % len(pieces)),
                "a2a": (_AlgoView(prim_ex, "a2a"), False, "native C-ABI exchange: per bucket RCCL "
                        "all-to-all -> HIP rank-order fold with /np -> RCCL all-gather, the "
                        "buckets of a step in one call"),
                "pipelined": (_AlgoView(prim_ex, "rs", PIPE_GROUPS), False,
                              "native C-ABI exchange: per bucket RCCL reduce-scatter -> HIP /np "
                              "-> RCCL all-gather, pipelined in %d groups (HIP /np on a second "
                              "stream between the groups' collectives)" % PIPE_GROUPS),
            }
            # rs_avg (ncclAvg, the /np inside the collective) is not a candidate:
            # it is not bit-exact on overflowing sums and subnormals
            # (test_rs_avg_special_values_decide_the_default), so it stays an
            # opt-in, timed beside as the c4_rs_avg sub-benchmark
            if args.c3_schedule != "auto":
                cands = {args.c3_schedule: cands[args.c3_schedule]}
            trial = {}
            for name, (ex_c, co_c, _) in cands.items():
                prim_ex, coalesce = ex_c, co_c
                gb.views[0].copy_(x)
                if name != "grouped" and not parity():
                    trial[name] = None
                    continue
                gb.views[0].copy_(x)
                trial[name] = _timed(lambda: ex_c.all_reduce_(pieces, average=True,
                                                              coalesce=co_c), 10, 3, dev, world)
            best = min((t, nm) for nm, t in trial.items() if t is not None)[1]
            prim_ex, coalesce, how = cands[best]
            _progress(rank, "C3 schedule %s (trial ms %s)" % (
                best, {k: None if v is None else round(v * 1e3, 3) for k, v in trial.items()}))
        del want, absum
        if not ok:
            raise SystemExit("C3 all-reduce parity check failed (N=2 bit-exact / N>2 bound)")
        _progress(rank, "C3 parity ok; timing %d steps" % args.steps)
        gb.views[0].copy_(x)
        step_s, phase_us = _timed_phases(
            prim_ex, lambda: prim_ex.all_reduce_(pieces, average=True, coalesce=coalesce),
            args.steps, args.warmup, dev, world)
        value = s_bytes / step_s / 2**30  # per GPU, as the metric says
        busbw = 2 * (world - 1) / world * s_bytes / step_s / 1e9
        _progress(rank, "C3 %.3f ms per step" % (step_s * 1e3))
        out["value_aggregate"] = round(world * value, 3)
        out["collective"] = {
            "busbw_GBps": round(busbw, 2),
            "algbw_GiBps_per_gpu": round(s_bytes / step_s / 2**30, 3),
            "xgmi_bound_GBps": round(XGMI_LINK_GBPS * (world - 1), 1),
            "frac_of_xgmi": _xgmi_frac(busbw, world),
            "buckets": args.buckets,
            "exchange": how,
            "correct": bool(ok),
        }
        if phase_us is not None:
            out["collective"]["phase_us"] = phase_us
        out["collective"].update(_rccl_report(_NATIVE.get("ex") if fallback is None else None,
                                              world, fallback))
        if trial is not None:
            out["collective"]["schedule_trial_ms"] = {
                k: None if v is None else round(v * 1e3, 4) for k, v in trial.items()}
        if fallback is not None:
            out["collective"]["native_exchange_error"] = fallback
        workload = ("C3: S-SGD all-reduce of %d fp32 buckets (%d MiB) per rank: %s"
                    % (len(pieces), s_bytes >> 20, how))
        parallelism = "dp%d" % world
        kt = torch.tensor([kernel_s], dtype=torch.float64, device=dev)
        dist.all_reduce(kt, op=dist.ReduceOp.MAX)
        kernel_s = kt.item()
        native = _NATIVE.get("ex")
        steps_x = min(args.steps, 50)
        # the other multi-GPU configs of BASELINE.json, reported beside `value`
        extra = (("c4", lambda: bench_c4(world, rank, dev, steps_x, 5, exchange="native")),
                 ("c5", lambda: bench_c5(world, rank, dev, steps_x, 5, exchange="native")),
                 ("c5_pipe", lambda: bench_c5(world, rank, dev, steps_x, 5,
                                              exchange="native_pipe")),
                 ("c5_overlap", lambda: bench_c5_overlap(world, rank, dev, min(steps_x, 20), 3)),
                 ("c4_overlap", lambda: bench_c4_overlap(world, rank, dev, min(steps_x, 20), 3)),
                 ("c4_pipe", lambda: bench_c4(world, rank, dev, steps_x, 5,
                                              exchange="native_pipe")),
                 ("c4_rs_avg", lambda: bench_c4(world, rank, dev, steps_x, 5,
                                                exchange="native_rs_avg")),
                 ("c3_pipe", lambda: bench_c3_native(world, rank, dev, steps_x, 5, n, x, "rs",
                                                     args.buckets, pipe=True)),
                 ("c3_a2a", lambda: bench_c3_native(world, rank, dev, steps_x, 5, n, x,
                                                    "a2a", args.buckets)),
                 ("c3_fused", lambda: bench_c3_native(world, rank, dev, steps_x, 5, n, x,
                                                      "rs", args.buckets, fused=True)),
                 ("c3_torch_fused", lambda: bench_c3_torch(world, dev, min(args.steps, 20), n, x,
                                                           args.buckets, True)),
                 ("c3_per_bucket", lambda: bench_c3_torch(world, dev, min(args.steps, 20), n, x,
                                                          args.buckets, False)),
                 ("c4_torch", lambda: bench_c4(world, rank, dev, steps_x, 5, exchange="torch")),
                 ("c5_torch", lambda: bench_c5(world, rank, dev, steps_x, 5, exchange="torch")),
                 ("c3_ar", lambda: bench_c3_ar(world, rank, dev, steps_x, 5, n, x)))
        # last: the experimental peer-to-peer paths, in child processes
        extra += tuple(_p2p_runs(world, rank, dev, steps_x, n, x).items())
        child_keys = P2P_KEYS
        if args.test_transport == "ipc":
            # the ranks already share one GPU: c4_named runs in these
            # processes, on an exchange of its own (a child group would put
            # 2N processes' queues on the GPU, which then time-slices them)
            child_keys = tuple(k for k in P2P_KEYS if k != "c4_named")
            extra = tuple((k, (lambda: _named_ipc(world, rank, dev, steps_x)) if k == "c4_named"
                           else fn) for k, fn in extra)
        # The primary number is measured by now: a sub-benchmark that hangs
        # (a peer mapping refused in a way that blocks, a stuck collective)
        # must not take it down. Past --extras-timeout every rank dumps its
        # stacks and stops with a non-zero status; rank 0 first prints the
        # line with what was measured so far.
        prim = dict(value=value, step_s=step_s, kernel_s=kernel_s, workload=workload,
                    parallelism=parallelism)
        dog = threading.Timer(args.extras_timeout, _extras_timeout,
                              (args, rank, world, sets, s_bytes, n, hot_s, prim, out))
        dog.daemon = True
        dog.start()
        t_extras = time.perf_counter()
        wanted = args.extras.split(",")
        for key, fn in extra:
            if args.no_extra:
                break
            if key not in wanted or key in child_keys:
                continue
            _progress(rank, "sub-benchmark %s" % key)
            out["_running"] = key
            t0 = time.perf_counter()
            try:
                res, err = fn(), None
            except Exception as e:  # keep the primary line; say what failed
                res, err = None, repr(e)[:300]
                # every rank names its own failure (the line carries rank 0's,
                # which may only be "failed earlier" after another rank's)
                print("[bench] rank %d: sub-benchmark %s failed: %s" % (rank, key, err),
                      file=sys.stderr, flush=True)
            # every rank learns whether every rank got through, before any
            # starts the next sub-benchmark's collectives
            if not _agree(err is None, dev):
                res = {"error": err or "failed on another rank"}
            res["wall_s"] = round(time.perf_counter() - t0, 2)
            out[key] = res
        p2p = [k for k, _ in extra if k in child_keys and k in wanted and not args.no_extra]
        if p2p:
            _progress(rank, "sub-benchmarks %s (child processes)" % ",".join(p2p))
            out["_running"] = "p2p children"
            left = args.extras_timeout - (time.perf_counter() - t_extras) - 20.0
            out.update(p2p_extras(args, rank, world, local_rank, dev, p2p, left))
        out.pop("_running", None)
        dog.cancel()
        if native is not None:
            native.close()

    res = _result(args, world, sets, s_bytes, n, hot_s,
                  dict(value=value, step_s=step_s, kernel_s=kernel_s, workload=workload,
                       parallelism=parallelism))
    res.update(out)
    if rank == 0 and not multi:
        if not args.no_kernels:
            _progress(rank, "kernel families")
            try:
                res["kernels"] = kernel_families(lib, dev)
            except Exception as e:  # the C2 line stands on its own
                res["kernels"] = {"error": repr(e)[:300]}
        if not args.no_host_staged:
            res["host_staged"] = host_staged(lib, x, y)
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(x, y, args.cpu_seconds)
        if not args.no_c1:
            _progress(rank, "C1 (np=2 localhost, device and reference-CPU folds)")
            try:
                res["c1"] = c1_summary()
            except Exception as e:  # the C2 line stands on its own
                res["c1"] = {"error": repr(e)[:300]}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if multi:
        dist.barrier()
        dist.destroy_process_group()


def _result(args, world, sets, s_bytes, n, hot_s, prim):
    """The bench line's primary fields (everything but the sub-benchmarks)."""
    value, step_s, kernel_s = prim["value"], prim["step_s"], prim["kernel_s"]
    workload, parallelism = prim["workload"], prim["parallelism"]
    traffic, tsrc = load_traffic() if n == BUCKET_ELEMS else (None, None)
    achieved = 3 * s_bytes / kernel_s / 1e9
    return {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: N(0,1) fp32 from torch.Generator, %d bucket sets" % len(sets),
        "config": {
            "workload": workload,
            "bucket_bytes": s_bytes,
            "elements": n,
            "parallelism": parallelism,
        },
        "note": ("BASELINE configs: N = 1 times the local two-input reduce (C2, HBM-bound); "
                 "N > 1 times the S-SGD all-reduce of 64 x 4 MiB buckets over xGMI (C3, "
                 "link-bound). value is per GPU at every N (the metric's unit): bucket bytes "
                 "/ step; value_aggregate = N x value is the whole job. The two steps differ, "
                 "so value(N) / value(1) is the exchange's cost relative to one local reduce, "
                 "not a scaling efficiency of one kernel (DESIGN.md section 7); "
                 "collective.frac_of_xgmi grades the N > 1 step against its own bound"),
        "roofline": {
            "bound": "hbm",
            "kernel": REDUCE_KERNEL,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "traffic_source": tsrc,
            "bytes_per_launch": 3 * s_bytes,
            "kernel_us": round(kernel_s * 1e6, 2),
            "rotate": len(sets),
            "same_buffer_GBps": round(3 * s_bytes / hot_s / 1e9, 1),
        },
    }


def _extras_timeout(args, rank, world, sets, s_bytes, n, hot_s, prim, out):
    """Watchdog of the N>1 sub-benchmarks (a thread): dump every thread's
    stack (so the stall names itself), print the line with the primary number
    and whatever finished, then end this rank with a non-zero status — a
    stuck sub-benchmark is a failure, not a success."""
    import faulthandler
    stuck = out.pop("_running", "?")
    print("[bench] rank %d: sub-benchmark %s not finished within --extras-timeout %.0f s; "
          "stacks:" % (rank, stuck, args.extras_timeout), file=sys.stderr, flush=True)
    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
    res = _result(args, world, sets, s_bytes, n, hot_s, prim)
    res.update(out)
    res[stuck] = {"error": "not finished within --extras-timeout %.0f s; stopped" %
                  args.extras_timeout}
    if rank == 0:
        print(json.dumps(res), flush=True)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(3)


def _progress(rank, what):
    """One line on stderr per phase (rank 0), so a long multi-GPU run shows
    it is alive; stdout carries only the JSON line."""
    if rank == 0:
        print("[bench] %.1f s: %s" % (time.perf_counter() - _T0, what), file=sys.stderr, flush=True)


_T0 = time.perf_counter()


def _models():
    with open(os.path.join(ROOT, "tests", "golden", "models.json")) as f:
        return json.load(f)


def _within(got, want, absum, world):
    """Two fp32 averages of the same `world` addends summed in different
    orders: each sum is within (world-1)*u*sum|x| of the exact sum (u = 2^-24),
    and each /world adds one rounding (u*|avg|)."""
    u = 2.0 ** -24
    bound = 2 * (world - 1) * u * absum / world + 2 * u * want.abs() + 1e-38
    return bool(((got - want).abs() <= bound * 1.0001).all())


def _xgmi_frac(busbw, world):
    """busbw against the xGMI bound: one 153 GB/s link per peer (world - 1
    links per GPU on a fully connected node); None for a single rank."""
    return round(busbw / (XGMI_LINK_GBPS * (world - 1)), 4) if world > 1 else None


def _agree(ok, dev):
    """All ranks learn whether every rank's check passed (no one-rank hang)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def _timed(fn, steps, warmup, dev, world, on_timed=None):
    """Seconds per step, the max over ranks. on_timed: called once the
    warmup is done, right before the timed region starts."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    if on_timed is not None:
        on_timed()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item() / steps


def _timed_phases(ex, fn, steps, warmup, dev, world):
    """_timed over the exchange's per-phase timing window (set_timing /
    phase_times: HIP events at the phase boundaries on the launch stream):
    (seconds per step, {phase: us per step, ...} of this rank, or None when
    the exchange has no timing). The phases of an un-pipelined call partition
    its stream time, so their sum is the step minus the host's gaps between
    calls; pipelined calls overlap two streams and are counted, not split."""
    if not hasattr(ex, "set_timing"):
        return _timed(fn, steps, warmup, dev, world), None
    step_s = _timed(fn, steps, warmup, dev, world, on_timed=lambda: ex.set_timing(True))
    ph = ex.phase_times()
    ex.set_timing(False)
    calls, untimed = ph.pop("calls"), ph.pop("untimed_calls")
    out = {k: round(v / steps, 2) for k, v in ph.items()}
    out["sum"] = round(sum(ph.values()) / steps, 2)
    out["timed_calls_per_step"] = round(calls / steps, 3)
    if untimed:
        out["pipelined_calls_untimed"] = untimed
    out["step_us"] = round(step_s * 1e6, 2)
    return step_s, out


def _fill(gb, rank_seed, dev, dtype):
    g = torch.Generator(device=dev).manual_seed(rank_seed)
    for v in gb.views:
        v.copy_(torch.randn(v.numel(), device=dev, generator=g).to(dtype))


_NATIVE = {}  # the primary's NativeExchange, reused by the sub-benchmarks
_OPTS = {"test_transport": "none"}  # --test-transport, for the helpers below

# The peer-to-peer sub-benchmarks map every peer's buckets and signal words
# over xGMI (HIP IPC) and spin on device barriers: the one part of the line
# that has never run across devices before the driver's multi-GPU node. They
# run in one child process per rank (own process group on its own port), so a
# fault or an abort there ends the child, not the ranks holding the line.
# run in child processes (their own process group and bounded waits): the
# xGMI peer mappings and the name negotiation, which run across devices for
# the first time on the driver's node
P2P_KEYS = ("c3_p2p", "c3_p2p_push", "c3_p2p_hostbar", "c4_p2p", "c5_p2p", "c4_named")


def _p2p_runs(world, rank, dev, steps, n, x):
    return {
        "c3_p2p": lambda: bench_c3_p2p(world, rank, dev, steps, 5, n, x),
        "c3_p2p_push": lambda: bench_c3_p2p(world, rank, dev, steps, 5, n, x, mode="push"),
        "c3_p2p_hostbar": lambda: bench_c3_p2p(world, rank, dev, steps, 5, n, x, barrier="host"),
        "c4_p2p": lambda: bench_c4(world, rank, dev, steps, 5, exchange="p2p"),
        "c5_p2p": lambda: bench_c5(world, rank, dev, steps, 5, exchange="p2p"),
        "c4_named": lambda: _named_in_child(world, rank, dev, steps),
    }


def _named_in_child(world, rank, dev, steps):
    """c4_named in a child process: its first run across devices is the
    name negotiation's first over RCCL (a split-off control communicator and
    a negotiation thread), so it is isolated like the P2P paths — a hang or
    fault there ends the child, not the line."""
    if "ex" not in _NATIVE:
        if dist.get_backend() != "nccl":
            raise RuntimeError("the name-keyed path needs the native exchange (nccl backend)")
        from kungfu_amd.exchange import NativeExchange
        _NATIVE["ex"] = NativeExchange(algo="auto", device=dev)
    return bench_c4_named(world, rank, dev, steps, 5)


def _named_ipc(world, rank, dev, steps):
    """c4_named under --test-transport ipc, in this process, over an ipc
    exchange of its own (the name-keyed path must not interleave with the
    primary's ordered calls on one exchange)."""
    ex = _ipc_exchange(rank, world, dev, "auto")
    try:
        return bench_c4_named(world, rank, dev, steps, 5, ex=ex)
    finally:
        ex.close()


def p2p_extras(args, rank, world, local_rank, dev, keys, seconds):
    """Every rank starts `bench.py --p2p-child` and waits for it (bounded);
    rank 0 returns the children's results, or an error per sub-benchmark."""
    import subprocess
    import tempfile
    if not _agree(seconds >= 30.0, dev):
        return {k: {"error": "not run: %.0f s of --extras-timeout left" % seconds} for k in keys}
    port = torch.tensor([_free_port() if rank == 0 else 0], dtype=torch.int64, device=dev)
    dist.broadcast(port, 0)
    port = int(port.item())
    path = os.path.join(tempfile.gettempdir(), "kf_bench_p2p_%d_%d.json" % (port, rank))
    # not the launcher's rendezvous: the child group has its own TCP store
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC")}
    env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(local_rank),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    cmd = [sys.executable, os.path.abspath(__file__), "--p2p-child", ",".join(keys),
           "--p2p-out", path, "--p2p-timeout", str(seconds - 10.0),
           "--elems", str(args.elems), "--steps", str(min(args.steps, 50)),
           "--dist-backend", args.dist_backend, "--test-transport", args.test_transport]
    if args.device_index is not None:
        cmd += ["--device-index", str(args.device_index)]
    t0 = time.perf_counter()
    # the child's stdout (gloo prints there) goes to stderr: stdout carries
    # only the line
    p = subprocess.Popen(cmd, env=env, stdout=sys.stderr.fileno())
    try:
        rc = p.wait(timeout=seconds)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()
        rc = "timeout"
    ok = _agree(rc == 0, dev)
    res = {}
    if rank == 0 and os.path.exists(path):
        with open(path) as f:
            res = json.load(f)
    if os.path.exists(path):
        os.unlink(path)
    for k in keys:
        if k not in res:
            res[k] = {"error": "child process of rank %d ended with %s before finishing it" %
                      (rank, rc) if rc != 0 else ("failed on another rank's child" if not ok
                                                  else "no result written")}
    res["p2p_children"] = {"rc_rank0": rc, "all_ok": ok, "wall_s": round(time.perf_counter() - t0, 2)}
    return res


def _quiet(fn, *a, **kw):
    """fn with file descriptor 1 pointed at stderr: gloo announces its mesh on
    stdout, which carries only the JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        return fn(*a, **kw)
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def p2p_child(args):
    """One rank of the peer-to-peer sub-benchmarks (see P2P_KEYS): its own
    process group, the same synthetic x as the parent, the results of rank 0
    written to --p2p-out. Bounded by its own watchdog."""
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    _OPTS["test_transport"] = args.test_transport

    def give_up():
        print("[bench] p2p child rank %d: not done within %.0f s" % (rank, args.p2p_timeout),
              file=sys.stderr, flush=True)
        import faulthandler
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        os._exit(5)

    dog = threading.Timer(args.p2p_timeout, give_up)
    dog.daemon = True
    dog.start()
    dev_index = local_rank if args.device_index is None else args.device_index
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    init = "tcp://127.0.0.1:%s" % os.environ["MASTER_PORT"]
    if args.dist_backend == "nccl":
        _quiet(dist.init_process_group, "nccl", init_method=init, rank=rank, world_size=world,
               device_id=dev)
    else:
        _quiet(dist.init_process_group, args.dist_backend, init_method=init, rank=rank,
               world_size=world)
    _progress(rank, "p2p children: process group of %d up" % world)
    n = args.elems
    x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(2 * rank))
    runs = _p2p_runs(world, rank, dev, args.steps, n, x)
    out = {}
    for key in args.p2p_child.split(","):
        _progress(rank, "sub-benchmark %s" % key)
        t0 = time.perf_counter()
        try:
            res, err = runs[key](), None
        except Exception as e:
            res, err = None, repr(e)[:300]
        if not _agree(err is None, dev):
            res = {"error": err or "failed on another rank"}
        res["wall_s"] = round(time.perf_counter() - t0, 2)
        out[key] = res
        if rank == 0:  # what finished survives a later fault
            with open(args.p2p_out, "w") as f:
                json.dump(out, f)
    dog.cancel()
    if "ex" in _NATIVE:
        _NATIVE.pop("ex").close()
    dist.barrier()
    dist.destroy_process_group()
    return 0


def _primary_exchange(args, rank, world, dev):
    """(exchange, description, why the native path is not used or None).
    The native C-ABI exchange needs RCCL with one GPU per rank; its
    communicator is created on a helper thread so that an init that never
    returns costs --native-timeout seconds and the torch.distributed path,
    not the whole line. The id is shared on this thread (a torch collective)."""
    from kungfu_amd.collective import Exchange
    how_torch = "torch.distributed RCCL RS -> HIP /np -> AG, contiguous buckets fused into one"
    if args.test_transport == "ipc":
        ex = _ipc_exchange(rank, world, dev, "rs")
        _NATIVE["ex"] = ex
        return ex, ("native C-ABI exchange (kf_exchange_all_reduce_batch) over the TEST-ONLY "
                    "cross-process IPC transport (tests/c/kf_testing_ipc.hip, every rank on "
                    "one GPU): per bucket reduce-scatter -> HIP /np -> all-gather, the "
                    "buckets of a step in one call"), None
    if args.dist_backend != "nccl" or args.device_index is not None:
        return Exchange(), how_torch, "not tried: ranks share a GPU (rehearsal)"
    from kungfu_amd.exchange import NativeExchange
    box = {}
    try:
        uid = NativeExchange.shared_id()
    except Exception as e:
        uid, box["err"] = None, repr(e)[:300]
    if uid is not None:
        def make():
            try:
                box["ex"] = NativeExchange(algo="rs", device=dev, uid=uid,
                                           timeout_s=args.native_timeout)
            except Exception as e:
                box["err"] = repr(e)[:300]
        th = threading.Thread(target=make, daemon=True)
        th.start()
        th.join(args.native_timeout + 15)
    ex = box.get("ex")
    if _agree(ex is not None, dev):
        _NATIVE["ex"] = ex
        return ex, ("native C-ABI exchange (kf_exchange_all_reduce_batch): per bucket RCCL "
                    "reduce-scatter -> HIP /np -> RCCL all-gather, the buckets of a step in "
                    "one call (grouped RCCL launches, one batched HIP epilogue)"), None
    if ex is not None:
        ex.close()
    return Exchange(), how_torch, box.get("err", "not ready within %.0f s or failed on "
                                                 "another rank" % args.native_timeout)


def _ipc_exchange(rank, world, dev, algo):
    """The native exchange of this rank over the test-only cross-process IPC
    transport (tests/c/kf_testing_ipc.hip through kf_exchange_create_transport):
    every rank a process on the same GPU, the group named by a token rank 0
    draws and broadcasts. Test infrastructure, loaded only under
    --test-transport ipc."""
    tok = torch.tensor([int.from_bytes(os.urandom(6), "little") if rank == 0 else 0],
                       dtype=torch.int64, device=dev)
    dist.broadcast(tok, 0)
    tests = os.path.join(ROOT, "tests")
    if tests not in sys.path:
        sys.path.insert(0, tests)
    from loopback import ipc_exchange
    # a rendezvous may wait out the other ranks' time slices on the shared
    # GPU; the line's own watchdog (--extras-timeout) bounds the whole run
    return ipc_exchange("/kf_bench_ipc_%x" % int(tok.item()), rank, world, algo=algo,
                        device=dev.index, timeout_s=300.0)


def _rccl_report(native, world, fallback):
    """What RCCL itself says about the primary exchange, for the N > 1 line:
    the communicator's rank count (ncclCommCount), RCCL's version
    (ncclGetVersion) and which exchange ran. A communicator whose count is
    not N means the ranks did not form one N-rank RCCL world (each may be
    timing a one-rank communicator), so the line would measure nothing of
    xGMI: that ends the run loudly instead of printing a number."""
    if native is None:
        return {"exchange_kind": "torch.distributed", "rccl_world": None, "rccl_version": None,
                "why_not_native": fallback}
    count, ver = native.transport_info()
    if count == -1 and _OPTS.get("test_transport") == "ipc":
        return {"exchange_kind": "native (test transport)", "rccl_world": None,
                "rccl_version": None,
                "transport": "ipc: tests/c/kf_testing_ipc.hip, the N ranks are processes on "
                             "one GPU; rates are not xGMI rates (no performance claim)"}
    if count == -1:  # a host-provided transport (tests' rccl1): RCCL not asked
        return {"exchange_kind": "native C-ABI (kf_exchange), host transport",
                "rccl_world": None, "rccl_version": None}
    if count != world:
        raise SystemExit("bench.py: the native exchange's RCCL communicator holds %d ranks, not "
                         "WORLD_SIZE %d: no N-rank collective would be timed" % (count, world))
    vs = None
    if ver:  # NCCL_VERSION_CODE: major * 10000 + minor * 100 + patch
        vs = "%d.%d.%d" % (ver // 10000, ver // 100 % 100, ver % 100)
    return {"exchange_kind": "native C-ABI (kf_exchange)", "rccl_world": count,
            "rccl_version": vs, "rccl_version_code": ver}


def _exchange(kind):
    """native: the C-ABI exchange (RCCL + HIP epilogue / rank-order fold);
    torch: collective.Exchange over torch.distributed; p2p: the xGMI
    peer-mapped pull exchange with device barriers (p2p.PeerExchange). Every
    one picks algo "auto": f32 sums go through RCCL's reduce-scatter, bf16
    through the all-to-all + rank-order fold (bit-exact at every N)."""
    if kind == "p2p":
        from kungfu_amd.p2p import PeerExchange
        return PeerExchange(timeout_s=5.0)
    if kind in ("native", "native_pipe", "native_rs_avg"):
        ex = _NATIVE.get("ex")
        if ex is None:
            raise RuntimeError("native exchange unavailable (see collective.native_exchange_error)")
        if kind == "native_rs_avg":
            return _AlgoView(ex, "rs_avg")
        return _AlgoView(ex, "auto", PIPE_GROUPS if kind == "native_pipe" else 1)
    from kungfu_amd.collective import Exchange
    return Exchange()


class _AlgoView:
    """The primary NativeExchange with another algo and pipeline setting (one
    communicator)."""

    def __init__(self, ex, algo, groups=1):
        self.ex, self.algo, self.groups, self.world = ex, algo, groups, ex.world

    def _run(self, fn, *a, **kw):
        saved, self.ex.algo = self.ex.algo, self.algo
        self.ex.set_pipeline(self.groups)
        try:
            return fn(*a, **kw)
        finally:
            self.ex.algo = saved
            self.ex.set_pipeline(1)

    def all_reduce_(self, *a, **kw):
        return self._run(self.ex.all_reduce_, *a, **kw)

    def sma_(self, *a, **kw):
        return self._run(self.ex.sma_, *a, **kw)

    def start_(self, *a, **kw):  # issued inside the call: the algo applies
        return self._run(self.ex.start_, *a, **kw)

    def start_into_(self, *a, **kw):
        return self._run(self.ex.start_into_, *a, **kw)

    def set_timing(self, on):
        return self.ex.set_timing(on)

    def phase_times(self):
        return self.ex.phase_times()


def bench_c3_native(world, rank, dev, steps, warmup, n, x, algo, nb, fused=False, pipe=False):
    """C3 through the native exchange with another algo or layout: "a2a" =
    RCCL all-to-all of every bucket's shards -> HIP rank-order fold (/np
    fused) -> RCCL all-gather, bit-exact against the local rank-order fold at
    every N; fused = the 64 contiguous buckets as ONE bucket (the reference's
    nccl_fusion, sync_sgd.py:87-92) instead of 64 grouped ones."""
    from kungfu_amd import ops
    from kungfu_amd.collective import GradBuckets
    ex = _exchange("native_pipe" if pipe else "native")
    ex.algo = algo
    gb = GradBuckets([n], torch.float32, dev, world, n_buckets=nb)
    gb.views[0].copy_(x)
    ex.all_reduce_(gb.buckets, average=True, coalesce=fused)
    allx = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(2 * r))
            for r in range(world)]
    want = ops.bucket_reduce_avg(allx, world)
    if algo == "a2a" or world == 2:
        ok = bool(torch.equal(gb.views[0], want))
    else:
        ok = _within(gb.views[0], want, sum(a.abs() for a in allx), world)
    del allx, want
    if not _agree(ok, dev):
        return {"error": "native %s exchange check failed (rank-order / N=2 bit-exact, "
                         "else the order bound)" % algo}
    step_s = _timed(lambda: ex.all_reduce_(gb.buckets, average=True, coalesce=fused),
                    steps, warmup, dev, world)
    s_bytes = n * 4
    busbw = 2 * (world - 1) / world * s_bytes / step_s / 1e9
    how = ("RCCL all-to-all -> HIP rank-order fold + /np -> RCCL all-gather" if algo == "a2a"
           else "RCCL reduce-scatter -> HIP /np -> RCCL all-gather")
    if pipe:
        how += ", pipelined in %d groups (HIP work on a second stream)" % PIPE_GROUPS
    return {"workload": "C3 via the native exchange, %s, algo %s (%s)" % (
                "one fused 256 MiB bucket" if fused else "%d grouped buckets" % nb, algo, how),
            "ms_per_step": round(step_s * 1e3, 4),
            "GiBps_per_gpu": round(s_bytes / step_s / 2**30, 3),
            "busbw_GBps": round(busbw, 2),
            "frac_of_xgmi": _xgmi_frac(busbw, world),
            "parity": ("bit-exact vs the rank-order fold (every N)" if algo == "a2a" else
                       "N=2 bit-exact, N>2 within the order bound"),
            "correct": True}


def bench_c3_torch(world, dev, steps, n, x, nb, fused):
    """C3 through torch.distributed (collective.Exchange, RCCL RS -> HIP /np
    -> AG): the 64 buckets coalesced into one collective (fused), or one RS ->
    /np -> AG per bucket, all reduce-scatters in flight first. Checked before
    timing; a progress line per timed step, so a slow step shows as slow and a
    stuck one is named by the watchdog's stack dump."""
    from kungfu_amd import ops
    from kungfu_amd.collective import Exchange, GradBuckets
    ex = Exchange()
    gb = GradBuckets([n], torch.float32, dev, world, n_buckets=nb)
    gb.views[0].copy_(x)
    ex.all_reduce_(gb.buckets, average=True, coalesce=fused)
    allx = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(2 * r))
            for r in range(world)]
    want = ops.bucket_reduce_avg(allx, world)
    ok = (bool(torch.equal(gb.views[0], want)) if world == 2 else
          _within(gb.views[0], want, sum(a.abs() for a in allx), world))
    del allx, want
    if not _agree(ok, dev):
        return {"error": "torch exchange check failed (N=2 bit-exact / N>2 bound)"}
    rank = dist.get_rank()

    def step():
        t0 = time.perf_counter()
        ex.all_reduce_(gb.buckets, average=True, coalesce=fused)
        if not fused:
            torch.cuda.synchronize()
            _progress(rank, "  c3 per-bucket step %.1f ms" % ((time.perf_counter() - t0) * 1e3))

    per_s = _timed(step, steps, 2, dev, world)
    s_bytes = n * 4
    return {"workload": "C3's %d buckets via torch.distributed, %s" % (
                nb, "coalesced into one RS -> /np -> AG" if fused else
                "one RS -> HIP /np -> AG per bucket"),
            "ms_per_step": round(per_s * 1e3, 4),
            "busbw_GBps": round(2 * (world - 1) / world * s_bytes / per_s / 1e9, 2),
            "correct": True}


def bench_c4(world, rank, dev, steps, warmup, exchange="native"):
    """C4: ResNet-50 gradient set (214 tensors, 25,583,592 fp32) fused into 16
    buckets (EvenPartition), S-SGD all-reduce."""
    from kungfu_amd import ops
    from kungfu_amd.collective import GradBuckets
    sizes = _models()["resnet50-imagenet"]
    ex = _exchange(exchange)
    gbs = [GradBuckets(sizes, torch.float32, dev, world, n_buckets=16) for _ in range(world)]
    for r, gb in enumerate(gbs):  # every rank's gradients, regenerated locally
        _fill(gb, 500 + r, dev, torch.float32)
    mine = gbs[rank]
    want = [ops.bucket_reduce_avg([gb.buckets[i] for gb in gbs], world)
            for i in range(len(mine.buckets))]
    absums = [sum(gb.buckets[i].abs() for gb in gbs) for i in range(len(mine.buckets))]
    orig = [b.clone() for b in mine.buckets] if exchange == "native_rs_avg" else None
    # the native exchange coalesces contiguous buckets into one run (the
    # reference's nccl_fusion) unless told not to; the pipelined schedule
    # needs them as separate buckets to have groups to overlap
    kw = {"coalesce": False} if exchange == "native_pipe" else {}
    ex.all_reduce_(mine.buckets, average=True, **kw)
    extra = {}
    if orig is not None:
        # the first real RCCL world's verdict on ncclAvg: the
        # opt-in rs_avg against the default rs (sum, then the exact /np) on
        # the same inputs, bit for bit
        got = [b.clone() for b in mine.buckets]
        for b, o in zip(mine.buckets, orig):
            b.copy_(o)
        _AlgoView(_NATIVE["ex"], "rs").all_reduce_(mine.buckets, average=True)
        extra["rs_avg_parity"] = _rs_avg_verdict(got, mine.buckets, mine.spans, world)
        for b, g in zip(mine.buckets, got):
            b.copy_(g)
        del got, orig
    ok = True
    for b, w, ab, sp in zip(mine.buckets, want, absums, mine.spans):
        if world == 2 or exchange == "p2p":  # rank order or two operands
            ok &= bool(torch.equal(b[:sp], w[:sp]))
        else:
            ok &= _within(b[:sp], w[:sp], ab[:sp], world)
    del want, absums
    gbs.clear()
    if not _agree(ok, dev):
        return {"error": "C4 parity check failed (N=2 or P2P bit-exact / N>2 bound)"}
    s_bytes = sum(sizes) * 4
    step_s, phase_us = _timed_phases(ex, lambda: ex.all_reduce_(mine.buckets, average=True, **kw),
                                     steps, warmup, dev, world)
    if exchange == "p2p":
        ex.close()
    busbw = 2 * (world - 1) / world * s_bytes / step_s / 1e9
    how = {"native": "native C-ABI exchange: RCCL RS -> HIP /np -> RCCL AG, the 16 contiguous "
                     "buckets coalesced into one run (nccl_fusion), one call",
           "native_pipe": "native C-ABI exchange: RCCL RS -> HIP /np -> RCCL AG, 16 buckets "
                          "in one call pipelined in %d groups (HIP /np on a second stream "
                          "between the groups' collectives)" % PIPE_GROUPS,
           "native_rs_avg": "native C-ABI exchange: RCCL RS with ncclAvg (no HIP epilogue) -> "
                            "RCCL AG, the 16 contiguous buckets coalesced into one run, one call",
           "torch": "torch.distributed RCCL RS -> HIP /np -> RCCL AG",
           "p2p": "xGMI P2P pull: rank-order shard fold from peers' HBM + gather, "
                  "device barriers"}[exchange]
    return {"workload": "C4: ResNet-50 grads, 25,583,592 fp32 in %d buckets, S-SGD "
                        "(%s)" % (len(mine.buckets), how),
            "bytes": s_bytes, "ms_per_step": round(step_s * 1e3, 4),
            "GiBps_per_gpu": round(s_bytes / step_s / 2**30, 3),
            "busbw_GBps": round(busbw, 2),
            "frac_of_xgmi": _xgmi_frac(busbw, world),
            "phase_us": phase_us, "correct": True, **extra}


def _rs_avg_verdict(got, ref, spans, world):
    """rs_avg (ncclAvg inside the reduce-scatter) against rs (sum, then the
    HIP /np) on the same buckets: bit-identical or not, and how many elements
    differ. The default stays rs either way; this records what the transport
    that ran actually does (transport: which one)."""
    bad = sum(int((a[:sp] != b[:sp]).sum().item()) for a, b, sp in zip(got, ref, spans))
    total = sum(int(sp) for sp in spans)
    kind = "test transport (ipc)" if _OPTS.get("test_transport") == "ipc" else (
        "RCCL, %d ranks" % world)
    return {"bit_exact_vs_rs": bad == 0, "mismatched_elements": bad, "elements": total,
            "transport": kind, "inputs": "N(0,1) fp32, no subnormal x / world"}


def bench_c4_named(world, rank, dev, steps, warmup, ex=None):
    """C4's 214 ResNet-50 gradient tensors one by one through the name-keyed
    all-reduce (kf_exchange_all_reduce_named, the torch op's path:
    all_reduce_cuda_async keyed by tensor name), every rank starting them in
    its OWN random order each step; the exchange negotiates the issue order
    and sends the names that become ready together as batched calls. S-SGD
    average, in place."""
    from kungfu_amd import ops
    from kungfu_amd.collective import GradBuckets
    sizes = _models()["resnet50-imagenet"]
    ex = _NATIVE.get("ex") if ex is None else ex
    if ex is None:
        raise RuntimeError("native exchange unavailable (see collective.native_exchange_error)")
    gbs = [GradBuckets(sizes, torch.float32, dev, world, n_buckets=16) for _ in range(world)]
    for r, gb in enumerate(gbs):
        _fill(gb, 600 + r, dev, torch.float32)
    mine = gbs[rank]
    views = mine.views
    want = [ops.bucket_reduce_avg([gb.views[i].reshape(-1) for gb in gbs], world)
            for i in range(len(views))]
    absums = [sum(gb.views[i].reshape(-1).abs() for gb in gbs) for i in range(len(views))]
    names = ["resnet50/grad/%d" % i for i in range(len(views))]
    flat = [v.reshape(-1) for v in views]
    rng = np.random.default_rng(1000 + rank)

    def step():
        for i in rng.permutation(len(flat)):
            ex.all_reduce_named(names[i], flat[i], average=True)
        ex.wait_named()

    inp = [f.clone() for f in flat]
    step()
    bad = [i for i, (v, w, ab) in enumerate(zip(flat, want, absums))
           if not (bool(torch.equal(v, w)) if world <= 2 else _within(v, w, ab, world))]
    detail = ""
    if bad:  # which tensors, and how far off (on this rank's stderr too)
        i = bad[0]
        off = int((flat[i] != want[i]).sum().item())
        detail = (" (rank %d: %d of %d tensors off; first %s, %d of %d elements, max |diff| "
                  "%.3g, equal to own input: %s)" % (
                      rank, len(bad), len(flat), names[i], off, flat[i].numel(),
                      (flat[i] - want[i]).abs().max().item(),
                      bool(torch.equal(flat[i], inp[i]))))
        print("[bench] c4_named" + detail, file=sys.stderr, flush=True)
    del want, absums, inp
    gbs.clear()
    if not _agree(not bad, dev):
        return {"error": "C4 named parity check failed (N<=2 bit-exact / N>2 bound)" + detail}
    s_bytes = sum(sizes) * 4
    step_s = _timed(step, steps, warmup, dev, world)
    busbw = 2 * (world - 1) / world * s_bytes / step_s / 1e9
    return {"workload": "C4: ResNet-50 grads, 214 fp32 tensors, each its own name-keyed "
                        "all-reduce started in a per-rank random order "
                        "(kf_exchange_all_reduce_named: negotiated order, batched issue, "
                        "RCCL RS -> HIP /np -> RCCL AG), S-SGD",
            "bytes": s_bytes, "tensors": len(flat), "ms_per_step": round(step_s * 1e3, 4),
            "GiBps_per_gpu": round(s_bytes / step_s / 2**30, 3),
            "busbw_GBps": round(busbw, 2),
            "frac_of_xgmi": _xgmi_frac(busbw, world), "correct": True}


def bench_c3_ar(world, rank, dev, steps, warmup, n, x):
    """C3 as ONE RCCL all-reduce (sum) of the 256 MiB bucket, then the HIP
    /np over the whole bucket: the alternative to RS -> /np on the shard -> AG,
    reported beside it to pick the faster exchange per N."""
    from kungfu_amd import ops
    b = x.clone()
    dist.all_reduce(b)
    ops.bucket_div_(b, world)
    allx = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(2 * r))
            for r in range(world)]
    want = ops.bucket_reduce_avg(allx, world)
    ok = bool(torch.equal(b, want)) if world == 2 else _within(b, want, sum(a.abs() for a in allx),
                                                                world)
    del allx, want
    if not _agree(ok, dev):
        return {"error": "all-reduce + /np check failed (N=2 bit-exact / N>2 bound)"}

    def step():
        b.copy_(x)
        dist.all_reduce(b)
        ops.bucket_div_(b, world)

    step_s = _timed(step, steps, warmup, dev, world)
    cp_s = _timed(lambda: b.copy_(x), steps, warmup, dev, world)  # refill, subtracted
    step_s = max(step_s - cp_s, 1e-9)
    s_bytes = n * 4
    busbw = 2 * (world - 1) / world * s_bytes / step_s / 1e9
    return {"workload": "C3 as RCCL all_reduce(sum) of the 256 MiB bucket + HIP /np over it",
            "ms_per_step": round(step_s * 1e3, 4),
            "GiBps_per_gpu": round(s_bytes / step_s / 2**30, 3),
            "busbw_GBps": round(busbw, 2),
            "frac_of_xgmi": _xgmi_frac(busbw, world), "correct": True}


def bench_c3_p2p(world, rank, dev, steps, warmup, n, x, mode="pull", barrier="device"):
    """C3 over xGMI peer mappings instead of RCCL (kungfu_amd/p2p.py). pull:
    each rank folds its shard straight from every peer's HBM in rank order,
    then gathers the other shards (remote reads, 3 barriers); push: shards
    are written into the owners' inboxes, folded locally, and written back
    into every peer's bucket (remote writes, 2 barriers). Deterministic, so
    checked bit-exact against a local fold of every rank's regenerated inputs
    at every N — before timing, and again after it on two fresh inputs (no
    shard may be served stale from a previous step)."""
    from kungfu_amd import ops
    from kungfu_amd.collective import GradBuckets
    from kungfu_amd.p2p import P2PExchange
    gb = GradBuckets([n], torch.float32, dev, world, n_buckets=1)
    gb.views[0].copy_(x)
    ex, err = None, ""
    try:
        ex = P2PExchange(gb.buckets, mode=mode, barrier=barrier, timeout_s=5.0)
    except Exception as e:  # e.g. IPC mapping refused on this node
        err = repr(e)[:300]
    if not _agree(ex is not None, dev):
        return {"error": "P2P setup failed on some rank: " + err}

    def check(seed):
        g = lambda r: torch.Generator(device=dev).manual_seed(seed + r)  # noqa: E731
        gb.views[0].copy_(torch.randn(n, device=dev, generator=g(rank)))
        ex.all_reduce_(average=True)
        want = ops.bucket_reduce_avg([torch.randn(n, device=dev, generator=g(r))
                                      for r in range(world)], world)
        return _agree(bool(torch.equal(gb.views[0], want)), dev)

    if not check(9000):
        st = ex.status()
        ex.close()
        return {"error": "P2P all-reduce not bit-exact against the rank-order fold"
                         + (" (device barrier status %d)" % st if st else "")}
    gb.views[0].copy_(x)
    step_s = _timed(lambda: ex.all_reduce_(average=True), steps, warmup, dev, world)
    after = check(9100) and check(9200)
    st = ex.status()
    ex.close()
    s_bytes = n * 4
    busbw = 2 * (world - 1) / world * s_bytes / step_s / 1e9
    how = ("shard fold from all peers' HBM (HIP k-input, rank order, fused /np) -> "
           "gather kernel; 3 barriers per step" if mode == "pull" else
           "shards written into the owners' inboxes -> local HIP k-input fold (rank "
           "order, fused /np) -> reduced shard written into every peer; 2 barriers per step")
    how += ("; barriers on the device (kf_peer_barrier: epoch stores into the peers' "
            "signal words over xGMI, bounded spin, no host sync)" if barrier == "device" else
            "; barriers on the host (torch.cuda.synchronize + dist.barrier)")
    return {"workload": "C3 via xGMI peer mappings (%s): %s" % (mode, how),
            "barrier": barrier, "barrier_status": st,
            "ms_per_step": round(step_s * 1e3, 4),
            "GiBps_per_gpu": round(s_bytes / step_s / 2**30, 3),
            "busbw_GBps": round(busbw, 2),
            "frac_of_xgmi": _xgmi_frac(busbw, world),
            "parity": "bit-exact vs rank-order fold before timing: yes; after timing, "
                      "two fresh inputs: %s" % ("yes" if after else "NO"),
            "correct": bool(after)}


def bench_c5(world, rank, dev, steps, warmup, alpha=0.1, exchange="native"):
    """C5: BERT-base (first 201 tensors of the fake model, 109,483,778
    params) in bf16 with SynchronousAveragingOptimizer semantics (sum, /np,
    alpha-blend), buckets pipelined."""
    from kungfu_amd import ops
    from kungfu_amd.collective import GradBuckets
    sizes = _models()["bert"][:201]
    ex = _exchange(exchange)
    mine = GradBuckets(sizes, torch.bfloat16, dev, world, bucket_bytes=16 << 20)
    _fill(mine, 700 + rank, dev, torch.bfloat16)
    # expected after one SMA step: the local rank-order fold of every rank's
    # variables (regenerated; fp32 accumulation, one bf16 rounding), then the
    # blend — every exchange folds bf16 that way (a2a or P2P): bit-exact
    others = []
    for r in range(world):
        gb = GradBuckets(sizes, torch.bfloat16, dev, world, bucket_bytes=16 << 20)
        _fill(gb, 700 + r, dev, torch.bfloat16)
        others.append(gb)
    v0 = [b.clone() for b in mine.buckets]
    ex.sma_(mine.buckets, alpha)
    ok = True
    for i, b in enumerate(mine.buckets):
        s = ops.bucket_reduce([gb.buckets[i] for gb in others])
        want = ops.sma_blend_(v0[i].clone(), s, world, alpha)
        ok &= bool(torch.equal(b, want))
    del others, v0
    if not _agree(ok, dev):
        return {"error": "C5 not bit-exact against the rank-order bf16 fold + blend"}
    s_bytes = sum(sizes) * 2
    step_s, phase_us = _timed_phases(ex, lambda: ex.sma_(mine.buckets, alpha), steps, warmup,
                                     dev, world)
    if exchange == "p2p":
        ex.close()
    busbw = 2 * (world - 1) / world * s_bytes / step_s / 1e9
    how = {"native": "native C-ABI exchange: RCCL all-to-all -> HIP rank-order bf16 fold "
                     "(fp32 accumulation) -> RCCL all-gather -> HIP blend, all buckets in one call",
           "native_pipe": "native C-ABI exchange: RCCL all-to-all -> HIP rank-order bf16 fold "
                          "(fp32 accumulation) -> RCCL all-gather -> HIP blend, all buckets in "
                          "one call pipelined in %d groups (folds and blends on a second stream "
                          "between the groups' collectives)" % PIPE_GROUPS,
           "torch": "torch.distributed all-to-all -> HIP rank-order fold -> all-gather -> "
                    "HIP blend, pipelined",
           "p2p": "xGMI P2P pull sum, device barriers -> HIP blend"}[exchange]
    return {"workload": "C5: BERT-base 109,483,778 params bf16, SMA alpha=%.2f, %d "
                        "pipelined buckets (%s)" % (alpha, len(mine.buckets), how),
            "bytes": s_bytes, "ms_per_step": round(step_s * 1e3, 4),
            "GiBps_per_gpu": round(s_bytes / step_s / 2**30, 3),
            "busbw_GBps": round(busbw, 2),
            "frac_of_xgmi": _xgmi_frac(busbw, world),
            "phase_us": phase_us, "correct": True,
            "parity": "bf16 unpinned (DESIGN.md); bit-exact vs the local rank-order fold "
                      "+ blend"}


def _gemm_standin(dev, world, t_target):
    """A stand-in for a training step's compute: bf16 GEMMs of 4096^3 on the
    current stream, as many as take about t_target seconds (at least one).
    Returns (run(k), k, n): run(k) queues k of them."""
    n = 4096
    a = torch.randn(n, n, device=dev, dtype=torch.bfloat16)
    w = torch.randn(n, n, device=dev, dtype=torch.bfloat16) / n
    t_mm = _timed(lambda: torch.mm(a, w), 20, 3, dev, world)

    def run(k):
        x = a
        for _ in range(k):
            x = torch.mm(x, w)
        return x
    return run, max(1, int(round(t_target / t_mm))), n


def bench_c4_overlap(world, rank, dev, steps, warmup):
    """C4's S-SGD exchange overlapped with backward, as
    SynchronousSGDOptimizer(overlap=True) runs it: a stand-in for backward
    (bf16 GEMMs, about the exchange's own time in all) produces the 16
    ResNet-50 buckets last to first, and each bucket's exchange starts on the
    exchange's own stream as soon as its share of the compute is queued
    (NativeExchange.start_); the step then waits for all. Against the serial
    step (the whole compute, then one all_reduce_ of the 16 buckets)."""
    from kungfu_amd import ops
    from kungfu_amd.collective import GradBuckets
    ex = _exchange("native")
    sizes = _models()["resnet50-imagenet"]
    gbs = [GradBuckets(sizes, torch.float32, dev, world, n_buckets=16) for _ in range(world)]
    for r, gb in enumerate(gbs):
        _fill(gb, 500 + r, dev, torch.float32)
    mine = gbs[rank]
    nb = len(mine.buckets)
    want = [ops.bucket_reduce_avg([gb.buckets[i] for gb in gbs], world) for i in range(nb)]
    absums = [sum(gb.buckets[i].abs() for gb in gbs) for i in range(nb)]

    def start_all(work=None, k=0):
        hs = []
        for i in reversed(range(nb)):  # backward produces the last bucket first
            if work is not None:
                work(k * (i + 1) // nb - k * i // nb)
            hs.append(ex.start_([mine.buckets[i]], average=True, coalesce=False, key=i))
        for h in hs:
            h.wait()

    start_all()
    ok = True
    for b, w, ab, sp in zip(mine.buckets, want, absums, mine.spans):
        ok &= (bool(torch.equal(b[:sp], w[:sp])) if world <= 2 else _within(b[:sp], w[:sp],
                                                                          ab[:sp], world))
    del want, absums
    gbs.clear()
    if not _agree(ok, dev):
        return {"error": "overlapped C4 exchange failed its parity check"}
    t_x = _timed(lambda: ex.all_reduce_(mine.buckets, average=True), steps, warmup, dev, world)
    work, k, n = _gemm_standin(dev, world, t_x)
    t_c = _timed(lambda: work(k), steps, warmup, dev, world)

    def serial():
        work(k)
        ex.all_reduce_(mine.buckets, average=True)

    t_s = _timed(serial, steps, warmup, dev, world)
    t_o = _timed(lambda: start_all(work, k), steps, warmup, dev, world)
    hidden = (t_s - t_o) / min(t_c, t_x) if min(t_c, t_x) > 0 else None
    return {"workload": "C4: ResNet-50 grads in %d buckets, S-SGD, each bucket's exchange started "
                        "as a backward stand-in (%d bf16 GEMMs of %d^3 in all) produces it "
                        "(SynchronousSGDOptimizer(overlap=True)) vs serial" % (nb, k, n),
            "exchange_ms": round(t_x * 1e3, 4), "compute_ms": round(t_c * 1e3, 4),
            "serial_ms": round(t_s * 1e3, 4), "overlapped_ms": round(t_o * 1e3, 4),
            "ms_per_step": round(t_o * 1e3, 4),
            "hidden_frac": round(hidden, 3) if hidden is not None else None,
            "parity": "N=2 bit-exact / N>2 order bound vs the rank-order average",
            "correct": True}


def bench_c5_overlap(world, rank, dev, steps, warmup, alpha=0.1):
    """C5's SMA exchange overlapped with compute, as
    SynchronousAveragingOptimizer(overlap=True) runs it: the sum of the
    variables starts on the exchange's own stream (NativeExchange.start_into_,
    out of place), a stand-in for the step's forward and backward (bf16 GEMMs sized
    to about the exchange's own time) runs on the current stream meanwhile,
    then the step waits and blends (the batched HIP kernel). Against the
    serial step (compute, then the synchronous sma_). Checked first: the
    overlapped blend equals the synchronous one bit for bit."""
    from kungfu_amd import ops
    from kungfu_amd.collective import GradBuckets
    ex = _exchange("native")
    sizes = _models()["bert"][:201]
    mine = GradBuckets(sizes, torch.bfloat16, dev, world, bucket_bytes=16 << 20)
    _fill(mine, 700 + rank, dev, torch.bfloat16)
    sums = [torch.empty_like(b) for b in mine.buckets]
    v0 = [b.clone() for b in mine.buckets]

    def start():  # out of place, as the optimizer does on the native exchange
        return ex.start_into_(mine.buckets, sums, op="sum")

    def finish(h):
        h.wait()
        ops.sma_blend_batch_(mine.buckets, sums, world, alpha)

    finish(start())
    over = [b.clone() for b in mine.buckets]
    for b, v in zip(mine.buckets, v0):
        b.copy_(v)
    ex.sma_(mine.buckets, alpha)
    ok = all(torch.equal(a, b) for a, b in zip(over, mine.buckets))
    del over, v0
    if not _agree(ok, dev):
        return {"error": "overlapped SMA differs from the synchronous sma_"}
    t_x = _timed(lambda: ex.sma_(mine.buckets, alpha), steps, warmup, dev, world)
    work, k, n = _gemm_standin(dev, world, t_x)

    def compute():
        return work(k)

    t_c = _timed(compute, steps, warmup, dev, world)

    def serial():
        compute()
        ex.sma_(mine.buckets, alpha)

    def overlapped():
        h = start()
        compute()
        finish(h)

    t_s = _timed(serial, steps, warmup, dev, world)
    t_o = _timed(overlapped, steps, warmup, dev, world)
    hidden = (t_s - t_o) / min(t_c, t_x) if min(t_c, t_x) > 0 else None
    return {"workload": "C5: BERT-base bf16 SMA (%d buckets) beside %d bf16 GEMMs of %d^3 on the "
                        "current stream, overlapped (the sum on the exchange's stream, "
                        "SynchronousAveragingOptimizer(overlap=True)) vs serial"
                        % (len(mine.buckets), k, n),
            "exchange_ms": round(t_x * 1e3, 4), "compute_ms": round(t_c * 1e3, 4),
            "serial_ms": round(t_s * 1e3, 4), "overlapped_ms": round(t_o * 1e3, 4),
            "ms_per_step": round(t_o * 1e3, 4),
            "hidden_frac": round(hidden, 3) if hidden is not None else None,
            "parity": "overlapped blend == synchronous sma_ bit for bit",
            "correct": True}


if __name__ == "__main__":
    sys.exit(main())
