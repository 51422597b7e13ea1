#!/usr/bin/env python3
"""Achieved HBM rate of every kernel family behind the C ABI, against the
8 TB/s roofline. Each sample: HIP events around 20 launches cycling over 3
independent buffer sets (cold Infinity Cache, as bench.py), median of 5.

  python tools/kernel_rates.py > profiles/r01/kernel_rates.jsonl
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

PEAK = 8000.0
BYTES = 256 << 20  # per input buffer


def timeit(fn, sets, launches=20, rounds=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        fn(*sets[i % len(sets)])
    ts = []
    for _ in range(rounds):
        e0.record()
        for i in range(launches):
            fn(*sets[i % len(sets)])
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / launches)
    return statistics.median(ts)


def main():
    from kungfu_amd import _lib, ops
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    rows = []

    def report(name, algo_bytes, us, **kw):
        gbps = algo_bytes / us / 1e3
        rows.append(dict(kernel=name, us=round(us, 2), algorithmic_bytes=algo_bytes,
                         GBps=round(gbps, 1), frac=round(gbps / PEAK, 4), **kw))

    n = BYTES // 4
    for k in (2, 4, 8):  # the P2P fold kernel (all loads in flight) on local HBM
        sets = []
        for _ in range(3):
            ins = [torch.randn(n, device=dev) for _ in range(k)]
            out = torch.empty_like(ins[0])
            sets.append((_lib.ptr_array([t.data_ptr() for t in ins]), out, ins))

        def run_p(ptrs, out, ins, k=k):
            lib.kf_bucket_reduce_peers(ptrs, k, out.data_ptr(), out.numel(), 0x20408, 0, k, s)
        report("reduce_peers avg k=%d (P2P fold, local HBM)" % k, (k + 1) * BYTES,
               timeit(run_p, sets), dtype="torch.float32")
        del sets
        torch.cuda.empty_cache()
    if "--peers-only" in sys.argv:
        for r in rows:
            print(json.dumps(r))
        return
    for dtype, code in ((torch.float32, 0x20408), (torch.float16, 0x20208),
                        (torch.bfloat16, 0x20209), (torch.float64, 0x20808),
                        (torch.int32, 0x10408), (torch.int8, 0x10108)):
        esz = torch.empty((), dtype=dtype).element_size()
        n = BYTES // esz
        for k in (2, 4, 8):
            sets = []
            for _ in range(3):
                ins = [torch.randn(n, device=dev).to(dtype) if dtype.is_floating_point
                       else torch.randint(-100, 100, (n,), device=dev, dtype=dtype)
                       for _ in range(k)]
                out = torch.empty_like(ins[0])
                sets.append((_lib.ptr_array([t.data_ptr() for t in ins]), out, ins))

            def run(ptrs, out, ins, k=k, code=code):
                lib.kf_bucket_reduce(ptrs, k, out.data_ptr(), out.numel(), code, 0, s)
            us = timeit(run, sets)
            report("reduce SUM k=%d" % k, (k + 1) * BYTES, us, dtype=str(dtype))
            del sets
            torch.cuda.empty_cache()
    n = BYTES // 4
    sets = [(torch.randn(n, device=dev),) for _ in range(3)]
    report("div_ (S-SGD shard epilogue) f32", 2 * BYTES,
           timeit(lambda x: ops.bucket_div_(x, 8), sets), dtype="torch.float32")
    sets = [(torch.randn(n, device=dev), torch.randn(n, device=dev), torch.randn(n, device=dev))
            for _ in range(3)]
    report("reduce_avg k=2 f32 (fused /np, np=3: IEEE division)", 3 * BYTES,
           timeit(lambda a, b, c: ops.bucket_reduce_avg([a, b], 3, out=c), sets),
           dtype="torch.float32")
    report("reduce_avg k=2 f32 (fused /np, np=2: exact multiply)", 3 * BYTES,
           timeit(lambda a, b, c: ops.bucket_reduce_avg([a, b], 2, out=c), sets),
           dtype="torch.float32")
    sets = [(torch.randn(n, device=dev), torch.randn(n, device=dev)) for _ in range(3)]
    report("sma_blend f32", 3 * BYTES,
           timeit(lambda v, sm: ops.sma_blend_(v, sm, 8, 0.1), sets), dtype="torch.float32")
    nb = BYTES // 2
    sets = [(torch.randn(nb, device=dev).bfloat16(), torch.randn(nb, device=dev).bfloat16())
            for _ in range(3)]
    report("sma_blend bf16", 3 * BYTES,
           timeit(lambda v, sm: ops.sma_blend_(v, sm, 8, 0.1), sets), dtype="torch.bfloat16")
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
