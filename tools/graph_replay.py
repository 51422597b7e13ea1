#!/usr/bin/env python3
"""Launch-bound per-bucket epilogues, four ways: the shard /np of C3 at N = 8
(64 buckets of 4 MiB -> 64 shards of 512 KiB) and of N = 64 (64 KiB shards),
as 64 kf_bucket_div launches, as kf_bucket_reduce_batch (16 shards per
launch), and each of those captured once in a HIP graph and replayed
(torch.cuda.CUDAGraph). Time per step from HIP events over 50 steps, median
of 5; every variant checked against the eager result.

  python tools/graph_replay.py > profiles/r02/graph_replay.jsonl
"""
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    for shard_kib in (512, 64):
        n = shard_kib * 1024 // 4
        base = [torch.randn(n, device=dev) for _ in range(64)]
        shards = [b.clone() for b in base]
        ptrs = _lib.ptr_array([t.data_ptr() for t in shards])
        counts = (ctypes.c_size_t * 64)(*[n] * 64)

        def per_bucket(s):
            for t in shards:
                lib.kf_bucket_div(t.data_ptr(), n, 0x20408, 8, s.cuda_stream)

        def batched(s):
            lib.kf_bucket_reduce_batch(ptrs, 1, ptrs, counts, 64, 0x20408, 0, 8, s.cuda_stream)

        def reset():
            for t, b in zip(shards, base):
                t.copy_(b)

        reset()
        per_bucket(torch.cuda.current_stream())
        torch.cuda.synchronize()
        want = [t.clone() for t in shards]
        rows = []
        for name, fn in (("per_bucket", per_bucket), ("batched", batched)):
            for graphed in (False, True):
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                if graphed:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.stream(s):
                        with torch.cuda.graph(g, stream=s):
                            fn(s)
                    run = g.replay
                else:
                    def run(fn=fn, s=s):
                        fn(s)
                torch.cuda.synchronize()
                reset()
                torch.cuda.synchronize()
                with torch.cuda.stream(s):
                    run()
                torch.cuda.synchronize()
                ok = all(torch.equal(a, b) for a, b in zip(shards, want))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ts = []
                for _ in range(5):
                    with torch.cuda.stream(s):
                        e0.record(s)
                        for _ in range(50):
                            run()
                        e1.record(s)
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3 / 50)
                us = statistics.median(ts)
                algo = 2 * 64 * n * 4
                rows.append({"shard_KiB": shard_kib, "shards": 64, "variant": name,
                             "graph": graphed, "us_per_step": round(us, 2),
                             "frac": round(algo / us / 1e3 / 8000.0, 4), "correct": ok})
        for r in rows:
            print(json.dumps(r), flush=True)
        del base, shards, want
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
