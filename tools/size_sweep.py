#!/usr/bin/env python3
"""C2's kernel (fp32 z = x + y through kf_bucket_reduce) over bucket sizes
from 64 KiB to 1 GiB: where the launch stops dominating and where HBM takes
over. Launches cycle over enough independent bucket sets that together they
exceed 1 GiB (4x the 256 MiB Infinity Cache), so no size is timed out of the
cache; HIP events around 50 back-to-back launches, median of 5.

  python tools/size_sweep.py > profiles/r01/size_sweep.jsonl
  python tools/size_sweep.py --batch 16 > profiles/r02/size_sweep_batch16.jsonl

--batch B: each timed launch is ONE kf_bucket_reduce_batch over B independent
buckets of that size (the multi-bucket launch the exchanges use for their
per-bucket epilogues), against B separate kf_bucket_reduce launches of the
same buckets, interleaved in one process. --div: the shard epilogue instead
(k = 1, x /= np in place), as kf_exchange issues it after a reduce-scatter.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

PEAK = 8000.0


def batch_main(nb, div):
    import ctypes
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    k, np_ = (1, 2) if div else (2, 0)
    for kib in (256, 1024, 2048, 4096, 16384):
        nbytes = kib << 10
        n = nbytes // 4
        per_set = nb * (k + (0 if div else 1)) * nbytes
        nsets = max(2, -(-(1 << 30) // per_set))
        sets = []
        for _ in range(nsets):
            ts = [[torch.randn(n, device=dev) for _ in range(k)] for _ in range(nb)]
            outs = [t[0] if div else torch.empty(n, device=dev) for t in ts]
            ins = _lib.ptr_array([t.data_ptr() for row in ts for t in row])
            op = _lib.ptr_array([o.data_ptr() for o in outs])
            singles = [(_lib.ptr_array([t.data_ptr() for t in row]), o.data_ptr())
                       for row, o in zip(ts, outs)]
            sets.append((ins, op, singles, ts, outs))
        cnts = (ctypes.c_size_t * nb)(*([n] * nb))

        def batched(i):
            ins, op = sets[i % nsets][:2]
            return lib.kf_bucket_reduce_batch(ins, k, op, cnts, nb, 0x20408, 0, np_, s)

        def single(i):
            for p, o in sets[i % nsets][2]:
                if div:
                    lib.kf_bucket_div(o, n, 0x20408, np_, s)
                else:
                    lib.kf_bucket_reduce(p, k, o, n, 0x20408, 0, s)
            return 0

        res = {}
        for name, fn in (("batch", batched), ("single", single)) * 2:
            assert fn(0) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            tms = []
            for _ in range(5):
                e0.record()
                for i in range(reps):
                    fn(i)
                e1.record()
                torch.cuda.synchronize()
                tms.append(e0.elapsed_time(e1) * 1e3 / reps)
            res[name] = statistics.median(tms)
        traffic = nb * (k + 1) * nbytes
        ok = True
        if not div:  # sets 0..reps-1 were written (both forms write x + y)
            ok = all(bool(torch.equal(o, a + b)) for st in sets[:20]
                     for (a, b), o in zip(st[3], st[4]))
        print(json.dumps({"bucket_KiB": kib, "buckets": nb, "kind": "div" if div else "sum k=2",
                          "sets": nsets,
                          "batch_us": round(res["batch"], 2),
                          "batch_frac": round(traffic / res["batch"] / 1e3 / PEAK, 4),
                          "single_launches_us": round(res["single"], 2),
                          "single_frac": round(traffic / res["single"] / 1e3 / PEAK, 4),
                          "correct": ok}), flush=True)
        del sets
        torch.cuda.empty_cache()


def main():
    if "--batch" in sys.argv:
        nb = int(sys.argv[sys.argv.index("--batch") + 1])
        return batch_main(nb, "--div" in sys.argv)
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for kib in (64, 256, 1024, 4096, 16384, 65536, 262144, 1048576):
        nbytes = kib << 10
        n = nbytes // 4
        nsets = max(3, -(-(1 << 30) // (3 * nbytes)))
        sets = []
        for _ in range(nsets):
            x, y, z = (torch.randn(n, device=dev) for _ in range(3))
            sets.append((_lib.ptr_array([x.data_ptr(), y.data_ptr()]), z.data_ptr(), (x, y, z)))
        launches = 50
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(nsets):
            lib.kf_bucket_reduce(sets[i][0], 2, sets[i][1], n, 0x20408, 0, s)
        ts = []
        for _ in range(5):
            e0.record()
            for i in range(launches):
                p, zp, _ = sets[i % nsets]
                lib.kf_bucket_reduce(p, 2, zp, n, 0x20408, 0, s)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / launches)
        us = statistics.median(ts)
        x, y, z = sets[0][2]
        ok = bool(torch.equal(z, x + y))
        gbps = 3 * nbytes / us / 1e3
        print(json.dumps({"bucket_KiB": kib, "sets": nsets, "us": round(us, 2),
                          "GBps": round(gbps, 1), "frac": round(gbps / PEAK, 4),
                          "bucket_GiBps": round(nbytes / us / 1e3 / 1.073741824, 1),
                          "correct": ok}), flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
