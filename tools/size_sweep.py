#!/usr/bin/env python3
"""C2's kernel (fp32 z = x + y through kf_bucket_reduce) over bucket sizes
from 64 KiB to 1 GiB: where the launch stops dominating and where HBM takes
over. Launches cycle over enough independent bucket sets that together they
exceed 1 GiB (4x the 256 MiB Infinity Cache), so no size is timed out of the
cache; HIP events around 50 back-to-back launches, median of 5.

  python tools/size_sweep.py > profiles/r01/size_sweep.jsonl
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

PEAK = 8000.0


def main():
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
