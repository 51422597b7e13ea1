#!/usr/bin/env python3
"""Sweep the launch geometry of the fp32 2-input SUM reduce on one GPU.

All variants run in ONE process, interleaved over R rounds (cdna guide §5.4
rule 24); each sample = HIP-event time of K back-to-back launches on the
launch stream over the C2 bucket (256 MiB fp32 per input, random data).
Prints one JSON line per variant (median / min µs and GB/s) sorted by median.

  python tools/tune_reduce.py [--rounds 5] [--launches 50] [--elems N]
"""
import argparse
import itertools
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--elems", type=int, default=64 << 20)
    ap.add_argument("--unroll", default="1,2,4,8")
    ap.add_argument("--grid", default="1024,2048,4096,8192,16384,65536")
    ap.add_argument("--loadnt", default="0,1")
    ap.add_argument("--stplain", default="0,1")
    ap.add_argument("--rotate", type=int, default=3,
                    help="cycle launches over this many independent (x,y,z) sets "
                         "so no launch finds its buffers in the 256 MiB Infinity Cache")
    args = ap.parse_args()

    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    sets = []
    for _ in range(args.rotate):
        x = torch.randn(args.elems, device=dev, generator=g)
        y = torch.randn(args.elems, device=dev, generator=g)
        z = torch.empty_like(x)
        sets.append((_lib.ptr_array([x.data_ptr(), y.data_ptr()]), z, x, y))
    s = torch.cuda.current_stream()
    ints = lambda v: [int(t) for t in v.split(",")]  # noqa: E731
    variants = list(itertools.product(ints(args.unroll), ints(args.grid),
                                      ints(args.loadnt), ints(args.stplain)))
    samples = {v: [] for v in variants}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(args.rounds):
        for v in variants:
            _lib.check(lib.kf_set_geometry(*v), "kf_set_geometry")
            for i in range(3):
                p, z, _, _ = sets[i % len(sets)]
                lib.kf_bucket_reduce(p, 2, z.data_ptr(), z.numel(), 0x20408, 0, s.cuda_stream)
            e0.record(s)
            for i in range(args.launches):
                p, z, _, _ = sets[i % len(sets)]
                lib.kf_bucket_reduce(p, 2, z.data_ptr(), z.numel(), 0x20408, 0, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            samples[v].append(e0.elapsed_time(e1) * 1e3 / args.launches)
            if r == 0:
                for _, z, x, y in sets:
                    assert torch.equal(z, x + y), v
                    z.zero_()
    bytes_ = 3 * args.elems * 4
    rows = []
    for v, ts in samples.items():
        med = statistics.median(ts)
        rows.append(dict(unroll=v[0], grid_cap=v[1], loadnt=v[2], stplain=v[3],
                         median_us=round(med, 2), min_us=round(min(ts), 2),
                         gbps_median=round(bytes_ / med / 1e3, 1),
                         gbps_best=round(bytes_ / min(ts) / 1e3, 1)))
    rows.sort(key=lambda d: d["median_us"])
    for d in rows:
        print(json.dumps(d))


if __name__ == "__main__":
    main()
