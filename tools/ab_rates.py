#!/usr/bin/env python3
"""A/B of kf_bucket_reduce between builds of libkungfu_amd.so, interleaved in
ONE process (same box, same buffers, same clocks): for each k, launches cycle
over 3 independent input sets (cold Infinity Cache), HIP events around 20
launches, 7 rounds alternating the libraries, median.

  python tools/ab_rates.py A.so B.so [--k 3,4,8] [--dtype f32]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

PEAK = 8000.0
CODES = {"f32": (0x20408, torch.float32), "bf16": (0x20209, torch.bfloat16),
         "f16": (0x20208, torch.float16), "i32": (0x10408, torch.int32),
         "i8": (0x10108, torch.int8), "u8": (0x00108, torch.uint8)}
OPS = {"sum": 0, "min": 1, "max": 2, "prod": 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--k", default="3,4,8")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--op", default="sum", choices=sorted(OPS))
    a = ap.parse_args()
    libs = []
    for p in a.libs:
        l = ctypes.CDLL(os.path.abspath(p))
        l.kf_bucket_reduce.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p]
        libs.append(l)
    code, tdt = CODES[a.dtype]
    op = OPS[a.op]
    lo, hi = (0, 256) if tdt == torch.uint8 else (-128, 128) if tdt == torch.int8 else (-1000, 1000)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    esz = torch.tensor([], dtype=tdt).element_size()
    n = (a.mib << 20) // esz
    for k in [int(x) for x in a.k.split(",")]:
        sets = []
        for _ in range(3):
            ins = [torch.randn(n, device=dev).to(tdt) if tdt.is_floating_point
                   else torch.randint(lo, hi, (n,), device=dev, dtype=tdt)
                   for _ in range(k)]
            out = torch.empty_like(ins[0])
            arr = (ctypes.c_void_p * k)(*[t.data_ptr() for t in ins])
            sets.append((arr, out, ins))
        results = [[] for _ in libs]
        outs = []
        for li, l in enumerate(libs):  # same answer from every build
            l.kf_bucket_reduce(sets[0][0], k, sets[0][1].data_ptr(), n, code, op, s.cuda_stream)
            torch.cuda.synchronize()
            outs.append(sets[0][1].clone())
        same = all(torch.equal(outs[0], o) for o in outs[1:])
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for li, l in enumerate(libs):
                for i in range(3):
                    arr, out, _ = sets[i % 3]
                    l.kf_bucket_reduce(arr, k, out.data_ptr(), n, code, op, s.cuda_stream)
                e0.record(s)
                for i in range(20):
                    arr, out, _ = sets[i % 3]
                    l.kf_bucket_reduce(arr, k, out.data_ptr(), n, code, op, s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                results[li].append(e0.elapsed_time(e1) * 1e3 / 20)
        algo = (k + 1) * n * esz
        for li, p in enumerate(a.libs):
            us = statistics.median(results[li])
            print(json.dumps({"lib": os.path.basename(p), "k": k, "dtype": a.dtype, "op": a.op,
                              "us": round(us, 2), "GBps": round(algo / us / 1e3, 1),
                              "frac": round(algo / us / 1e3 / PEAK, 4), "same_result": same}))
        sys.stdout.flush()
        del sets


if __name__ == "__main__":
    main()
