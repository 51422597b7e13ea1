#!/usr/bin/env python3
"""The one-input streaming kernels (the shard /np in place, the SMA blend
f32 and bf16) with the k <= 2 occupancy cap off and at 24 / 32 KiB
(kf_set_occupancy), same buffers, settings alternated over 15 rounds of 20
launches over 3 rotating sets. (The C2 sum showed no gain,
ab_c2_occupancy.jsonl; one earlier sample had the /np at +1.7 %.)

  python tools/ab_k1_occupancy.py > profiles/r02/ab_k1_occupancy.jsonl
"""
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

F32, BF16 = 0x20408, 0x20209


def main():
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    n = 64 << 20
    xs = [torch.randn(n, device=dev) for _ in range(3)]
    sv = [(torch.randn(n, device=dev), torch.randn(n, device=dev)) for _ in range(3)]
    bv = [(torch.randn(2 * n, device=dev).to(torch.bfloat16),
           torch.randn(2 * n, device=dev).to(torch.bfloat16)) for _ in range(3)]
    fams = {
        "div_np8_f32": (lambda i: lib.kf_bucket_div(xs[i].data_ptr(), n, F32, 8, s), 8 * n),
        "sma_f32": (lambda i: lib.kf_sma_blend(sv[i][0].data_ptr(), sv[i][1].data_ptr(), n, F32, 8,
                                               ctypes.c_double(0.1), s), 12 * n),
        "sma_bf16": (lambda i: lib.kf_sma_blend(bv[i][0].data_ptr(), bv[i][1].data_ptr(), 2 * n, BF16,
                                                8, ctypes.c_double(0.1), s), 12 * n),
    }
    settings = {"none": 0, "lds24K": 24 << 10, "lds32K": 32 << 10}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = {(f, c): [] for f in fams for c in settings}
    wins = {(f, c): 0 for f in fams for c in settings}
    for r in range(15):
        for f, (fn, _) in fams.items():
            order = list(settings.items())
            if r % 2:
                order.reverse()
            rnd = {}
            for c, lds in order:
                lib.kf_set_occupancy(lds, 32 << 10)
                fn(0)
                e0.record()
                for i in range(20):
                    fn(i % 3)
                e1.record()
                torch.cuda.synchronize()
                rnd[c] = e0.elapsed_time(e1) * 1e3 / 20
                ts[(f, c)].append(rnd[c])
            wins[(f, min(rnd, key=rnd.get))] += 1
    lib.kf_set_occupancy(0, 32 << 10)
    for (f, c), t in ts.items():
        us = statistics.median(t)
        print(json.dumps({"family": f, "setting": c, "us": round(us, 2), "min_us": round(min(t), 2),
                          "frac": round(fams[f][1] / us / 8e6, 4), "round_wins": wins[(f, c)],
                          "rounds": len(t)}), flush=True)


if __name__ == "__main__":
    main()
