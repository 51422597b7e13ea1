#!/usr/bin/env python3
"""C2 (k = 2 fp32 sum, 256 MiB, the bench's 3 rotating sets) with the k <= 2
occupancy cap off and at 32 / 48 KiB (kf_set_occupancy), same buffers,
settings alternated over 21 rounds of 20 launches: is the small gain seen in
the probes real for the headline kernel?

  python tools/ab_c2_occupancy.py > profiles/r02/ab_c2_occupancy.jsonl
"""
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
    s = torch.cuda.current_stream().cuda_stream
    n = 64 << 20
    sets = []
    for j in range(3):
        x, y = torch.randn(n, device=dev), torch.randn(n, device=dev)
        sets.append((_lib.ptr_array([x.data_ptr(), y.data_ptr()]), torch.empty_like(x), x, y))
    settings = {"none": 0, "lds32K": 32 << 10, "lds48K": 48 << 10}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = {c: [] for c in settings}
    wins = {c: 0 for c in settings}
    for r in range(21):
        order = list(settings.items())
        if r % 2:
            order.reverse()
        rnd = {}
        for c, lds in order:
            lib.kf_set_occupancy(lds, 48 << 10)
            lib.kf_bucket_reduce(sets[0][0], 2, sets[0][1].data_ptr(), n, 0x20408, 0, s)
            e0.record()
            for i in range(20):
                p, o = sets[i % 3][:2]
                lib.kf_bucket_reduce(p, 2, o.data_ptr(), n, 0x20408, 0, s)
            e1.record()
            torch.cuda.synchronize()
            rnd[c] = e0.elapsed_time(e1) * 1e3 / 20
            ts[c].append(rnd[c])
        wins[min(rnd, key=rnd.get)] += 1
    lib.kf_set_occupancy(0, 32 << 10)
    ok = all(torch.equal(o, x + y) for _, o, x, y in sets)
    for c, t in ts.items():
        us = statistics.median(t)
        print(json.dumps({"setting": c, "us": round(us, 2), "min_us": round(min(t), 2),
                          "frac": round(12 * n / us / 8e6, 4), "round_wins": wins[c],
                          "rounds": len(t), "correct": ok}), flush=True)


if __name__ == "__main__":
    main()
