#!/usr/bin/env python3
"""Does writing the fold's result over one of its inputs (the reference's
recvOnto is in place: RecvBuf = RecvBuf + received, session.go:255-264) change
the k-input fold's rate? Same buffers for every variant (placement moves a
streaming kernel by up to 5 %): out-of-place (a separate output), in place
over input 0, in place over input k-1; k = 2, 4, 8, 256 MiB fp32 per stream,
3 rotating sets, rounds interleaved, median of 7 x 10 launches.

  python tools/ab_inplace.py > profiles/r02/ab_inplace.jsonl
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k in (2, 4, 8):
        sets = []
        for _ in range(3):
            ins = [torch.randn(n, device=dev) for _ in range(k)]
            sets.append((ins, torch.empty_like(ins[0]), _lib.ptr_array([t.data_ptr() for t in ins])))
        outs = {"out_of_place": lambda st: st[1], "in_place_0": lambda st: st[0][0],
                "in_place_last": lambda st: st[0][-1]}
        ts = {v: [] for v in outs}
        for _ in range(7):
            for v, pick in outs.items():
                assert lib.kf_bucket_reduce(sets[0][2], k, pick(sets[0]).data_ptr(), n, 0x20408, 0, s) == 0
                e0.record()
                for i in range(10):
                    st = sets[i % 3]
                    lib.kf_bucket_reduce(st[2], k, pick(st).data_ptr(), n, 0x20408, 0, s)
                e1.record()
                torch.cuda.synchronize()
                ts[v].append(e0.elapsed_time(e1) * 1e3 / 10)
        # correctness of the in-place fold on fresh data (left fold in input order)
        ins = [torch.randn(n, device=dev) for _ in range(k)]
        want = ins[0].clone()
        for t in ins[1:]:
            want = want + t
        assert lib.kf_bucket_reduce(_lib.ptr_array([t.data_ptr() for t in ins]), k,
                                    ins[0].data_ptr(), n, 0x20408, 0, s) == 0
        torch.cuda.synchronize()
        ok = bool(torch.equal(ins[0], want))
        for v, t in ts.items():
            us = statistics.median(t)
            print(json.dumps({"k": k, "variant": v, "us": round(us, 2), "min_us": round(min(t), 2),
                              "frac": round((k + 1) * 4 * n / us / 8e6, 4),
                              "in_place_correct": ok}), flush=True)
        del sets, ins, want
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
