#!/usr/bin/env python3
"""The product's k-input fold (kf_bucket_reduce, fp32 SUM) across bucket
sizes, after its schedule became size-dependent (batched loads below 2048
blocks, one vector in flight from 2048, the residency cap from 8192; see
kSerialMinBlocks in kf_capi.hip): k = 3, 4, 8 at 1 MiB .. 256 MiB per input,
3 rotating sets, HIP events around 20 launches, median of 5.

  python tools/fold_size_sweep.py > profiles/r02/fold_size_sweep.jsonl
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for mib in (1, 4, 16, 32, 64, 128, 256):
        n = mib << 18
        for k in (3, 4, 8):
            sets = []
            for _ in range(3):
                ins = [torch.randn(n, device=dev) for _ in range(k)]
                sets.append((_lib.ptr_array([t.data_ptr() for t in ins]), torch.empty(n, device=dev),
                             ins))
            ts = []
            for _ in range(5):
                e0.record()
                for i in range(20):
                    p, o, _ = sets[i % 3]
                    lib.kf_bucket_reduce(p, k, o.data_ptr(), n, 0x20408, 0, s)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 20)
            want = sets[2][2][0].clone()
            for t in sets[2][2][1:]:
                want += t
            us = statistics.median(ts)
            print(json.dumps({"mib_per_input": mib, "k": k, "blocks": n // 4096, "us": round(us, 2),
                              "frac": round((k + 1) * 4 * n / us / 8e6, 4),
                              "correct": bool(torch.equal(sets[2][1], want))}), flush=True)
            del sets, want
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
