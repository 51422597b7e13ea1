#!/usr/bin/env python3
"""C5's SMA blend step on one GPU: BERT-base's first 201 tensors in bf16 laid
out as the bench lays them out (16 MiB buckets), blended with one
kf_sma_blend per bucket against one kf_sma_blend_batch, same buffers,
alternated over 15 rounds of 20 steps.

  python tools/ab_sma_batch.py > profiles/r02/ab_sma_batch.jsonl
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main():
    from kungfu_amd import ops
    from kungfu_amd.collective import GradBuckets
    dev = torch.device("cuda:0")
    sizes = json.load(open(os.path.join(ROOT, "tests", "golden", "models.json")))["bert"][:201]
    gb = GradBuckets(sizes, torch.bfloat16, dev, 8, bucket_bytes=16 << 20)
    vs = gb.buckets
    ss = [torch.randn(b.numel(), device=dev).to(torch.bfloat16) for b in vs]
    for v in vs:
        v.copy_(torch.randn(v.numel(), device=dev).to(torch.bfloat16))
    var = {"per_bucket": lambda: [ops.sma_blend_(v, s, 8, 0.1) for v, s in zip(vs, ss)],
           "batched": lambda: ops.sma_blend_batch_(vs, ss, 8, 0.1)}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = {k: [] for k in var}
    for r in range(15):
        for k, fn in (list(var.items()) if r % 2 == 0 else list(var.items())[::-1]):
            fn()
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) * 1e3 / 20)
    nbytes = 3 * sum(b.numel() for b in vs) * 2
    for k, t in ts.items():
        us = statistics.median(t)
        print(json.dumps({"variant": k, "buckets": len(vs), "us_per_step": round(us, 2),
                          "min_us": round(min(t), 2), "frac": round(nbytes / us / 8e6, 4)}))


if __name__ == "__main__":
    main()
