#!/usr/bin/env python3
"""bench.py's c4_overlap / c5_overlap on ONE GPU over a one-rank librccl
communicator (the test library's rccl1 transport: the exchange calls RCCL's
own reduce-scatter / all-to-all / all-gather kernels, no world-1 copy), so
the overlap of the exchange's stream with GEMMs on the current stream is
measured on real hardware before any multi-GPU node: serial vs overlapped
step, hidden_frac. Each with the exchange's side stream at default and at
high priority. One JSON line per (case, priority).

    python tools/overlap_w1.py > profiles/r03/overlap_w1.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    import bench
    from loopback import rccl1_exchange
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    for prio in (0, -1):
        ex = rccl1_exchange("auto")
        ex._side = torch.cuda.Stream(dev, priority=prio)
        bench._NATIVE["ex"] = ex
        for name, fn in (("c5_overlap", bench.bench_c5_overlap),
                         ("c4_overlap", bench.bench_c4_overlap)):
            r = fn(1, 0, dev, 20, 3)
            r.update(case=name, side_stream_priority=prio,
                     transport="one-rank librccl communicator (rccl1)")
            print(json.dumps(r), flush=True)
        bench._NATIVE.pop("ex").close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
