"""Probe: can two ranks on ONE GPU form an RCCL communicator through the native
exchange (kf_exchange_create)? NCCL/RCCL normally refuse a duplicate GPU; if
this RCCL allows it, run the world-2 native exchange against the rank-order
fold. Run: torchrun --nproc-per-node 2 tools/native_same_gpu_probe.py"""
import json
import os
import sys
import threading

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from kungfu_amd import ops
    from kungfu_amd.exchange import NativeExchange
    uid = NativeExchange.shared_id()
    box = {}

    def make():
        try:
            box["ex"] = NativeExchange(algo="rs", device=dev, uid=uid)
        except Exception as e:
            box["err"] = repr(e)[:400]

    th = threading.Thread(target=make, daemon=True)
    th.start()
    th.join(60)
    res = {"rank": rank, "created": "ex" in box, "error": box.get("err")}
    if "ex" in box:
        ex = box["ex"]
        out = {}
        for algo in ("rs", "a2a"):
            ex.algo = algo
            n = (1 << 22) + 3
            xs = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(r))
                  for r in range(world)]
            b = xs[rank].clone()
            ex.all_reduce_([b], average=True)
            torch.cuda.synchronize()
            out[algo] = bool(torch.equal(b, ops.bucket_reduce_avg(xs, world)))
        res["bit_exact"] = out
    print(json.dumps(res), flush=True)
    os._exit(0)


if __name__ == "__main__":
    main()
