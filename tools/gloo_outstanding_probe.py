"""Probe for the N=4 same-GPU gloo stall of C3's per-bucket exchange
(profiles/r01/rehearsal_n4_same_gpu_watchdog.json, profiles/r02/): 64 buckets
of 1 MiB, reduce_scatter_tensor(async) issued in windows of k outstanding
works, k = 1, 2, 4, 8, 64, first on CPU tensors, then on cuda:0 tensors. Each
variant runs under a watchdog that dumps every thread's stack and exits 3.
Run: torchrun --nproc-per-node 4 tools/gloo_outstanding_probe.py"""
import faulthandler
import os
import sys
import threading
import time

import torch
import torch.distributed as dist


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    nb, n = 64, 1 << 18  # 64 buckets of 1 MiB fp32
    for devname in ("cpu", "cuda:0"):
        dev = torch.device(devname)
        bufs = [torch.randn(n, device=dev) for _ in range(nb)]
        outs = [torch.empty(n // world, device=dev) for _ in range(nb)]
        for k in (1, 2, 4, 8, 64):
            tag = "%s k=%d" % (devname, k)
            dog = threading.Timer(40.0, _stuck, (rank, tag))
            dog.daemon = True
            dog.start()
            dist.barrier()
            t0 = time.perf_counter()
            for i in range(0, nb, k):
                ws = [dist.reduce_scatter_tensor(outs[j], bufs[j], async_op=True)
                      for j in range(i, min(nb, i + k))]
                for w in ws:
                    w.wait()
            if devname != "cpu":
                torch.cuda.synchronize()
            dist.barrier()
            dog.cancel()
            if rank == 0:
                print("[probe] %s: 64 reduce-scatters in %.1f ms" %
                      (tag, (time.perf_counter() - t0) * 1e3), file=sys.stderr, flush=True)
    if rank == 0:
        print("[probe] all variants finished", file=sys.stderr, flush=True)
    dist.destroy_process_group()


def _stuck(rank, tag):
    print("[probe] rank %d stuck in %s; stacks:" % (rank, tag), file=sys.stderr, flush=True)
    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
    sys.stderr.flush()
    os._exit(3)


if __name__ == "__main__":
    main()
