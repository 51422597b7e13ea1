"""BASELINE.json's multi-GPU configs at FULL size through the HIP path, with
ranks as processes sharing cuda:0 (HIP IPC and gloo both work between
processes on one device; RCCL refuses two ranks on one GPU, so its own
transport runs in bench.py on the driver's node), checked against the oracle.

  C3  64 x 4 MiB fp32 buckets (256 MiB), S-SGD (sum, / np), world 2:
      the xGMI P2P exchange (rank-order fold from the peers' HBM, fused /np)
      and the RCCL-shaped path (gloo moving GPU tensors: reduce-scatter ->
      HIP /np -> all-gather, and all-to-all -> HIP rank-order fold ->
      all-gather), every one bit-exact against oracle.reduce_avg.
  C4  ResNet-50's 214 gradients (25,583,592 fp32) in 16 buckets, world 2
      and 4: P2P and all-to-all + fold, bit-exact (rank order) at both worlds.
  C5  BERT-base (first 201 tensors, 109,483,778 params) in bf16, SMA with
      alpha = 0.1, world 2: P2P and all-to-all + fold give the same bits as
      the oracle's fp32-accumulated rank-order sum followed by the blend.

Inputs are N(0,1) from per-rank seeds; every rank regenerates all ranks'
inputs to build the expected values (reference semantics: sync_sgd.py:103-104,
sma_sgd.py:60-65; shapes: tests/go/fakemodel/resnet50-imagenet.go, bert.go)."""
import json
import os
import sys
import traceback

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
from procs import hung_msg, join_all

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.gpu


def _models():
    with open(os.path.join(HERE, "golden", "models.json")) as f:
        return json.load(f)


def _run(target, world, *args):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    ps = [ctx.Process(target=target, args=(r, world, port, errq) + args) for r in range(world)]
    for p in ps:
        p.start()
    hung = join_all(ps, 600)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


def _init(rank, world, port):
    sys.path[:0] = [ROOT, HERE]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _fill(gb, seed, dev, dtype):
    """Every tensor view of `gb` from one generator, in order (bench.py _fill)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    for v in gb.views:
        v.copy_(torch.randn(v.numel(), device=dev, generator=g).to(dtype))


def _host(t):
    t = t.cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def _c3_body(rank, world, port, errq):
    try:
        dist = _init(rank, world, port)
        from kungfu_amd.collective import Exchange, GradBuckets
        from kungfu_amd.p2p import P2PExchange
        from oracle import oracle
        dev = torch.device("cuda:0")
        n = 64 << 20  # 256 MiB of fp32 per rank
        gb = GradBuckets([n], torch.float32, dev, world, n_buckets=64)
        assert len(gb.buckets) == 64 and all(b.numel() * 4 == 4 << 20 for b in gb.buckets)

        def gen(r, step):
            g = torch.Generator(device=dev).manual_seed(1000 * step + r)
            return torch.randn(n, device=dev, generator=g)

        def expect(step):
            return oracle.reduce_avg([gen(r, step).cpu().numpy() for r in range(world)],
                                     "f32", world)

        step = 0
        # P2P, the 64 buckets as one run and one by one
        for coalesce in (True, False):
            ex = P2PExchange(gb.buckets, coalesce=coalesce)
            assert len(ex.buckets) == (1 if coalesce else 64)
            for _ in range(2):  # fresh data: no stale shard survives a step
                gb.views[0].copy_(gen(rank, step))
                ex.all_reduce_(average=True)
                ex.finish()
                assert np.array_equal(gb.views[0].cpu().numpy(), expect(step)), (coalesce, step)
                step += 1
            ex.close()
        # RCCL's shape over gloo with GPU tensors: RS -> HIP /np -> AG (two
        # operands: bit-exact) and all-to-all -> HIP fold -> AG, per bucket
        for algo in ("rs", "a2a"):
            rex = Exchange(algo=algo)
            gb.views[0].copy_(gen(rank, step))
            rex.all_reduce_(gb.buckets, average=True, coalesce=False)
            torch.cuda.synchronize()
            assert np.array_equal(gb.views[0].cpu().numpy(), expect(step)), algo
            step += 1
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def test_c3_full_size_world2():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(_c3_body, 2)


def _c4_body(rank, world, port, errq):
    try:
        dist = _init(rank, world, port)
        from kungfu_amd.collective import Exchange, GradBuckets
        from kungfu_amd.p2p import PeerExchange
        from oracle import oracle
        dev = torch.device("cuda:0")
        sizes = _models()["resnet50-imagenet"]
        assert len(sizes) == 214 and sum(sizes) == 25583592
        for name, ex in (("p2p", PeerExchange()), ("a2a", Exchange(algo="a2a"))):
            seed = 500 if name == "p2p" else 600
            gbs = [GradBuckets(sizes, torch.float32, dev, world, n_buckets=16)
                   for _ in range(world)]
            for r, gb in enumerate(gbs):
                _fill(gb, seed + r, dev, torch.float32)
            want = [oracle.reduce_avg([gb.buckets[j].cpu().numpy() for gb in gbs], "f32", world)
                    for j in range(16)]
            mine = gbs[rank]
            assert len(mine.buckets) == 16
            ex.all_reduce_(mine.buckets, average=True)
            if hasattr(ex, "finish"):
                ex.finish()
            torch.cuda.synchronize()
            for j, (b, sp) in enumerate(zip(mine.buckets, mine.spans)):
                assert np.array_equal(b[:sp].cpu().numpy(), want[j][:sp]), (name, j)
            if name == "p2p":
                ex.close()
            del gbs
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 4])
def test_c4_resnet50_16_buckets(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(_c4_body, world)


def _c5_body(rank, world, port, errq):
    try:
        dist = _init(rank, world, port)
        from kungfu_amd.collective import Exchange, GradBuckets
        from kungfu_amd.p2p import PeerExchange
        from oracle import oracle
        dev = torch.device("cuda:0")
        sizes = _models()["bert"][:201]
        assert sum(sizes) == 109483778
        alpha = 0.1
        results = {}
        for name, ex in (("p2p", PeerExchange()), ("rccl", Exchange())):
            gbs = [GradBuckets(sizes, torch.bfloat16, dev, world, bucket_bytes=16 << 20)
                   for _ in range(world)]
            for r, gb in enumerate(gbs):
                _fill(gb, 700 + r, dev, torch.bfloat16)
            mine = gbs[rank]
            before = [_host(b) for b in mine.buckets]
            sums = [oracle.reduce_k([_host(gb.buckets[j]) for gb in gbs], "bf16", "sum")
                    for j in range(len(mine.buckets))]
            ex.sma_(mine.buckets, alpha)
            if hasattr(ex, "finish"):
                ex.finish()
            torch.cuda.synchronize()
            got = [_host(b) for b in mine.buckets]
            for j in range(len(got)):
                want = oracle.sma_blend(before[j], sums[j], "bf16", world, alpha)
                assert np.array_equal(got[j], want), (name, j)
            results[name] = got
            if name == "p2p":
                ex.close()
            del gbs
        # transport-independent bits
        assert all(np.array_equal(a, b) for a, b in zip(results["p2p"], results["rccl"]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def test_c5_bert_bf16_sma_world2():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(_c5_body, 2)
