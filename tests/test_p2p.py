"""xGMI peer-to-peer all-reduce (kungfu_amd/p2p.py) with ranks as processes
sharing cuda:0 (HIP IPC works between processes on one device), gloo for the
barriers. The fold order is rank order, so results are bit-exact against the
oracle for every world size."""
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


def _body(rank, world, port, errq, mode, barrier="device"):
    sys.path[:0] = [ROOT, HERE]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kungfu_amd.collective import GradBuckets
        from kungfu_amd.p2p import P2PExchange
        from oracle import oracle
        dev = torch.device("cuda:0")
        sizes = [100003, 5000, 777777, 64]
        gb = GradBuckets(sizes, torch.float32, dev, world, n_buckets=4)
        ex = P2PExchange(gb.buckets, mode=mode, barrier=barrier)
        assert len(ex.buckets) == 1  # the 4 contiguous buckets run as one
        assert ex.all_local  # every rank on cuda:0: the register-shape fold
        for step in range(3):  # fresh data every step: no stale shard survives
            xs = [[np.random.default_rng(1000 * r + 100 * step + i).standard_normal(n)
                   .astype(np.float32) for i, n in enumerate(sizes)] for r in range(world)]
            for v, x in zip(gb.views, xs[rank]):
                v.copy_(torch.from_numpy(x))
            ex.all_reduce_(average=True)
            for i, v in enumerate(gb.views):
                want = oracle.reduce_avg([xs[r][i] for r in range(world)], "f32", world)
                assert np.array_equal(v.cpu().numpy(), want), (step, i)
        # int32 MAX, a second exchange on other buckets, twice (buffer reuse)
        gi = GradBuckets([4099], torch.int32, dev, world, n_buckets=3)
        ex2 = P2PExchange(gi.buckets, mode=mode, barrier=barrier, coalesce=False)
        ex2.all_local = False  # the link spreader (kf_bucket_reduce_peers), same bits
        for step in range(2):
            gi.views[0].copy_(torch.arange(4099, dtype=torch.int32, device=dev) * (rank + 1 + step))
            ex2.all_reduce_(op="max")
            assert torch.equal(gi.views[0].cpu(), torch.arange(4099, dtype=torch.int32) * (world + step))
        ex.close()
        ex2.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


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
    hung = join_all(ps, 300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


@pytest.mark.parametrize("barrier", ["device", "host"])
@pytest.mark.parametrize("mode", ["pull", "push"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_p2p_all_reduce_bit_exact(world, mode, barrier):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(_body, world, mode, barrier)


def _timeout_body(rank, world, port, errq):
    sys.path[:0] = [ROOT, HERE]
    import time
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kungfu_amd._lib import KungFuAMDError
        from kungfu_amd.collective import GradBuckets
        from kungfu_amd.p2p import P2PExchange
        dev = torch.device("cuda:0")
        gb = GradBuckets([4096], torch.float32, dev, world, n_buckets=1)
        ex = P2PExchange(gb.buckets, timeout_s=0.2)
        if rank == 0:
            # rank 1 never joins: the device barrier must give up on its own
            t0 = time.perf_counter()
            ex.all_reduce_()
            torch.cuda.synchronize()
            assert time.perf_counter() - t0 < 5.0
            assert ex.status() == 8  # KF_ERR_TIMEOUT
            with pytest.raises(KungFuAMDError):
                ex.all_reduce_()
        dist.barrier()
        ex.close()
        dist.destroy_process_group()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def test_p2p_device_barrier_times_out():
    """A peer that never arrives: the bounded wait ends, the status word says
    KF_ERR_TIMEOUT, the next call raises (no wave left spinning)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(_timeout_body, 2)


def _opt_body(rank, world, port, errq):
    """SynchronousSGDOptimizer / SynchronousAveragingOptimizer over the P2P
    exchange: rank-order sum / np (S-SGD) and the SMA blend, bit-exact
    against the same arithmetic done locally on every rank's regenerated
    gradients / variables."""
    sys.path[:0] = [ROOT, HERE]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kungfu_amd import ops
        from kungfu_amd.optimizers import (SynchronousAveragingOptimizer,
                                           SynchronousSGDOptimizer)
        from kungfu_amd.p2p import PeerExchange
        from bounds import assert_within, sgd_bound
        dev = torch.device("cuda:0")

        def model(seed):
            torch.manual_seed(seed)
            return torch.nn.Sequential(torch.nn.Linear(33, 65), torch.nn.Tanh(),
                                       torch.nn.Linear(65, 7)).to(dev)

        def loss(m, r, step):
            g = torch.Generator(device=dev).manual_seed(100 * step + r)
            return (m(torch.randn(16, 33, device=dev, generator=g)) ** 2).mean()

        for mode in ("pull", "push"):
            ex = PeerExchange(mode=mode)
            m = model(0)
            opt = SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                          named_parameters=m.named_parameters(), exchange=ex)
            for step in range(3):
                snap = [p.detach().clone() for p in m.parameters()]
                grads = []
                for r in range(world):
                    mr = model(0)
                    with torch.no_grad():
                        for a, b in zip(mr.parameters(), snap):
                            a.copy_(b)
                    loss(mr, r, step).backward()
                    grads.append([p.grad.detach().clone() for p in mr.parameters()])
                opt.zero_grad()
                loss(m, rank, step).backward()
                opt.step()
                for j, p in enumerate(m.parameters()):
                    avg = ops.bucket_reduce_avg([grads[r][j].reshape(-1)
                                                 for r in range(world)], world).view_as(p)
                    assert torch.equal(p.grad, avg), (mode, step, j)  # the exchange: exact
                    # the SGD update may round differently (FMA): its own bound only
                    assert_within(p.detach(), snap[j] - 0.1 * avg,
                                  sgd_bound(torch.zeros_like(avg, dtype=torch.float64), 0.1,
                                            snap[j], avg), "param")
                flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu()
                allf = [torch.empty_like(flat) for _ in range(world)]
                dist.all_gather(allf, flat)
                assert all(torch.equal(f, flat) for f in allf), (mode, step)
            ex.close()

        ex = PeerExchange()
        alpha = 0.1
        m = model(rank)
        allp = [[p.detach().clone() for p in model(r).parameters()] for r in range(world)]
        opt = SynchronousAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.0),
                                            alpha=alpha, exchange=ex)
        loss(m, rank, 0).backward()
        opt.step()
        for j, p in enumerate(m.parameters()):
            s = ops.bucket_reduce([allp[r][j].reshape(-1) for r in range(world)])
            want = allp[rank][j].reshape(-1).clone()
            ops.sma_blend_(want, s, world, alpha)
            assert torch.equal(p.detach().reshape(-1), want), j
        ex.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_p2p_optimizers(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(_opt_body, world)


def _auto_body(rank, world, port, errq):
    """AutoExchange on GPU buckets: RCCL's paths (gloo here) and P2P are timed
    on the first call, whose result must still be the plain all-reduce (the
    trial restores the buckets); the pick is the same on every rank, and
    bit-exact whichever it is (only same-bits candidates compete)."""
    sys.path[:0] = [ROOT, HERE]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kungfu_amd import ops
        from kungfu_amd.collective import GradBuckets
        from kungfu_amd.p2p import AutoExchange
        dev = torch.device("cuda:0")
        sizes = [70001, 333, 120000]
        gb = GradBuckets(sizes, torch.float32, dev, world, n_buckets=3)
        ex = AutoExchange(trials=2)
        for step in range(2):
            xs = [[torch.randn(n, device=dev, generator=torch.Generator(device=dev)
                               .manual_seed(1000 * r + 10 * step + i)) for i, n in enumerate(sizes)]
                  for r in range(world)]
            for v, x in zip(gb.views, xs[rank]):
                v.copy_(x)
            ex.all_reduce_(gb.buckets, average=True)
            for i, v in enumerate(gb.views):
                # every candidate folds in rank order (or is exact at N = 2):
                # the pick cannot change a bit
                want = ops.bucket_reduce_avg([xs[r][i] for r in range(world)], world)
                assert torch.equal(v, want), (step, i, ex.picked)
        picks = [None] * world
        dist.all_gather_object(picks, sorted(ex.picked.values()))
        assert all(p == picks[0] for p in picks), picks
        ex.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_auto_exchange_gpu(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(_auto_body, world)


def _auto_guard_body(rank, world, port, errq):
    """AutoExchange's same-bits guard on GPU buckets: an extra candidate that
    runs the P2P pull exchange and then flips one bit on the last rank (a
    stand-in for a shard served stale over xGMI) is dropped on EVERY rank,
    the rank that saw the difference says where, and the result is the
    oracle's rank-order average."""
    sys.path[:0] = [ROOT, HERE]
    import contextlib
    import io
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from kungfu_amd.collective import GradBuckets
        from kungfu_amd.p2p import AutoExchange, PeerExchange
        from oracle import oracle
        dev = torch.device("cuda:0")

        class Perturbing:
            def __init__(self):
                self.inner = PeerExchange()

            def all_reduce_(self, buckets, op="sum", average=False, coalesce=True):
                self.inner.all_reduce_(buckets, op=op, average=average)
                if rank == world - 1:
                    buckets[2].view(torch.int32)[4097] ^= 1
                return buckets

            def finish(self):
                self.inner.finish()

        sizes = [70001, 333, 120000]
        gb = GradBuckets(sizes, torch.float32, dev, world, n_buckets=3)
        ex = AutoExchange(trials=1, extra=[("p2p_stale", Perturbing())])
        xs = [[np.random.default_rng(100 * r + i).standard_normal(n).astype(np.float32)
               for i, n in enumerate(sizes)] for r in range(world)]
        for v, x in zip(gb.views, xs[rank]):
            v.copy_(torch.from_numpy(x))
        err = io.StringIO()
        with contextlib.redirect_stderr(err):
            ex.all_reduce_(gb.buckets, average=True)
        assert "p2p_stale" not in ex.picked.values(), ex.picked
        assert "p2p_stale" in [n for n, _ in ex.dropped], ex.dropped
        if rank == world - 1:
            assert "drops candidate p2p_stale" in err.getvalue(), err.getvalue()
            assert "bucket 2 at element 4097" in err.getvalue(), err.getvalue()
        for i, v in enumerate(gb.views):
            want = oracle.reduce_avg([xs[r][i] for r in range(world)], "f32", world)
            assert np.array_equal(v.cpu().numpy(), want), i
        ex.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_auto_exchange_drops_wrong_bits_gpu(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(_auto_guard_body, world)
