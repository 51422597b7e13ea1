"""Hierarchical all-reduce (kungfu_amd/hierarchical.py; the reference's
ScheduledHierarchicalNcclAllReduce, tensorflow/ops/gpu/collective.cpp:108-162)
with hosts emulated by loopback addresses: gloo stands in for RCCL inside a
host, the native session (host mode, the oracle's restatement of the reference
reduce as the fold) runs across hosts, the oracle does the /np epilogue.
Expected values: integer sums exactly (the reference's known answers sum to
np·x / iota·np, fake_agent.cpp:15-44); float averages within the order bound
(np-1)·2^-24·Σ|x| + one rounding for the division."""
import ctypes
import os
import socket
import sys
import tempfile
import traceback

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from procs import hung_msg, join_all

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _peers(hosts_sizes, base):
    out = []
    for h, n in enumerate(hosts_sizes):
        out += ["127.0.0.%d:%d" % (h + 1, base + len(out) + i) for i in range(n)]
    return out


def _addr(peer):
    ip, port = peer.rsplit(":", 1)
    return ip, int(port)


def _x(rank, n):
    return np.random.default_rng(300 + rank).standard_normal(n).astype(np.float32)


def _body(rank, hosts_sizes, port, sock_dir, errq, use_gpu, first=None):
    import faulthandler
    faulthandler.dump_traceback_later(100, exit=True)  # a hung rank dies loudly
    sys.path[:0] = [ROOT, HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=sum(hosts_sizes))
        # the session ports: a block every rank could bind, agreed over gloo
        from ports import agreed_block
        base, rounds = agreed_block(lambda b: [_addr(_peers(hosts_sizes, b)[rank])], first=first)
        if first is not None:  # the test holds rank 0's first port: redrawn
            assert rounds >= 2 and base != first, (rounds, base, first)
        peers = _peers(hosts_sizes, base)
        from cpu_epilogue import CpuEpilogue
        from kungfu_amd.hierarchical import HierarchicalExchange
        from oracle import oracle
        world = len(peers)
        if use_gpu:
            dev = torch.device("cuda:0")
            ex = HierarchicalExchange(peers, rank, sock_dir=sock_dir, mode="device")
        else:
            dev = torch.device("cpu")
            fn = ctypes.cast(oracle.lib().oracle_transform2, ctypes.c_void_p)
            ex = HierarchicalExchange(peers, rank, sock_dir=sock_dir, mode="host",
                                      epilogue=CpuEpilogue(), host_reduce_fn=fn)
        # fp32 S-SGD average over a 3-chunk bucket and a small one
        for step, n in enumerate(((3 << 20) // 4 + 11, 1000)):
            m = ex.padded_count(n, 4)
            b = torch.zeros(m, dtype=torch.float32, device=dev)
            b[:n] = torch.from_numpy(_x(rank + 10 * step, n)).to(dev)
            ex.all_reduce_([b], average=True, name="grad%d" % step)
            xs = [_x(r + 10 * step, n) for r in range(world)]
            exact = np.sum([x.astype(np.float64) for x in xs], axis=0) / world
            absum = np.sum([np.abs(x).astype(np.float64) for x in xs], axis=0)
            got = b[:n].cpu().numpy().astype(np.float64)
            bound = (world - 1) * 2.0 ** -24 * absum / world + 2.0 ** -24 * np.abs(exact) + 1e-37
            assert np.all(np.abs(got - exact) <= bound * 1.0001), step
            assert np.all(b[n:].cpu().numpy() == 0)
        # int32 SUM and MAX: exact
        n = 4099
        m = ex.padded_count(n, 4)
        bi = torch.zeros(m, dtype=torch.int32, device=dev)
        bi[:n] = torch.arange(n, dtype=torch.int32, device=dev) + rank
        ex.all_reduce_([bi], op="sum", name="iota")
        want = (np.arange(n) * world + world * (world - 1) // 2).astype(np.int32)
        assert np.array_equal(bi[:n].cpu().numpy(), want)
        bi[:n] = torch.full((n,), rank * 7, dtype=torch.int32, device=dev)
        ex.all_reduce_([bi], op="max", name="max")
        assert torch.all(bi[:n].cpu() == (world - 1) * 7)
        # the optimizer surface on top: S-SGD averages, SMA blends
        from kungfu_amd.optimizers import (SynchronousAveragingOptimizer,
                                           SynchronousSGDOptimizer)
        w = torch.nn.Parameter(torch.zeros(3000, device=dev))
        opt = SynchronousSGDOptimizer(torch.optim.SGD([w], lr=1.0), exchange=ex)
        w.grad = torch.full((3000,), float(rank + 1), device=dev)
        opt.step()  # w = 0 - mean(rank + 1)
        assert torch.all(w.detach().cpu() == -(world + 1) / 2)
        v = torch.nn.Parameter(torch.full((777,), float(2 * rank), device=dev))
        sma = SynchronousAveragingOptimizer(torch.optim.SGD([v], lr=0.0), alpha=0.5, exchange=ex)
        v.grad = torch.zeros(777, device=dev)
        sma.step()  # 0.5 * 2r + 0.5 * mean(2r) = r + (world - 1) / 2
        assert torch.allclose(v.detach().cpu(), torch.full((777,), rank + (world - 1) / 2))
        ex.close()
        dist.barrier()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(hosts_sizes, use_gpu=False, first=None):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_body, args=(r, hosts_sizes, port, d, errq, use_gpu, first))
              for r in range(sum(hosts_sizes))]
        for p in ps:
            p.start()
        hung = join_all(ps, 300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


def test_host_layout_matches_partition_by_host():
    from kungfu_amd.hierarchical import host_layout
    peers = ["10.0.0.1:1", "10.0.0.2:1", "10.0.0.1:2", "10.0.0.3:1", "10.0.0.2:2"]
    # PartitionByHost: masters are the first rank seen on each host
    assert host_layout(peers) == [[0, 2], [1, 4], [3]]


def test_two_equal_hosts_2d():
    # 2 hosts x 2 ranks: local reduce-scatter, per-local-rank cross sessions
    _run([2, 2])


def test_uneven_hosts_via_master():
    # hosts of 2 and 1 ranks: the reference's reduce -> masters -> broadcast
    _run([2, 1])


def test_one_rank_per_host():
    # every host one rank: the whole exchange is the cross-host session
    _run([1, 1, 1])


def test_session_port_taken_is_redrawn():
    """Another process listens on the first port chosen for rank 0's session:
    the ranks see it in their bind check, agree to redraw, and the run
    passes."""
    sys.path[:0] = [HERE]
    from ports import taken_port
    s, p = taken_port()
    try:
        _run([1, 1], first=p)
    finally:
        s.close()


@pytest.mark.gpu
def test_cross_host_device_sessions():
    # device-mode cross sessions (HIP folds in HBM) + HIP /np epilogue; one rank
    # per emulated host so no intra-host collective is needed on a shared GPU
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run([1, 1], use_gpu=True)
    _run([1, 1, 1], use_gpu=True)


@pytest.mark.gpu
def test_two_hosts_two_gpus_each_device():
    """2 emulated hosts x 2 ranks, all on cuda:0: the intra-host step moves GPU
    tensors (gloo standing in for RCCL, which refuses ranks sharing a device),
    the HIP /np epilogue runs on the shard, the cross-host step is a
    device-mode native session per local rank (HIP folds in HBM) — the whole
    2-D path on the GPU; and 2 + 1 ranks through the masters."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run([2, 2], use_gpu=True)
    _run([2, 1], use_gpu=True)


@pytest.mark.gpu
def test_native_hierarchical_threads_two_hosts_two_ranks():
    """kungfu_amd.hierarchical.NativeHierarchicalExchange — kf_hier_all_reduce
    behind the C ABI — with 2 emulated hosts x 2 ranks as threads of one
    process on cuda:0: device-mode sessions across hosts (127.0.0.1 / .2),
    the test library's loopback inside each host. S-SGD average (f32, both
    algos, a ragged count), i32 MAX, and SMA through the exchange: bit-exact
    against the per-host rank-order fold added across the two hosts."""
    import socket
    import tempfile
    import threading
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path[:0] = [ROOT, HERE]
    from loopback import LoopbackGroup
    from kungfu_amd.hierarchical import NativeHierarchicalExchange
    from kungfu_amd.session import Session
    from oracle import oracle
    from ports import draw_block
    hosts = [[0, 1], [2, 3]]

    def mk(base):
        return ["127.0.0.%d:%d" % (h + 1, base + g) for h, hs in enumerate(hosts) for g in hs]
    peers = mk(draw_block(lambda b: [_addr(p) for p in mk(b)]))  # all bindable now
    groups = [LoopbackGroup(2), LoopbackGroup(2)]
    d = tempfile.mkdtemp(prefix="kfnh")
    dev = torch.device("cuda:0")
    n = 100003
    xs = [np.random.default_rng(500 + r).standard_normal(n).astype(np.float32) for r in range(4)]
    ys = [np.random.default_rng(900 + r).integers(-2 ** 31, 2 ** 31 - 1, 4097).astype(np.int32)
          for r in range(4)]

    def combine(arrs, name, op):
        per_host = [oracle.reduce_k([arrs[g] for g in h], name, op) for h in hosts]
        return oracle.reduce_k(per_host, name, op)

    errs = []

    def run(g):
        try:
            torch.cuda.set_device(0)
            h = 0 if g < 2 else 1
            local = groups[h].exchange(g % 2)
            sess = Session(peers=peers, self_spec=peers[g], sock_dir=d, mode="device")
            ex = NativeHierarchicalExchange(sess, local=local)
            assert (ex.rank, ex.np, ex.local_rank, ex.local_size, ex.host_count) == \
                (g, 4, g % 2, 2, 2)
            for algo in (1, 2):  # reduce-scatter, all-to-all
                ex.algo = algo
                b = torch.from_numpy(xs[g].copy()).to(dev)
                ex.all_reduce_([b], average=True, name="w%d" % algo)
                torch.cuda.synchronize()
                want = oracle.reduce_avg([combine(xs, "f32", "sum")], "f32", 4)
                assert np.array_equal(b.cpu().numpy(), want), algo
            c = torch.from_numpy(ys[g].copy()).to(dev)
            ex.all_reduce_([c], op="max", name="imax")
            torch.cuda.synchronize()
            assert np.array_equal(c.cpu().numpy(), np.max(np.array(ys), axis=0))
            v = torch.from_numpy(xs[g].copy()).to(dev)
            ex.sma_([v], 0.1)
            torch.cuda.synchronize()
            want = oracle.sma_blend(xs[g], combine(xs, "f32", "sum"), "f32", 4, 0.1)
            assert np.array_equal(v.cpu().numpy(), want)
            ex.close()
            sess.close()
        except Exception:
            import traceback
            errs.append("rank %d: %s" % (g, traceback.format_exc()))

    ts = [threading.Thread(target=run, args=(g,), daemon=True) for g in range(4)]
    for t in ts:
        t.start()
    import time
    deadline = time.monotonic() + 100  # inside pytest's 120 s, so the errors print
    for t in ts:
        t.join(timeout=max(0.0, deadline - time.monotonic()))
    alive = [g for g, t in enumerate(ts) if t.is_alive()]
    assert not alive, "ranks %s did not finish; the others reported:\n%s" % (alive, "\n".join(errs))
    for gr in groups:
        gr.close()
    assert not errs, "\n".join(errs)
