"""N>1 path over gloo on CPU (world sizes 2 and 3): bucketing, sharding,
reduce-scatter -> epilogue -> all-gather, the optimizer wrappers. Expected
values come from the oracle / the reference's known answers."""
import json
import os
import socket
import tempfile
import sys
import traceback

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from procs import hung_msg, join_all

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, store, fn_name, errq, use_gpu):
    sys.path[:0] = [ROOT, HERE]
    try:
        # a file store, not a TCP port: parallel test workers (pytest -n) once
        # raced for the same free port
        dist.init_process_group("gloo", init_method="file://" + store, rank=rank,
                                world_size=world)
        import test_collective_gloo as mod
        getattr(mod, fn_name)(rank, world, use_gpu)
        dist.barrier()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_world(fn_name, world, use_gpu=False):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    store = os.path.join(tempfile.mkdtemp(prefix="kfgloo"), "store")
    procs = [ctx.Process(target=_entry, args=(r, world, store, fn_name, errq, use_gpu))
             for r in range(world)]
    for p in procs:
        p.start()
    hung = join_all(procs, 600)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in procs), hung_msg(hung, [p.exitcode for p in procs])


def _epilogue(use_gpu):
    import cpu_epilogue
    if use_gpu:
        return cpu_epilogue.GpuShardEpilogue(torch.device("cuda:0"))
    return cpu_epilogue.CpuEpilogue()


def _inputs(rank, n, dtype=np.float32):
    rng = np.random.default_rng(100 + rank)
    return rng.standard_normal(n).astype(dtype)


# ---- per-rank bodies ---------------------------------------------------------

def body_all_reduce(rank, world, use_gpu):
    from kungfu_amd.collective import Exchange, padded_count
    from oracle import oracle
    ex = Exchange(epilogue=_epilogue(use_gpu))
    n = 100003
    L = padded_count(n, world, 4)
    xs = [_inputs(r, n) for r in range(world)]
    b = torch.zeros(L)
    b[:n] = torch.from_numpy(xs[rank])
    ex.all_reduce_([b], average=True)
    got = b[:n].numpy()
    if world == 2:  # two operands: commutative, so bit-exact
        assert np.array_equal(got, oracle.reduce_avg(xs, "f32", 2))
    else:
        exact = np.sum(np.array(xs, np.float64), axis=0) / world
        bound = (world - 1) * 2.0 ** -24 * np.sum(np.abs(np.array(xs, np.float64)), axis=0) / world
        assert np.all(np.abs(got - exact) <= bound + 2.0 ** -24 * np.abs(exact))
    # sum only, int32: bit-exact for every world size and order
    ints = [np.random.default_rng(r).integers(-2**31, 2**31 - 1, n, dtype=np.int32)
            for r in range(world)]
    bi = torch.zeros(L, dtype=torch.int32)
    bi[:n] = torch.from_numpy(ints[rank])
    ex.all_reduce_([bi], op="sum")
    assert np.array_equal(bi[:n].numpy(), oracle.reduce_k(ints, "i32"))
    # MAX
    bm = torch.zeros(L)
    bm[:n] = torch.from_numpy(xs[rank])
    ex.all_reduce_([bm], op="max")
    assert np.array_equal(bm[:n].numpy(), np.max(np.array(xs), axis=0))


def body_resnet50_buckets(rank, world, use_gpu):
    # C4 layout: ResNet-50 gradient set fused into 16 buckets (EvenPartition)
    from kungfu_amd.collective import Exchange, GradBuckets
    sizes = json.load(open(os.path.join(HERE, "golden", "models.json")))["resnet50-imagenet"]
    ex = Exchange(epilogue=_epilogue(use_gpu))
    gb = GradBuckets(sizes, torch.float32, torch.device("cpu"), world, n_buckets=16)
    assert len(gb.buckets) == 16 and sum(gb.spans) == 25583592
    lens = [b.numel() for b in gb.buckets]
    assert max(lens) - min(lens) <= world * 64  # EvenPartition of aligned units
    for i, v in enumerate(gb.views):
        assert v.numel() == sizes[i]
        v.fill_(float((rank + 1) * (i % 7 + 1)))
    for b in gb.buckets:
        assert b.numel() % world == 0 and (b.numel() // world) * 4 % 256 == 0
    ex.all_reduce_(gb.buckets, average=True)
    tot = world * (world + 1) / 2
    for i, v in enumerate(gb.views):
        want = np.float32(np.float32(tot * (i % 7 + 1)) / np.float32(world))
        assert torch.all(v == want), i


def body_group_all_reduce(rank, world, use_gpu):
    # ops/collective.py:71-73 mirror; KAT of fake_agent.cpp:15-44 (iota * np)
    from kungfu_amd.collective import Exchange, group_all_reduce
    ex = Exchange(epilogue=_epilogue(use_gpu))
    ts = [torch.arange(world * 4, dtype=torch.int32),
          torch.ones(1 << 20, dtype=torch.int32),
          torch.full((3, 5), float(rank + 1))]
    out = group_all_reduce(ts, exchange=ex)
    assert torch.equal(out[0], torch.arange(world * 4, dtype=torch.int32) * world)
    assert torch.all(out[1] == world)  # kungfu-test-public-apis.go:87-104
    assert torch.all(out[2] == world * (world + 1) / 2)
    assert out[2].shape == (3, 5)


def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(17, 9), torch.nn.Tanh(), torch.nn.Linear(9, 3))


def _loss(m, rank):
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(8, 17, generator=g)
    return (m(x) ** 2).mean()


def body_sync_sgd(rank, world, use_gpu):
    from kungfu_amd.collective import Exchange
    from kungfu_amd.optimizers import SynchronousSGDOptimizer
    m = _model()
    opt = SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                  named_parameters=m.named_parameters(),
                                  exchange=Exchange(epilogue=_epilogue(use_gpu)))
    # expected: every rank's gradients, summed, / np, then SGD
    grads = []
    for r in range(world):
        mr = _model()
        _loss(mr, r).backward()
        grads.append([p.grad.clone() for p in mr.parameters()])
    ref = _model()
    from bounds import assert_within, avg_bound, sgd_bound
    for steps in range(2):
        opt.zero_grad()
        _loss(m, rank).backward()
        opt.step()
        if steps == 0:
            tols = []
            with torch.no_grad():
                for j, p in enumerate(ref.parameters()):
                    s = grads[0][j].clone()
                    for r in range(1, world):
                        s = s + grads[r][j]
                    avg = s / world
                    gb = avg_bound([grads[r][j] for r in range(world)], world)
                    tols.append((gb, avg))
                    p -= 0.1 * avg
            for (p, q), (gb, avg) in zip(zip(m.parameters(), ref.parameters()), tols):
                assert_within(p.grad, avg, gb, "gradient")  # the exchange
                assert_within(p.detach(), q.detach(), sgd_bound(gb, 0.1, q.detach(), avg), "param")
    # all ranks hold identical parameters after synchronous steps
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    allf = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(allf, flat)
    for f in allf:
        assert torch.equal(f, flat)


def body_sma(rank, world, use_gpu):
    from kungfu_amd.collective import Exchange
    from kungfu_amd.optimizers import SynchronousAveragingOptimizer
    alpha = 0.1
    m = _model(seed=rank)  # replicas start different
    before = [p.detach().clone() for p in m.parameters()]
    allp = []
    for r in range(world):
        allp.append([p.detach().clone() for p in _model(seed=r).parameters()])
    opt = SynchronousAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.0),
                                        alpha=alpha,
                                        exchange=Exchange(epilogue=_epilogue(use_gpu)))
    _loss(m, rank).backward()
    opt.step()  # lr 0: only the model averaging acts
    from bounds import assert_within, avg_bound, sma_bound
    for j, p in enumerate(m.parameters()):
        s = allp[0][j].clone()
        for r in range(1, world):
            s = s + allp[r][j]
        avg = s / world
        want = np.float32(1 - alpha) * before[j] + np.float32(alpha) * avg
        ab = avg_bound([allp[r][j] for r in range(world)], world)
        assert_within(p.detach(), want, sma_bound(ab, alpha, before[j], avg), "sma %d" % j)


def body_sma_overlap(rank, world, use_gpu):
    """SMA with overlap=True (the next step's sum started at the end of
    step()) gives the same parameters, bit for bit, as overlap=False, over
    three SGD steps from replicas that start different."""
    from kungfu_amd.collective import Exchange
    from kungfu_amd.optimizers import SynchronousAveragingOptimizer
    ms = [_model(seed=rank), _model(seed=rank)]
    opts = [SynchronousAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), alpha=0.1,
                                          exchange=Exchange(epilogue=_epilogue(use_gpu)),
                                          overlap=ov)
            for m, ov in zip(ms, (False, True))]
    for step in range(3):
        for m, opt in zip(ms, opts):
            opt.zero_grad()
            _loss(m, rank + 10 * step).backward()
            opt.step()
        for a, b in zip(ms[0].parameters(), ms[1].parameters()):
            assert torch.equal(a.detach(), b.detach()), step


# ---- tests -------------------------------------------------------------------

@pytest.mark.parametrize("world", [2, 3])
def test_all_reduce(world):
    run_world("body_all_reduce", world)


def test_resnet50_16_buckets():
    run_world("body_resnet50_buckets", 2)


@pytest.mark.parametrize("world", [2, 3])
def test_group_all_reduce(world):
    run_world("body_group_all_reduce", world)


@pytest.mark.parametrize("world", [2, 3])
def test_sync_sgd_optimizer(world):
    run_world("body_sync_sgd", world)


@pytest.mark.parametrize("world", [2, 3])
def test_sma_optimizer(world):
    run_world("body_sma", world)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sma_optimizer_overlap_same_bits(world):
    run_world("body_sma_overlap", world)


def test_world1_identity():
    from kungfu_amd.collective import Exchange
    ex = Exchange()
    b = torch.arange(64, dtype=torch.float32)
    ex.all_reduce_([b], average=True)
    assert torch.equal(b, torch.arange(64, dtype=torch.float32))


@pytest.mark.gpu
def test_all_reduce_with_hip_epilogue():
    # gloo moves the shards, the real HIP /np epilogue runs on the GPU
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run_world("body_all_reduce", 2, use_gpu=True)
    run_world("body_sync_sgd", 3, use_gpu=True)
    run_world("body_sma", 2, use_gpu=True)
    run_world("body_sync_sgd_overlap", 2, use_gpu=True)


def test_coalesce_runs():
    from kungfu_amd.collective import GradBuckets, coalesce_runs
    gb = GradBuckets([1000, 3000, 5000], torch.float32, torch.device("cpu"), 2, n_buckets=3)
    runs = coalesce_runs(gb.buckets)
    assert len(runs) == 1 and runs[0].numel() == sum(b.numel() for b in gb.buckets)
    assert runs[0].data_ptr() == gb.buckets[0].data_ptr()
    gb2 = GradBuckets([1000, 3000], torch.float32, torch.device("cpu"), 2, bucket_bytes=4000)
    assert len(coalesce_runs(gb2.buckets)) == len(gb2.buckets)  # separate storages
    # order matters: reversed buckets are not one run
    assert len(coalesce_runs(gb.buckets[::-1])) == 3


def test_workspace_like_mirrors_a_contiguous_run():
    """SMA's sum workspaces: for GradBuckets' contiguous buckets, views of ONE
    flat allocation in the same order (so the blend launches once over both
    ranges); otherwise one tensor per bucket."""
    from kungfu_amd.collective import GradBuckets, workspace_like
    gb = GradBuckets([1000, 3000, 5000], torch.float32, torch.device("cpu"), 2, n_buckets=3)
    ws = workspace_like(gb.buckets)
    assert [w.shape for w in ws] == [b.shape for b in gb.buckets]
    for w0, w1 in zip(ws, ws[1:]):
        assert w1.data_ptr() == w0.data_ptr() + w0.numel() * w0.element_size()
    assert all(w.data_ptr() != b.data_ptr() for w, b in zip(ws, gb.buckets))
    ws2 = workspace_like(gb.buckets[::-1])  # not one run: separate tensors
    assert [w.shape for w in ws2] == [b.shape for b in gb.buckets[::-1]]
    assert len({w.untyped_storage().data_ptr() for w in ws2}) == 3


def body_coalesced_equals_per_bucket(rank, world, use_gpu):
    from kungfu_amd.collective import Exchange, GradBuckets
    ex = Exchange(epilogue=_epilogue(use_gpu))
    sizes = [5000, 123457, 77, 64000]
    a = GradBuckets(sizes, torch.float32, torch.device("cpu"), world, n_buckets=6)
    b = GradBuckets(sizes, torch.float32, torch.device("cpu"), world, n_buckets=6)
    for i, (va, vb) in enumerate(zip(a.views, b.views)):
        x = torch.from_numpy(_inputs(rank * 10 + i, va.numel()))
        va.copy_(x)
        vb.copy_(x)
    ex.all_reduce_(a.buckets, average=True, coalesce=True)
    ex.all_reduce_(b.buckets, average=True, coalesce=False)
    from bounds import assert_within, avg_bound
    for i, (va, vb) in enumerate(zip(a.views, b.views)):
        if world == 2:
            assert torch.equal(va, vb)
        else:
            xs = [torch.from_numpy(_inputs(r * 10 + i, va.numel())) for r in range(world)]
            assert_within(va, vb, avg_bound(xs, world), "bucket %d" % i)


@pytest.mark.parametrize("world", [2, 3])
def test_coalesced_equals_per_bucket(world):
    run_world("body_coalesced_equals_per_bucket", world)


def body_per_bucket_many_outstanding(rank, world, use_gpu):
    # bench.py's c3_per_bucket shape: 64 buckets, all 64 reduce-scatters in
    # flight before the first wait, then 64 all-gathers in flight
    from kungfu_amd.collective import Exchange, GradBuckets
    ex = Exchange(epilogue=_epilogue(use_gpu))
    n = 64 * 4096 * world
    a = GradBuckets([n], torch.float32, torch.device("cpu"), world, n_buckets=64)
    b = GradBuckets([n], torch.float32, torch.device("cpu"), world, n_buckets=64)
    x = torch.from_numpy(_inputs(rank, n))
    a.views[0].copy_(x)
    b.views[0].copy_(x)
    assert len(a.buckets) == 64
    ex.all_reduce_(a.buckets, average=True, coalesce=False)
    ex.all_reduce_(b.buckets, average=True, coalesce=True)
    from bounds import assert_within, avg_bound
    xs = [torch.from_numpy(_inputs(r, n)) for r in range(world)]
    assert_within(a.views[0], b.views[0], avg_bound(xs, world), "per bucket vs fused")
    for _ in range(2):  # many outstanding again, on the averaged values
        ex.all_reduce_(a.buckets, average=True, coalesce=False)


@pytest.mark.parametrize("world", [4])
def test_per_bucket_many_outstanding(world):
    run_world("body_per_bucket_many_outstanding", world)


def body_torch_ops(rank, world, use_gpu):
    # kungfu.torch.ops surface (srcs/python/kungfu/torch/ops/collective.py)
    from kungfu_amd.torch import ops
    x = torch.arange(10, dtype=torch.float32).reshape(2, 5) + rank
    y = ops.all_reduce_fn(x)
    assert torch.equal(y, torch.arange(10, dtype=torch.float32).reshape(2, 5) * world
                       + world * (world - 1) / 2)
    z = torch.full((7,), float(rank + 1))
    ops.inplace_all_reduce_op(z, "max")
    assert torch.all(z == world)
    hs = [ops.inplace_all_reduce_async_op(torch.ones(1000, dtype=torch.int32) * (rank + 1), "a")]
    t = torch.ones(33) * (rank + 1)
    hs.append(ops.inplace_all_reduce_async_op(t, "t"))
    ops.wait_all_handles(hs)
    assert torch.all(t == world * (world + 1) / 2)
    sd = {"w": torch.full((4,), float(rank))}
    ops.broadcast_parameters(sd)
    assert torch.all(sd["w"] == 0)
    g = ops.all_gather(torch.tensor([rank, rank * 10]))
    assert g.shape == (world, 2) and g[world - 1, 1].item() == (world - 1) * 10
    # package-level peer queries (kungfu/torch/__init__.py:1-16)
    import kungfu_amd.torch as kf
    assert (kf.current_rank(), kf.current_cluster_size()) == (rank, world)
    assert (kf.current_local_rank(), kf.current_local_size()) == (rank, world)  # one host
    assert kf.get_cuda_index() == kf.current_local_rank()
    assert kf.nccl_built() is False
    kf.run_barrier()


@pytest.mark.parametrize("world", [2, 3])
def test_torch_ops_surface(world):
    run_world("body_torch_ops", world)


def body_sync_sgd_overlap(rank, world, use_gpu):
    # buckets exchanged from backward hooks (overlap=True) give the same
    # parameters as the exchange in step(); small buckets so a step has many,
    # a layer that gets no gradient (zeros contributed), three steps with
    # zero_grad(set_to_none) in between
    from kungfu_amd.collective import Exchange
    from kungfu_amd.optimizers import SynchronousSGDOptimizer

    def model():
        torch.manual_seed(3)
        m = torch.nn.Sequential(torch.nn.Linear(17, 40), torch.nn.Tanh(),
                                torch.nn.Linear(40, 30), torch.nn.Tanh(),
                                torch.nn.Linear(30, 3))
        m.register_parameter("unused", torch.nn.Parameter(torch.ones(25)))
        return m

    a, b = model(), model()
    # rank-order folds (a2a): the two bucket layouts give the same bits at
    # every world size, so the parameters must be identical, not close
    oa = SynchronousSGDOptimizer(torch.optim.SGD(a.parameters(), lr=0.1, momentum=0.9),
                                 exchange=Exchange(epilogue=_epilogue(use_gpu), algo="a2a"),
                                 bucket_bytes=2048, overlap=True)
    ob = SynchronousSGDOptimizer(torch.optim.SGD(b.parameters(), lr=0.1, momentum=0.9),
                                 exchange=Exchange(epilogue=_epilogue(use_gpu), algo="a2a"),
                                 bucket_bytes=2048)
    assert len(oa._kf_slots) > 3
    for step in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            _loss(m, rank + 7 * step).backward()
            if o is oa:  # every bucket with gradients went out during backward
                assert oa._kf_next == len(oa._kf_slots) - 1  # all but `unused`'s
            o.step()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
    flat = torch.cat([p.detach().reshape(-1) for p in a.parameters()])
    allf = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(allf, flat)
    for f in allf:
        assert torch.equal(f, flat)


@pytest.mark.parametrize("world", [2, 3])
def test_sync_sgd_overlap(world):
    run_world("body_sync_sgd_overlap", world)


def body_torch_sync_sgd_sums(rank, world, use_gpu):
    # kungfu.torch.optimizers.SynchronousSGDOptimizer sums the gradients and
    # does not divide by np (reference torch/optimizers/sync_sgd.py:12-22);
    # named_parameters is required as there (sync_sgd.py:31)
    from kungfu_amd.torch.optimizers import SynchronousSGDOptimizer
    w = torch.nn.Parameter(torch.zeros(5))
    opt = SynchronousSGDOptimizer(torch.optim.SGD([w], lr=1.0), [("w", w)])
    w.grad = torch.full((5,), float(rank + 1))
    opt.step()
    # w = 0 - lr * sum_r (r + 1)
    assert torch.equal(w.detach(), torch.full((5,), -world * (world + 1) / 2.0))
    w2 = torch.nn.Parameter(torch.zeros(3))
    opt2 = SynchronousSGDOptimizer(torch.optim.SGD([w2], lr=1.0), [("w2", w2)], op="max")
    w2.grad = torch.full((3,), float(rank))
    opt2.step()
    assert torch.equal(w2.detach(), torch.full((3,), -(world - 1.0)))
    try:
        SynchronousSGDOptimizer(torch.optim.SGD([w], lr=1.0))
    except TypeError:
        pass
    else:
        raise AssertionError("named_parameters must be required")


@pytest.mark.parametrize("world", [2, 3])
def test_torch_sync_sgd_sums_like_reference(world):
    run_world("body_torch_sync_sgd_sums", world)


def sgd_bound0(p, g, lr=0.1):
    """p - lr·g with an exact g on both sides: only the update's roundings."""
    from bounds import sgd_bound
    return sgd_bound(torch.zeros_like(p, dtype=torch.float64), lr, p, g)


def body_auto_exchange_cpu(rank, world, use_gpu):
    # AutoExchange on host tensors: P2P is no candidate, RCCL's path (gloo
    # here) is picked, S-SGD values as with Exchange
    from kungfu_amd.optimizers import SynchronousSGDOptimizer
    from kungfu_amd.p2p import AutoExchange
    ex = AutoExchange(epilogue=_epilogue(use_gpu))
    m = _model()
    opt = SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                  named_parameters=m.named_parameters(), exchange=ex)
    grads = []
    for r in range(world):
        mr = _model()
        _loss(mr, r).backward()
        grads.append([p.grad.clone() for p in mr.parameters()])
    opt.zero_grad()
    _loss(m, rank).backward()
    opt.step()
    ref = _model()
    avgs = []
    with torch.no_grad():
        for j, p in enumerate(ref.parameters()):
            s = grads[0][j].clone()
            for r in range(1, world):
                s = s + grads[r][j]
            avgs.append(s / world)
            p -= 0.1 * avgs[-1]
    # every candidate folds in rank order: the exchanged gradient IS the
    # rank-order average; the update itself may round differently (FMA)
    from bounds import assert_within
    for p, q, avg in zip(m.parameters(), ref.parameters(), avgs):
        assert torch.equal(p.grad, avg)
        assert_within(p.detach(), q.detach(), sgd_bound0(q.detach(), avg), "param")
    # RCCL's paths only (no P2P for host buckets); reduce-scatter only where
    # its order cannot change a bit (two ranks)
    assert set(ex.picked.values()) <= ({"rccl", "rccl_rs"} if world == 2 else {"rccl"})


@pytest.mark.parametrize("world", [2, 3])
def test_auto_exchange_host_buckets(world):
    run_world("body_auto_exchange_cpu", world)


@pytest.mark.parametrize("world", [4, 8])
def test_more_ranks_all_reduce(world):
    # the N = 4 / 8 shapes of the driver's multi-GPU run, rehearsed on CPU:
    # fp32 within the order bound, int32 / MAX bit-exact, ResNet-50's 16
    # buckets (C4 layout), the fake_agent KATs, S-SGD
    run_world("body_all_reduce", world)
    run_world("body_group_all_reduce", world)


def test_eight_ranks_resnet50_and_sgd():
    run_world("body_resnet50_buckets", 8)
    run_world("body_sync_sgd", 8)


def body_a2a_rank_order(rank, world, use_gpu):
    # algo "a2a": all-to-all of the shards, then the rank-order fold — the
    # oracle's reduce over ranks 0..world-1 bit for bit at EVERY world size
    # (bf16: fp32 accumulation, one rounding; f16: per-hop rounding; f32: the
    # rank-order sum), both for S-SGD (sum, / np) and SMA
    from kungfu_amd.collective import Exchange, GradBuckets
    from oracle import oracle
    import cpu_epilogue
    ex = Exchange(epilogue=_epilogue(use_gpu), algo="a2a")
    auto = Exchange(epilogue=_epilogue(use_gpu))  # auto: bf16/f16 -> a2a
    sizes = [1000, 33333, 7]
    for dtype, name in ((torch.bfloat16, "bf16"), (torch.float16, "f16"),
                        (torch.float32, "f32")):
        xs = [[torch.from_numpy(_inputs(100 * r + i, n)).to(dtype) for i, n in enumerate(sizes)]
              for r in range(world)]
        for e in ((ex, auto) if dtype != torch.float32 else (ex,)):
            gb = GradBuckets(sizes, dtype, torch.device("cpu"), world, n_buckets=2)
            for v, x in zip(gb.views, xs[rank]):
                v.copy_(x)
            e.all_reduce_(gb.buckets, average=True, coalesce=False)
            for i, v in enumerate(gb.views):
                want = oracle.reduce_avg([cpu_epilogue._np(xs[r][i]).copy() for r in range(world)],
                                         name, world)
                assert np.array_equal(cpu_epilogue._np(v), want), (name, i)
        # SMA: v <- (1-a) v + a sum/np, sum folded in rank order
        alpha = 0.1
        gb = GradBuckets(sizes, dtype, torch.device("cpu"), world, bucket_bytes=40000)
        for v, x in zip(gb.views, xs[rank]):
            v.copy_(x)
        before = [cpu_epilogue._np(b).copy() for b in gb.buckets]
        allb = []
        for r in range(world):
            g2 = GradBuckets(sizes, dtype, torch.device("cpu"), world, bucket_bytes=40000)
            for v, x in zip(g2.views, xs[r]):
                v.copy_(x)
            allb.append([cpu_epilogue._np(b).copy() for b in g2.buckets])
        ex.sma_(gb.buckets, alpha)
        for j, b in enumerate(gb.buckets):
            s = oracle.reduce_k([allb[r][j] for r in range(world)], name, "sum")
            want = oracle.sma_blend(before[j], s, name, world, alpha)
            assert np.array_equal(cpu_epilogue._np(b), want), (name, "sma", j)
    # integers: the fold and RCCL's order agree
    n = 5000
    ints = [np.random.default_rng(7 + r).integers(-2**31, 2**31 - 1, n, dtype=np.int32)
            for r in range(world)]
    from kungfu_amd.collective import padded_count
    bi = torch.zeros(padded_count(n, world, 4), dtype=torch.int32)
    bi[:n] = torch.from_numpy(ints[rank])
    ex.all_reduce_([bi], op="max")
    assert np.array_equal(bi[:n].numpy(), np.max(np.array(ints), axis=0))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_a2a_rank_order_bit_exact(world):
    run_world("body_a2a_rank_order", world)


class _Perturbing:
    """A candidate that runs the real exchange and then flips the low bit of
    one element on rank 1 only — a stand-in for a transport that serves a
    stale shard on one node. It is the fastest (it IS the reference's path,
    minus nothing); the pick must still drop it."""

    def __init__(self, inner):
        self.inner = inner

    def all_reduce_(self, buckets, op="sum", average=False, coalesce=True):
        self.inner.all_reduce_(buckets, op=op, average=average)
        if dist.get_rank() == 1:
            v = buckets[1].view(torch.int32) if buckets[1].dtype == torch.float32 else buckets[1]
            v[17] ^= 1
        return buckets

    def sma_(self, buckets, alpha):
        self.inner.sma_(buckets, alpha)
        if dist.get_rank() == 1:
            buckets[0].view(torch.int32)[3] ^= 1
        return buckets


def body_auto_exchange_drops_wrong_bits(rank, world, use_gpu):
    import contextlib
    import io
    from kungfu_amd.collective import Exchange
    from kungfu_amd.p2p import AutoExchange
    from oracle import oracle
    ep = _epilogue(use_gpu)
    bad = _Perturbing(Exchange(epilogue=ep, algo="a2a"))
    ex = AutoExchange(epilogue=ep, extra=[("bad", bad)], trials=1)
    sizes = [1000 * world, 4096 * world, 111 * world]
    xs = [[_inputs(10 * r + j, n) for j, n in enumerate(sizes)] for r in range(world)]
    buckets = [torch.from_numpy(xs[rank][j].copy()) for j in range(len(sizes))]
    err = io.StringIO()
    with contextlib.redirect_stderr(err):
        ex.all_reduce_(buckets, average=True)
    assert ex.picked[tuple((b.data_ptr(), b.numel(), b.dtype) for b in buckets)] != "bad"
    assert [n for n, _ in ex.dropped] == ["bad"], ex.dropped
    if rank == 1:
        assert "rank 1 drops candidate bad" in err.getvalue(), err.getvalue()
        assert "bucket 1 at element 17" in err.getvalue(), err.getvalue()
    for j in range(len(sizes)):
        want = oracle.reduce_avg([xs[r][j] for r in range(world)], "f32", world)
        assert np.array_equal(buckets[j].numpy(), want), j
    # SMA picks separately, with the same check
    vs = [torch.from_numpy(xs[rank][j].copy()) for j in range(len(sizes))]
    with contextlib.redirect_stderr(io.StringIO()):
        ex.sma_(vs, 0.1)
    assert "bad" not in [ex.picked[k] for k in ex.picked]
    for j in range(len(sizes)):
        s = oracle.reduce_k([xs[r][j] for r in range(world)], "f32", "sum")
        assert np.array_equal(vs[j].numpy(), oracle.sma_blend(xs[rank][j], s, "f32", world, 0.1))


@pytest.mark.parametrize("world", [2, 3])
def test_auto_exchange_drops_a_candidate_with_other_bits(world):
    run_world("body_auto_exchange_drops_wrong_bits", world)


def body_auto_exchange_past_16_ranks(rank, world, use_gpu):
    # past KF_MAX_INPUTS ranks the rank-order fold cannot run: RCCL's
    # reduce-scatter is the base candidate and the call goes through
    from kungfu_amd.p2p import AutoExchange
    ex = AutoExchange(epilogue=_epilogue(use_gpu))
    b = torch.full((world * 64,), float(rank + 1))
    ex.all_reduce_([b])
    assert torch.equal(b, torch.full_like(b, world * (world + 1) / 2))
    assert list(ex.picked.values()) == ["rccl_rs"]


def test_auto_exchange_past_16_ranks():
    run_world("body_auto_exchange_past_16_ranks", 17)


def body_native_bring_up(rank, world, use_gpu):
    """kungfu_amd.torch.ops.bring_up over gloo with injected failures: a
    failure on ONE rank at any step sends every rank to the torch path
    (None), nobody enters the (blocking) communicator init unless every rank
    got ready, and nobody hangs; no failure: every rank gets the module."""
    from kungfu_amd.torch import ops as tops

    class Mod:
        def __init__(self):
            self.inits, self.finals = [], 0

        def initialized(self):
            return bool(self.inits)

    def run(fail_where, fail_rank):
        mod = Mod()

        def load_module():
            if fail_where == "import" and rank == fail_rank:
                raise ImportError("injected")
            return mod

        def make_uid():
            if fail_where == "uid":
                raise RuntimeError("injected")
            return b"u" * 128

        def init(m, uid, r, w):
            assert uid == b"u" * 128 and r == rank and w == world
            m.inits.append(uid)
            if fail_where == "init" and rank == fail_rank:
                raise RuntimeError("injected")

        def finalize(m):
            m.finals += 1

        got = tops.bring_up(load_module, make_uid, init, finalize)
        return got, mod

    for where in ("import", "uid", "init"):
        for fail_rank in range(world):
            if where == "uid" and fail_rank != 0:
                continue  # only rank 0 makes the id
            got, mod = run(where, fail_rank)
            assert got is None, (where, fail_rank)
            # the blocking init only after every rank got ready
            assert bool(mod.inits) == (where == "init"), (where, fail_rank, mod.inits)
            assert mod.finals == (1 if where == "init" else 0)
    got, mod = run(None, -1)
    assert got is mod and len(mod.inits) == 1 and mod.finals == 0


@pytest.mark.parametrize("world", [2, 3])
def test_native_bring_up_agrees_before_init(world):
    run_world("body_native_bring_up", world)
