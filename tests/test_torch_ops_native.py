"""The torch C++ op module with the reference's signatures
(kungfu_amd/csrc/torch_ops.cpp; reference srcs/cpp/src/torch/module_cuda.cpp:28-40,
ops/cuda/collective.cpp:20-55): all_reduce_cuda(input, output, type, op),
all_reduce_cuda_async(input, output, type, op, name) -> handle, wait_handle,
and kungfu_amd.torch.ops routing CUDA tensors through it. The multi-rank
arithmetic underneath is kf_exchange's (tests/test_exchange.py)."""
import pytest
import torch


def _mod():
    try:
        from kungfu_amd import kungfu_amd_torch_ops as m
    except ImportError as e:
        pytest.fail("torch op module not built: %s (__graft_entry__.build())" % e)
    return m


def test_module_surface_and_uninitialised_errors():
    m = _mod()
    for name in ("all_reduce_cuda", "all_reduce_cuda_async", "wait_handle", "wait_all_handles",
                 "init_exchange", "unique_id", "finalize", "initialized"):
        assert hasattr(m, name), name
    if m.initialized():
        pytest.skip("already initialised in this process")
    x = torch.zeros(4)
    with pytest.raises(RuntimeError, match="init_exchange"):
        m.all_reduce_cuda(x, x, x.type(), "sum")
    with pytest.raises(RuntimeError, match="128 bytes"):
        m.init_exchange(b"short", 0, 1, 0)


@pytest.mark.parametrize("bad", ["0", "-5", "abc", "2.5", "99999999"])
def test_init_timeout_env_is_validated(bad, monkeypatch):
    """KUNGFU_AMD_INIT_TIMEOUT_S was read with atoi and
    multiplied in int, so "0" or junk timed every init out at once and huge
    values overflowed to "wait forever". Now anything but whole seconds in
    [1, 86400] is refused, with a message, before RCCL is touched."""
    m = _mod()
    if m.initialized():
        pytest.skip("already initialised in this process")
    monkeypatch.setenv("KUNGFU_AMD_INIT_TIMEOUT_S", bad)
    with pytest.raises(RuntimeError, match="KUNGFU_AMD_INIT_TIMEOUT_S"):
        m.init_exchange(b"\0" * 128, 0, 1, 0)


@pytest.mark.gpu
def test_cuda_ops_world1():
    """One rank: the all-reduce is the identity for every op and dtype; the
    type string must match the tensor; handles complete; the Python mirror's
    CUDA path goes through the C++ op."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist
    from kungfu_amd.torch import ops
    assert not dist.is_initialized()
    m = ops.native_ops()
    assert m is not None and m.initialized()
    dev = torch.device("cuda:0")
    for dtype in (torch.float32, torch.bfloat16, torch.float16, torch.int32, torch.float64):
        x = (torch.randn(100003, device=dev) * 100).to(dtype)
        y = torch.empty_like(x)
        for op in ("sum", "min", "max", "prod"):
            if dtype == torch.float16 and op != "sum":
                continue  # fp16 is SUM only (op.cpp:45-54)
            m.all_reduce_cuda(x, y, x.type(), op)
            torch.cuda.synchronize()
            assert torch.equal(y, x), (dtype, op)
    x = torch.randn(4097, device=dev)
    with pytest.raises(RuntimeError):
        m.all_reduce_cuda(x, x, "torch.cuda.DoubleTensor", "sum")  # size mismatch
    with pytest.raises(RuntimeError):
        m.all_reduce_cuda(x, x, x.type(), "mean")
    hs = [m.all_reduce_cuda_async(x, x, x.type(), "sum", "w%d" % i) for i in range(4)]
    m.wait_all_handles(hs)
    with pytest.raises(RuntimeError):
        m.wait_handle(hs[0])  # already waited
    # the kungfu.torch.ops mirror: CUDA tensors through the C++ op
    x0 = torch.arange(10, dtype=torch.float32, device=dev).reshape(2, 5)
    assert torch.equal(ops.all_reduce_fn(x0), x0)
    h = ops.inplace_all_reduce_async_op(x0, "x0")
    ops.wait_handle(h)
    assert torch.equal(x0, torch.arange(10, dtype=torch.float32, device=dev).reshape(2, 5))
    ar, ara = ops._op_maps()
    assert ar["torch.cuda.FloatTensor"] is m.all_reduce_cuda


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["auto", "a2a"])
@pytest.mark.parametrize("world", [2, 4])
def test_cuda_ops_multi_rank_by_name(world, algo):
    """all_reduce_cuda_async pairs tensors by NAME across ranks, as the
    reference's does (collective.cpp:32-55 hands tensor_name to
    Peer::AllReduce, whose messages pair by name): `world` ranks (threads,
    each with its own exchange over the test library's loopback transport,
    bound with bind_exchange) start the same named tensors in different
    random orders with random gaps; every result equals the oracle's
    rank-order fold of that name's tensors — f32 sum, i32 max, bf16 sum. Then
    the blocking all_reduce_cuda in one order, and the kungfu.torch.ops mirror
    (inplace_all_reduce_async_op) over the same binding. algo "a2a"
    (set_algo): the f32 and i32 names too go through the all-to-all and the
    HIP rank-order fold, not the loopback's host reduce-scatter, so the
    product's arithmetic is what is compared at world > 1."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import time
    import numpy as np
    from loopback import loop_ranks
    from oracle import oracle
    from kungfu_amd.torch import ops
    m = _mod()
    dev = torch.device("cuda:0")
    kinds = [("f32", "sum"), ("i32", "max"), ("bf16", "sum")]
    sizes = [1, 1000, 65537, 7, 300001, 4096, 33, 2 * 4096 + 3, 5]
    names = ["layer%d.%s" % (i, kinds[i % 3][0]) for i in range(len(sizes))]

    def host(r, step, i):
        name = kinds[i % 3][0]
        rng = np.random.default_rng(1000 * step + 10 * r + i)
        if name == "i32":
            return rng.integers(-2 ** 31, 2 ** 31 - 1, sizes[i]).astype(np.int32)
        x = rng.standard_normal(sizes[i]).astype(np.float32)
        return oracle.f32_to_bf16_bits(x) if name == "bf16" else x

    def dev_t(a, name):
        t = torch.from_numpy(np.ascontiguousarray(a))
        if name == "bf16":
            t = t.view(torch.int16).view(torch.bfloat16)
        return t.to(dev)

    def back(t, name):
        t = t.cpu()
        return t.view(torch.int16).numpy().view(np.uint16) if name == "bf16" else t.numpy()

    def want(step, i):
        name, op = kinds[i % 3]
        return oracle.reduce_k([host(r, step, i) for r in range(world)], name, op)

    def body(rank, ex):
        m.bind_exchange(ex._h)
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for step in range(2):
                    rng = np.random.default_rng(77 * rank + step)
                    xs = [dev_t(host(rank, step, i), kinds[i % 3][0]) for i in range(len(sizes))]
                    outs = [torch.empty_like(x) for x in xs]
                    hs = []
                    for i in rng.permutation(len(sizes)):
                        time.sleep(float(rng.random()) * 0.003)
                        x = xs[i]
                        hs.append(m.all_reduce_cuda_async(x, outs[i], x.type(), kinds[i % 3][1],
                                                          names[i]))
                    m.wait_all_handles(hs)
                    for i in range(len(sizes)):
                        assert np.array_equal(back(outs[i], kinds[i % 3][0]), want(step, i)), \
                            (rank, step, names[i])
                # the blocking op: same order on every rank (the reference's "" name)
                for i in range(len(sizes)):
                    x = dev_t(host(rank, 5, i), kinds[i % 3][0])
                    m.all_reduce_cuda(x, x, x.type(), kinds[i % 3][1])
                    assert np.array_equal(back(x, kinds[i % 3][0]), want(5, i)), (rank, i)
                # the Python mirror, in place, any order
                rng = np.random.default_rng(5 + rank)
                xs = [dev_t(host(rank, 9, i), kinds[i % 3][0]) for i in range(len(sizes))]
                hs = {}
                for i in rng.permutation(len(sizes)):
                    hs[i] = ops.inplace_all_reduce_async_op(xs[i], names[i], kinds[i % 3][1])
                ops.wait_all_handles([hs[i] for i in range(len(sizes))])
                for i in range(len(sizes)):
                    assert np.array_equal(back(xs[i], kinds[i % 3][0]), want(9, i)), (rank, i)
            torch.cuda.synchronize()
        finally:
            m.bind_exchange(0)

    m.set_algo(algo)
    try:
        loop_ranks(world, body)
    finally:
        m.set_algo("auto")
