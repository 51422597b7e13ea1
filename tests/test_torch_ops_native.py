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
