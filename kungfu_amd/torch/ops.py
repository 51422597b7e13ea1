"""``kungfu.torch.ops`` mirror (srcs/python/kungfu/torch/ops/collective.py:8-52).

The reference moves a CUDA tensor to the host, all-reduces it there through
Peer::AllReduce and copies it back (srcs/cpp/src/torch/ops/cuda/collective.cpp:
20-55). Here the tensor stays in HBM: it is staged into an aligned bucket and
reduced by RCCL reduce-scatter + all-gather over xGMI (op 'sum' / 'min' /
'max' / 'prod'); the handle API is kept for the async variants.
"""
import threading

import torch
import torch.distributed as dist

from ..collective import Exchange, padded_count

_exchange = None
_native = [None, False]  # the C++ op module once its exchange is up; tried?
_native_lock = threading.Lock()


def native_ops():
    """The C++ extension with the reference's op signatures
    (kungfu_amd/csrc/torch_ops.cpp: all_reduce_cuda(input, output, type, op),
    all_reduce_cuda_async(..., name) -> handle, wait_handle), its exchange
    initialised from the process group: RCCL needs one GPU per rank, so only
    with the nccl backend (or a single process). None where it cannot run —
    decided the same way on every rank: a rank whose import or exchange setup
    fails says why, every rank agrees on the outcome (all_gather_object), and
    all of them take the torch.distributed path from then on."""
    with _native_lock:
        if not _native[1]:
            _native[0] = _init_native()
            _native[1] = True
        return _native[0]


def _init_native():
    if not torch.cuda.is_available():
        return None
    if dist.is_initialized() and dist.get_backend() != "nccl":
        return None

    def load_module():
        from .. import kungfu_amd_torch_ops as m
        return m

    def make_uid():
        import ctypes
        from .. import _lib
        uid = (ctypes.c_char * 128)()
        _lib.check(_lib.load().kf_exchange_unique_id(uid), "kf_exchange_unique_id")
        return bytes(uid)

    def init(m, uid, rank, world):
        m.init_exchange(uid, rank, world, torch.cuda.current_device())

    def finalize(m):
        if m.initialized():
            m.finalize()

    return bring_up(load_module, make_uid, init, finalize)


def bring_up(load_module, make_uid, init, finalize):
    """The native op's start-up, decided the same way on every rank. RCCL's
    communicator init blocks until every rank has joined, so no rank may
    enter it unless every rank is known to get there: each step that can
    fail on one rank alone (the module import, rank 0's unique id, anything
    before the init) is followed by an agreement (all_gather_object), and a
    failure anywhere sends every rank to the torch.distributed path together.
    The reference's init blocks the same way with no such check
    (gpu_collective.cpp:105). Returns the module, or None."""
    import sys
    rank = dist.get_rank() if dist.is_initialized() else 0
    world = _world()
    m, uid, ok = None, None, True

    def say(what, e):
        print("kungfu_amd.torch.ops: %s on rank %d: %r" % (what, rank, e), file=sys.stderr)

    try:
        m = load_module()
    except ImportError as e:
        say("C++ op module unavailable", e)
        ok = False
    if ok and rank == 0:
        try:
            uid = make_uid()
        except RuntimeError as e:  # KungFuAMDError is one
            say("unique id failed", e)
            ok = False
    # every rank is ready to join (and rank 0 has an id) before any shares it
    if not _agree(ok):
        return None
    if world > 1:
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    try:
        init(m, uid, rank, world)
    except RuntimeError as e:
        say("exchange setup failed", e)
        ok = False
    if not _agree(ok):
        try:
            finalize(m)
        except RuntimeError as e:
            say("finalize failed", e)
        return None
    return m


def _agree(flag):
    """True iff `flag` holds on every rank."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bool(flag)
    flags = [None] * dist.get_world_size()
    dist.all_gather_object(flags, bool(flag))
    return all(flags)


def _op_maps():
    """clib.py's maps (srcs/python/kungfu/torch/ops/clib.py:13-38): tensor
    type string -> op, for the CUDA types the C++ op serves."""
    m = native_ops()
    if m is None:
        return {}, {}
    types = ("torch.cuda.FloatTensor", "torch.cuda.DoubleTensor", "torch.cuda.HalfTensor",
             "torch.cuda.BFloat16Tensor", "torch.cuda.IntTensor", "torch.cuda.LongTensor")
    return ({t: m.all_reduce_cuda for t in types},
            {t: m.all_reduce_cuda_async for t in types})


def _ex():
    global _exchange
    if _exchange is None:
        _exchange = Exchange()
    return _exchange


def _world():
    return dist.get_world_size() if dist.is_initialized() else 1


class _Handle:
    def __init__(self, works, finish):
        self.works, self.finish = works, finish


_handles = {}
_next = [0]


def _staged(x):
    n = x.numel()
    L = padded_count(max(n, 1), _world(), x.element_size())
    buf = torch.zeros(L, dtype=x.dtype, device=x.device)
    buf[:n].copy_(x.reshape(-1))
    return buf


def all_reduce_fn(x, op=None):
    """Returns the all-reduced copy of x (collective.py:8-13)."""
    y = x.clone()
    inplace_all_reduce_op(y, op)
    return y


def inplace_all_reduce_op(x, op=None):
    """x <- all-reduce(x) in place (collective.py:16-19)."""
    op = op or "sum"
    if x.is_cuda and x.is_contiguous():
        m = native_ops()
        if m is not None:
            m.all_reduce_cuda(x, x, x.type(), op)
            return x
    if _world() == 1:
        return x
    buf = _staged(x)
    _ex().all_reduce_([buf], op=op)
    x.copy_(buf[:x.numel()].view_as(x))
    return x


def inplace_all_reduce_async_op(x, name, op=None):
    """Starts x <- all-reduce(x); returns a handle for wait_handle
    (collective.py:22-25). CUDA tensors go through the C++ op, which pairs
    them across ranks by `name` (any start order per rank, as the
    reference). The torch.distributed stand-in (no C++ op: CPU tensors, gloo)
    queues reduce-scatter and all-gather at once and pairs by call order, so
    there every rank must start its names in one order."""
    op = op or "sum"
    h = _next[0]
    _next[0] += 1
    if x.is_cuda and x.is_contiguous():
        m = native_ops()
        if m is not None:
            nh = m.all_reduce_cuda_async(x, x, x.type(), op, name)
            _handles[h] = _Handle([], lambda: m.wait_handle(nh))
            return h
    if _world() == 1:
        _handles[h] = _Handle([], lambda: None)
        return h
    from ..base import OP_NAMES
    from ..collective import _RED_OPS
    buf = _staged(x)
    world = _world()
    shard = torch.empty(buf.numel() // world, dtype=buf.dtype, device=buf.device)
    w1 = dist.reduce_scatter_tensor(shard, buf, op=_RED_OPS[OP_NAMES[op]], async_op=True)
    if dist.get_backend() == "nccl":
        # RCCL ops of one communicator run in order on its stream: queue the
        # all-gather right behind the reduce-scatter
        works = [w1, dist.all_gather_into_tensor(buf, shard, async_op=True)]

        def finish(x=x, buf=buf):
            x.copy_(buf[:x.numel()].view_as(x))
    else:
        # other backends may run async ops concurrently: gather after the wait
        works = [w1]

        def finish(x=x, buf=buf, shard=shard):
            dist.all_gather_into_tensor(buf, shard)
            x.copy_(buf[:x.numel()].view_as(x))

    _handles[h] = _Handle(works, finish)
    return h


def inplace_broadcast_async_op(x, name):
    """Starts x <- rank 0's x (collective.py:28-29); returns a handle."""
    h = _next[0]
    _next[0] += 1
    works = [dist.broadcast(x, src=0, async_op=True)] if _world() > 1 else []
    _handles[h] = _Handle(works, lambda: None)
    return h


def wait_handle(handle):
    hd = _handles.pop(handle)
    for w in hd.works:
        w.wait()
    hd.finish()


def wait_all_handles(handles):
    for h in handles:
        wait_handle(h)


def broadcast_parameters(state_dict):
    """Every rank takes rank 0's parameters (collective.py:40-45)."""
    wait_all_handles([inplace_broadcast_async_op(v, k) for k, v in state_dict.items()])


def all_gather(x):
    """[np] + x.shape tensor of every rank's x (collective.py:48-52)."""
    world = _world()
    y = x.new_empty(torch.Size([world] + list(x.shape)))
    if world == 1:
        y[0].copy_(x)
        return y
    dist.all_gather_into_tensor(y.reshape(-1), x.contiguous().reshape(-1))
    return y
