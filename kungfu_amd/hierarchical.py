"""Hierarchical all-reduce for peers on several hosts.

The reference's hierarchical path is the TF op ScheduledHierarchicalNcclAllReduce
(srcs/cpp/src/tensorflow/ops/gpu/collective.cpp:108-162), used by
SynchronousSGDOptimizer(nccl=True, hierarchical_nccl=True) (sync_sgd.py:68-72,
ops/collective.py:113-139). Per gradient tensor:
  1. ncclReduce to the host's local rank 0                (controller_->Reduce)
  2. CrossAllReduceGpu (srcs/cpp/src/nccl/controller.cpp:7-39) on local rank 0:
     D2H copy, Session.CrossAllReduce over the host masters only
     (session/allreduce.go:46-48; graphs: a ring per master for RING, else a
     binary tree over the masters, session/strategy.go:188-210), the host reduce
     std_transform_2 at every graph node, H2D copy back
  3. ncclBroadcast from local rank 0                      (controller_->Broadcast)
and the optimizer divides by np afterwards (sync_sgd.py:103-104).

MI355X-first restatement (HierarchicalExchange):
  * equal hosts (every host runs L ranks): a 2-D all-reduce. RCCL
    reduce-scatter over xGMI inside the host leaves each local rank with 1/L of
    the host's sum; local rank i then all-reduces ITS shard across hosts with
    its own native session (kungfu_amd.session, device mode: peer chunks land
    in page-locked slots and are folded in HBM by the HIP kernel), so the
    cross-host bytes leave every GPU of the host in parallel instead of all
    through local rank 0; the 1/np epilogue runs on the shard (HIP); RCCL
    all-gather inside the host. A session whose peers are one per host runs
    exactly the reference's cross graphs: its BINARY_TREE_STAR is a binary tree
    over the masters and its RING the masters' rings (session.go:55,
    strategy.go:188-210);
  * uneven hosts: the reference's shape — RCCL reduce to the local master, the
    masters' session all-reduce, 1/np on the master, RCCL broadcast.
Sums are the same element-wise sum as the flat all-reduce; the fp32 order
differs (RCCL inside hosts, the session's graph across them), so float results
are within (np-1)·2^-24·Σ|x| of the exact sum, integers exact.

Ranks of torch.distributed and of the peer list (KUNGFU_INIT_PEERS order) are
the same numbering. The epilogue is injectable only for the CPU tests (gloo +
host-mode sessions); the product path is HIP + RCCL.
"""
import torch
import torch.distributed as dist

from .base import OP, OP_NAMES
from .collective import ALIGN_BYTES, HipEpilogue, _RED_OPS
from .session import Session


def host_layout(peers):
    """hosts (first-seen order), each a list of global ranks; PartitionByHost
    (plan/peerlist.go:166-178) keeps the same masters (first rank per host)."""
    order, by_host = [], {}
    for r, p in enumerate(peers):
        ip = p.rsplit(":", 1)[0]
        if ip not in by_host:
            by_host[ip] = []
            order.append(ip)
        by_host[ip].append(r)
    return [by_host[ip] for ip in order]


def hier_padded_count(count, local_size, itemsize):
    """Smallest length >= count that splits into `local_size` shards that each
    start on a 256-byte boundary."""
    unit = local_size * max(1, ALIGN_BYTES // itemsize)
    return ((count + unit - 1) // unit) * unit


class HierarchicalExchange:
    """Hierarchical all-reduce of flat buckets (see module docstring).

    peers      the KUNGFU_INIT_PEERS list ("ip:port", rank order)
    rank       this process's rank (torch.distributed and peer list)
    mode       "device" (GPU buckets, the product) or "host" (CPU tests)
    Every rank must construct it (it creates the per-host process groups)."""

    def __init__(self, peers, rank, sock_dir="/tmp", mode="device", epilogue=None,
                 host_reduce_fn=None, token=0):
        peers = peers.split(",") if isinstance(peers, str) else list(peers)
        self.peers, self.rank, self.np = peers, rank, len(peers)
        self.world = self.np  # GradBuckets pads to world shards: a multiple of L
        self.hosts = host_layout(peers)
        self.mode = mode
        self.epilogue = epilogue if epilogue is not None else HipEpilogue()
        self.host = next(h for h in self.hosts if rank in h)
        self.local_rank = self.host.index(rank)
        self.local_size = len(self.host)
        self.equal = len({len(h) for h in self.hosts}) == 1
        # one process group per host, created by every rank in the same order
        self.local_group = None
        for h in self.hosts:
            g = dist.new_group(h) if len(h) > 1 else None
            if rank in h:
                self.local_group = g
        # the cross-host session of this rank: local rank i of every host
        # (2-D), or the masters (uneven hosts; only masters take part)
        if self.equal:
            cross = [h[self.local_rank] for h in self.hosts]
        else:
            cross = [h[0] for h in self.hosts] if self.local_rank == 0 else None
        self.session = None
        if cross is not None and len(cross) > 1:
            self.session = Session(peers=[peers[r] for r in cross], self_spec=peers[rank],
                                   sock_dir=sock_dir, mode=mode, token=token,
                                   host_reduce_fn=host_reduce_fn)
        self._ws = {}

    def padded_count(self, count, itemsize):
        """Bucket length to allocate for `count` elements; the same on every
        rank (equal hosts: a multiple of the local size in aligned units;
        uneven hosts: no constraint)."""
        if self.equal:
            return hier_padded_count(count, self.local_size, itemsize)
        return count

    def close(self):
        if self.session is not None:
            self.session.close()
            self.session = None

    def _cross(self, t, name, red):
        if self.session is None:
            return
        buf = t if self.mode == "device" else t.numpy()
        self.session.all_reduce(buf, buf, name, op=red)

    def _shard(self, key, n, like):
        t = self._ws.get(key)
        if t is None or t.numel() < n or t.dtype != like.dtype or t.device != like.device:
            t = torch.empty(n, dtype=like.dtype, device=like.device)
            self._ws[key] = t
        return t[:n]

    def all_reduce_(self, buckets, op="sum", average=False, name="hier"):
        """In place. Buckets must be flat and, on equal hosts, of a length
        divisible by the local size (hier_padded_count). `name` keys the
        cross-host messages; every rank must pass the same."""
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        if average and red != OP.SUM:
            raise ValueError("average requires op='sum'")
        for i, b in enumerate(buckets):
            if b.dim() != 1 or not b.is_contiguous():
                raise ValueError("bucket must be a flat contiguous tensor")
            key = "%s/%d:%d" % (name, i, b.numel())
            if self.equal:
                self._two_d(b, key, red, average)
            else:
                self._via_master(b, key, red, average)
        return buckets

    def sma_(self, buckets, alpha, name="hier-sma"):
        """SMA (sma_sgd.py:60-65): v <- (1-alpha) v + alpha * sum_ranks(v) / np,
        the sum by the hierarchical all-reduce into a workspace."""
        sums = []
        for i, b in enumerate(buckets):
            s = self._shard(("sum", i), b.numel(), b)
            s.copy_(b)
            sums.append(s)
        self.all_reduce_(sums, op="sum", name=name)
        for b, s in zip(buckets, sums):
            self.epilogue.sma_blend_(b, s, self.np, alpha)
        return buckets

    def _two_d(self, b, key, red, average):
        L = self.local_size
        if b.numel() % L:
            raise ValueError("bucket length %d not divisible by the local size %d; use "
                             "hier_padded_count()" % (b.numel(), L))
        if L == 1:
            shard = b
        else:
            shard = self._shard(key, b.numel() // L, b)
            dist.reduce_scatter_tensor(shard, b, op=_RED_OPS[red], group=self.local_group)
        self._cross(shard, key, red)
        if average:
            self.epilogue.div_(shard, self.np)
        if L > 1:
            dist.all_gather_into_tensor(b, shard, group=self.local_group)

    def _via_master(self, b, key, red, average):
        master = self.host[0]
        if self.local_size > 1:
            dist.reduce(b, dst=master, op=_RED_OPS[red], group=self.local_group)
        if self.rank == master:
            self._cross(b, key, red)
            if average:
                self.epilogue.div_(b, self.np)
        if self.local_size > 1:
            dist.broadcast(b, src=master, group=self.local_group)


class NativeHierarchicalExchange:
    """The hierarchical all-reduce behind the C ABI (kf_hier_all_reduce,
    include/kungfu_amd.h): one native call per bucket does the host's
    reduce-scatter (RCCL, or the all-to-all + HIP rank-order fold), the
    cross-host all-reduce of the shard over the device-mode session (one tree
    of ranks per local rank, kf_session_subset_all_reduce), / np and the host's
    all-gather; hosts of different sizes take the reference's masters path.
    The same code a C++ or Go host runs.

    session   a device-mode kungfu_amd.session.Session over ALL peers
    local     the host's exchange (kungfu_amd.exchange.NativeExchange);
              default kf_exchange_create_local(session) — gpu_collective::
              new_local, its RCCL id shared over the session."""

    def __init__(self, session, local=None, device=None, algo="auto"):
        import ctypes
        from . import _lib
        from .exchange import ALGOS, NativeExchange
        self.lib = _lib.load()
        self.session = session
        r, n, lr, ls, hc = (ctypes.c_int() for _ in range(5))
        _lib.check(self.lib.kf_session_info(session._h, ctypes.byref(r), ctypes.byref(n),
                                            ctypes.byref(lr), ctypes.byref(ls),
                                            ctypes.byref(hc)), "kf_session_info")
        self.rank, self.np, self.world = r.value, n.value, n.value
        self.local_rank, self.local_size, self.host_count = lr.value, ls.value, hc.value
        if local is None:
            dev = torch.device(device if device is not None else
                               ("cuda:%d" % torch.cuda.current_device()))
            h = self.lib.kf_exchange_create_local(session._h, dev.index)
            if not h:
                raise _lib.KungFuAMDError("kf_exchange_create_local: " +
                                          self.lib.kf_exchange_last_error().decode())
            local = NativeExchange.from_handle(h, algo)
        self.local = local
        self.algo = ALGOS[algo]
        self._sums = {}

    def padded_count(self, count, itemsize):
        return hier_padded_count(count, self.local_size, itemsize)

    def all_reduce_(self, buckets, op="sum", average=False, name="hier"):
        """In place, queued on the current stream; every rank passes the same
        buckets (counts), op and name, in the same order."""
        from . import _lib
        from .ops import kungfu_dtype
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        if average and red != OP.SUM:
            raise ValueError("average requires op='sum'")
        for i, b in enumerate(buckets):
            if not b.is_cuda or b.dim() != 1 or not b.is_contiguous():
                raise ValueError("buckets must be flat contiguous GPU tensors")
            rc = self.lib.kf_hier_all_reduce(
                self.local._h, self.session._h, b.data_ptr(), b.data_ptr(), b.numel(),
                int(kungfu_dtype(b)), int(red), 1 if average else 0, self.algo,
                ("%s/%d" % (name, i)).encode(), torch.cuda.current_stream(b.device).cuda_stream)
            _lib.check(rc, "kf_hier_all_reduce")
        return buckets

    def sma_(self, buckets, alpha, name="hier-sma"):
        from . import ops
        sums = []
        for i, b in enumerate(buckets):
            key = (i, b.numel(), b.dtype)
            s = self._sums.get(key)
            if s is None:
                s = self._sums[key] = torch.empty_like(b)
            s.copy_(b)
            sums.append(s)
        self.all_reduce_(sums, name=name)
        for b, s in zip(buckets, sums):
            ops.sma_blend_(b, s, self.np, alpha)
        return buckets

    def close(self):
        if self.local is not None:
            self.local.close()
            self.local = None
