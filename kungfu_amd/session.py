"""Single-host KungFu session with the reduce on the GPU — Python face of the
native engine in kungfu_amd/csrc/kf_session.hip (kf_session_* C ABI).

Mirrors ``Session.AllReduce`` (srcs/go/kungfu/session/allreduce.go:10-12 ->
session.go:231-326) for peers that share a host: 1 MiB chunks by
EvenPartition named ``part::<name>[b:e]``, each chunk's strategy picked by the
reference's name hash, reduce-graph folds in arrival order, bcast with
WaitRecvBuf. Strategies: the star family (the single-host default:
BINARY_TREE_STAR / AUTO), CLIQUE, RING, BINARY_TREE. Peers are processes on
unix sockets speaking the reference's rchannel framing.

Modes:
  "device": send/recv are GPU tensors; chunks land in page-locked slots, are
            copied to HBM and folded by the HIP kernel.
  "host":   send/recv are host numpy arrays; the fold is std_transform_2 (the
            drop-in, GPU offload) or, if given, a C function pointer with the
            kf_host_reduce_fn signature (bench.py's CPU baseline leg).
"""
import ctypes
import threading

from . import _lib
from .base import OP, OP_NAMES

CHUNK_SIZE = 1 << 20  # session.go:301-304
PORT_BASE = 10000

# KungFu_Strategy codes (srcs/cpp/include/kungfu/strategy.h:7-17) by the names
# kungfu-run accepts (srcs/go/kungfu/base/strategy.go:24-36)
STRATEGIES = {
    "TREE": 0, "BINARY_TREE": 1, "RING": 2, "STAR": 3, "MULTI_STAR": 4,
    "CLIQUE": 5, "BINARY_TREE_STAR": 6, "MULTI_BINARY_TREE_STAR": 7, "AUTO": 8,
}


class Session:
    """Peer `rank` of `size` on this host, or — with ``peers`` (the
    KUNGFU_INIT_PEERS list, "ip:port,...") and ``self_spec`` (KUNGFU_SELF_SPEC)
    — a peer of a multi-host cluster: colocated peers use unix sockets under
    ``sock_dir``, the others TCP; multi-host strategies follow the hosts."""

    def __init__(self, rank=None, size=None, sock_dir="/tmp", mode="device", token=0,
                 host_reduce_fn=None, strategy=None, hash_method="NAME",
                 peers=None, self_spec=None):
        if mode not in ("device", "host"):
            raise ValueError(mode)
        self.mode = mode
        self.lib = _lib.load()
        dm = 1 if mode == "device" else 0
        if peers is not None:
            plist = peers.split(",") if isinstance(peers, str) else list(peers)
            if self_spec not in plist:
                raise ValueError("self %r not in peer list" % (self_spec,))
            self.rank, self.size = plist.index(self_spec), len(plist)
            self._h = self.lib.kf_session_create_peers(",".join(plist).encode(),
                                                       self_spec.encode(), sock_dir.encode(),
                                                       token, dm)
        else:
            self.rank, self.size = rank, size
            self._h = self.lib.kf_session_create(rank, size, sock_dir.encode(), token, dm)
        if not self._h:
            raise _lib.KungFuAMDError("kf_session_create: " +
                                      self.lib.kf_session_last_error().decode())
        if strategy is not None:  # else KUNGFU_ALLREDUCE_STRATEGY / default
            _lib.check(self.lib.kf_session_set_strategy(
                self._h, STRATEGIES[strategy], 1 if hash_method == "NAME" else 0),
                "kf_session_set_strategy", "session")
        self._pending = []  # async handles: keep buffers and callbacks alive
        self._plock = threading.Lock()
        if host_reduce_fn is not None:
            if mode != "host":
                raise ValueError("host_reduce_fn needs mode='host'")
            _lib.check(self.lib.kf_session_set_host_reduce(self._h, host_reduce_fn),
                       "kf_session_set_host_reduce", "session")

    @classmethod
    def from_env(cls, sock_dir="/tmp", **kw):
        """As a peer started by kungfu-run: KUNGFU_INIT_PEERS / KUNGFU_SELF_SPEC
        (srcs/go/kungfu/env/envs.go:9-11)."""
        import os
        return cls(peers=os.environ["KUNGFU_INIT_PEERS"],
                   self_spec=os.environ["KUNGFU_SELF_SPEC"], sock_dir=sock_dir, **kw)

    def close(self):
        if self._h:
            self.lib.kf_session_destroy(self._h)  # runs what is still queued
            self._h = None
            self._pending = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _meta(self, buf):
        if self.mode == "device":
            from .ops import kungfu_dtype
            if not buf.is_cuda or not buf.is_contiguous():
                raise ValueError("device mode needs contiguous GPU tensors")
            return buf.numel(), int(kungfu_dtype(buf)), buf.data_ptr()
        from .base import dtype_of
        if not buf.flags["C_CONTIGUOUS"]:
            raise ValueError("host mode needs contiguous numpy arrays")
        return buf.size, int(dtype_of(buf)), buf.ctypes.data

    def all_reduce(self, send, recv, name, op="sum"):
        """Synchronous all-reduce of one bucket (send is recv: in place)."""
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        count, dt, sp = self._meta(send)
        rcount, rdt, rp = self._meta(recv)
        if (rcount, rdt) != (count, dt):
            raise ValueError("send/recv mismatch")
        stream = None
        if self.mode == "device":
            import torch
            stream = torch.cuda.current_stream(send.device).cuda_stream
        rc = self.lib.kf_session_all_reduce(self._h, sp, rp, count, dt, int(red),
                                            name.encode(), stream)
        _lib.check(rc, "kf_session_all_reduce", "session")
        return recv

    def _stream(self, t):
        if self.mode != "device":
            return None
        import torch
        return torch.cuda.current_stream(t.device).cuda_stream

    def subset_all_reduce(self, send, recv, forest, name, op="sum"):
        """Session.SubsetAllReduce (allreduce.go:14-24): each tree of `forest`
        (forest[i] = father of i, a root is its own) all-reduces within itself."""
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        count, dt, sp = self._meta(send)
        rcount, rdt, rp = self._meta(recv)
        if (rcount, rdt) != (count, dt):
            raise ValueError("send/recv mismatch")
        if len(forest) != self.size:
            raise ValueError("forest needs one entry per peer")
        f = (ctypes.c_int32 * self.size)(*forest)
        _lib.check(self.lib.kf_session_subset_all_reduce(self._h, sp, rp, count, dt, int(red), f,
                                                         name.encode(), self._stream(send)),
                   "kf_session_subset_all_reduce", "session")
        return recv

    def reduce(self, send, recv, name, op="sum"):
        """Session.Reduce (session.go:159-162): the first strategy's reduce
        graph only; its root's recv holds the reduction."""
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        count, dt, sp = self._meta(send)
        rcount, rdt, rp = self._meta(recv)
        if (rcount, rdt) != (count, dt):
            raise ValueError("send/recv mismatch")
        _lib.check(self.lib.kf_session_reduce(self._h, sp, rp, count, dt, int(red),
                                              name.encode(), self._stream(send)),
                   "kf_session_reduce", "session")
        return recv

    def broadcast(self, send, recv, name):
        """Session.Broadcast (session.go:164-167): every recv becomes the
        first strategy's root's send."""
        count, dt, sp = self._meta(send)
        rcount, rdt, rp = self._meta(recv)
        if (rcount, rdt) != (count, dt):
            raise ValueError("send/recv mismatch")
        _lib.check(self.lib.kf_session_broadcast(self._h, sp, rp, count, dt, name.encode(),
                                                 self._stream(send)),
                   "kf_session_broadcast", "session")
        return recv

    def all_reduce_async(self, send, recv, name, op="sum", callback=None):
        """Start an all-reduce and return at once (GoKungfuAllReduce with a
        done callback, libkungfu-comm/collective.go:34-45): the session's
        worker thread runs every started all-reduce at once, pairing peers'
        messages by name as the reference's goroutine per call does, so peers
        may start their names in different orders (a name started again waits
        for its previous call). ``callback(status)`` runs on that thread when
        the all-reduce is done, in completion order; ``handle.wait()`` blocks
        until then and raises on failure. send/recv must not be touched
        before that."""
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        count, dt, sp = self._meta(send)
        rcount, rdt, rp = self._meta(recv)
        if (rcount, rdt) != (count, dt):
            raise ValueError("send/recv mismatch")
        stream = None
        if self.mode == "device":
            import torch
            stream = torch.cuda.current_stream(send.device).cuda_stream
        h = AsyncHandle(send, recv, name, callback)
        rc = self.lib.kf_session_all_reduce_async(self._h, sp, rp, count, dt, int(red),
                                                  name.encode(), stream, h._cfn, None)
        _lib.check(rc, "kf_session_all_reduce_async", "session")
        with self._plock:
            self._pending = [p for p in self._pending if not p.done()] + [h]
        return h

    def barrier(self):
        """Session.Barrier (session.go:98-115): returns once every peer has
        entered it."""
        _lib.check(self.lib.kf_session_barrier(self._h), "kf_session_barrier", "session")

    def wait_all(self):
        """Block until every queued all-reduce has finished."""
        rc = self.lib.kf_session_wait_all(self._h)
        with self._plock:
            self._pending = [p for p in self._pending if not p.done()]
        _lib.check(rc, "kf_session_wait_all", "session")


class AsyncHandle:
    """One queued all-reduce (Session.all_reduce_async)."""

    def __init__(self, send, recv, name, callback):
        self.bufs = (send, recv)
        self.name = name
        self.status = None
        self._cb = callback
        self._ev = threading.Event()
        self._cfn = _lib.DONE_FN(self._done)

    def _done(self, status, _arg):
        self.status = status
        try:
            if self._cb is not None:
                self._cb(status)
        finally:
            self._ev.set()

    def done(self):
        return self._ev.is_set()

    def wait(self, timeout=None):
        if not self._ev.wait(timeout):
            raise TimeoutError("all-reduce %r not done" % self.name)
        _lib.check(self.status, "all-reduce %r" % self.name, "session")
        return self.bufs[1]


def c_reduce_fn(addr):
    """Wrap a C function address with the kf_host_reduce_fn signature."""
    return ctypes.c_void_p(addr)
