"""Multi-GPU bucket exchange through the native C-ABI (kf_exchange_*,
kungfu_amd/csrc/kf_exchange.hip): RCCL over xGMI for the data movement, the
build's HIP kernels for the element-wise sum.

The reference's GPU path is native too: gpu_collective_nccl
(srcs/cpp/src/nccl/gpu_collective.cpp:91-188) owns an NCCL communicator whose
id rank 0 creates and KungFu broadcasts (:190-200). ``NativeExchange`` does the
same with torch.distributed carrying the 128-byte id, then hands every step's
buckets to ONE native call:

  algo="rs"   ncclReduceScatter -> HIP /np on the shard -> ncclAllGather
  algo="a2a"  ncclAllToAll -> HIP rank-order fold (/np fused) -> ncclAllGather
  algo="auto" rs for integers and f32/f64, a2a for f16/bf16 (the build's
              defined semantics: bf16 accumulates in fp32 and rounds once,
              bit-identical to the P2P exchange and the oracle)
  algo="rs_avg" (opt-in) average calls as ncclReduceScatter(ncclAvg) ->
              ncclAllGather, no HIP epilogue: rs's bits when the world is a
              power of two and no x / world is subnormal

Each phase of a call is one grouped RCCL launch and all shard epilogues one
batched HIP launch, so a step of 64 buckets costs 3 launches whatever the
bucket size. Same interface as collective.Exchange (all_reduce_, start_, sma_,
world), so the optimizers take it as ``exchange=NativeExchange()``.
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from .base import OP, OP_NAMES
from .ops import kungfu_dtype

ALGOS = {"auto": 0, "rs": 1, "a2a": 2, "rs_avg": 3}
# kf_exchange_phase_times' order: phase 1 (reduce-scatter, or all-to-all for
# the rank-order fold), phase 2 (/np epilogue or the fold), phase 3
# (all-gather), the SMA blend
PHASES = ("reduce_scatter", "epilogue", "all_gather", "blend")
_NO_DONE = _lib.DONE_FN()  # a NULL kf_done_fn


def _arr(t, vals):
    return (t * len(vals))(*vals)


class NativeExchange:
    @staticmethod
    def shared_id(group=None):
        """Rank 0's unique id, broadcast to the group (gpu_collective.cpp:
        196-198); every rank of the group calls it."""
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        lib = _lib.load()
        uid = (ctypes.c_char * 128)()
        if rank == 0:
            _lib.check(lib.kf_exchange_unique_id(uid), "kf_exchange_unique_id")
        if world > 1:
            obj = [bytes(uid) if rank == 0 else None]
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(obj, src=src, group=group)
            return obj[0]
        return bytes(uid)

    def __init__(self, group=None, algo="auto", device=None, uid=None, timeout_s=None):
        """uid: the bytes of shared_id(group), when the caller shared it
        already (e.g. to create the communicator on another thread).
        timeout_s: give up (KungFuAMDError) if not every rank joined the
        communicator's init in time (kf_exchange_create_timeout)."""
        if algo not in ALGOS:
            raise ValueError("algo must be one of %s" % sorted(ALGOS))
        self.algo = algo
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.lib = _lib.load()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if uid is None:
            uid = self.shared_id(group)
        buf = (ctypes.c_char * 128).from_buffer_copy(uid)
        ms = -1 if timeout_s is None else max(0, int(timeout_s * 1000))
        h = self.lib.kf_exchange_create_timeout(buf, self.rank, self.world, self.device.index, ms)
        if not h:
            raise _lib.KungFuAMDError("kf_exchange_create: " +
                                      self.lib.kf_exchange_last_error().decode())
        self._h = h
        self._side = None
        self._sums = {}

    @classmethod
    def from_handle(cls, h, algo="auto", device=None):
        """Wrap a kf_exchange_t* made elsewhere — kf_exchange_create_session by
        a C++/Go host, kf_exchange_split, kf_exchange_create_transport over a
        host's own transport; this object owns (destroys) it."""
        if not h:
            raise _lib.KungFuAMDError("no exchange handle")
        if algo not in ALGOS:
            raise ValueError("algo must be one of %s" % sorted(ALGOS))
        self = cls.__new__(cls)
        self.lib = _lib.load()
        r, w, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.kf_exchange_info(h, ctypes.byref(r), ctypes.byref(w),
                                             ctypes.byref(d)), "kf_exchange_info")
        self.algo, self.group, self.rank, self.world = algo, None, r.value, w.value
        self.device = torch.device("cuda", d.value) if device is None else torch.device(device)
        self._h, self._side, self._sums = h, None, {}
        return self

    def transport_info(self):
        """(communicator rank count, RCCL version) as the transport reports
        them (kf_exchange_transport_info: ncclCommCount, ncclGetVersion);
        (-1, 0) over a host's own transport."""
        c, v = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.kf_exchange_transport_info(self._h, ctypes.byref(c), ctypes.byref(v)),
                   "kf_exchange_transport_info")
        return c.value, v.value

    def split(self, color, key=None):
        """kf_exchange_split (gpu_collective::new_local / new_group,
        gpu_collective.cpp:202-243): the ranks passing the same color form a
        new exchange, ordered by key; color < 0 joins none (None)."""
        st = ctypes.c_int(0)
        h = self.lib.kf_exchange_split(self._h, int(color), int(self.rank if key is None else key),
                                       ctypes.byref(st))
        _lib.check(st.value, "kf_exchange_split")
        return NativeExchange.from_handle(h, self.algo, self.device) if h else None

    def set_pipeline(self, groups):
        """kf_exchange_set_pipeline: split every batch call into `groups`
        groups of buckets whose HIP work (folds, /np, SMA blends) overlaps the
        next group's RCCL phases (1 = off, the default). Same bits."""
        _lib.check(self.lib.kf_exchange_set_pipeline(self._h, int(groups)),
                   "kf_exchange_set_pipeline")
        self.groups = int(groups)
        return self

    def set_timing(self, on):
        """kf_exchange_set_timing: start (zeroed) or stop the per-phase timing
        window of the un-pipelined batch calls."""
        _lib.check(self.lib.kf_exchange_set_timing(self._h, 1 if on else 0),
                   "kf_exchange_set_timing")

    def phase_times(self):
        """kf_exchange_phase_times: the window's per-phase sums in us
        (PHASES order) and the number of timed / pipelined (untimed) calls."""
        us = (ctypes.c_double * 4)()
        calls, untimed = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self.lib.kf_exchange_phase_times(self._h, us, ctypes.byref(calls),
                                                    ctypes.byref(untimed)),
                   "kf_exchange_phase_times")
        out = dict(zip(PHASES, (float(v) for v in us)))
        out.update(calls=calls.value, untimed_calls=untimed.value)
        return out

    # -- the optimizers' interface (collective.Exchange) --------------------
    def _check(self, buckets):
        for b in buckets:
            if not b.is_cuda or b.dim() != 1 or not b.is_contiguous():
                raise ValueError("buckets must be flat contiguous GPU tensors")
            if b.dtype != buckets[0].dtype:
                raise ValueError("one dtype per call")

    def _issue(self, buckets, op, average, stream, recvs=None):
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        if average and red != OP.SUM:
            raise ValueError("average requires op='sum'")
        ptrs = [b.data_ptr() for b in buckets]
        rptrs = ptrs if recvs is None else [r.data_ptr() for r in recvs]
        rc = self.lib.kf_exchange_all_reduce_batch(
            self._h, _lib.ptr_array(ptrs), _lib.ptr_array(rptrs),
            _arr(ctypes.c_size_t, [b.numel() for b in buckets]), len(buckets),
            int(kungfu_dtype(buckets[0])), int(red), 1 if average else 0, ALGOS[self.algo],
            stream.cuda_stream)
        _lib.check(rc, "kf_exchange_all_reduce_batch")

    def _runs(self, buckets, coalesce):
        from .collective import coalesce_runs
        return coalesce_runs(buckets) if coalesce else list(buckets)

    def all_reduce_(self, buckets, op="sum", average=False, coalesce=True):
        """In place, queued on the current stream (no host sync)."""
        buckets = list(buckets)
        if not buckets:
            return buckets
        self._check(buckets)
        self._issue(self._runs(buckets, coalesce), op, average,
                    torch.cuda.current_stream(self.device))
        return buckets

    def start_(self, buckets, op="sum", average=False, coalesce=True, key=None):
        """Queue the all-reduce on the exchange's own stream, after the work
        already queued on the current one (the gradients), so it overlaps the
        rest of backward; handle.wait() orders the current stream after it."""
        buckets = list(buckets)
        self._check(buckets)
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        cur = torch.cuda.current_stream(self.device)
        self._side.wait_stream(cur)
        self._issue(self._runs(buckets, coalesce), op, average, self._side)
        ev = torch.cuda.Event()
        ev.record(self._side)
        for b in buckets:
            b.record_stream(self._side)
        return _Handle(ev, self.device)

    def start_into_(self, sends, recvs, op="sum", average=False):
        """start_ out of place: recvs[i] <- all-reduce(sends[i]), on the
        exchange's stream after the current one's queued work; sends are only
        read. (SMA's overlapped sum: the variables stay where they are, no copy
        of them is made first.)"""
        sends, recvs = list(sends), list(recvs)
        self._check(sends)
        self._check(recvs)
        if len(sends) != len(recvs) or any(a.numel() != b.numel() or a.dtype != b.dtype
                                           for a, b in zip(sends, recvs)):
            raise ValueError("sends and recvs must pair up in size and dtype")
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        cur = torch.cuda.current_stream(self.device)
        self._side.wait_stream(cur)
        self._issue(sends, op, average, self._side, recvs=recvs)
        ev = torch.cuda.Event()
        ev.record(self._side)
        for b in sends + recvs:
            b.record_stream(self._side)
        return _Handle(ev, self.device)

    def sma_(self, buckets, alpha):
        """SMA (sma_sgd.py:60-65) over flat variable buckets, in place."""
        buckets = list(buckets)
        if not buckets:
            return buckets
        self._check(buckets)
        key = tuple((b.data_ptr(), b.numel()) for b in buckets)
        sums = self._sums.get(key)
        if sums is None:
            from .collective import workspace_like
            sums = workspace_like(buckets)  # flat when the buckets are
            self._sums[key] = sums
        vp = [b.data_ptr() for b in buckets]
        sp = [s.data_ptr() for s in sums]
        rc = self.lib.kf_exchange_sma_batch(
            self._h, _lib.ptr_array(vp), _lib.ptr_array(sp),
            _arr(ctypes.c_size_t, [b.numel() for b in buckets]), len(buckets),
            int(kungfu_dtype(buckets[0])), float(alpha), ALGOS[self.algo],
            torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(rc, "kf_exchange_sma_batch")
        return buckets

    def all_reduce_named(self, name, buf, op="sum", average=False, stream=None, callback=None):
        """kf_exchange_all_reduce_named: in place, paired with the peers' calls
        of the same name whatever order each rank starts its names in
        (GoKungfuAllReduce with a done callback). callback(name, status) runs
        on the exchange's completion thread; wait_named() blocks for all."""
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        s = stream if stream is not None else torch.cuda.current_stream(buf.device)
        self._named_keep = getattr(self, "_named_keep", [])
        if callback is not None:
            def done(status, _arg):
                callback(name, status)
            cfn = _lib.DONE_FN(done)
            self._named_keep.append((cfn, buf))
        else:  # no callback: a NULL done (no Python call per completion)
            cfn = _NO_DONE
            self._named_keep.append(buf)
        rc = self.lib.kf_exchange_all_reduce_named(
            self._h, name.encode(), buf.data_ptr(), buf.data_ptr(), buf.numel(),
            int(kungfu_dtype(buf)), int(red), 1 if average else 0, ALGOS[self.algo],
            s.cuda_stream, cfn, None)
        _lib.check(rc, "kf_exchange_all_reduce_named")

    def wait_named(self):
        """Block until every name started so far completed; raise on failure."""
        rc = self.lib.kf_exchange_wait_named(self._h)
        self._named_keep = []
        _lib.check(rc, "kf_exchange_wait_named")

    def check(self):
        """Raise if RCCL reported an asynchronous error."""
        _lib.check(self.lib.kf_exchange_check(self._h), "kf_exchange_check")

    def finish(self):
        """RCCL and the HIP epilogues are stream-ordered, so nothing waits;
        an asynchronous RCCL error is raised here (the optimizers call this
        before their update)."""
        self.check()

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            self.lib.kf_exchange_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Handle:
    def __init__(self, ev, device):
        self.ev = ev
        self.device = device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.ev)


class Scheduler:
    """Ordered issue of all-reduces that become ready in any order — the
    reference's NCCLScheduler (srcs/cpp/src/nccl/scheduler.cpp:8-130) on
    kf_exchange_begin_step / kf_exchange_start. ``begin_step(names)`` fixes
    the step's names (same list on every rank); ``start(name, buf)`` may come
    in any order; the native thread issues them in the agreed order (with
    ``auto_order``, rank 0's arrival order of the first step from the second
    step on)."""

    def __init__(self, exchange, auto_order=True):
        self.ex = exchange
        self.auto_order = bool(auto_order)
        self._keep = []

    def begin_step(self, names):
        arr = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
        self.names = list(names)
        _lib.check(self.ex.lib.kf_exchange_begin_step(self.ex._h, arr, len(names),
                                                      1 if self.auto_order else 0),
                   "kf_exchange_begin_step")
        self._keep = []

    def start(self, name, buf, op="sum", average=False, stream=None, callback=None):
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        s = stream if stream is not None else torch.cuda.current_stream(buf.device)

        def done(status, _arg):
            if callback is not None:
                callback(name, status)

        cfn = _lib.DONE_FN(done)
        self._keep.append((cfn, buf))
        rc = self.ex.lib.kf_exchange_start(self.ex._h, name.encode(), buf.data_ptr(),
                                           buf.data_ptr(), buf.numel(), int(kungfu_dtype(buf)),
                                           int(red), 1 if average else 0,
                                           ALGOS[self.ex.algo], s.cuda_stream, cfn, None)
        _lib.check(rc, "kf_exchange_start")

    def wait_all(self):
        """Block until the step's all-reduces completed; returns the issue
        order (names)."""
        order = (ctypes.c_int32 * len(self.names))()
        rc = self.ex.lib.kf_exchange_wait_all(self.ex._h, order)
        _lib.check(rc, "kf_exchange_wait_all")
        return [self.names[i] for i in order]
