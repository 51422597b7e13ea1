"""All-reduce of persistent device buckets over xGMI peer mappings (no RCCL).

Every rank maps every peer's bucket (HIP IPC, kf_ipc_export / kf_ipc_import)
once. One all-reduce is then:

  1. barrier                      — every rank's gradients are written;
  2. reduce my shard              — the k-input HIP fold reads shard `rank`
                                    of all `world` buckets straight from the
                                    peers' HBM over their xGMI links, in rank
                                    order, and writes it (with the S-SGD /np
                                    epilogue fused) into my own bucket; the
                                    loads of all peers are in flight together
                                    (kf_bucket_reduce_peers) so every link
                                    carries traffic at once;
  3. barrier                      — every shard is reduced;
  4. gather the other shards      — one kernel pulls shard r from rank r's
                                    bucket for every r != rank, consecutive
                                    blocks on different peers;
  5. barrier                      — nobody rewrites a bucket a peer still reads.

The fold order is fixed (rank 0, 1, ..., n-1), so results are deterministic and
equal the oracle's reduce_avg over the ranks in order, bit for bit, for every
world size — unlike a ring/tree collective whose order depends on the shard.
On a fully connected 8-GPU MI355X node each phase spreads its reads over all 7
links. Experimental in round 1: bench.py reports it beside the RCCL path
(``c3_p2p``); DESIGN.md §6.

mode="push" moves the same bytes as remote WRITES instead of reads (posted
over the fabric, no round trip per request), through a per-bucket inbox of
`world` shard slots:

  1. scatter   — one kernel writes my shard j of every bucket into rank j's
                 inbox slot `rank`, for every j != rank (kf_copy_segments);
  2. barrier   — every push into my inbox has landed;
  3. reduce    — the k-input fold over (inbox slot j, or my own shard for
                 j == rank) in rank order, /np fused, into my shard — local
                 HBM only;
  4. all-gather — one kernel writes my reduced shard into every peer's
                 bucket at offset `rank`;
  5. barrier   — every peer's shard has landed in my bucket.

Two barriers instead of three: the scatter reads only local data, and the
previous call's last barrier already ordered every peer's fold (its inbox
reads) before this call's pushes. Same rank-order fold, so the same bits as
mode="pull". Extra HBM: one inbox per bucket ((world-1)/world of it used).

barrier="device" (default) runs every barrier on the GPU, in stream order
(kf_peer_barrier): one workgroup stores the barrier's epoch into each peer's
signal array over xGMI (fine-grained, uncached memory mapped like the
buckets) and spins on its own until every peer has arrived. No host sync and
no RCCL round trip, so a whole all-reduce is queued without blocking the host.
The wait is bounded (timeout_s, 60 s by default: a peer may legitimately
still be in its forward/backward pass): a peer that never arrives makes the barrier
record KF_ERR_TIMEOUT in a host-visible status word, which the next call (or
check()) raises. barrier="host" is the torch.cuda.synchronize() +
dist.barrier() of the first version, kept for comparison.
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from .ops import kungfu_dtype


def _device_identity(dev):
    """(host, PCI domain/bus/device) of a GPU, or None when torch does not
    report the PCI location (every peer is then treated as remote)."""
    import socket
    p = torch.cuda.get_device_properties(dev)
    pci = tuple(getattr(p, a, None) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if any(x is None for x in pci):
        return None
    return (socket.gethostname(), pci)


class P2PExchange:
    def __init__(self, buckets, group=None, mode="pull", barrier="device", timeout_s=60.0,
                 coalesce=True):
        if mode not in ("pull", "push"):
            raise ValueError("mode must be 'pull' or 'push'")
        if barrier not in ("device", "host"):
            raise ValueError("barrier must be 'device' or 'host'")
        self.mode = mode
        self.barrier = barrier
        self.timeout_us = int(timeout_s * 1e6)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.lib = _lib.load()
        self.given = list(buckets)
        # buckets that lie back to back in one storage are exchanged as one:
        # every element's result is the same rank-order fold whichever rank
        # owns its shard, so the bits do not change, and a run costs one fold
        # and one gather launch instead of one per bucket
        from .collective import coalesce_runs
        self.buckets = coalesce_runs(self.given) if coalesce else list(self.given)
        for b in self.buckets:
            if not b.is_cuda or b.dim() != 1 or not b.is_contiguous():
                raise ValueError("P2P buckets must be flat contiguous GPU tensors")
            if b.numel() % self.world or (b.numel() // self.world * b.element_size()) % 16:
                raise ValueError("bucket does not split into 16-B aligned shards")
        # push mode: one inbox of `world` shard slots per bucket (slot `rank`
        # unused: my own shard is read in place)
        self.inboxes = ([torch.empty_like(b) for b in self.buckets]
                        if mode == "push" else [])
        self._bases = {}  # (rank, handle) -> mapped base (one mapping per allocation)
        # Peers whose buckets live on THIS device (ranks sharing one GPU) are
        # read from local HBM: the pull fold then takes the register-shape
        # kernel (kf_bucket_reduce, 0.76 of the roofline at k = 8) rather than
        # the all-loads-in-flight link spreader (kf_bucket_reduce_peers, 0.72
        # locally), which exists for inputs behind different xGMI links. Both
        # are the same rank-order left fold, bit for bit.
        ids = [None] * self.world
        dist.all_gather_object(ids, _device_identity(self.buckets[0].device)
                               if self.buckets else None, group=self.group)
        self.all_local = ids[0] is not None and all(i == ids[0] for i in ids)
        self.ptrs = self._share([b.data_ptr() for b in self.buckets])  # ptrs[j][r]: bucket j of rank r
        self.inbox_ptrs = self._share([b.data_ptr() for b in self.inboxes])  # same for inboxes
        self.epoch = 0
        self._sig = self._status = None
        if barrier == "device":
            sig, st = ctypes.c_void_p(), ctypes.c_void_p()
            _lib.check(self.lib.kf_signal_alloc(64, 0, ctypes.byref(sig)), "kf_signal_alloc")
            self._sig = sig.value
            _lib.check(self.lib.kf_signal_alloc(1, 1, ctypes.byref(st)), "kf_signal_alloc")
            self._status = st.value
            self.sig_ptrs = _lib.ptr_array(self._share([self._sig])[0])

    def _share(self, ptrs):
        """Export my allocations, import every peer's: rows[j][r] = address of
        rank r's buffer j as seen from this process."""
        mine = []
        for p in ptrs:
            h = (ctypes.c_char * 64)()
            off = ctypes.c_size_t()
            _lib.check(self.lib.kf_ipc_export(p, h, ctypes.byref(off)), "kf_ipc_export")
            mine.append((bytes(h), off.value))
        everyone = [None] * self.world
        dist.all_gather_object(everyone, mine, group=self.group)
        rows = []
        for j, p in enumerate(ptrs):
            row = []
            for r in range(self.world):
                if r == self.rank:
                    row.append(p)
                    continue
                h, off = everyone[r][j]
                key = (r, h)
                if key not in self._bases:
                    base = ctypes.c_void_p()
                    _lib.check(self.lib.kf_ipc_import(h, ctypes.byref(base)), "kf_ipc_import")
                    self._bases[key] = base.value
                row.append(self._bases[key] + off)
            rows.append(row)
        return rows

    def close(self):
        torch.cuda.synchronize()
        for base in self._bases.values():
            self.lib.kf_ipc_close(base)
        self._bases = {}
        if self._sig is not None:
            # every peer's store into my array landed before my last barrier
            # returned, and no peer reads it: free once my stream is idle
            self.lib.kf_signal_free(self._sig, 0)
            self.lib.kf_signal_free(self._status, 1)
            self._sig = self._status = None

    def status(self):
        """KF_OK, or KF_ERR_TIMEOUT once a device barrier gave up (no sync)."""
        if self._status is None:
            return 0
        return ctypes.c_uint64.from_address(self._status).value

    def check(self):
        st = self.status()
        if st:
            raise _lib.KungFuAMDError("P2P device barrier: %s after %.1f s (a peer never "
                                      "arrived)" % (_lib.STATUS.get(st, st),
                                                    self.timeout_us / 1e6))

    def finish(self):
        """Wait for the queued exchange and raise if one of its barriers gave
        up. A timed-out barrier lets the fold and gather behind it run on peer
        buffers nobody synchronised, so a result must not be used before this
        returns (the optimizers call it before their update)."""
        torch.cuda.current_stream().synchronize()
        self.check()

    def _barrier(self):
        if self.barrier == "host":
            torch.cuda.synchronize()
            dist.barrier(group=self.group)
            return
        self.epoch += 1
        s = torch.cuda.current_stream().cuda_stream
        _lib.check(self.lib.kf_peer_barrier(self.sig_ptrs, self.world, self.rank, self.epoch,
                                            self.timeout_us, self._status, s),
                   "kf_peer_barrier")

    def all_reduce_(self, op="sum", average=False):
        """In place on the buckets given at construction."""
        self.check()
        if self.mode == "push":
            return self._all_reduce_push(op, average)
        from .base import OP_NAMES
        world, rank = self.world, self.rank
        s = torch.cuda.current_stream().cuda_stream
        self._barrier()
        for b, row in zip(self.buckets, self.ptrs):
            isz = b.element_size()
            shard = b.numel() // world
            off = rank * shard * isz
            ins = _lib.ptr_array([p + off for p in row])
            out = b.data_ptr() + off
            dt = int(kungfu_dtype(b))
            if self.all_local:
                rc = (self.lib.kf_bucket_reduce_avg(ins, world, out, shard, dt, world, s)
                      if average else
                      self.lib.kf_bucket_reduce(ins, world, out, shard, dt, int(OP_NAMES[op]), s))
            else:
                # every peer's load in flight at once (all links busy), adds
                # in rank order
                rc = self.lib.kf_bucket_reduce_peers(ins, world, out, shard, dt,
                                                     int(OP_NAMES[op]), world if average else 0, s)
            _lib.check(rc, "p2p shard reduce")
        self._barrier()
        for b, row in zip(self.buckets, self.ptrs):
            isz = b.element_size()
            nbytes = b.numel() // world * isz
            peers = [r for r in range(world) if r != rank]
            srcs = _lib.ptr_array([row[r] for r in peers])
            offs = (ctypes.c_size_t * len(peers))(*[r * nbytes for r in peers])
            lens = (ctypes.c_size_t * len(peers))(*[nbytes] * len(peers))
            _lib.check(self.lib.kf_gather_segments(b.data_ptr(), srcs, offs, lens,
                                                   len(peers), s), "kf_gather_segments")
        self._barrier()
        return self.given

    def _all_reduce_push(self, op, average):
        from .base import OP_NAMES
        world, rank = self.world, self.rank
        s = torch.cuda.current_stream().cuda_stream
        peers = [r for r in range(world) if r != rank]

        def copy(dsts, srcs, nbytes):
            _lib.check(self.lib.kf_copy_segments(
                _lib.ptr_array(dsts), _lib.ptr_array(srcs),
                (ctypes.c_size_t * len(dsts))(*[nbytes] * len(dsts)), len(dsts), s),
                "kf_copy_segments")

        for b, ibox in zip(self.buckets, self.inbox_ptrs):
            nbytes = b.numel() // world * b.element_size()
            # my shard j -> rank j's inbox slot `rank`
            copy([ibox[r] + rank * nbytes for r in peers],
                 [b.data_ptr() + r * nbytes for r in peers], nbytes)
        self._barrier()
        for b, ib in zip(self.buckets, self.inboxes):
            shard = b.numel() // world
            nbytes = shard * b.element_size()
            mine = b.data_ptr() + rank * nbytes
            ins = _lib.ptr_array([mine if r == rank else ib.data_ptr() + r * nbytes
                                  for r in range(world)])
            if average:
                rc = self.lib.kf_bucket_reduce_avg(ins, world, mine, shard,
                                                   int(kungfu_dtype(b)), world, s)
            else:
                rc = self.lib.kf_bucket_reduce(ins, world, mine, shard, int(kungfu_dtype(b)),
                                               int(OP_NAMES[op]), s)
            _lib.check(rc, "p2p shard reduce")
        for b, row in zip(self.buckets, self.ptrs):
            nbytes = b.numel() // world * b.element_size()
            # my reduced shard -> every peer's bucket at offset `rank`
            copy([row[r] + rank * nbytes for r in peers],
                 [b.data_ptr() + rank * nbytes] * len(peers), nbytes)
        self._barrier()
        return self.given


class PeerExchange:
    """The optimizers' exchange interface (``all_reduce_(buckets, op, average)``,
    ``sma_(buckets, alpha)``, ``world``; see collective.Exchange) over
    P2PExchange, so ``SynchronousSGDOptimizer(opt, exchange=PeerExchange())``
    and ``SynchronousAveragingOptimizer(...)`` reduce over xGMI peer mappings
    instead of RCCL.

    The optimizers hand over the same persistent buckets every step
    (collective.GradBuckets), so each distinct bucket list is mapped once (a
    collective call: every rank meets the same lists in the same order) and
    reused. Results are the rank-order fold, bit-identical at every world
    size. SMA sums into a persistent workspace copy of the variables, then
    runs the fused blend (sma_sgd.py:60-65)."""

    def __init__(self, group=None, mode="pull", barrier="device", timeout_s=60.0):
        from .collective import HipEpilogue
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.kw = dict(mode=mode, barrier=barrier, timeout_s=timeout_s)
        self.epilogue = HipEpilogue()
        self._ex = {}
        self._sums = {}

    def _get(self, buckets):
        key = tuple((b.data_ptr(), b.numel(), b.dtype) for b in buckets)
        ex = self._ex.get(key)
        if ex is None:
            ex = P2PExchange(buckets, group=self.group, **self.kw)
            self._ex[key] = ex
        return ex

    def all_reduce_(self, buckets, op="sum", average=False, coalesce=True):
        buckets = list(buckets)
        if average and op != "sum":
            raise ValueError("average requires op='sum'")
        if self.world > 1:
            self._get(buckets).all_reduce_(op=op, average=average)
        return buckets

    def sma_(self, buckets, alpha):
        from .collective import coalesce_runs
        runs = coalesce_runs(list(buckets))  # copy and blend once per run
        key = tuple(b.data_ptr() for b in runs)
        sums = self._sums.get(key)
        if sums is None:
            if all(b.dtype == runs[0].dtype and b.device == runs[0].device for b in runs):
                # one flat workspace laid out like the runs, so the P2P sum
                # of it is a single run as well
                flat = torch.empty(sum(b.numel() for b in runs), dtype=runs[0].dtype,
                                   device=runs[0].device)
                sums, off = [], 0
                for b in runs:
                    sums.append(flat[off:off + b.numel()])
                    off += b.numel()
            else:
                sums = [torch.empty_like(b) for b in runs]
            self._sums[key] = sums
        for s, b in zip(sums, runs):
            s.copy_(b)
        if self.world > 1:
            self._get(sums).all_reduce_(op="sum")
        for b, s in zip(runs, sums):
            self.epilogue.sma_blend_(b, s, self.world, alpha)
        return list(buckets)

    def finish(self):
        for ex in self._ex.values():
            ex.finish()

    def close(self):
        for ex in self._ex.values():
            ex.close()
        self._ex = {}


def _same_host(group=None):
    """True when every rank of the group runs on this host (the P2P exchange
    maps peers' HBM through HIP IPC, which only reaches the node's GPUs)."""
    import socket
    names = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, socket.gethostname(), group=group)
    return len(set(names)) == 1


class AutoExchange:
    """Exchange that picks, per bucket list, the fastest of candidates that
    give the SAME bits, by timing them on the real buckets the first time it
    sees them — the way RCCL itself tunes its algorithm per size, lifted one
    level. The candidates are RCCL's all-to-all + HIP rank-order fold, through
    torch.distributed (collective.Exchange(algo="a2a")) and through the native
    C-ABI exchange (exchange.NativeExchange(algo="a2a"), nccl backend only),
    and the xGMI P2P exchange (PeerExchange), which all fold the ranks in order
    0..n-1 with the same kernel; RCCL's
    reduce-scatter joins them only where its own order cannot change a bit
    (integer dtypes; two ranks summing f32/f64). So the result never depends
    on which transport won on a given box.

    "Same bits" is checked, not assumed: every candidate's warm-up starts from
    the same snapshot of the buckets, and its result is compared bit for bit
    with the first candidate's (rank-agreed: a mismatch on any rank drops the
    candidate on every rank, and the rank, the candidate, the bucket and the
    first differing element are printed to stderr). So a transport that
    returns a stale or wrong shard on some node (the P2P push
    mode's cross-device coherence) is never adopted, however fast it is.

    The trial runs `trials` exchanges with each candidate on the buckets, then
    restores their contents from the snapshot, so the first call returns the
    same values as any later one. The choice is rank-agreed (the slowest
    rank's time decides), so every rank keeps issuing the same collectives.
    P2P is a candidate only for GPU buckets with every rank on one host; if
    its setup fails on any rank, RCCL is used. Past KF_MAX_INPUTS (16) ranks
    the rank-order fold cannot run, and RCCL's reduce-scatter is the only
    candidate. `extra` adds (name, exchange) candidates a host offers (its own
    transport, say); they are held to the same check. ``picked`` maps each
    bucket list (by address) to the winner's name; ``dropped`` lists
    (candidate, reason) of those that failed or differed."""

    def __init__(self, group=None, trials=3, mode="pull", epilogue=None, extra=()):
        from .collective import Exchange, HipEpilogue
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.trials = int(trials)
        self.epilogue = epilogue if epilogue is not None else HipEpilogue()
        self.rccl = Exchange(group, epilogue=self.epilogue, algo="a2a")
        self.rccl_rs = Exchange(group, epilogue=self.epilogue, algo="rs")
        self.mode = mode
        self._p2p = None
        self._host_ok = None
        self._native, self._native_tried = None, False
        self.picked = {}
        self.dropped = []
        self.extra = list(extra)
        self._choice = {}

    def _p2p_candidate(self, buckets):
        if self.world == 1 or not all(b.is_cuda for b in buckets):
            return None
        if self._host_ok is None:
            self._host_ok = _same_host(self.group)
        if not self._host_ok:
            return None
        if self._p2p is None:
            self._p2p = PeerExchange(self.group, mode=self.mode)
        return self._p2p

    def _native_candidate(self, buckets):
        """The native C-ABI exchange with the all-to-all + rank-order fold
        (kungfu_amd.exchange.NativeExchange(algo="a2a")): the same bits as the
        other candidates, one call per step. Needs RCCL with one GPU per rank
        (the nccl backend); created once, dropped on every rank if any fails."""
        if (self.world == 1 or not all(b.is_cuda for b in buckets)
                or dist.get_backend(self.group) != "nccl"):
            return None
        if not self._native_tried:
            self._native_tried = True
            nx, ok = None, True
            try:
                from .exchange import NativeExchange
                nx = NativeExchange(self.group, algo="a2a")
            except Exception as e:
                import sys
                print("kungfu_amd AutoExchange: native exchange unavailable on rank %d: %r"
                      % (self.rank, e), file=sys.stderr)
                ok = False
            if not self._agree_all(ok):
                if nx is not None:
                    nx.close()
                nx = None
            self._native = nx
        return self._native

    def _agree_all(self, flag):
        flags = [None] * self.world
        dist.all_gather_object(flags, bool(flag), group=self.group)
        return all(flags)

    def _rs_exact(self, buckets, op):
        """RCCL's reduce-scatter gives the rank-order bits: integer sums and
        selects in any order, or a single addition of two f32/f64 values."""
        if all(not b.dtype.is_floating_point for b in buckets):
            return True
        return (self.world == 2 and op == "sum" and
                all(b.dtype in (torch.float32, torch.float64) for b in buckets))

    def _candidates(self, buckets, op):
        from ._lib import MAX_INPUTS
        if self.world > MAX_INPUTS:  # no rank-order fold of more than 16 inputs
            return [("rccl_rs", self.rccl_rs)] + self.extra
        cands = [("rccl", self.rccl)]
        if self._rs_exact(buckets, op):
            cands.append(("rccl_rs", self.rccl_rs))
        native = self._native_candidate(buckets)
        if native is not None:
            cands.append(("native", native))
        p2p = self._p2p_candidate(buckets)
        if p2p is not None:
            cands.append(("p2p", p2p))
        return cands + self.extra

    def _drop(self, name, why):
        import sys
        self.dropped.append((name, why))
        print("kungfu_amd AutoExchange: rank %d drops candidate %s: %s" % (self.rank, name, why),
              file=sys.stderr)

    @staticmethod
    def _first_difference(ref, res):
        """None if every bucket holds the same bytes, else (bucket, element)."""
        for j, (a, b) in enumerate(zip(ref, res)):
            x, y = a.reshape(-1).view(torch.uint8), b.reshape(-1).view(torch.uint8)
            if not torch.equal(x, y):
                byte = int((x != y).nonzero()[0])
                return j, byte // a.element_size()
        return None

    def _pick(self, buckets, step, op="sum"):
        import time
        key = tuple((b.data_ptr(), b.numel(), b.dtype) for b in buckets)
        ex = self._choice.get(key)
        if ex is not None:
            return ex
        cands = self._candidates(buckets, op)
        on_gpu = any(b.is_cuda for b in buckets)

        def sync():
            if on_gpu:
                torch.cuda.synchronize()

        if len(cands) > 1:
            snap = [b.clone() for b in buckets]
            times, ref = [], None
            for name, cand in cands:
                for b, s in zip(buckets, snap):  # every warm-up from the same inputs
                    b.copy_(s)
                ok = True
                try:
                    step(cand)  # warm-up; maps the buckets for P2P
                    sync()
                    if hasattr(cand, "finish"):
                        cand.finish()
                except Exception as e:  # say why; the other candidates still run
                    self._drop(name, "failed: %r" % (e,))
                    ok = False
                if not self._agree_all(ok):
                    times.append(float("inf"))
                    continue
                if ref is None:  # the first candidate that ran everywhere is the reference
                    ref, ref_name = [b.clone() for b in buckets], name
                else:
                    diff = self._first_difference(ref, buckets)
                    if diff is not None:
                        self._drop(name, "result differs from %s's in bucket %d at element %d"
                                   % (ref_name, diff[0], diff[1]))
                    if not self._agree_all(diff is None):
                        if diff is None:
                            self.dropped.append((name, "differs on another rank"))
                        times.append(float("inf"))
                        continue
                dist.barrier(group=self.group)
                t0 = time.perf_counter()
                for _ in range(self.trials):
                    step(cand)
                sync()
                times.append(time.perf_counter() - t0)
                if hasattr(cand, "finish"):
                    cand.finish()
            every = [None] * self.world
            dist.all_gather_object(every, times, group=self.group)
            worst = [max(t[i] for t in every) for i in range(len(cands))]
            best = min(range(len(cands)), key=lambda i: worst[i])
            for b, s in zip(buckets, snap):
                b.copy_(s)
            del snap, ref
            if worst[best] == float("inf"):
                from ._lib import KungFuAMDError
                raise KungFuAMDError("AutoExchange: no candidate ran on every rank (%s)"
                                     % self.dropped)
        else:
            best = 0
        self.picked[key] = cands[best][0]
        self._choice[key] = cands[best][1]
        return cands[best][1]

    def all_reduce_(self, buckets, op="sum", average=False, coalesce=True):
        buckets = list(buckets)
        if self.world == 1:
            return self.rccl.all_reduce_(buckets, op=op, average=average)
        ex = self._pick(buckets, lambda e: e.all_reduce_(buckets, op=op, average=average), op)
        ex.all_reduce_(buckets, op=op, average=average)
        return buckets

    def finish(self):
        if self._p2p is not None:
            self._p2p.finish()

    def sma_(self, buckets, alpha):
        buckets = list(buckets)
        if self.world == 1:
            return self.rccl.sma_(buckets, alpha)
        ex = self._pick(buckets, lambda e: e.sma_(buckets, alpha))
        ex.sma_(buckets, alpha)
        return buckets

    def close(self):
        if self._p2p is not None:
            self._p2p.close()
        if self._native is not None:
            self._native.close()
