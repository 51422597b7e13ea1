"""Bucketed data-parallel all-reduce across the GPUs of a node.

What the reference does (per gradient tensor, on the host):
  AllReduce op -> Session.AllReduce -> 1 MiB chunks -> strategy graphs ->
  std_transform_2 per received chunk (session.go:231-326), then the optimizer
  divides by np in a separate TF op (sync_sgd.py:103-104) or blends
  (sma_sgd.py:60-65).

What this module does instead: gradients live in a few large
flat device buckets; each bucket is split evenly into one shard per rank and
  1. RCCL reduce-scatter (sum)  — each rank receives the sum of its shard
  2. HIP epilogue on the shard  — /np (S-SGD) via kf_bucket_div, bit-exact
                                  against "sum, then g / np"
  3. RCCL all-gather            — every rank gets the full reduced bucket
over xGMI, one process per GPU. Buckets are issued back to back so the
epilogue of bucket i overlaps the reduce-scatter of bucket i+1 (all RS on the
RCCL stream first, each AG queued behind its own epilogue).

For f16/bf16 (and float MIN/MAX) step 1 is instead an all-to-all of the
shards followed by the HIP k-input fold of the `world` received shards in rank
order (algo "a2a"): RCCL's reduce-scatter would add in its own order and, for
bf16, round to bf16 at every hop, while the build defines bf16 as fp32
accumulation with one rounding (the oracle's semantics and the P2P path's).
Same xGMI bytes as the reduce-scatter; the bits no longer depend on the
transport (kungfu_amd/csrc/kf_exchange.hip does the same natively).

The epilogue runs through ``kungfu_amd.ops`` (HIP kernels). It is injectable
only so the orchestration can be exercised over gloo on CPU in tests; the
product default is the HIP path and it raises on CPU tensors.
"""
import torch
import torch.distributed as dist

from . import ops
from .base import OP_NAMES, OP, EvenPartition

# Shards start on 256-byte boundaries so every shard pointer is 16-B aligned
# for the vector path and RCCL's preferred alignment.
ALIGN_BYTES = 256

_RED_OPS = {
    OP.SUM: dist.ReduceOp.SUM,
    OP.MIN: dist.ReduceOp.MIN,
    OP.MAX: dist.ReduceOp.MAX,
    OP.PROD: dist.ReduceOp.PRODUCT,
}


class HipEpilogue:
    """The shard epilogues as HIP kernels (default, product path)."""

    def div_(self, x, np_):
        return ops.bucket_div_(x, np_)

    def fold_(self, inputs, out, op, np_):
        """out = left fold of inputs (rank order); np_ > 0: SUM then / np_."""
        if np_:
            return ops.bucket_reduce_avg(inputs, np_, out=out)
        return ops.bucket_reduce(inputs, out=out, op=op)

    def sma_blend_(self, v, summed, np_, alpha):
        return ops.sma_blend_(v, summed, np_, alpha)


def coalesce_runs(buckets):
    """Maximal runs of buckets that are consecutive in one storage, each as
    one flat view."""
    runs, cur = [], []

    def flush():
        if not cur:
            return
        if len(cur) == 1:
            runs.append(cur[0])
        else:
            first = cur[0]
            n = sum(t.numel() for t in cur)
            runs.append(torch.empty(0, dtype=first.dtype, device=first.device).set_(
                first.untyped_storage(), first.storage_offset(), (n,)))
        cur.clear()

    for b in buckets:
        if cur:
            last = cur[-1]
            adjacent = (b.dtype == last.dtype and b.device == last.device and
                        b.untyped_storage().data_ptr() == last.untyped_storage().data_ptr() and
                        b.storage_offset() == last.storage_offset() + last.numel())
            if not adjacent:
                flush()
        cur.append(b)
    flush()
    return runs


def workspace_like(buckets):
    """One workspace tensor per bucket (e.g. SMA's sum of each variable
    bucket). When the buckets are one contiguous run (GradBuckets' flat
    layout), the workspaces are views of ONE flat allocation in the same
    order, so a kernel over (bucket, workspace) pairs sees two contiguous
    ranges and launches once over them (kf_sma_blend_batch merges such
    buckets)."""
    buckets = list(buckets)
    if len(buckets) > 1 and len(coalesce_runs(buckets)) == 1:
        flat = torch.empty(sum(b.numel() for b in buckets), dtype=buckets[0].dtype,
                           device=buckets[0].device)
        out, off = [], 0
        for b in buckets:
            out.append(flat[off:off + b.numel()].view_as(b))
            off += b.numel()
        return out
    return [torch.empty_like(b) for b in buckets]


def resolve_algo(algo, dtype, op, world):
    """"rs" (RCCL reduce-scatter) or "a2a" (all-to-all + HIP rank-order fold)
    for one bucket dtype; "auto" keeps RCCL's reduce-scatter where its order
    cannot change what the result means (integers; f32/f64, the north_star's
    path; for MIN/MAX only NaN inputs could select differently) and folds on
    the GPU where the build defines the arithmetic: f16 (per-hop rounding) and
    bf16 (fp32 accumulation, one rounding) — kf_exchange.hip resolve_algo."""
    if algo in ("rs", "a2a"):
        return algo
    if algo != "auto":
        raise ValueError("algo must be 'auto', 'rs' or 'a2a'")
    own = dtype in (torch.float16, torch.bfloat16)
    return "a2a" if own and world <= 16 else "rs"


def padded_count(count, world, itemsize):
    """Smallest length >= count that splits into `world` aligned shards."""
    unit = world * max(1, ALIGN_BYTES // itemsize)
    return ((count + unit - 1) // unit) * unit


PHASES = ("reduce_scatter", "epilogue", "all_gather", "blend")


class _PhaseClock:
    """Per-phase timing of the calls in a window (Exchange.set_timing): timing
    events on the current stream at every point where it moves from one phase
    to the next, so the segments partition the stream's time from a call's
    first launch to its last wait. A segment counts for the phase that ends
    at its closing mark: waiting on a reduce-scatter (or all-to-all) is
    phase 1, the HIP shard work phase 2, waiting on the all-gathers phase 3."""

    def __init__(self):
        self.calls = []

    def begin(self):
        marks = []
        self.calls.append(marks)
        self.mark(marks, "start")
        return marks

    @staticmethod
    def mark(marks, label):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((label, ev))

    def sums(self):
        out = dict.fromkeys(PHASES, 0.0)
        for marks in self.calls:
            marks[-1][1].synchronize()
            for (_, a), (label, b) in zip(marks, marks[1:]):
                out[label] += 1e3 * a.elapsed_time(b)
        out["calls"] = len(self.calls)
        out["untimed_calls"] = 0
        return out


class Exchange:
    """One process group, its shard workspaces and the epilogue."""

    def __init__(self, group=None, epilogue=None, algo="auto"):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.epilogue = epilogue if epilogue is not None else HipEpilogue()
        self.algo = algo
        resolve_algo(algo, torch.float32, OP.SUM, self.world)  # validates
        self._ws = {}
        self._clock = None

    def set_timing(self, on):
        """Start (zeroed) or stop the per-phase timing window (the native
        exchange's kf_exchange_set_timing, for this path)."""
        self._clock = _PhaseClock() if on else None

    def phase_times(self):
        """The window's per-phase sums in us (PHASES) and the timed calls."""
        if self._clock is None:
            return dict(dict.fromkeys(PHASES, 0.0), calls=0, untimed_calls=0)
        return self._clock.sums()

    def _marks(self):
        return self._clock.begin() if self._clock is not None else None

    @staticmethod
    def _mark(marks, label):
        if marks is not None:
            _PhaseClock.mark(marks, label)

    def _workspace(self, key, n, like):
        t = self._ws.get(key)
        if t is None or t.numel() < n or t.dtype != like.dtype or t.device != like.device:
            t = torch.empty(n, dtype=like.dtype, device=like.device)
            self._ws[key] = t
        return t[:n]

    def _check(self, buf):
        if buf.dim() != 1 or not buf.is_contiguous():
            raise ValueError("bucket must be a flat contiguous tensor")
        if buf.numel() % self.world:
            raise ValueError("bucket length %d not divisible by world %d; use "
                             "padded_count()" % (buf.numel(), self.world))

    def all_reduce_(self, buckets, op="sum", average=False, coalesce=True):
        """In-place all-reduce of flat padded buckets. average=True applies the
        S-SGD epilogue (sum, then / np) on each shard.

        coalesce=True merges buckets that lie back to back in one storage
        (GradBuckets(n_buckets=k) lays them out that way) into one
        reduce-scatter -> epilogue -> all-gather run: the same values with
        one RCCL launch pair instead of one per bucket — the fusion the
        reference's S-SGD applies to ready gradients (nccl_fusion,
        sync_sgd.py:87-92). Buckets handed over one call at a time (e.g. as
        backward produces them) are reduced as they come."""
        self.start_(buckets, op=op, average=average, coalesce=coalesce).wait()
        return buckets

    def start_(self, buckets, op="sum", average=False, coalesce=True, key="ar"):
        """Queue the all-reduce of `buckets` and return a handle whose wait()
        completes it. With RCCL nothing here blocks the host: each shard
        epilogue is ordered behind its reduce-scatter on the device, and each
        all-gather behind its epilogue, so this can be called from a backward
        hook while later gradients are still being computed. Concurrent calls
        must use different `key`s (their shard workspaces)."""
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        if average and red != OP.SUM:
            raise ValueError("average requires op='sum'")
        for b in buckets:
            self._check(b)
        if self.world == 1:
            # a single peer: the reduce is the identity; g / 1 == g exactly
            return _Handle([])
        if coalesce:
            runs = coalesce_runs(buckets)
            if len(runs) < len(buckets):
                return self.start_(runs, op=op, average=average, coalesce=False, key=key)
        marks = self._marks()
        shards = []
        works = []
        for i, b in enumerate(buckets):
            shard = self._workspace((key, "rs", i), b.numel() // self.world, b)
            works.append(self._scatter(b, shard, red, (key, "a2a", i)))
            shards.append(shard)
        gathers = []
        for b, shard, (w, recv) in zip(buckets, shards, works):
            w.wait()
            self._mark(marks, "reduce_scatter")
            if recv is not None:  # the rank-order fold of the received shards
                self.epilogue.fold_(list(recv.chunk(self.world)), shard, red,
                                    self.world if average else 0)
            elif average:
                self.epilogue.div_(shard, self.world)
            self._mark(marks, "epilogue")
            gathers.append(dist.all_gather_into_tensor(b, shard, group=self.group,
                                                       async_op=True))
        return _Handle(gathers, None if marks is None else
                       (lambda: _PhaseClock.mark(marks, "all_gather")))

    def _scatter(self, b, shard, red, key):
        """Step 1 for one bucket: (work, None) for RCCL's reduce-scatter into
        `shard`, or (work, recv) for the all-to-all whose `recv` holds the
        `world` shards (rank order) still to be folded."""
        if resolve_algo(self.algo, b.dtype, red, self.world) == "rs":
            return (dist.reduce_scatter_tensor(shard, b, op=_RED_OPS[red], group=self.group,
                                               async_op=True), None)
        recv = self._workspace(key, b.numel(), b)
        return dist.all_to_all_single(recv, b, group=self.group, async_op=True), recv

    def sma_(self, buckets, alpha):
        """SMA over flat variable buckets (sma_sgd.py:60-65): each rank's v
        becomes (1-alpha) v + alpha * (sum_ranks v) / np."""
        for b in buckets:
            self._check(b)
        sums = []
        if self.world == 1:
            for i, b in enumerate(buckets):
                s = self._workspace(("sum", i), b.numel(), b)
                s.copy_(b)
                sums.append(s)
            for b, s in zip(buckets, sums):
                self.epilogue.sma_blend_(b, s, self.world, alpha)
            return buckets
        # pipelined: every reduce-scatter is queued first, each all-gather
        # right behind its reduce-scatter, and each bucket's blend waits only
        # for its own all-gather, so blends overlap later buckets' transfers.
        # The reduce-scatter reads v before any blend of that bucket runs.
        marks = self._marks()
        rs = []
        for i, b in enumerate(buckets):
            shard = self._workspace(("rs", i), b.numel() // self.world, b)
            rs.append((shard, self._scatter(b, shard, OP.SUM, ("a2a", i))))
        ags = []
        for i, (b, (shard, (w, recv))) in enumerate(zip(buckets, rs)):
            w.wait()
            self._mark(marks, "reduce_scatter")
            if recv is not None:
                self.epilogue.fold_(list(recv.chunk(self.world)), shard, OP.SUM, 0)
                self._mark(marks, "epilogue")
            s = self._workspace(("sum", i), b.numel(), b)
            ags.append((s, dist.all_gather_into_tensor(s, shard, group=self.group,
                                                       async_op=True)))
        for b, (s, w) in zip(buckets, ags):
            w.wait()
            self._mark(marks, "all_gather")
            self.epilogue.sma_blend_(b, s, self.world, alpha)
            self._mark(marks, "blend")
        return buckets


class _Handle:
    """Pending collectives of one start_() call."""

    def __init__(self, works, on_done=None):
        self.works = works
        self.on_done = on_done

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []
        if self.on_done is not None:
            self.on_done()
            self.on_done = None


class GradBuckets:
    """Flat, padded device storage for a list of same-dtype tensors.

    Two layouts:
      * ``bucket_bytes`` (default): tensors are grouped, in order, into buckets
        of about that size at tensor boundaries (a larger tensor gets a bucket
        of its own); each bucket is its own flat buffer, padded to split into
        ``world`` aligned shards.
      * ``n_buckets=k``: all tensors are laid out back to back in ONE flat
        buffer, which is cut into k contiguous buckets by EvenPartition
        (interval.go:12-27) of its aligned units — tensors may straddle bucket
        boundaries (the reduce is element-wise). This is SURVEY §8(a) C4:
        ResNet-50's 25,583,592 fp32 in 16 buckets of ~1.6 M elements.
    ``views[i]`` is tensor i's view into the flat storage, so gradients can be
    written in place and reduced without fuse/defuse copies (the reference's
    NCCL path concatenates and slices instead, ops/__init__.py:29-46).
    ``spans[j]`` is the number of real (non-padding) elements of bucket j,
    which always precede its padding.
    """

    def __init__(self, numels, dtype, device, world, bucket_bytes=32 << 20,
                 n_buckets=None):
        itemsize = torch.empty((), dtype=dtype).element_size()
        self.buckets, self.views, self.spans, self.flats = [], [None] * len(numels), [], []
        if n_buckets is not None:
            total = sum(numels)
            unit = world * max(1, ALIGN_BYTES // itemsize)
            units = max(1, (total + unit - 1) // unit)
            flat = torch.zeros(units * unit, dtype=dtype, device=device)
            self.flats.append(flat)
            off = 0
            for i, n in enumerate(numels):
                self.views[i] = flat[off:off + n]
                off += n
            for ub, ue in EvenPartition(0, units, min(n_buckets, units)):
                b, e = ub * unit, ue * unit
                self.buckets.append(flat[b:e])
                self.spans.append(max(0, min(e, total) - b))
            return
        for g in self._groups_greedy(numels, max(1, bucket_bytes // itemsize)):
            count = sum(numels[i] for i in g)
            b = torch.zeros(padded_count(max(count, 1), world, itemsize),
                            dtype=dtype, device=device)
            off = 0
            for i in g:
                self.views[i] = b[off:off + numels[i]]
                off += numels[i]
            self.flats.append(b)
            self.buckets.append(b)
            self.spans.append(count)

    @staticmethod
    def _groups_greedy(numels, cap):
        groups, cur, size = [], [], 0
        for i, n in enumerate(numels):
            if cur and size + n > cap:
                groups.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += n
        if cur:
            groups.append(cur)
        return groups


def group_all_reduce(tensors, op="sum", average=False, exchange=None,
                     bucket_bytes=32 << 20):
    """Mirror of the reference's group_all_reduce (ops/collective.py:71-73):
    returns all-reduced copies of `tensors`. Fuses them into flat buckets
    (copy in, reduce, copy out); optimizers that own their gradient storage
    use GradBuckets directly and skip the copies."""
    ex = exchange or Exchange()
    if not tensors:
        return []
    by_dtype = {}
    for i, t in enumerate(tensors):
        by_dtype.setdefault((t.dtype, t.device), []).append(i)
    out = [None] * len(tensors)
    for (dtype, device), idx in by_dtype.items():
        gb = GradBuckets([tensors[i].numel() for i in idx], dtype, device,
                         ex.world, bucket_bytes=bucket_bytes)
        for j, i in enumerate(idx):
            gb.views[j].copy_(tensors[i].reshape(-1))
        ex.all_reduce_(gb.buckets, op=op, average=average)
        for j, i in enumerate(idx):
            out[i] = gb.views[j].view_as(tensors[i]).clone()
    return out


def all_reduce(t, op="sum", exchange=None):
    """Mirror of all_reduce(t, op) (ops/collective.py:22-24)."""
    return group_all_reduce([t], op=op, exchange=exchange)[0]
