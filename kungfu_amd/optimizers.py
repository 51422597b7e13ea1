"""Synchronous data-parallel optimizers whose gradient/variable reduction runs on
the MI355X bucket path (RCCL reduce-scatter + HIP epilogue + RCCL all-gather).

Operator surface kept from the reference:

* ``SynchronousSGDOptimizer(optimizer, named_parameters=None, op=None, ...)``
  — torch signature of srcs/python/kungfu/torch/optimizers/sync_sgd.py:31-34
  (wraps an optimizer instance, reduces every gradient in ``step()``). The
  arithmetic is that of the TF S-SGD (sync_sgd.py:78-109): all-reduce-sum of
  each gradient, then ``g / np`` — here fused into the shard epilogue and
  bit-exact against "sum, then divide". ``average=False`` gives the torch
  reference's sum-only behaviour (torch/optimizers/sync_sgd.py:12-22).
* ``SynchronousAveragingOptimizer(optimizer, named_parameters=None, alpha=0.1)``
  — SMA (sma_sgd.py:9-74): before the local update every variable with a
  gradient becomes ``(1 - alpha) * v + alpha * allreduce_sum(v) / np``.

Buckets: parameters are grouped (in registration order, per dtype/device) into
flat padded device buckets (``collective.GradBuckets``); ``p.grad`` (S-SGD) or
``p.data`` (SMA) are made views into them so the reduction needs no fuse /
defuse copies. If a training loop replaces ``p.grad`` (``zero_grad`` with
``set_to_none=True``), the new gradient is copied into the bucket view once.
"""

from .collective import Exchange, GradBuckets


def _wrap(optimizer, mixin):
    # same trick as the reference (torch/optimizers/sync_sgd.py:31-34): a
    # subclass of the user's optimizer class, sharing its param_groups/state
    cls = type(optimizer.__class__.__name__, (mixin, optimizer.__class__), {})
    obj = cls.__new__(cls)
    obj.__dict__.update(optimizer.__dict__)
    return obj


def _finish(exchange):
    """An exchange whose queued work can fail without the host seeing it
    (the P2P device barriers) settles and raises here, before the update
    consumes the reduced values."""
    fin = getattr(exchange, "finish", None)
    if fin is not None:
        fin()


class _Bucketed:
    def _kf_setup(self, named_parameters, exchange, bucket_bytes):
        if named_parameters is None:
            params = [p for g in self.param_groups for p in g["params"]]
        else:
            params = [p for _, p in named_parameters]
        self._kf_params = [p for p in params if p.requires_grad]
        self._kf_ex = exchange if exchange is not None else Exchange()
        self._kf_bucket_bytes = bucket_bytes
        self._kf_groups = None

    def _kf_build(self, tensors_of):
        groups = {}
        for p in self._kf_params:
            groups.setdefault((p.dtype, p.device), []).append(p)
        self._kf_groups = []
        for (dtype, device), ps in groups.items():
            gb = GradBuckets([p.numel() for p in ps], dtype, device,
                             self._kf_ex.world, bucket_bytes=self._kf_bucket_bytes)
            self._kf_groups.append((ps, gb))


class _SyncSGD(_Bucketed):
    def _kf_setup_overlap(self):
        """Buckets in backward order (parameters reversed) with one
        post-accumulate-grad hook per parameter: when the last gradient of a
        bucket is in, that bucket's RS -> /np -> AG is queued at once, while
        backward goes on computing earlier layers. Buckets are launched strictly
        in index order (a ready bucket waits for the ones before it), so every
        rank issues the same collectives in the same order."""
        groups = {}
        for p in reversed(self._kf_params):
            groups.setdefault((p.dtype, p.device), []).append(p)
        self._kf_slots = []  # (bucket, [(param, view)]) in launch order
        self._kf_slot_of = {}
        for (dtype, device), ps in groups.items():
            gb = GradBuckets([p.numel() for p in ps], dtype, device,
                             self._kf_ex.world, bucket_bytes=self._kf_bucket_bytes)
            members = [[] for _ in gb.buckets]
            for p, v in zip(ps, gb.views):
                j = next(j for j, b in enumerate(gb.buckets)
                         if b.data_ptr() <= v.data_ptr() < b.data_ptr() + b.numel() * b.element_size())
                members[j].append((p, v.view_as(p)))
            for b, m in zip(gb.buckets, members):
                for p, v in m:
                    self._kf_slot_of[p] = (len(self._kf_slots), v)
                self._kf_slots.append((b, m))
        self._kf_reset_overlap()
        for p in self._kf_params:
            p.register_post_accumulate_grad_hook(self._kf_grad_ready)

    def _kf_reset_overlap(self):
        self._kf_missing = [len(m) for _, m in self._kf_slots]
        self._kf_next = 0
        self._kf_handles = []

    def _kf_grad_ready(self, p):
        i, v = self._kf_slot_of[p]
        if p.grad.data_ptr() != v.data_ptr():
            v.copy_(p.grad)
        self._kf_missing[i] -= 1
        self._kf_launch_ready()

    def _kf_launch_ready(self):
        # every bucket that is ready in index order goes out in ONE start_
        # call: the native exchange runs a call's buckets as one grouped RCCL
        # launch per phase and one batched HIP epilogue (kf_bucket_reduce_batch)
        first = self._kf_next
        while self._kf_next < len(self._kf_slots) and self._kf_missing[self._kf_next] <= 0:
            self._kf_next += 1
        if self._kf_next > first:
            self._kf_handles.append(self._kf_ex.start_(
                [b for b, _ in self._kf_slots[first:self._kf_next]], op=self._kf_op,
                average=self._kf_average, coalesce=False, key="ovl%d" % first))

    def _kf_finish_overlap(self):
        # parameters that got no gradient this step contribute zeros
        # (sync_gradients' rule); then every remaining bucket goes, in order
        for i, (b, m) in enumerate(self._kf_slots):
            if i >= self._kf_next and self._kf_missing[i] > 0:
                for p, v in m:
                    if p.grad is None:
                        v.zero_()
                self._kf_missing[i] = 0
        self._kf_launch_ready()
        for h in self._kf_handles:
            h.wait()
        for b, m in self._kf_slots:
            for p, v in m:
                p.grad = v
        self._kf_reset_overlap()

    def sync_gradients(self):
        if self._kf_overlap:
            return self._kf_finish_overlap()
        if self._kf_groups is None:
            self._kf_build(None)
        for ps, gb in self._kf_groups:
            for p, view in zip(ps, gb.views):
                g = p.grad
                v = view.view_as(p)
                if g is None:
                    v.zero_()
                    p.grad = v
                elif g.data_ptr() != v.data_ptr():
                    v.copy_(g)
                    p.grad = v
            self._kf_ex.all_reduce_(gb.buckets, op=self._kf_op,
                                    average=self._kf_average)

    def step(self, closure=None):
        self.sync_gradients()
        _finish(self._kf_ex)
        return super().step(closure)


def SynchronousSGDOptimizer(optimizer, named_parameters=None, op=None,
                            average=True, exchange=None, bucket_bytes=32 << 20,
                            overlap=False):
    """S-SGD: all-reduce gradients (sum, then / np when average) before each
    step. Returns the wrapped optimizer (reference: sync_sgd.py:81-84).

    overlap=True starts each bucket's exchange from a backward hook as soon as
    its gradients are complete (one backward per step), so the RCCL traffic
    of late layers hides behind the backward of early ones; step() waits for
    the rest. Same values as overlap=False up to the bucket grouping."""
    opt = _wrap(optimizer, _SyncSGD)
    opt._kf_setup(named_parameters, exchange, bucket_bytes)
    opt._kf_op = op if op is not None else "sum"
    opt._kf_average = bool(average)
    if opt._kf_average and opt._kf_op != "sum":
        raise ValueError("average=True needs op='sum'")
    opt._kf_overlap = bool(overlap)
    if opt._kf_overlap:
        if not hasattr(opt._kf_ex, "start_"):
            raise ValueError("overlap=True needs an exchange with start_() "
                             "(collective.Exchange)")
        opt._kf_setup_overlap()
    return opt


class _SMA(_Bucketed):
    def _kf_build_sma(self):
        self._kf_build(None)
        for ps, gb in self._kf_groups:  # move the variables into buckets
            for p, view in zip(ps, gb.views):
                v = view.view_as(p)
                v.copy_(p.data)
                p.data = v

    def sync_variables(self):
        if self._kf_groups is None:
            self._kf_build_sma()
        if self._kf_overlap:
            return self._kf_sync_overlapped()
        for ps, gb in self._kf_groups:
            # sma_sgd.py:53-57: only variables that have a gradient take part;
            # others are restored after the blend
            saved = [(p, p.data.clone()) for p in ps if p.grad is None]
            self._kf_ex.sma_(gb.buckets, self._kf_alpha)
            for p, d in saved:
                p.data.copy_(d)

    # overlap=True: the sum of the variables is all-reduced while the next
    # step's forward and backward run. SMA reduces v_t, the variables the
    # step's forward used (sma_sgd.py:60-65: group_all_reduce(variables)
    # before the blend and the gradient update), and they do not change
    # between the end of step t-1 and the blend of step t, so the sum can
    # start as soon as step t-1 has updated them — on the exchange's own
    # stream, into a workspace per bucket (out of place on the native
    # exchange; a copy, then in place, on collective.Exchange) — and step t
    # only waits for it and blends. The collectives and the blend kernel are those of sma_(), so the
    # result is the same bit for bit.
    def _kf_start_sums(self):
        if self._kf_sums is None:
            from .collective import workspace_like
            self._kf_sums = [workspace_like(gb.buckets) for _, gb in self._kf_groups]
        self._kf_pending = []
        into = getattr(self._kf_ex, "start_into_", None)
        for gi, ((_, gb), sums) in enumerate(zip(self._kf_groups, self._kf_sums)):
            if into is not None:  # the native exchange: out of place, no copy
                self._kf_pending.append(into(gb.buckets, sums, op="sum"))
                continue
            for s, b in zip(sums, gb.buckets):
                s.copy_(b)
            self._kf_pending.append(self._kf_ex.start_(sums, op="sum", average=False,
                                                       coalesce=False, key=("sma", gi)))

    def _kf_sync_overlapped(self):
        if self._kf_pending is None:  # the first step: nothing started yet
            self._kf_start_sums()
        world = self._kf_ex.world
        epilogue = getattr(self._kf_ex, "epilogue", None)
        for (ps, gb), sums, h in zip(self._kf_groups, self._kf_sums, self._kf_pending):
            saved = [(p, p.data.clone()) for p in ps if p.grad is None]
            h.wait()
            if epilogue is not None:  # collective.Exchange: its own epilogue
                for b, s in zip(gb.buckets, sums):
                    epilogue.sma_blend_(b, s, world, self._kf_alpha)
            else:  # the native exchange's blend: the batched HIP kernel
                from . import ops
                ops.sma_blend_batch_(gb.buckets, sums, world, self._kf_alpha)
            for p, d in saved:
                p.data.copy_(d)
        self._kf_pending = None

    def step(self, closure=None):
        self.sync_variables()
        _finish(self._kf_ex)
        out = super().step(closure)
        if self._kf_overlap:  # v_{t+1} is final: start its sum now
            self._kf_start_sums()
        return out


def SynchronousAveragingOptimizer(optimizer, named_parameters=None, alpha=0.1,
                                  exchange=None, bucket_bytes=32 << 20, overlap=False):
    """SMA: v <- (1 - alpha) v + alpha * mean_ranks(v) before each local step
    (sma_sgd.py:50-74).

    overlap=True starts the all-reduce of the next step's variables at the
    end of step() on the exchange's stream, so it runs during that step's
    forward and backward; step() then waits for it and blends. Same values as
    overlap=False, provided the variables change only through step() (the
    first step reduces synchronously)."""
    opt = _wrap(optimizer, _SMA)
    opt._kf_setup(named_parameters, exchange, bucket_bytes)
    opt._kf_alpha = float(alpha)
    opt._kf_overlap = bool(overlap)
    opt._kf_sums = None
    opt._kf_pending = None
    if opt._kf_overlap and not hasattr(opt._kf_ex, "start_"):
        raise ValueError("overlap=True needs an exchange with start_() "
                         "(collective.Exchange or exchange.NativeExchange)")
    return opt
