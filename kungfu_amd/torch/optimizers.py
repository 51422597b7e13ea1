"""``kungfu.torch.optimizers`` mirror.

``SynchronousSGDOptimizer(optimizer, named_parameters, op=None)`` keeps the
reference torch wrapper's signature AND arithmetic
(srcs/python/kungfu/torch/optimizers/sync_sgd.py:12-34): ``named_parameters``
is required, and every gradient is all-reduced with ``op`` (default 'sum')
and NOT divided by np — unlike the TF S-SGD (tensorflow/optimizers/
sync_sgd.py:103-104), whose averaging variant is
``kungfu_amd.optimizers.SynchronousSGDOptimizer`` (average=True). Extra
keyword arguments (``overlap``, ``exchange``, ``bucket_bytes``, ``average``)
pass through to it.

``SynchronousAveragingOptimizer`` is the SMA wrapper (sma_sgd.py:9-74); the
reference has no torch version, so it is the package's own.
"""
from .. import optimizers as _opt
from ..optimizers import SynchronousAveragingOptimizer

__all__ = ["SynchronousSGDOptimizer", "SynchronousAveragingOptimizer"]


def SynchronousSGDOptimizer(optimizer, named_parameters, op=None, **kwargs):
    """Reference torch S-SGD (sync_sgd.py:31-34): sum (or `op`) of every
    gradient across peers before the wrapped optimizer's step; no /np."""
    kwargs.setdefault("average", False)
    return _opt.SynchronousSGDOptimizer(optimizer, named_parameters=named_parameters, op=op,
                                        **kwargs)
