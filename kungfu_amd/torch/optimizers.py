"""``kungfu.torch.optimizers`` mirror: the S-SGD and SMA wrappers
(srcs/python/kungfu/torch/optimizers/sync_sgd.py:31-34; SMA as in
srcs/python/kungfu/tensorflow/optimizers/sma_sgd.py:9-74)."""
from ..optimizers import SynchronousAveragingOptimizer, SynchronousSGDOptimizer

__all__ = ["SynchronousSGDOptimizer", "SynchronousAveragingOptimizer"]
