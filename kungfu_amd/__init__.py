"""kungfu_amd — MI355X-native gradient-bucket reduce for KungFu.

A drop-in for KungFu's host element reduce (std_transform_2 and the sum-and-
scale of SynchronousSGDOptimizer / SynchronousAveragingOptimizer), built as
hand-written gfx950 HIP kernels behind a C ABI (include/kungfu_amd.h) with
RCCL reduce-scatter + all-gather across the GPUs of a node.

Modules:
  base        mirror of srcs/go/kungfu/base (DataType, OP, Vector, Workspace,
              Transform2 -> std_transform_2 on the GPU)
  ops         device bucket-reduce ops on torch tensors
  collective  bucketed RCCL all-reduce with the fused HIP epilogues
  optimizers  SynchronousSGDOptimizer / SynchronousAveragingOptimizer (torch)
"""
__version__ = "0.1.0"
