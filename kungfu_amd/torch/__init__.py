"""PyTorch surface mirroring the reference's ``kungfu.torch`` package
(srcs/python/kungfu/torch/{__init__,ops,optimizers}.py): same names, arguments
and meaning, with the reduction on the MI355X bucket path.

The package-level peer queries of the reference (``kungfu.python``,
srcs/python/kungfu/python/__init__.py:60-86, re-exported by
srcs/python/kungfu/torch/__init__.py:1-16) read the cluster kungfu-run set
up; here the cluster is the torch.distributed process group that
``torch.distributed.run`` set up (one process per GPU), so they answer from
it: rank / size from the group, local rank / size from LOCAL_RANK /
LOCAL_WORLD_SIZE (one host if unset), the CUDA index is the local rank (one GPU per process), and
the barrier is the group's barrier. Without an initialised group they answer
as a single peer, as the reference does without kungfu-run
(env/config.go:54-56)."""
import os

import torch.distributed as dist

from . import ops, optimizers  # noqa: F401


def _group():
    return dist.is_available() and dist.is_initialized()


def current_rank():
    """Rank of this peer (kungfu.python.current_rank)."""
    return dist.get_rank() if _group() else 0


def current_cluster_size():
    """Number of peers (kungfu.python.current_cluster_size)."""
    return dist.get_world_size() if _group() else 1


def current_local_rank():
    """Rank of this peer among the peers of its host."""
    if not _group():
        return 0
    # launched without torch.distributed.run (e.g. spawned): one host
    return int(os.environ.get("LOCAL_RANK", str(dist.get_rank())))


def current_local_size():
    """Number of peers on this host."""
    if not _group():
        return 1
    return int(os.environ.get("LOCAL_WORLD_SIZE", str(dist.get_world_size())))


def get_cuda_index():
    """The GPU this peer drives (kungfu.python._get_cuda_index): one per process."""
    return current_local_rank()


def run_barrier():
    """Barrier over every peer, eagerly (kungfu.python.run_barrier)."""
    if _group():
        dist.barrier()


def nccl_built():
    """As the reference's torch package (torch/__init__.py:10-11): the KungFu
    NCCL op library is not part of it; RCCL is used through torch.distributed."""
    return False


broadcast_parameters = ops.broadcast_parameters
