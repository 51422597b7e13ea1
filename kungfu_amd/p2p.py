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
"""
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from .ops import kungfu_dtype


class P2PExchange:
    def __init__(self, buckets, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.lib = _lib.load()
        self.buckets = list(buckets)
        for b in self.buckets:
            if not b.is_cuda or b.dim() != 1 or not b.is_contiguous():
                raise ValueError("P2P buckets must be flat contiguous GPU tensors")
            if b.numel() % self.world or (b.numel() // self.world * b.element_size()) % 16:
                raise ValueError("bucket does not split into 16-B aligned shards")
        mine = []
        for b in self.buckets:
            h = (ctypes.c_char * 64)()
            off = ctypes.c_size_t()
            _lib.check(self.lib.kf_ipc_export(b.data_ptr(), h, ctypes.byref(off)),
                       "kf_ipc_export")
            mine.append((bytes(h), off.value))
        everyone = [None] * self.world
        dist.all_gather_object(everyone, mine, group=group)
        self._bases = {}  # handle -> mapped base (one mapping per allocation)
        self.ptrs = []    # ptrs[j][r]: bucket j of rank r, as seen from here
        for j, b in enumerate(self.buckets):
            row = []
            for r in range(self.world):
                if r == self.rank:
                    row.append(b.data_ptr())
                    continue
                h, off = everyone[r][j]
                key = (r, h)
                if key not in self._bases:
                    base = ctypes.c_void_p()
                    _lib.check(self.lib.kf_ipc_import(h, ctypes.byref(base)), "kf_ipc_import")
                    self._bases[key] = base.value
                row.append(self._bases[key] + off)
            self.ptrs.append(row)

    def close(self):
        for base in self._bases.values():
            self.lib.kf_ipc_close(base)
        self._bases = {}

    def _barrier(self):
        torch.cuda.synchronize()
        dist.barrier(group=self.group)

    def all_reduce_(self, op="sum", average=False):
        """In place on the buckets given at construction."""
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
            # every peer's load in flight at once (all links busy), adds in
            # rank order
            rc = self.lib.kf_bucket_reduce_peers(ins, world, out, shard, int(kungfu_dtype(b)),
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
        return self.buckets
