"""Test-only CPU stand-in for collective.HipEpilogue, so the N>1 orchestration
(bucketing, sharding, RS -> epilogue -> AG) runs over gloo on CPU tensors. It
delegates to the oracle, i.e. the exact semantics the HIP kernels are
parity-tested against on the GPU (tests/test_gpu_parity.py)."""
import numpy as np
import torch

from oracle import oracle

_DT = {torch.float32: "f32", torch.float64: "f64", torch.float16: "f16",
       torch.bfloat16: "bf16", torch.int32: "i32", torch.int64: "i64", torch.uint8: "u8",
       torch.int8: "i8", torch.int16: "i16"}


def _np(t):
    if t.dtype in (torch.float16, torch.bfloat16):
        return t.view(torch.int16).numpy().view(np.uint16 if t.dtype == torch.bfloat16 else np.float16)
    return t.numpy()


class CpuEpilogue:
    def div_(self, x, np_):
        a = _np(x)
        a[...] = oracle.reduce_avg([np.ascontiguousarray(a)], _DT[x.dtype], np_)
        return x

    def fold_(self, inputs, out, op, np_):
        arrs = [np.ascontiguousarray(_np(t)) for t in inputs]
        if np_:
            res = oracle.reduce_avg(arrs, _DT[out.dtype], np_)
        else:
            res = oracle.reduce_k(arrs, _DT[out.dtype], int(op))
        _np(out)[...] = res
        return out

    def sma_blend_(self, v, summed, np_, alpha):
        a = _np(v)
        a[...] = oracle.sma_blend(np.ascontiguousarray(a), np.ascontiguousarray(_np(summed)),
                                  _DT[v.dtype], np_, alpha)
        return v


class GpuShardEpilogue:
    """Runs the REAL HIP epilogue on a GPU copy of each CPU shard (used by the
    gpu-marked multi-process test: gloo moves the data, HIP does the math)."""

    def __init__(self, device):
        from kungfu_amd.collective import HipEpilogue
        self.hip = HipEpilogue()
        self.device = device

    def div_(self, x, np_):
        g = x.to(self.device)
        self.hip.div_(g, np_)
        x.copy_(g.cpu())
        return x

    def fold_(self, inputs, out, op, np_):
        g = out.to(self.device)
        self.hip.fold_([t.to(self.device) for t in inputs], g, op, np_)
        out.copy_(g.cpu())
        return out

    def sma_blend_(self, v, summed, np_, alpha):
        g = v.to(self.device)
        self.hip.sma_blend_(g, summed.to(self.device), np_, alpha)
        v.copy_(g.cpu())
        return v
