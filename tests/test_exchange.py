"""The native multi-GPU exchange (kf_exchange_*, kungfu_amd/csrc/kf_exchange.hip)
and the multi-bucket launch (kf_bucket_reduce_batch).

CPU: the RCCL id travels over a host-mode KungFu session exactly as
gpu_collective.cpp:190-200 broadcasts it (world 2 and 3 processes), creation
without a device fails with a status instead of crashing.
GPU (one MI355X): the batch kernel bit-exact against the oracle; a world-1
communicator through the C ABI (all-reduce, batch, SMA, both algorithms and
the ordered scheduler). RCCL refuses two ranks on one device, so the N > 1
exchange runs in bench.py on the driver's multi-GPU node, where it is checked
against the rank-order fold before it is timed."""
import ctypes
import multiprocessing as mp
import os
import sys
import tempfile
import traceback

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _share_body(rank, world, sock_dir, errq):
    sys.path[:0] = [ROOT, HERE]
    try:
        from kungfu_amd import _lib
        from kungfu_amd.session import Session
        s = Session(rank, world, sock_dir, mode="host", strategy="STAR")
        lib = _lib.load()
        uid = (ctypes.c_char * 128)()
        if rank == 0:
            ctypes.memmove(uid, bytes(range(128)), 128)
        _lib.check(lib.kf_exchange_share_id(ctypes.c_void_p(s._h), uid), "share_id")
        assert bytes(uid) == bytes(range(128)), rank
        s.close()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_share_id_over_session(world):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_share_body, args=(r, world, d, errq)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in ps)


def test_create_without_device_is_an_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("has a GPU")
    from kungfu_amd import _lib
    lib = _lib.load()
    uid = (ctypes.c_char * 128)()
    assert not lib.kf_exchange_create(uid, 0, 1, 0)
    msg = lib.kf_exchange_last_error().decode()
    assert msg, "no reason given"
    # bad arguments are refused before anything is touched
    assert not lib.kf_exchange_create(uid, 2, 2, 0)
    assert lib.kf_exchange_all_reduce(None, None, None, 0, 0x20408, 0, 0, 0, None) == 3


# ---- GPU --------------------------------------------------------------------

def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


DTS = {"f32": "float32", "bf16": "bfloat16", "f16": "float16", "i32": "int32", "i8": "int8",
       "f64": "float64", "u8": "uint8"}


def _rand(name, n, seed):
    rng = np.random.default_rng(seed)
    if name in ("f32", "f64", "f16"):
        return rng.standard_normal(n).astype({"f32": np.float32, "f64": np.float64,
                                              "f16": np.float16}[name])
    if name == "bf16":
        from oracle import oracle
        return oracle.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32))
    info = np.iinfo({"i32": np.int32, "i8": np.int8, "u8": np.uint8}[name])
    return rng.integers(info.min, info.max, n, endpoint=True).astype(info.dtype)


def _to_dev(a, name, dev):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a))
    if name == "bf16":
        t = t.view(torch.int16).view(torch.bfloat16)
    return t.to(dev)


def _to_np(t, name):
    import torch
    t = t.cpu()
    if name == "bf16":
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("name,k,avg", [("f32", 2, False), ("f32", 1, True), ("f32", 5, True),
                                        ("bf16", 4, True), ("bf16", 2, False), ("f16", 3, False),
                                        ("i32", 3, False), ("i8", 2, False), ("u8", 8, False),
                                        ("f64", 2, True)])
def test_batch_kernel_matches_oracle(name, k, avg):
    """20 buckets (more than one launch of 16), ragged sizes incl. 0, 1 and a
    misaligned bucket, against the oracle's fold / reduce_avg per bucket."""
    import torch
    from kungfu_amd import _lib
    from oracle import oracle
    dev = _gpu()
    lib = _lib.load()
    sizes = [0, 1, 7, 4099, 1 << 20, 262147, 33] + [4096 * (i + 1) + i for i in range(13)]
    ins_h = [[_rand(name, n, 100 * b + j) for j in range(k)] for b, n in enumerate(sizes)]
    ins_d = [[_to_dev(a, name, dev) for a in row] for row in ins_h]
    # bucket 3: every pointer one element past an aligned start (same residue)
    ins_d[3] = [torch.cat([t[:1], t])[1:] for t in ins_d[3]]
    outs = [torch.empty_like(row[0]) if row else None for row in ins_d]
    ptrs = [t.data_ptr() for row in ins_d for t in row]
    rc = lib.kf_bucket_reduce_batch(
        _lib.ptr_array(ptrs), k, _lib.ptr_array([o.data_ptr() for o in outs]),
        (ctypes.c_size_t * len(sizes))(*sizes), len(sizes), oracle.DT[name], 0,
        k if avg else 0, torch.cuda.current_stream().cuda_stream)
    _lib.check(rc, "kf_bucket_reduce_batch")
    torch.cuda.synchronize()
    for b, n in enumerate(sizes):
        if avg:
            want = oracle.reduce_avg(ins_h[b], name, k)
        else:
            want = oracle.reduce_k(ins_h[b], name, "sum")
        assert np.array_equal(_to_np(outs[b], name), want), (name, b, n)
    # MIN goes bucket by bucket through the same entry point
    if name in ("f32", "i32"):
        rc = lib.kf_bucket_reduce_batch(
            _lib.ptr_array(ptrs), k, _lib.ptr_array([o.data_ptr() for o in outs]),
            (ctypes.c_size_t * len(sizes))(*sizes), len(sizes), oracle.DT[name], 1, 0,
            torch.cuda.current_stream().cuda_stream)
        _lib.check(rc, "kf_bucket_reduce_batch(min)")
        torch.cuda.synchronize()
        for b in range(len(sizes)):
            assert np.array_equal(_to_np(outs[b], name), oracle.reduce_k(ins_h[b], name, "min"))


@pytest.mark.gpu
def test_world1_native_exchange():
    """A one-rank communicator through the C ABI: every call is the identity
    (a sum of one, / 1), for both algorithms, batch and SMA, out of place too;
    the ordered scheduler issues in the agreed order and, with auto_order,
    adopts the first step's arrival order."""
    import torch
    import torch.distributed as dist
    from kungfu_amd import _lib
    from kungfu_amd.exchange import NativeExchange, Scheduler
    from oracle import oracle
    dev = _gpu()
    assert not dist.is_initialized()
    lib = _lib.load()
    for algo in ("auto", "rs", "a2a"):
        ex = NativeExchange(algo=algo, device=dev)
        r, w, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(lib.kf_exchange_info(ex._h, ctypes.byref(r), ctypes.byref(w),
                                        ctypes.byref(d)), "info")
        assert (r.value, w.value, d.value) == (0, 1, 0)
        bs = [torch.randn(n, device=dev) for n in (1 << 20, 1001, 5)]
        want = [b.clone() for b in bs]
        ex.all_reduce_(bs, average=True)
        bf = torch.randn(4097, device=dev).to(torch.bfloat16)
        bfw = bf.clone()
        ex.all_reduce_([bf], average=True)
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(bs, want))
        assert torch.equal(bf, bfw)
        # out of place through the single-bucket entry
        y = torch.empty_like(bs[0])
        _lib.check(lib.kf_exchange_all_reduce(ex._h, bs[0].data_ptr(), y.data_ptr(), y.numel(),
                                              0x20408, 0, 1, 0,
                                              torch.cuda.current_stream().cuda_stream), "ar")
        torch.cuda.synchronize()
        assert torch.equal(y, bs[0])
        # SMA of one rank: v <- (1-a) v + a v (the blend's own rounding)
        v = torch.randn(30001, device=dev)
        v0 = v.cpu().numpy().copy()
        ex.sma_([v], 0.1)
        torch.cuda.synchronize()
        assert np.array_equal(v.cpu().numpy(), oracle.sma_blend(v0, v0, "f32", 1, 0.1))
        h = ex.start_([bs[1]], average=True)
        h.wait()
        ex.check()
        # the scheduler: names started in reverse, issued in the agreed order
        sch = Scheduler(ex, auto_order=True)
        names = ["g%d" % i for i in range(6)]
        bufs = [torch.full((1000 + i,), float(i), device=dev) for i in range(6)]
        seen = []
        for step in range(3):
            sch.begin_step(names)
            arrival = names[::-1] if step == 0 else names[2:] + names[:2]
            for nm in arrival:
                i = names.index(nm)
                sch.start(nm, bufs[i], callback=lambda n, st: seen.append((n, st)))
            order = sch.wait_all()
            # step 0: the given order; afterwards rank 0's arrival of step 0
            assert order == (names if step == 0 else names[::-1]), (step, order)
        assert all(st == 0 for _, st in seen) and len(seen) == 18
        assert all(torch.all(b == i) for i, b in enumerate(bufs))
        ex.close()
