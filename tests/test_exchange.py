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
from procs import join_all

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
        hung = join_all(ps, 120)
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


def _rand(name, n, seed):
    rng = np.random.default_rng(seed)
    if name in ("f32", "f64", "f16"):
        return rng.standard_normal(n).astype({"f32": np.float32, "f64": np.float64,
                                              "f16": np.float16}[name])
    if name == "bf16":
        from oracle import oracle
        return oracle.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32))
    info = np.iinfo({"i32": np.int32, "i8": np.int8, "u8": np.uint8, "u16": np.uint16}[name])
    return rng.integers(info.min, info.max, n, endpoint=True).astype(info.dtype)


def _to_dev(a, name, dev):
    import torch
    if name == "u16":
        return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).to(dev)
    t = torch.from_numpy(np.ascontiguousarray(a))
    if name == "bf16":
        t = t.view(torch.int16).view(torch.bfloat16)
    return t.to(dev)


def _to_np(t, name):
    import torch
    t = t.cpu()
    if name in ("bf16", "u16"):
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("name,k,avg", [("f32", 2, False), ("f32", 1, True), ("f32", 5, True),
                                        ("bf16", 4, True), ("bf16", 2, False), ("f16", 3, False),
                                        ("i32", 3, False), ("i8", 2, False), ("u8", 8, False),
                                        ("f64", 2, True), ("u16", 4, False), ("u16", 8, False)])
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
@pytest.mark.parametrize("k,avg", [(1, True), (2, False), (8, True), (3, False)])
def test_batch_kernel_equal_buckets(k, avg):
    """Buckets of one size (the exchange's shards of equal buckets) take the
    launch's common block count: the kernel finds a block's bucket by one
    division instead of searching the argument table. 70 equal f32 buckets
    (two launches at k = 1, five at k >= 2) with one misaligned bucket in the
    middle (a launch of its own), /np and plain, against the oracle."""
    import torch
    from kungfu_amd import _lib
    from oracle import oracle
    dev = _gpu()
    lib = _lib.load()
    nb, n = 70, 49968 * 4 + 3
    hs = [[_rand("f32", n, 9000 + 10 * b + j) for j in range(k)] for b in range(nb)]
    ins = [[_to_dev(a, "f32", dev) for a in row] for row in hs]
    ins[33] = [torch.cat([t[:1], t])[1:] for t in ins[33]]
    outs = [torch.empty_like(row[0]) for row in ins]
    rc = lib.kf_bucket_reduce_batch(
        _lib.ptr_array([t.data_ptr() for row in ins for t in row]), k,
        _lib.ptr_array([o.data_ptr() for o in outs]), (ctypes.c_size_t * nb)(*[n] * nb), nb,
        oracle.DT["f32"], 0, 8 if avg else 0, torch.cuda.current_stream().cuda_stream)
    _lib.check(rc, "kf_bucket_reduce_batch")
    torch.cuda.synchronize()
    for b in range(nb):
        want = oracle.reduce_avg(hs[b], "f32", 8) if avg else oracle.reduce_k(hs[b], "f32", "sum")
        assert np.array_equal(_to_np(outs[b], "f32"), want), b


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["f32", "bf16"])
def test_batch_kernel_k1_past_64_buckets(name):
    """k = 1 (the shard /np) packs up to 64 buckets per launch (kBatchSeg1):
    150 ragged buckets — three launches, the last partial — with one
    misaligned bucket in the middle (a launch of its own), /np and plain."""
    import torch
    from kungfu_amd import _lib
    from oracle import oracle
    dev = _gpu()
    lib = _lib.load()
    sizes = [(4099 * (i % 7) + 13 * i) % 70000 for i in range(150)]
    hs = [_rand(name, n, 7000 + b) for b, n in enumerate(sizes)]
    for np_ in (8, 3, 0):
        ins = [_to_dev(h, name, dev) for h in hs]
        ins[77] = torch.cat([ins[77][:1], ins[77]])[1:]
        outs = [torch.empty_like(t) for t in ins]
        rc = lib.kf_bucket_reduce_batch(
            _lib.ptr_array([t.data_ptr() for t in ins]), 1,
            _lib.ptr_array([o.data_ptr() for o in outs]),
            (ctypes.c_size_t * len(sizes))(*sizes), len(sizes), oracle.DT[name], 0, np_,
            torch.cuda.current_stream().cuda_stream)
        _lib.check(rc, "kf_bucket_reduce_batch")
        torch.cuda.synchronize()
        for b, h in enumerate(hs):
            want = oracle.reduce_avg([h], name, np_) if np_ else h
            assert np.array_equal(_to_np(outs[b], name), want), (np_, b)


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


# ---- the exchange's multi-rank logic over the loopback transport ------------

def _loop_ranks(world, body):
    """body(rank, ex) on `world` threads over the test library's loopback
    transport (tests/loopback.py, tests/c/kf_testing.cpp)."""
    from loopback import loop_ranks
    loop_ranks(world, body)


_LONE_RANK = r"""
import ctypes, os, sys, time
sys.path.insert(0, %r)
from kungfu_amd import _lib
lib = _lib.load()
uid = (ctypes.c_char * 128)()
assert lib.kf_exchange_unique_id(uid) == 0
t0 = time.monotonic()
h = lib.kf_exchange_create_timeout(uid, 0, 2, 0, 3000)
dt = time.monotonic() - t0
print("RESULT", bool(h), round(dt, 2), lib.kf_exchange_last_error().decode(), flush=True)
os._exit(0)  # the abandoned init is still waiting for rank 1
"""


@pytest.mark.gpu
def test_create_timeout_when_a_rank_never_joins():
    """kf_exchange_create_timeout: rank 0 of a world of 2 whose rank 1 never
    comes gets NULL and KF_ERR_TIMEOUT's message after the deadline instead
    of blocking in ncclCommInitRank (the torch op's start-up uses it, so a
    missing rank costs its peers KUNGFU_AMD_INIT_TIMEOUT_S, then every rank
    takes the torch.distributed path together)."""
    import subprocess
    _gpu()
    r = subprocess.run([sys.executable, "-c", _LONE_RANK % ROOT], capture_output=True,
                       text=True, timeout=90)
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
    assert line, r.stdout + r.stderr[-2000:]
    _, ok, dt, msg = line[0].split(" ", 3)
    assert ok == "False" and 2.5 <= float(dt) <= 30, line
    assert "not every rank joined" in msg, msg


@pytest.mark.gpu
@pytest.mark.parametrize("world,groups", [(2, 1), (4, 1), (4, 2), (3, 1)])
def test_rs_avg_folds_the_division_into_the_collective(world, groups):
    """KF_ALGO_REDUCE_SCATTER_AVG: the average's /np inside the reduce-scatter
    (ncclAvg; the loopback premultiplies by 1/world and sums in rank order)
    and no shard epilogue. At a power-of-two world it has the bits of the
    rank-order sum then /np (the oracle's reduce_avg) for normal inputs; at
    world 3 each input adds one rounding (|err| <= world * u * sum|x|/world
    + u*|avg|). Tails (count % world) still take the rank-order fold with /np.
    Non-average calls under it are plain reduce-scatters."""
    import torch
    from oracle import oracle
    dev = _gpu()
    counts = [world * 5000, world * 777 + 2, 1, world * 65536]

    def body(rank, ex):
        ex.set_pipeline(groups)
        ex.algo = "rs_avg"
        hs = [[_rand("f32", n, 40 * r + b) for b, n in enumerate(counts)] for r in range(world)]
        bufs = [_to_dev(hs[rank][b], "f32", dev) for b in range(len(counts))]
        ex.set_timing(True)
        ex.all_reduce_(bufs, average=True, coalesce=False)
        torch.cuda.synchronize()
        ph = ex.phase_times()
        ex.set_timing(False)
        for b, n in enumerate(counts):
            ins = [hs[r][b] for r in range(world)]
            want = oracle.reduce_avg(ins, "f32", world)
            got = _to_np(bufs[b], "f32")
            if world & (world - 1) == 0:
                assert np.array_equal(got, want), (b, n)
            else:
                u = 2.0 ** -24
                absum = np.sum([np.abs(x.astype(np.float64)) for x in ins], axis=0)
                bound = 2 * world * u * absum / world + 2 * u * np.abs(want.astype(np.float64))
                assert np.all(np.abs(got.astype(np.float64) - want) <= bound + 1e-38), (b, n)
        if groups == 1:
            assert ph["calls"] == 1, ph
        # a plain sum under rs_avg is the reduce-scatter's
        xi = [_rand("i32", world * 999, 7 + r) for r in range(world)]
        bi = _to_dev(xi[rank], "i32", dev)
        ex.all_reduce_([bi], average=False)
        torch.cuda.synchronize()
        assert np.array_equal(_to_np(bi, "i32"), oracle.reduce_k(xi, "i32", "sum"))

    _loop_ranks(world, body)


def _special_inputs(world, q, seed):
    """Per-rank fp32 shards whose rank-order sum then /np and whose
    premultiplied sum (ncclAvg's PreMulSum for floating types) can part: a
    normal block, pairs near FLT_MAX whose sum overflows, subnormals (x/np
    loses bits), NaN and +-inf lanes."""
    rng = np.random.default_rng(seed)
    big = np.float32(3.0e38)
    ins = []
    for r in range(world):
        x = rng.standard_normal(world * q).astype(np.float32)
        x[0:64] = big * (1 + np.float32(0.01) * np.float32(r))           # overflow on the sum
        # subnormals with odd mantissas: x / np is inexact in every one
        x[64:128] = (rng.integers(0, 1 << 20, 64) * 2 + 1).astype(np.uint32).view(np.float32)
        x[128:136] = np.float32("nan") if r == world - 1 else np.float32(1.0)
        x[136:144] = np.float32("inf") if r == 0 else np.float32(-1.0)
        ins.append(x)
    return ins


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rs_avg_special_values_decide_the_default(world):
    """may KF_ALGO_REDUCE_SCATTER_AVG (the /np inside the
    reduce-scatter as ncclAvg, which RCCL runs for floats as a premultiply by
    1/np before the sum) replace the shard /np epilogue at power-of-two
    worlds? Only if its bits equal sum-then-/np (oracle.reduce_avg,
    sync_sgd.py:103-104) on every input. On normal values they do (x * 2^-k is
    exact, every partial sum scales by the same power of two). They do NOT on
    sums that overflow (inf in the reference, finite premultiplied) nor on
    subnormals (x / np drops bits before the sum). NaN and inf lanes agree. So
    the default stays "rs" (sum, then the exact /np epilogue), and rs_avg stays
    an opt-in whose difference this test pins."""
    import torch
    from oracle import oracle
    dev = _gpu()
    q = 4096
    ins = _special_inputs(world, q, 11 + world)
    want = oracle.reduce_avg(ins, "f32", world)
    got = {}

    def body(rank, ex):
        for algo in ("rs", "rs_avg"):
            ex.algo = algo
            b = _to_dev(ins[rank], "f32", dev)
            ex.all_reduce_([b], average=True, coalesce=False)
            torch.cuda.synchronize()
            if rank == 0:
                got[algo] = _to_np(b, "f32")

    _loop_ranks(world, body)
    same = lambda a, b: (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))  # noqa: E731
    # the default: bit-exact everywhere, specials included
    assert same(got["rs"], want).all()
    eq = same(got["rs_avg"], want)
    normal = np.ones(world * q, bool)
    normal[:144] = False
    assert eq[normal].all()                      # normal range: identical bits
    assert eq[128:144].all()                     # NaN / inf lanes agree
    assert not eq[0:64].any()                    # overflow: reference inf, premultiplied finite
    assert np.isinf(want[0:64]).all() and np.isfinite(got["rs_avg"][0:64]).all()
    assert not eq[64:128].all()                  # subnormals: bits dropped by the premultiply


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["rs", "a2a"])
def test_pipelined_failure_at_every_call_then_reusable(algo):
    """a transport failure at ANY collective of the
    pipelined schedule (3 groups of 2 buckets: p1(0) p1(1) p3(0) p1(2) p3(1)
    p3(2), 12 calls) comes back as the call's error on every rank, with the
    folds already queued on the exchange's second stream joined and the
    workspace released: the next call on the same exchange is bit-exact."""
    import threading
    import torch
    from loopback import LoopbackGroup, loop_ranks
    from oracle import oracle
    from kungfu_amd._lib import KungFuAMDError
    dev = _gpu()
    world, nb = 2, 6
    counts = [world * (40000 + 1000 * b) for b in range(nb)]  # no tails
    g = LoopbackGroup(world)
    bar = threading.Barrier(world)
    per_call = 2 * nb  # one phase-1 and one phase-3 collective per bucket

    def body(rank, ex):
        ex.set_pipeline(3)
        ex.algo = algo
        done = 0  # collective calls made so far (the same on every rank)
        for k in range(per_call):
            hs = [[_rand("f32", n, 100 * r + b + k) for b, n in enumerate(counts)]
                  for r in range(world)]
            bufs = [_to_dev(hs[rank][b], "f32", dev) for b in range(nb)]
            bar.wait()
            if rank == 0:
                g.fail_at(done + k)
            bar.wait()
            with pytest.raises(KungFuAMDError, match="injected failure"):
                ex.all_reduce_(bufs, average=True, coalesce=False)
            done += k + 1
            # the same exchange, workspace and streams: bit-exact next call
            bufs = [_to_dev(hs[rank][b], "f32", dev) for b in range(nb)]
            ex.all_reduce_(bufs, average=True, coalesce=False)
            torch.cuda.synchronize()
            done += per_call
            for b in range(nb):
                want = oracle.reduce_avg([hs[r][b] for r in range(world)], "f32", world)
                assert np.array_equal(_to_np(bufs[b], "f32"), want), (k, b)

    loop_ranks(world, body, group=g)


@pytest.mark.gpu
@pytest.mark.parametrize("world,groups", [(2, 1), (3, 1), (4, 1), (8, 1), (2, 3), (3, 2),
                                          (8, 4)])
def test_exchange_multi_rank_loopback(world, groups):
    """The N > 1 code of kf_exchange (shards, tails of count % world, the
    workspace, batched folds, in-place all-gather, SMA) at worlds 2-8 on one
    GPU: the loopback transport moves the bytes where RCCL would, its
    reduce-scatter folds in rank order, so every algo is bit-exact against the
    oracle's rank-order fold. groups > 1: the pipelined schedule
    (kf_exchange_set_pipeline), whose folds and blends run on the exchange's
    own stream between the groups' collectives — the same bits."""
    import torch
    from oracle import oracle
    dev = _gpu()
    counts = [1, 7, world * 1000 + 3, 262147, world * 4096]

    def body(rank, ex):
        ex.set_pipeline(groups)
        for algo in ("rs", "a2a", "auto"):
            for name, avg in (("f32", True), ("bf16", True), ("f16", False), ("i32", False)):
                if algo == "rs" and name in ("bf16", "f16"):
                    continue  # the loopback has no half-precision reduce-scatter
                seeds = [[1000 * r + 10 * b + len(algo) for b in range(len(counts))]
                         for r in range(world)]
                hs = [[_rand(name, n, seeds[r][b]) for b, n in enumerate(counts)]
                      for r in range(world)]
                bufs = [_to_dev(hs[rank][b], name, dev) for b in range(len(counts))]
                ex.algo = algo
                ex.all_reduce_(bufs, average=avg, coalesce=False)
                torch.cuda.synchronize()
                for b in range(len(counts)):
                    ins = [hs[r][b] for r in range(world)]
                    want = (oracle.reduce_avg(ins, name, world) if avg else
                            oracle.reduce_k(ins, name, "sum"))
                    assert np.array_equal(_to_np(bufs[b], name), want), (algo, name, b)
        # MAX on i32 (RCCL's reduce-scatter under auto) and u16 SUM (no RCCL
        # reduction type: the all-to-all fold)
        ex.algo = "auto"
        hs = [_rand("i32", 50001, 77 + r) for r in range(world)]
        b = _to_dev(hs[rank], "i32", dev)
        ex.all_reduce_([b], op="max")
        torch.cuda.synchronize()
        assert np.array_equal(_to_np(b, "i32"), np.max(np.array(hs), axis=0))
        us = [np.random.default_rng(5 + r).integers(0, 65535, 9999).astype(np.uint16)
              for r in range(world)]
        ub = torch.from_numpy(us[rank].view(np.int16)).to(dev)
        lib = ex.lib
        from kungfu_amd import _lib
        _lib.check(lib.kf_exchange_all_reduce(ex._h, ub.data_ptr(), ub.data_ptr(), ub.numel(),
                                              0x00208, 0, 0, 0,
                                              torch.cuda.current_stream().cuda_stream), "u16")
        torch.cuda.synchronize()
        assert np.array_equal(ub.cpu().numpy().view(np.uint16), oracle.reduce_k(us, "u16", "sum"))
        # out of place: send untouched, recv = the average
        xs = [_rand("f32", 30011, 900 + r) for r in range(world)]
        x = _to_dev(xs[rank], "f32", dev)
        y = torch.empty_like(x)
        _lib.check(lib.kf_exchange_all_reduce(ex._h, x.data_ptr(), y.data_ptr(), x.numel(),
                                              0x20408, 0, 1, 0,
                                              torch.cuda.current_stream().cuda_stream), "oop")
        torch.cuda.synchronize()
        assert np.array_equal(_to_np(x, "f32"), xs[rank])
        assert np.array_equal(_to_np(y, "f32"), oracle.reduce_avg(xs, "f32", world))
        # SMA, bf16 (auto: the all-to-all fold, fp32 accumulation), one and
        # five buckets (the pipelined schedule blends group by group)
        for sizes in ([20003], [20003, 5, world * 777, 65536 + 1, 3]):
            vs = [[_rand("bf16", n, 300 + 10 * r + j) for j, n in enumerate(sizes)]
                  for r in range(world)]
            v = [_to_dev(vs[rank][j], "bf16", dev) for j in range(len(sizes))]
            ex.sma_(v, 0.1)
            torch.cuda.synchronize()
            for j in range(len(sizes)):
                s = oracle.reduce_k([vs[r][j] for r in range(world)], "bf16", "sum")
                assert np.array_equal(_to_np(v[j], "bf16"),
                                      oracle.sma_blend(vs[rank][j], s, "bf16", world, 0.1)), j

    _loop_ranks(world, body)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_scheduler_orders_across_ranks(world):
    """NCCLScheduler semantics with several ranks: every rank starts the
    step's names in its own order; the issue order is the agreed one (step 0:
    the given order; from step 1 on, rank 0's arrival order of step 0,
    broadcast over the communicator), the same on every rank, and every
    all-reduce is right."""
    import torch
    from kungfu_amd.exchange import Scheduler
    dev = _gpu()
    names = ["grad/%d" % i for i in range(7)]
    orders = {}

    def body(rank, ex):
        sch = Scheduler(ex, auto_order=True)
        rng = np.random.default_rng(rank)
        got = []
        for step in range(3):
            bufs = [torch.full((5000 + i,), float(rank + 1), device=dev) for i in range(7)]
            sch.begin_step(names)
            arrival = list(names) if step else [names[i] for i in rng.permutation(7)]
            if rank == 0 and step == 0:
                arrival = names[3:] + names[:3]
            for nm in arrival:
                sch.start(nm, bufs[names.index(nm)])
            got.append(sch.wait_all())
            torch.cuda.synchronize()
            assert all(torch.all(b == world * (world + 1) / 2) for b in bufs)
        orders[rank] = got

    _loop_ranks(world, body)
    for r in range(world):
        assert orders[r][0] == names
        assert orders[r][1] == names[3:] + names[:3] == orders[r][2]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 3])
def test_sma_overlap_native_same_bits(world):
    """SynchronousAveragingOptimizer(overlap=True) over the native exchange
    (loopback ranks; the next step's sum on the exchange's stream, then the
    batched HIP blend) equals overlap=False (kf_exchange_sma_batch) bit for
    bit, f32 and bf16, over three SGD steps from different replicas."""
    import torch
    from kungfu_amd.optimizers import SynchronousAveragingOptimizer
    dev = _gpu()

    def model(seed, dtype):
        g = torch.Generator(device=dev).manual_seed(seed)
        m = torch.nn.Sequential(torch.nn.Linear(33, 65), torch.nn.Tanh(),
                                torch.nn.Linear(65, 7)).to(dev)
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(torch.randn(p.shape, device=dev, generator=g) * 0.1)
        return m.to(dtype)

    def body(rank, ex):
        for dtype in (torch.float32, torch.bfloat16):
            ms = [model(rank, dtype), model(rank, dtype)]
            opts = [SynchronousAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                                  alpha=0.1, exchange=ex, overlap=ov)
                    for m, ov in zip(ms, (False, True))]
            for step in range(3):
                for m, opt in zip(ms, opts):
                    g = torch.Generator(device=dev).manual_seed(100 * step + rank)
                    x = torch.randn(16, 33, device=dev, generator=g).to(dtype)
                    opt.zero_grad()
                    (m(x).float() ** 2).mean().backward()
                    opt.step()
                torch.cuda.synchronize()
                for a, b in zip(ms[0].parameters(), ms[1].parameters()):
                    assert torch.equal(a.detach(), b.detach()), (dtype, step)

    if world == 1:
        from kungfu_amd.exchange import NativeExchange
        body(0, NativeExchange())
    else:
        _loop_ranks(world, body)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_optimizers_over_native_exchange(world):
    """SynchronousSGDOptimizer / SynchronousAveragingOptimizer with
    exchange=NativeExchange (loopback ranks): the exchanged gradients are the
    rank-order average bit for bit (both algos fold in rank order here), and
    SMA gives the oracle's blend of the rank-order sum."""
    import torch
    from kungfu_amd import ops
    from kungfu_amd.optimizers import SynchronousAveragingOptimizer, SynchronousSGDOptimizer
    dev = _gpu()

    def model(seed):
        g = torch.Generator(device=dev).manual_seed(seed)
        m = torch.nn.Sequential(torch.nn.Linear(33, 65), torch.nn.Tanh(),
                                torch.nn.Linear(65, 7)).to(dev)
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(torch.randn(p.shape, device=dev, generator=g) * 0.1)
        return m

    def loss(m, r, step):
        g = torch.Generator(device=dev).manual_seed(100 * step + r)
        return (m(torch.randn(16, 33, device=dev, generator=g)) ** 2).mean()

    def body(rank, ex):
        for algo in ("auto", "a2a"):
            ex.algo = algo
            m = model(0)
            opt = SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                          named_parameters=m.named_parameters(), exchange=ex)
            for step in range(2):
                snap = [p.detach().clone() for p in m.parameters()]
                grads = []
                for r in range(world):
                    mr = model(0)
                    with torch.no_grad():
                        for a, b in zip(mr.parameters(), snap):
                            a.copy_(b)
                    loss(mr, r, step).backward()
                    grads.append([p.grad.detach().clone() for p in mr.parameters()])
                opt.zero_grad()
                loss(m, rank, step).backward()
                opt.step()
                for j, p in enumerate(m.parameters()):
                    avg = ops.bucket_reduce_avg([grads[r][j].reshape(-1) for r in range(world)],
                                                world).view_as(p)
                    assert torch.equal(p.grad, avg), (algo, step, j)
        m = model(rank)
        allp = [[p.detach().clone() for p in model(r).parameters()] for r in range(world)]
        opt = SynchronousAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.0), alpha=0.1,
                                            exchange=ex)
        loss(m, rank, 0).backward()
        opt.step()
        for j, p in enumerate(m.parameters()):
            s = ops.bucket_reduce([allp[r][j].reshape(-1) for r in range(world)])
            want = allp[rank][j].reshape(-1).clone()
            ops.sma_blend_(want, s, world, 0.1)
            assert torch.equal(p.detach().reshape(-1), want), j

    _loop_ranks(world, body)


@pytest.mark.gpu
def test_native_exchange_configs_full_size():
    """The bench's N > 1 code path at BASELINE's sizes, over the loopback
    transport: C3 (64 x 4 MiB fp32 as 64 grouped buckets, S-SGD, world 2, the
    primary's reduce-scatter algo), C4 (ResNet-50 in 16 buckets, world 4) and C5
    (BERT-base bf16 SMA, world 2, all-to-all fold). The loopback's
    reduce-scatter folds in rank order, so all three are bit-exact against the
    oracle."""
    import json
    import torch
    from kungfu_amd.collective import GradBuckets
    from oracle import oracle
    dev = _gpu()
    models = json.load(open(os.path.join(HERE, "golden", "models.json")))

    def fill(gb, seed, dtype):
        g = torch.Generator(device=dev).manual_seed(seed)
        for v in gb.views:
            v.copy_(torch.randn(v.numel(), device=dev, generator=g).to(dtype))

    # C3, world 2
    n = 64 << 20

    def c3(rank, ex):
        ex.algo = "rs"
        gb = GradBuckets([n], torch.float32, dev, 2, n_buckets=64)
        fill(gb, 40 + rank, torch.float32)
        ex.all_reduce_(gb.buckets, average=True, coalesce=False)
        torch.cuda.synchronize()
        xs = []
        for r in range(2):
            g2 = GradBuckets([n], torch.float32, dev, 2, n_buckets=64)
            fill(g2, 40 + r, torch.float32)
            xs.append(g2.views[0].cpu().numpy())
        assert np.array_equal(gb.views[0].cpu().numpy(), oracle.reduce_avg(xs, "f32", 2))

    _loop_ranks(2, c3)
    # C4, world 4
    sizes = models["resnet50-imagenet"]

    def c4(rank, ex):
        ex.algo = "auto"
        gbs = [GradBuckets(sizes, torch.float32, dev, 4, n_buckets=16) for _ in range(4)]
        for r, gb in enumerate(gbs):
            fill(gb, 500 + r, torch.float32)
        want = [oracle.reduce_avg([gb.buckets[j].cpu().numpy() for gb in gbs], "f32", 4)
                for j in range(16)]
        mine = gbs[rank]
        ex.all_reduce_(mine.buckets, average=True, coalesce=False)
        torch.cuda.synchronize()
        for j, (b, sp) in enumerate(zip(mine.buckets, mine.spans)):
            assert np.array_equal(b[:sp].cpu().numpy(), want[j][:sp]), j

    _loop_ranks(4, c4)
    # C5, world 2
    bert = models["bert"][:201]

    def c5(rank, ex):
        ex.algo = "auto"
        gbs = [GradBuckets(bert, torch.bfloat16, dev, 2, bucket_bytes=16 << 20) for _ in range(2)]
        for r, gb in enumerate(gbs):
            fill(gb, 700 + r, torch.bfloat16)
        mine = gbs[rank]
        before = [_to_np(b, "bf16") for b in mine.buckets]
        sums = [oracle.reduce_k([_to_np(gb.buckets[j], "bf16") for gb in gbs], "bf16", "sum")
                for j in range(len(mine.buckets))]
        ex.sma_(mine.buckets, 0.1)
        torch.cuda.synchronize()
        for j, b in enumerate(mine.buckets):
            assert np.array_equal(_to_np(b, "bf16"),
                                  oracle.sma_blend(before[j], sums[j], "bf16", 2, 0.1)), j

    _loop_ranks(2, c5)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,groups", [("c4", 1), ("c5", 1), ("c4", 4), ("c5", 4)])
def test_native_exchange_configs_world8(cfg, groups):
    """C4 and C5 at the world size BASELINE names for them (8 GPUs), full size,
    through the native exchange over the loopback transport: C4 = ResNet-50's
    25,583,592 fp32 in 16 buckets, S-SGD /np, both algos (auto -> RCCL-shaped
    reduce-scatter, a2a -> rank-order fold); C5 = BERT-base's first 201 tensors
    (109,483,778 bf16), SMA alpha 0.1 (auto -> a2a). The oracle's rank-order
    fold of all 8 ranks is computed once; every rank's buckets must equal it
    bit for bit, with the pipelined schedule (groups = 4) as without it."""
    import json
    import torch
    from kungfu_amd.collective import GradBuckets
    from oracle import oracle
    dev = _gpu()
    world = 8
    models = json.load(open(os.path.join(HERE, "golden", "models.json")))

    def filled(sizes, dtype, seed, **kw):
        gb = GradBuckets(sizes, dtype, dev, world, **kw)
        g = torch.Generator(device=dev).manual_seed(seed)
        for v in gb.views:
            v.copy_(torch.randn(v.numel(), device=dev, generator=g).to(dtype))
        return gb

    if cfg == "c4":
        sizes = models["resnet50-imagenet"]
        assert sum(sizes) == 25583592
        mk = [lambda r=r: filled(sizes, torch.float32, 900 + r, n_buckets=16) for r in range(world)]
        ref = [mk[r]() for r in range(world)]
        want = [oracle.reduce_avg([gb.buckets[j].cpu().numpy() for gb in ref], "f32", world)
                for j in range(16)]
        del ref
        for algo in ("auto", "a2a"):
            def body(rank, ex, algo=algo):
                ex.algo = algo
                ex.set_pipeline(groups)
                mine = mk[rank]()
                ex.all_reduce_(mine.buckets, average=True, coalesce=False)
                torch.cuda.synchronize()
                for j, (b, sp) in enumerate(zip(mine.buckets, mine.spans)):
                    assert np.array_equal(b[:sp].cpu().numpy(), want[j][:sp]), (algo, j)

            _loop_ranks(world, body)
    else:
        bert = models["bert"][:201]
        assert sum(bert) == 109483778
        kw = dict(bucket_bytes=16 << 20)
        mk = [lambda r=r: filled(bert, torch.bfloat16, 1700 + r, **kw) for r in range(world)]
        ref = [mk[r]() for r in range(world)]
        nb = len(ref[0].buckets)
        sums = [oracle.reduce_k([_to_np(gb.buckets[j], "bf16") for gb in ref], "bf16", "sum")
                for j in range(nb)]
        before = [[_to_np(b, "bf16") for b in gb.buckets] for gb in ref]
        del ref

        def body(rank, ex):
            ex.algo = "auto"
            ex.set_pipeline(groups)
            mine = mk[rank]()
            ex.sma_(mine.buckets, 0.1)
            torch.cuda.synchronize()
            for j, b in enumerate(mine.buckets):
                assert np.array_equal(_to_np(b, "bf16"),
                                      oracle.sma_blend(before[rank][j], sums[j], "bf16", world,
                                                       0.1)), (rank, j)

        _loop_ranks(world, body)


_W1_CHILD = r"""
import ctypes, sys
import numpy as np
import torch
sys.path[:0] = [%r, %r]
from kungfu_amd import _lib
from loopback import rccl1_exchange
from kungfu_amd.collective import GradBuckets
from kungfu_amd.exchange import NativeExchange, Scheduler
from oracle import oracle
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
lib = _lib.load()
g = torch.Generator(device=dev).manual_seed(7)
def rnd(n, dt):
    if dt.is_floating_point:
        return torch.randn(n, device=dev, generator=g).to(dt)
    info = torch.iinfo(dt)
    return torch.randint(max(info.min, -2**31), min(info.max, 2**31 - 1), (n,), device=dev,
                         generator=g).to(dt)
for algo in ("rs", "a2a", "auto"):
    ex = rccl1_exchange(algo)
    # C3's shape: 64 grouped 4 MiB buckets, S-SGD average (x / 1 == x)
    gb = GradBuckets([64 << 20], torch.float32, dev, 1, n_buckets=64)
    gb.views[0].copy_(rnd(64 << 20, torch.float32))
    want = gb.views[0].clone()
    ex.all_reduce_(gb.buckets, average=True, coalesce=False)
    torch.cuda.synchronize()
    assert torch.equal(gb.views[0], want), (algo, "c3")
    ex.set_pipeline(4)  # the pipelined schedule: a second stream, events per group
    ex.all_reduce_(gb.buckets, average=True, coalesce=False)
    torch.cuda.synchronize()
    assert torch.equal(gb.views[0], want), (algo, "c3 pipelined")
    vs = [rnd(n, torch.bfloat16) for n in (30001, 1 << 18, 5, 4097)]
    v0 = [v.clone() for v in vs]
    ex.sma_(vs, 0.1)
    torch.cuda.synchronize()
    for v, a in zip(vs, v0):
        want_b = oracle.sma_blend(a.cpu().view(torch.int16).numpy().view(np.uint16),
                                  a.cpu().view(torch.int16).numpy().view(np.uint16),
                                  "bf16", 1, 0.1)
        assert np.array_equal(v.cpu().view(torch.int16).numpy().view(np.uint16), want_b), algo
    ex.set_pipeline(1)
    cases = [(torch.bfloat16, "sum", True), (torch.float16, "sum", False),
             (torch.int32, "max", False), (torch.int64, "sum", False),
             (torch.uint8, "sum", False), (torch.float64, "sum", True),
             (torch.int16, "sum", False)]
    for dt, op, avg in cases:
        bs = [rnd(n, dt) for n in (1 << 20, 4097, 1, 333)]
        w = [b.clone() for b in bs]
        try:
            ex.all_reduce_(bs, op=op, average=avg, coalesce=False)
        except _lib.KungFuAMDError as e:
            # int16 has no RCCL reduction type: only the forced rs algo refuses it
            assert algo == "rs" and dt == torch.int16, (algo, dt, e)
            continue
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip(bs, w)), (algo, dt)
    # out of place, single-bucket entry
    x = rnd(1 << 20, torch.float32)
    y = torch.empty_like(x)
    _lib.check(lib.kf_exchange_all_reduce(ex._h, x.data_ptr(), y.data_ptr(), y.numel(),
                                          0x20408, 0, 1, {"auto": 0, "rs": 1, "a2a": 2}[algo],
                                          torch.cuda.current_stream().cuda_stream), "ar")
    torch.cuda.synchronize()
    assert torch.equal(x, y), (algo, "out of place")
    # SMA batch: v <- (1 - a) v + a (v / 1)
    for dt, name in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
        vs = [rnd(n, dt) for n in (30001, 1 << 18)]
        v0 = [v.cpu().view(torch.int16).numpy().view(np.uint16).copy() if name == "bf16"
              else v.cpu().numpy().copy() for v in vs]
        ex.sma_(vs, 0.1)
        torch.cuda.synchronize()
        for v, a in zip(vs, v0):
            got = (v.cpu().view(torch.int16).numpy().view(np.uint16) if name == "bf16"
                   else v.cpu().numpy())
            assert np.array_equal(got, oracle.sma_blend(a, a, name, 1, 0.1)), (algo, name)
    # overlap handle + the ordered scheduler (its order broadcast is an RCCL call)
    b = rnd(5000, torch.float32)
    w = b.clone()
    ex.start_([b], average=True).wait()
    sch = Scheduler(ex, auto_order=True)
    names = ["g%%d" %% i for i in range(4)]
    bufs = [rnd(1000 + i, torch.float32) for i in range(4)]
    keep = [t.clone() for t in bufs]
    for step in range(2):
        sch.begin_step(names)
        for nm in names[::-1]:
            sch.start(nm, bufs[names.index(nm)], average=True)
        sch.wait_all()
    torch.cuda.synchronize()
    assert torch.equal(b, w) and all(torch.equal(a, c) for a, c in zip(bufs, keep))
    # name-keyed through librccl: the control communicator split off by
    # ncclCommSplit and the negotiation's all-gathers run with one rank
    nb = [rnd(1000 + 7 * i, torch.float32) for i in range(5)]
    nk = [t.clone() for t in nb]
    for i in (3, 1, 4, 0, 2):
        ex.all_reduce_named("w%%d" %% i, nb[i], average=True)
    ex.wait_named()
    torch.cuda.synchronize()
    assert all(torch.equal(a, c) for a, c in zip(nb, nk)), (algo, "named")
    # gpu_collective::new_group through ncclCommSplit
    sub = ex.split(0)
    assert sub is not None and sub.world == 1
    t = rnd(4097, torch.float32)
    t0 = t.clone()
    sub.all_reduce_([t], average=True)
    torch.cuda.synchronize()
    assert torch.equal(t, t0), (algo, "split")
    sub.close()
    ex.check()
    ex.close()
print("W1_RCCL_OK")
"""


@pytest.mark.gpu
def test_world1_rccl_entry_points():
    """A one-rank exchange through librccl's own entry points (the test
    library's rccl1 transport, which has no world-1 copy: reduce-scatter / all-to-all /
    all-gather groups, the batched epilogue, the order broadcast) with the
    exchange's exact arguments — C3's 64 grouped buckets, every RCCL dtype
    and the all-to-all-only int16, in and out of place, SMA, the scheduler —
    so the real RCCL calls run on a one-GPU box (two ranks on one device
    are refused by RCCL; the multi-rank logic is the loopback tests')."""
    import subprocess
    import sys
    _gpu()
    r = subprocess.run([sys.executable, "-c", _W1_CHILD % (os.path.dirname(HERE), HERE)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "W1_RCCL_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.gpu
@pytest.mark.parametrize("name,np_", [("f32", 8), ("f32", 3), ("bf16", 8), ("bf16", 7),
                                      ("f16", 2), ("f64", 5)])
def test_sma_blend_batch_matches_single(name, np_):
    """kf_sma_blend_batch over 20 ragged buckets (more than one launch of 16;
    sizes 0, 1, 7, ...; one bucket whose v and sum sit at different residues,
    so it takes the element-wise body) equals one kf_sma_blend per bucket
    bit for bit, and the oracle's blend for f32 / bf16."""
    import torch
    from kungfu_amd import ops
    from oracle import oracle
    dev = _gpu()
    sizes = [0, 1, 7, 4099, 1 << 20, 262147, 33] + [4096 * (i + 1) + i for i in range(13)]
    vs0 = [_rand(name, n, 10 + b) for b, n in enumerate(sizes)]
    ss = [_rand(name, n, 500 + b) for b, n in enumerate(sizes)]
    a = [_to_dev(v, name, dev) for v in vs0]
    s = [_to_dev(x, name, dev) for x in ss]
    # bucket 3: the sum one element past an aligned start, v aligned
    s[3] = torch.cat([s[3][:1], s[3]])[1:]
    b = [t.clone() for t in a]
    ops.sma_blend_batch_(a, s, np_, 0.1)
    for v, x in zip(b, s):
        ops.sma_blend_(v, x, np_, 0.1)
    torch.cuda.synchronize()
    for j in range(len(sizes)):
        assert np.array_equal(_to_np(a[j], name), _to_np(b[j], name)), j
        if name in ("f32", "bf16"):
            want = oracle.sma_blend(vs0[j], ss[j], name, np_, 0.1)
            assert np.array_equal(_to_np(a[j], name), want), j


@pytest.mark.gpu
@pytest.mark.parametrize("name,np_", [("f32", 8), ("bf16", 8), ("bf16", 3), ("f16", 2),
                                      ("f64", 5)])
def test_sma_blend_batch_contiguous_runs(name, np_):
    """Buckets back to back in v AND in the sums (GradBuckets' flat layout,
    collective.workspace_like) are blended by kf_sma_blend_batch as merged
    ranges — here three runs: 5 ragged buckets, then a bucket whose sum is
    elsewhere (breaks the run), then 4 more, 20 k elements in the middle of a
    run starting at an odd offset — bit-identical to one kf_sma_blend per
    bucket and to the oracle."""
    import torch
    from kungfu_amd import ops
    from oracle import oracle
    dev = _gpu()
    sizes = [7, 4099, 1 << 18, 33, 262147, 1000, 3, 20001, 65536, 5]
    total = sum(sizes)
    v_np = _rand(name, total + 1, 31)[1:]  # the flat v starts one element in
    s_np = _rand(name, total + 1, 77)[1:]
    vflat = _to_dev(_rand(name, total + 1, 31), name, dev)[1:]
    sflat = _to_dev(_rand(name, total + 1, 77), name, dev)[1:]
    offs = np.cumsum([0] + sizes)
    a = [vflat[offs[i]:offs[i + 1]] for i in range(len(sizes))]
    s = [sflat[offs[i]:offs[i + 1]] for i in range(len(sizes))]
    s[5] = s[5].clone()  # its sum elsewhere: the run breaks around it
    b = [t.clone() for t in a]
    ops.sma_blend_batch_(a, s, np_, 0.1)
    for v, x in zip(b, s):
        ops.sma_blend_(v, x, np_, 0.1)
    torch.cuda.synchronize()
    for j, n in enumerate(sizes):
        assert np.array_equal(_to_np(a[j], name), _to_np(b[j], name)), j
        if name in ("f32", "bf16"):
            want = oracle.sma_blend(v_np[offs[j]:offs[j + 1]], s_np[offs[j]:offs[j + 1]], name,
                                    np_, 0.1)
            assert np.array_equal(_to_np(a[j], name), want), j


# ---- name-keyed all-reduce and splits ----------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["auto", "a2a"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_named_all_reduce_any_order(world, algo):
    """kf_exchange_all_reduce_named: every rank starts the step's names in its
    own random order, with random gaps, from its own thread; tensors pair by
    name (the reference's per-name mailbox, handler/collective.go:48-64), so
    each result is the oracle's rank-order fold of that name's buffers on
    every rank. Three steps reuse the names; f32 /np, bf16, i32 MAX and a u16
    SUM (all-to-all fold) are mixed, so one cycle can complete names of
    different kinds (one batched call per kind). algo "a2a": the f32 and i32
    names go through the all-to-all and the HIP rank-order fold too (under
    "auto" they take the transport's reduce-scatter, which the loopback does
    on the host), so the product's fold is what is checked at world > 1."""
    import time
    import torch
    from oracle import oracle
    dev = _gpu()
    kinds = [("f32", "sum", True), ("bf16", "sum", False), ("i32", "max", False),
             ("u16", "sum", False)]
    names = ["t%02d/%s" % (i, kinds[i % 4][0]) for i in range(14)]
    sizes = [1, 7, 4099, 100003, world * 1000 + 1, 65536, 3, 262147, 5, 777, 1 << 16, 9, 31,
             4096]

    def data(r, step, i):
        name = kinds[i % 4][0]
        if name == "u16":
            return np.random.default_rng(7 * r + 1000 * step + i).integers(
                0, 65535, sizes[i]).astype(np.uint16)
        return _rand(name, sizes[i], 10000 * step + 100 * r + i)

    def body(rank, ex):
        import torch
        ex.algo = algo
        s = torch.cuda.Stream()
        for step in range(3):
            rng = np.random.default_rng(31 * rank + step)
            hs = [data(rank, step, i) for i in range(len(names))]
            bufs = []
            for i, h in enumerate(hs):
                if kinds[i % 4][0] == "u16":
                    bufs.append(torch.from_numpy(h.view(np.int16)).to(dev))
                else:
                    bufs.append(_to_dev(h, kinds[i % 4][0], dev))
            torch.cuda.synchronize()
            seen = []
            with torch.cuda.stream(s):
                for i in rng.permutation(len(names)):
                    time.sleep(float(rng.random()) * 0.002)
                    name, op, avg = kinds[i % 4]
                    if name == "u16":
                        from kungfu_amd import _lib
                        cb = _lib.DONE_FN(lambda st, a: seen.append(st))
                        ex._named_keep = getattr(ex, "_named_keep", []) + [cb]
                        _lib.check(ex.lib.kf_exchange_all_reduce_named(
                            ex._h, names[i].encode(), bufs[i].data_ptr(), bufs[i].data_ptr(),
                            bufs[i].numel(), 0x00208, 0, 0, 2 if algo == "a2a" else 0,
                            s.cuda_stream, cb, None), "u16")
                    else:
                        ex.all_reduce_named(names[i], bufs[i], op=op, average=avg,
                                            callback=lambda n, st: seen.append(st))
            ex.wait_named()
            assert len(seen) == len(names) and all(st == 0 for st in seen), seen
            for i in range(len(names)):
                name, op, avg = kinds[i % 4]
                ins = [data(r, step, i) for r in range(world)]
                if avg:
                    want = oracle.reduce_avg(ins, name, world)
                else:
                    want = oracle.reduce_k(ins, name, op)
                got = (bufs[i].cpu().numpy().view(np.uint16) if name == "u16"
                       else _to_np(bufs[i], name))
                assert np.array_equal(got, want), (step, names[i])

    _loop_ranks(world, body)


@pytest.mark.gpu
def test_named_all_reduce_mismatch_fails_on_every_rank():
    """A name whose count differs across ranks fails with KF_ERR_ARG on every
    rank (no collective is issued for it); the other names still complete."""
    import threading
    import torch
    from kungfu_amd import _lib
    dev = _gpu()
    world = 2
    bar = threading.Barrier(world)

    def body(rank, ex):
        import torch
        ok = torch.full((1000,), float(rank + 1), device=dev)
        bad = torch.ones(100 + rank, device=dev)
        st = {}
        ex.all_reduce_named("bad", bad, callback=lambda n, s: st.__setitem__(n, s))
        ex.all_reduce_named("ok", ok, callback=lambda n, s: st.__setitem__(n, s))
        with pytest.raises(_lib.KungFuAMDError, match="differ across ranks"):
            ex.wait_named()
        assert st == {"bad": 3, "ok": 0}, st
        assert torch.all(ok == 3.0)
        # the exchange keeps working, and a name may be reused
        ex.all_reduce_named("bad", torch.ones(5, device=dev))
        ex.wait_named()
        # one name outstanding twice is refused at once (rank 1 starts it only
        # after rank 0 checked, so rank 0's cannot have been issued yet)
        x = torch.ones(8, device=dev)
        if rank == 0:
            ex.all_reduce_named("twice", x)
            with pytest.raises(_lib.KungFuAMDError, match="outstanding"):
                ex.all_reduce_named("twice", x)
            bar.wait()
        else:
            bar.wait()
            ex.all_reduce_named("twice", x)
        ex.wait_named()
        assert torch.all(x == 2.0)

    _loop_ranks(world, body)


@pytest.mark.gpu
def test_split_local_scope():
    """kf_exchange_split (gpu_collective::new_local / new_group): world 4 as 2
    emulated hosts of 2 ranks (color = rank // 2); each sub-exchange
    all-reduces within its host only, ranks ordered by key (here reversed), and
    color -1 joins none. A second split of the sub-exchange still works."""
    import torch
    from oracle import oracle
    dev = _gpu()
    world = 4
    xs = [_rand("f32", 30011, 50 + r) for r in range(world)]

    def body(rank, ex):
        import torch
        loc = ex.split(rank // 2, key=-rank)
        assert (loc.world, loc.rank) == (2, 1 - rank % 2), (loc.world, loc.rank)
        x = _to_dev(xs[rank], "f32", dev)
        loc.all_reduce_([x], average=True)
        torch.cuda.synchronize()
        host = [xs[2 * (rank // 2) + 1], xs[2 * (rank // 2)]]  # the sub-exchange's rank order
        assert np.array_equal(_to_np(x, "f32"), oracle.reduce_avg(host, "f32", 2))
        none = ex.split(-1 if rank == 3 else 0)
        assert (none is None) == (rank == 3)
        if none is not None:
            assert none.world == 3
            none.close()
        solo = loc.split(loc.rank)
        assert solo.world == 1
        solo.close()
        loc.close()

    _loop_ranks(world, body)
