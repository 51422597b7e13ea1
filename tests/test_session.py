"""Single-host Session (kungfu_amd/session.py) over the rchannel wire format:
np peers as processes on unix sockets, STAR strategy, chunked by 1 MiB.
Host mode runs on CPU with the oracle as the injected fold; device mode
(pinned ingest + HIP fold) is the -m gpu variant. Expected values: the
reference KATs and the oracle folded in every possible arrival order."""
import itertools
import os
import sys
import tempfile
import traceback

import numpy as np
import pytest
import multiprocessing as mp
from procs import hung_msg, join_all

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def oracle_reduce_fn():
    """C address of the oracle's transform2 (kf_host_reduce_fn signature)."""
    import ctypes
    from oracle import oracle
    return ctypes.cast(oracle.lib().oracle_transform2, ctypes.c_void_p)


def inputs(rank, n, kind):
    if kind == "iota":  # fake_agent.cpp:15-44
        return np.arange(n, dtype=np.int32)
    if kind == "c1":  # x_r[i] = (r+1) * (i mod 1024) / 1024
        return ((rank + 1) * (np.arange(n) % 1024) / 1024).astype(np.float32)
    return np.random.default_rng(40 + rank).standard_normal(n).astype(np.float32)


def _body(rank, size, sock_dir, mode, kind, n, errq, strategy=None, env=None):
    sys.path[:0] = [ROOT, HERE]
    os.environ.update(env or {})
    try:
        from kungfu_amd.session import Session
        if strategy is not None:
            os.environ["KUNGFU_ALLREDUCE_STRATEGY"] = strategy  # as kungfu-run sets it
        if mode == "device":
            import torch
            dev = torch.device("cuda:0")
            x = torch.from_numpy(inputs(rank, n, kind)).to(dev)
            y = torch.zeros_like(x)
            s = Session(rank, size, sock_dir, mode="device")
            s.all_reduce(x, y, "NegotiatedGrad_0/AllReduce")
            got = y.cpu().numpy()
            z = x.clone()
            s.all_reduce(z, z, "inplace")  # in place: SendBuf is RecvBuf
            got_inplace = z.cpu().numpy()
        else:
            x = inputs(rank, n, kind)
            y = np.zeros_like(x)
            s = Session(rank, size, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn())
            s.all_reduce(x, y, "NegotiatedGrad_0/AllReduce")
            got = y
            z = x.copy()
            s.all_reduce(z, z, "inplace")
            got_inplace = z
        s.close()
        # the parent checks every rank's results once (the expected chunks are
        # the same for every rank: one computation instead of one per rank)
        np.save(os.path.join(sock_dir, "got%d.npy" % rank), got)
        np.save(os.path.join(sock_dir, "inplace%d.npy" % rank), got_inplace)
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def check(rank, size, kind, n, got):
    from oracle import oracle
    xs = [inputs(r, n, kind) for r in range(size)]
    if kind == "iota":
        assert np.array_equal(got, np.arange(n, dtype=np.int32) * size)
        return
    if kind == "c1":
        assert np.array_equal(got, sum(xs))  # exact in fp32
        return
    # arrival order may differ per chunk: each chunk must equal the root's
    # fold x0 o x_a o x_b ... for SOME order of the peers
    k = (n * 4 + (1 << 20) - 1) >> 20
    from kungfu_amd.base import EvenPartition
    for b, e in EvenPartition(0, n, k):
        opts = [oracle.reduce_k([xs[0][b:e]] + [xs[p][b:e] for p in perm], "f32")
                for perm in itertools.permutations(range(1, size))]
        assert any(np.array_equal(got[b:e], o) for o in opts), (rank, b, e)


def check_strategy(size, kind, n, strategy, name, got):
    """Every chunk equals the reference schedule (oracle/schedule.py) for this
    strategy under SOME arrival order; RING has exactly one order."""
    from oracle import schedule
    xs = [inputs(r, n, kind) for r in range(size)]
    dt = "i32" if kind == "iota" else "f32"
    multi = [r for r in range(size)]  # nodes whose prevs may arrive in any order
    outs = []
    for perms in itertools.product(*[list(itertools.permutations(range(size)))] * 1):
        order = perms[0]

        def arrival(r, prevs, order=order):
            return sorted(prevs, key=order.index)
        outs.append(schedule.all_reduce(xs, dt, "sum", strategy=strategy, name=name,
                                        arrival=arrival)[0])
    del multi
    k = (n * 4 + (1 << 20) - 1) >> 20
    from kungfu_amd.base import EvenPartition
    for b, e in EvenPartition(0, n, k):
        assert any(np.array_equal(got[b:e], o[b:e]) for o in outs), (strategy, b, e)
    if strategy == "RING":
        assert all(np.array_equal(outs[0], o) for o in outs)  # order-free


def _matrix(axes, keep):
    """The product of `axes` (lists of tuples), each case flattened; every
    case not in `keep` is marked gpu_slow (conftest.py)."""
    import itertools
    out = []
    for combo in itertools.product(*axes):
        case = tuple(v for part in combo for v in part)
        marks = () if case in keep else (pytest.mark.gpu_slow,)
        out.append(pytest.param(*case, marks=marks))
    return out


def run(size, mode, kind, n, strategy=None, env=None):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_body, args=(r, size, d, mode, kind, n, errq, strategy, env))
              for r in range(size)]
        for p in ps:
            p.start()
        hung = join_all(ps, 180)
        errs = []
        while not errq.empty():
            errs.append(errq.get())
        assert not errs, "\n".join(errs)
        assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])
        gots = [(np.load(os.path.join(d, "got%d.npy" % r)),
                 np.load(os.path.join(d, "inplace%d.npy" % r))) for r in range(size)]
    # every rank ends with the same bucket (the bcast of each chunk's root)
    for r in range(1, size):
        assert np.array_equal(gots[r][0], gots[0][0]), ("rank differs", r)
        assert np.array_equal(gots[r][1], gots[0][1]), ("rank differs (in place)", r)
    if strategy is not None:
        check_strategy(size, kind, n, strategy, "NegotiatedGrad_0/AllReduce", gots[0][0])
        check_strategy(size, kind, n, strategy, "inplace", gots[0][1])
    else:
        check(0, size, kind, n, gots[0][0])
        check(0, size, kind, n, gots[0][1])


@pytest.mark.parametrize("size,kind,n", [(2, "iota", 8), (3, "iota", 12),
                                         (2, "c1", 1 << 20), (2, "rand", 300007),
                                         (3, "rand", 600011)])
def test_session_host_mode(size, kind, n):
    run(size, "host", kind, n)


@pytest.mark.parametrize("threads,strategy", [("0", "STAR"), ("1", "RING"), ("3", "BINARY_TREE"),
                                              ("3", "STAR")])
def test_session_host_fold_workers(threads, strategy):
    """Host mode folds each received chunk on a worker (the goroutine per
    chunk) while the poll thread reads the next one; 0 folds inline on the
    poll thread. Same schedule, same bits, at 4 peers and three chunks (the
    default pool of min(8, cores) workers runs every other host-mode test)."""
    run(4, "host", "rand", (3 << 20) // 4 + 7, strategy=strategy,
        env={"KUNGFU_AMD_HOST_FOLD_THREADS": threads})


@pytest.mark.parametrize("strategy", ["RING", "CLIQUE", "BINARY_TREE", "STAR",
                                      "BINARY_TREE_STAR", "AUTO"])
@pytest.mark.parametrize("size", [2, 3, 4])
def test_session_strategies_host(strategy, size):
    # 1 MiB chunks, so each chunk of the 5-chunk bucket picks its own root
    run(size, "host", "rand", (5 << 20) // 4 + 17, strategy=strategy)


def test_session_strategies_iota():
    for strategy in ("RING", "CLIQUE", "BINARY_TREE"):
        run(4, "host", "iota", 16, strategy=strategy)


def test_session_single_peer_forward():
    from kungfu_amd.session import Session
    with tempfile.TemporaryDirectory() as d:
        s = Session(0, 1, d, mode="host", host_reduce_fn=oracle_reduce_fn())
        x = np.arange(10, dtype=np.int32) + 1
        y = np.zeros_like(x)
        s.all_reduce(x, y, "t")
        assert np.array_equal(y, x)  # test_operations.cpp:3-26
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("size,kind,n", [(2, "c1", 1 << 20), (2, "rand", 300007),
                                         (3, "rand", 600011), (2, "iota", 8)])
def test_session_device_mode(size, kind, n):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(size, "device", kind, n)


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,size,batch_fold", _matrix(
    [[("RING", 3), ("RING", 4), ("CLIQUE", 3), ("BINARY_TREE", 4), ("STAR", 4), ("CLIQUE", 4)],
     [("1",), ("0",)]],
    keep={(st, n, "0") for st, n in [("RING", 3), ("RING", 4), ("CLIQUE", 3), ("BINARY_TREE", 4),
                                      ("STAR", 4), ("CLIQUE", 4)]} |
    {("STAR", 4, "1"), ("BINARY_TREE", 4, "1")}))
def test_session_device_strategies(strategy, size, batch_fold):
    # batch_fold=1: nodes with >= 2 reduce predecessors (star/clique roots,
    # binary-tree inner nodes) stage the arrivals in HBM and fold them in one
    # k-input launch; 0: the reference's chain of 2-input recvOnto folds.
    # Either way each chunk must equal the schedule for some arrival order.
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(size, "device", "rand", (5 << 20) // 4 + 17, strategy=strategy,
        env={"KUNGFU_AMD_BATCH_FOLD": batch_fold})


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,size,piece_kb", _matrix(
    [[("STAR", 2), ("RING", 3), ("BINARY_TREE", 4), ("CLIQUE", 3)], [("256",), ("64",), ("300",)]],
    keep={("CLIQUE", 3, "300"), ("BINARY_TREE", 4, "64")}))
def test_session_device_pieces(strategy, size, piece_kb):
    """Device mode can move a chunk through each stage in pieces
    (KUNGFU_AMD_PIECE_KB; default 0 = whole chunks): the D2H before a send,
    the fold or copy after a receive, the send of a fold's result written
    piece by piece as each piece's fold ends, one whole message per successor
    at a time (CLIQUE at np = 3 deadlocked when a root interleaved two
    successors' messages). 300 KiB (rounded down to 296 KiB, whole 4 KiB)
    leaves a ragged last piece in every chunk of the ragged bucket. Same
    schedule, same bits."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(size, "device", "rand", (5 << 20) // 4 + 17, strategy=strategy,
        env={"KUNGFU_AMD_PIECE_KB": piece_kb})


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,size,piece_kb,kind,batch_fold", _matrix(
    [[("STAR", 2), ("RING", 3), ("BINARY_TREE", 4), ("CLIQUE", 3), ("STAR", 4)],
     [("64", "rand", "1"), ("4", "rand", "0"), ("300", "iota", "1"), ("1024", "rand", "0")]],
    # r04's abort was [RING-3-4-rand-0] (driver) and [RING-3-1024-rand-0] (builder)
    keep={("RING", 3, "4", "rand", "0"), ("RING", 3, "1024", "rand", "0"),
          ("STAR", 4, "64", "rand", "1"), ("CLIQUE", 3, "300", "iota", "1"),
          ("BINARY_TREE", 4, "1024", "rand", "0")}))
def test_session_device_streamed(strategy, size, piece_kb, kind, batch_fold):
    """KUNGFU_AMD_STREAM=1: one kernel per received chunk, launched before
    its body arrives, folds (the completing 2-input fold) or copies (bcast)
    each 4 KiB as the socket delivers it, and marks pieces of
    KUNGFU_AMD_STREAM_PIECE_KB done in page-locked memory; the sender writes
    each piece of a folded chunk (and of a leaf's copy out of HBM, also one
    kernel) as soon as all its 4 KiB blocks are flagged. 4 KiB pieces are
    single blocks; 300 KiB leaves ragged pieces. Same schedule, same bits as
    the whole-chunk path."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(size, "device", kind, (5 << 20) // 4 + 17, strategy=strategy,
        env={"KUNGFU_AMD_STREAM": "1", "KUNGFU_AMD_STREAM_PIECE_KB": piece_kb,
             "KUNGFU_AMD_BATCH_FOLD": batch_fold, "KUNGFU_AMD_STREAM_TIMEOUT_MS": "20000"})


_DT_ITEM = {"f16": 2, "bf16": 2, "f32": 4, "f64": 8, "i8": 1, "u8": 1, "i16": 2, "u16": 2,
            "i32": 4, "i64": 8, "u32": 4, "u64": 8}


def _dt_inputs(rank, dt, n):
    from oracle import oracle
    rng = np.random.default_rng(700 + rank)
    if dt == "bf16":
        return oracle.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32))
    if dt in ("f16", "f32", "f64"):
        return rng.standard_normal(n).astype(oracle.NP[dt])
    info = np.iinfo(oracle.NP[dt])
    return rng.integers(info.min, info.max, n, endpoint=True, dtype=oracle.NP[dt])


def _dt_to_dev(a, dt):
    import torch
    if dt == "bf16":
        return torch.from_numpy(a.view(np.int16)).view(torch.bfloat16).to("cuda:0")
    if dt in ("u16", "u32", "u64"):
        signed = {"u16": np.int16, "u32": np.int32, "u64": np.int64}[dt]
        tdt = getattr(torch, {"u16": "uint16", "u32": "uint32", "u64": "uint64"}[dt])
        return torch.from_numpy(a.view(signed)).view(tdt).to("cuda:0")
    return torch.from_numpy(a).to("cuda:0")


def _dt_to_np(t, dt):
    import torch
    if dt in ("bf16", "u16"):
        return t.cpu().view(torch.int16).numpy().view(np.uint16)
    if dt in ("u32", "u64"):
        signed = {"u32": torch.int32, "u64": torch.int64}[dt]
        return t.cpu().view(signed).numpy().view({"u32": np.uint32, "u64": np.uint64}[dt])
    return t.cpu().numpy()


def _dtype_body(rank, size, sock_dir, dt, n, errq, env, op="sum", mode="device"):
    sys.path[:0] = [ROOT, HERE]
    os.environ.update(env)
    try:
        from kungfu_amd.session import Session
        if mode == "device":
            x = _dt_to_dev(_dt_inputs(rank, dt, n), dt)
            y = x.clone().zero_()
            s = Session(rank, size, sock_dir, mode="device")
        else:
            x = _dt_inputs(rank, dt, n)
            y = np.zeros_like(x)
            s = Session(rank, size, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn())
        s.all_reduce(x, y, "dt/%s" % dt, op=op)
        z = x.clone() if mode == "device" else x.copy()
        s.all_reduce(z, z, "dt/%s/inplace" % dt, op=op)
        s.close()
        conv = (lambda t: _dt_to_np(t, dt)) if mode == "device" else (lambda a: a)
        np.save(os.path.join(sock_dir, "got%d.npy" % rank), conv(y))
        np.save(os.path.join(sock_dir, "inplace%d.npy" % rank), conv(z))
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def _run_dtype(dt, n, env, op="sum", mode="device", size=3):
    """np = `size` peers under RING (fixed accumulation order); every rank's
    out-of-place and in-place results against the schedule oracle."""
    from oracle import schedule
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    env = dict(env, KUNGFU_ALLREDUCE_STRATEGY="RING")
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_dtype_body, args=(r, size, d, dt, n, errq, env, op, mode))
              for r in range(size)]
        for p in ps:
            p.start()
        hung = join_all(ps, 180)
        errs = []
        while not errq.empty():
            errs.append(errq.get())
        assert not errs, "\n".join(errs)
        assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])
        gots = [(np.load(os.path.join(d, "got%d.npy" % r)),
                 np.load(os.path.join(d, "inplace%d.npy" % r))) for r in range(size)]
    xs = [_dt_inputs(r, dt, n) for r in range(size)]
    for name, which in (("dt/%s" % dt, 0), ("dt/%s/inplace" % dt, 1)):
        want = schedule.all_reduce(xs, dt, op, strategy="RING", name=name)[0]
        for r in range(size):
            assert np.array_equal(gots[r][which], want), (dt, op, name, r)


@pytest.mark.gpu
@pytest.mark.parametrize("stages", ["fold", pytest.param("1", marks=pytest.mark.gpu_slow)])
@pytest.mark.parametrize("dt", ["f16", "bf16", "f64", "i8", "u8", "i16", "u16", "i64", "u64"])
def test_session_device_dtypes(dt, stages):
    """Every dtype the streamed fold supports (kf_stream.hip fold_kernel<T>,
    the dtype's own arithmetic: kf_reduce_kernels.hpp Elt<T>) through a
    device-mode session: np = 3 under RING, whose accumulation order is fixed,
    2.5 MiB + 3 elements per rank (three chunks, a ragged one), out of place
    and in place, each chunk equal bit for bit to the schedule oracle
    (oracle/schedule.py over the oracle's own two-input fold, pinned by the
    reference's compiled std_transform_2). bf16 has no reference (parity
    unpinned: the build's fp32-accumulate-then-round per hop)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if dt in ("u16", "u64") and not hasattr(torch, {"u16": "uint16", "u64": "uint64"}[dt]):
        pytest.skip("torch has no %s" % dt)
    _run_dtype(dt, (5 << 19) // _DT_ITEM[dt] + 3, {"KUNGFU_AMD_STREAM": stages})


_OP_CASES = [("f32", "min"), ("f32", "max"), ("f32", "prod"), ("i32", "min"), ("i32", "max"),
             ("i32", "prod"), ("f64", "max"), ("i8", "prod"), ("u16", "min")]


@pytest.mark.parametrize("dt,op", _OP_CASES)
def test_session_host_ops(dt, op):
    """MIN / MAX / PROD through the session engine (KungFu_Op reaches every
    fold; the reference's call_as<T>, op.cpp:22-43, via the oracle's fold as
    the host callback): np = 3 RING, three chunks, out of place and in place,
    against the schedule oracle."""
    _run_dtype(dt, (5 << 19) // _DT_ITEM[dt] + 3, {}, op=op, mode="host")


@pytest.mark.gpu
@pytest.mark.parametrize("dt,op", _OP_CASES)
def test_session_device_ops(dt, op):
    """The same through device-mode sessions: non-SUM ops take the
    whole-chunk HIP fold (the streamed fold is SUM only), bit-exact vs the
    schedule oracle (MIN / MAX select an input, so no rounding question)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if dt == "u16" and not hasattr(torch, "uint16"):
        pytest.skip("torch has no uint16")
    _run_dtype(dt, (5 << 19) // _DT_ITEM[dt] + 3, {}, op=op, mode="device")


@pytest.mark.gpu
@pytest.mark.gpu_slow  # a stress case (40 chunks, 4 KiB pieces); the streamed
# stages keep their default-tier cases in test_session_device_streamed_*
def test_session_device_streamed_stress():
    """the streamed kernels write page-locked memory the
    host sender reads after per-block flags. Every byte of a 40-chunk bucket
    per call, every stage streamed (copy out, fold, copy in), 4 KiB pieces
    (one block per piece: the most flags), np = 3 under RING, whose result is
    order-free, so each chunk is checked exactly against the schedule oracle;
    out of place and in place."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(3, "device", "rand", (40 << 20) // 4 + 5, strategy="RING",
        env={"KUNGFU_AMD_STREAM": "1", "KUNGFU_AMD_STREAM_PIECE_KB": "4"})


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["RING", pytest.param("BINARY_TREE",
                                                           marks=pytest.mark.gpu_slow)])
def test_session_device_streamed_launch_race(strategy):
    """rank 2 of [RING-3-4-rand-0] aborted in the HIP
    runtime ("Cannot create GlobalVar Obj for symbol ... g_seen") when the
    poll thread's first streamed launch resolved a module-scope __device__
    array while the sender thread launched copy_out_kernel. The words are now
    the session's (hipMalloc'd before its threads start) and every kf_stream
    kernel is resolved on the creating thread. KUNGFU_AMD_TEST_LAUNCH_RACE=1
    holds the first copy-out launch and the first streamed fold / copy-in
    launch of each rank until both are ready, so they are issued together,
    at np = 3 with every stage streamed; same bits as the schedule."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(3, "device", "rand", (5 << 20) // 4 + 17, strategy=strategy,
        env={"KUNGFU_AMD_STREAM": "1", "KUNGFU_AMD_STREAM_PIECE_KB": "4",
             "KUNGFU_AMD_TEST_LAUNCH_RACE": "1", "KUNGFU_AMD_STREAM_TIMEOUT_MS": "20000"})


@pytest.mark.gpu
@pytest.mark.parametrize("stages", ["0", "out", "fold", "in", "out+in", "fold+last+idle"])
def test_session_device_streamed_stages(stages):
    """KUNGFU_AMD_STREAM names the stages streamed (default "fold"); each
    alone (and the two that touch only one side of a hop) beside the
    whole-chunk others gives the same bits, at np = 3 under BINARY_TREE
    (inner fold, leaf copies); "0" moves every chunk whole."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(3, "device", "rand", (5 << 20) // 4 + 17, strategy="BINARY_TREE",
        env={"KUNGFU_AMD_STREAM": stages, "KUNGFU_AMD_BATCH_FOLD": "0"})


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,size,stages", [
    pytest.param("STAR", 2, "fold", marks=pytest.mark.gpu_slow),
    pytest.param("BINARY_TREE", 4, "0", marks=pytest.mark.gpu_slow),
    pytest.param("CLIQUE", 3, "fold", marks=pytest.mark.gpu_slow), ("RING", 3, "1")])
def test_session_device_copy_kernels(strategy, size, stages):
    """KUNGFU_AMD_COPY_KERNEL=1: a chunk's copies between HBM and page-locked
    memory (the D2H into a send slot, the H2D out of a landing slot, the
    mirror's copy to HBM) run as kernels instead of DMA copies; same bits,
    with and without the streamed stages (a ragged last chunk included)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(size, "device", "rand", (5 << 20) // 4 + 17, strategy=strategy,
        env={"KUNGFU_AMD_COPY_KERNEL": "1", "KUNGFU_AMD_STREAM": stages})


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["STAR", "BINARY_TREE", "CLIQUE"])
def test_session_device_lease_caps(strategy):
    """HBM staging and page-locked mirrors come from
    pools capped in bytes; a call that would pass the cap goes without (the
    chain of 2-input folds, the D2H send) instead of failing. Caps of 1 MiB
    refuse every lease of a 5 MiB bucket: same schedule, same bits."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(4, "device", "rand", (5 << 20) // 4 + 17, strategy=strategy,
        env={"KUNGFU_AMD_STAGE_CAP_MB": "1", "KUNGFU_AMD_MIRROR_CAP_MB": "1",
             "KUNGFU_AMD_BATCH_FOLD": "1"})


@pytest.mark.gpu
def test_session_async_any_order_device_capped():
    """Calls in flight at once share the capped pools: some get staging and a
    mirror, the rest fall back (12 MiB caps, six names of 1-6 chunks)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_any_order(3, "device", None, env={"KUNGFU_AMD_STAGE_CAP_MB": "12",
                                           "KUNGFU_AMD_MIRROR_CAP_MB": "6",
                                           "KUNGFU_AMD_BATCH_FOLD": "1"})


@pytest.mark.gpu
def test_session_device_batched_iota():
    # fake_agent.cpp:15-44 KAT (iota * np) through the k-input fold at np=4
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run(4, "device", "iota", (3 << 20) // 4 + 5, env={"KUNGFU_AMD_BATCH_FOLD": "1"})


def _repeat_body(rank, size, sock_dir, strategy, steps, errq):
    sys.path[:0] = [ROOT, HERE]
    try:
        os.environ["KUNGFU_ALLREDUCE_STRATEGY"] = strategy
        from kungfu_amd.session import Session
        s = Session(rank, size, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn())
        n = (3 << 20) // 4 + 5
        for t in range(steps):
            # the same name every step, as an optimizer's gradient all-reduce
            x = (np.arange(n) * (rank + 1) + t).astype(np.int32)
            y = np.zeros_like(x)
            s.all_reduce(x, y, "grad")
            want = (np.arange(n) * (size * (size + 1) // 2) + size * t).astype(np.int32)
            assert np.array_equal(y, want), (rank, t)
        s.close()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


@pytest.mark.parametrize("strategy,size", [("RING", 4), ("BINARY_TREE", 5), ("CLIQUE", 3),
                                           ("STAR", 4)])
def test_session_same_name_back_to_back(strategy, size):
    # a peer that finished step t may send step t+1's message for a chunk
    # while this peer still polls for step t: it must wait for step t+1
    # (the reference's per-name mailbox, handler/collective.go:27-61)
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_repeat_body, args=(r, size, d, strategy, 40, errq))
              for r in range(size)]
        for p in ps:
            p.start()
        hung = join_all(ps, 180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


def _fake_peer(sock_dir, token, msgs, n_bcast, out, err):
    """Rank 1 of 2 speaking the rchannel protocol by hand: sends `msgs`
    (name, flags, payload) in the given order, then reads n_bcast messages."""
    import socket
    import struct
    import threading
    import time
    try:
        me = os.path.join(sock_dir, "kungfu-amd-127.0.0.1-10001.sock")
        root = os.path.join(sock_dir, "kungfu-amd-127.0.0.1-10000.sock")
        srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        srv.bind(me)
        srv.listen(1)
        c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        for _ in range(500):
            try:
                c.connect(root)
                break
            except OSError:
                time.sleep(0.05)
        # connection header {u16 type=Collective, u16 port, u32 ipv4}, then ack
        c.sendall(struct.pack("<HHI", 2, 10001, 0x7F000001))
        assert struct.unpack("<I", c.recv(4))[0] == token
        a, _ = srv.accept()
        hdr = b""
        while len(hdr) < 8:
            hdr += a.recv(8 - len(hdr))
        a.sendall(struct.pack("<I", token))

        def exact(k):
            b = b""
            while len(b) < k:
                chunk = a.recv(k - len(b))
                assert chunk, "root closed early"
                b += chunk
            return b

        def reader():  # a real peer reads while it writes
            try:
                for _ in range(n_bcast):
                    nl = struct.unpack("<I", exact(4))[0]
                    name = exact(nl).decode()
                    flags, ln = struct.unpack("<II", exact(8))
                    out.append((name, flags, exact(ln)))
            except Exception:
                err.append(traceback.format_exc())
        rd = threading.Thread(target=reader)
        rd.start()
        for name, flags, payload in msgs:
            nb = name.encode()
            c.sendall(struct.pack("<I", len(nb)) + nb + struct.pack("<II", flags, len(payload))
                      + payload)
        rd.join(timeout=60)
        c.close()
        a.close()
        srv.close()
    except Exception:
        err.append(traceback.format_exc())


@pytest.mark.timeout(120)
def test_session_next_step_message_waits_for_its_call():
    # the fake peer interleaves step t+1's chunk-0 message between step t's
    # chunk-0 and chunk-1 messages, as messages from several peers can
    # interleave; the root must keep it for step t+1 (per-name mailbox,
    # handler/collective.go:27-61) instead of folding it twice into step t
    import threading
    from kungfu_amd.base import EvenPartition
    from kungfu_amd.session import Session
    n = (1 << 18) + 3  # 2 chunks of int32
    parts = list(EvenPartition(0, n, 2))
    names = ["part::grad[%d:%d]" % (b, e) for b, e in parts]
    x1 = [np.arange(n, dtype=np.int32) * 3, np.arange(n, dtype=np.int32) * 5 + 1]
    msgs = [(names[0], 0, x1[0][parts[0][0]:parts[0][1]].tobytes()),
            (names[0], 0, x1[1][parts[0][0]:parts[0][1]].tobytes()),  # step 1, early
            (names[1], 0, x1[0][parts[1][0]:parts[1][1]].tobytes()),
            (names[1], 0, x1[1][parts[1][0]:parts[1][1]].tobytes())]
    out, err = [], []
    with tempfile.TemporaryDirectory() as d:
        t = threading.Thread(target=_fake_peer, args=(d, 7, msgs, 4, out, err))
        t.start()
        os.environ.pop("KUNGFU_ALLREDUCE_STRATEGY", None)
        s = Session(0, 2, d, mode="host", token=7, host_reduce_fn=oracle_reduce_fn())
        x0 = [np.arange(n, dtype=np.int32) + 7, np.arange(n, dtype=np.int32) * 2]
        ys = []
        for step in range(2):
            y = np.zeros(n, np.int32)
            s.all_reduce(x0[step], y, "grad")
            ys.append(y)
        t.join(timeout=60)
        s.close()
    assert not err, err[0]
    for step in range(2):
        assert np.array_equal(ys[step], x0[step] + x1[step]), step
    # the bcast the peer received: step 0 then step 1, both chunks, WaitRecvBuf
    got = {}
    for name, flags, data in out:
        assert flags == 1
        got.setdefault(name, []).append(np.frombuffer(data, np.int32))
    for c, (b, e) in enumerate(parts):
        for step in range(2):
            assert np.array_equal(got[names[c]][step], (x0[step] + x1[step])[b:e])


def _async_body(rank, size, sock_dir, mode, errq):
    """GoKungfuAllReduce with a done callback: several named all-reduces
    queued at once (ints, an exact-in-fp32 float bucket of 3 chunks, an
    in-place one), then a synchronous one behind them."""
    sys.path[:0] = [ROOT, HERE]
    try:
        from kungfu_amd.session import Session
        specs = [("grad/a", "iota", 37), ("grad/b", "c1", (3 << 20) // 4 + 9),
                 ("grad/c", "iota", 4099)]
        xs = [inputs(rank, n, kind) for _, kind, n in specs]
        if mode == "device":
            import torch
            dev = torch.device("cuda:0")
            sends = [torch.from_numpy(x).to(dev) for x in xs]
            recvs = [torch.zeros_like(t) for t in sends[:2]] + [sends[2]]  # c in place
            s = Session(rank, size, sock_dir, mode="device")
        else:
            sends = [x.copy() for x in xs]
            recvs = [np.zeros_like(x) for x in xs[:2]] + [sends[2]]
            s = Session(rank, size, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn())
        seen = []
        nested = []

        def cb(st, name):
            seen.append((name, st))
            if name == "grad/a":  # a blocking call from the worker must not hang
                try:
                    s.wait_all()
                except Exception as e:
                    nested.append(str(e))

        hs = [s.all_reduce_async(snd, rcv, name, callback=lambda st, name=name: cb(st, name))
              for (name, _, _), snd, rcv in zip(specs, sends, recvs)]
        z = inputs(rank, 11, "iota")
        zr = np.zeros_like(z)
        if mode == "device":
            z, zr = torch.from_numpy(z).to(dev), torch.zeros(11, dtype=torch.int32, device=dev)
        s.all_reduce(z, zr, "after")  # waits for the queued ones first
        assert all(h.done() for h in hs)
        outs = [h.wait() for h in hs]
        s.wait_all()
        assert sorted(n for n, _ in seen) == sorted(n for n, _, _ in specs)  # completion order
        assert all(st == 0 for _, st in seen)
        assert len(nested) == 1 and "KF_ERR_ARG" in nested[0], nested
        s.close()
        if mode == "device":
            outs = [o.cpu().numpy() for o in outs]
            zr = zr.cpu().numpy()
        for (_, kind, n), got in zip(specs, outs):
            check(rank, size, kind, n, got)
        assert np.array_equal(zr, np.arange(11, dtype=np.int32) * size)
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def _run_async(size, mode):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_async_body, args=(r, size, d, mode, errq))
              for r in range(size)]
        for p in ps:
            p.start()
        hung = join_all(ps, 180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


@pytest.mark.parametrize("size", [2, 3])
def test_session_async_host(size):
    _run_async(size, "host")


@pytest.mark.gpu
def test_session_async_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_async(3, "device")


def _any_order_body(rank, size, sock_dir, mode, strategy, errq, steps=2, env=None):
    """Every peer starts the same named all-reduces in its OWN random order,
    two steps of them back to back (a name's second call waits for its
    first; the peers' step-2 chunks wait in the stash meanwhile), as the
    reference allows: each GoKungfuAllReduce is its own goroutine and peers'
    messages pair by name (handler/collective.go:48-64). Exact inputs (ints,
    and the C1 floats whose sums are exact in any order)."""
    sys.path[:0] = [ROOT, HERE]
    os.environ.update(env or {})
    try:
        import time
        if strategy is not None:
            os.environ["KUNGFU_ALLREDUCE_STRATEGY"] = strategy
        from kungfu_amd.session import Session
        specs = [("w%d" % j, "iota" if j % 2 else "c1", n)
                 for j, n in enumerate([5, 1 << 18, (5 << 20) // 4 + 3, 4099, 77, (3 << 20) // 4])]
        rng = np.random.default_rng(1000 + rank)
        if mode == "device":
            import torch
            dev = torch.device("cuda:0")
            s = Session(rank, size, sock_dir, mode="device")
        else:
            s = Session(rank, size, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn())
        hs = []
        noise, stop, spins = None, None, [0]
        if mode == "device" and os.environ.get("KF_TEST_NOISE") == "1":
            # torch work on the default (null) stream from a second thread
            # while the streamed folds wait for socket bodies (VERDICT r05
            # item 4: the lone session's waiting kernel may sit on the null
            # stream; nothing this thread queues there is needed for a body
            # to arrive, so both must finish)
            import threading
            stop = threading.Event()

            def churn():
                torch.cuda.set_device(0)
                a = torch.randn(512, 512, device=dev)
                while not stop.is_set():
                    (a @ a).sum().item()  # queued on the null stream, then a sync
                    spins[0] += 1
            noise = threading.Thread(target=churn, daemon=True)
            noise.start()
        opposite = os.environ.get("KF_TEST_ORDER") == "opposite"
        for step in range(steps):  # step t+1 starts while step t may be in flight
            order = (np.arange(len(specs)) if rank % 2 == 0 else np.arange(len(specs))[::-1]) \
                if opposite else rng.permutation(len(specs))
            for j in order:
                name, kind, n = specs[j]
                x = inputs(rank, n, kind) * (step + 1)
                if mode == "device":
                    snd = torch.from_numpy(x).to(dev)
                    rcv = torch.zeros_like(snd) if j % 3 else snd  # some in place
                else:
                    snd = x.copy()
                    rcv = np.zeros_like(x) if j % 3 else snd
                hs.append((step, j, s.all_reduce_async(snd, rcv, name)))
                if rng.random() < 0.3:
                    time.sleep(0.01)  # let some run before the rest start
        s.wait_all()
        if noise is not None:
            stop.set()
            noise.join(60)
            assert not noise.is_alive() and spins[0] > 0, ("noise thread", spins[0])
        for step, j, h in hs:
            name, kind, n = specs[j]
            got = h.wait()
            if mode == "device":
                got = got.cpu().numpy()
            want = sum(inputs(r, n, kind) for r in range(size)) * (step + 1)
            assert np.array_equal(got, want.astype(got.dtype)), (rank, step, name)
        s.close()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def _run_any_order(size, mode, strategy=None, steps=2, env=None):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_any_order_body,
                          args=(r, size, d, mode, strategy, errq, steps, env))
              for r in range(size)]
        for p in ps:
            p.start()
        hung = join_all(ps, 120)
        for p in ps:
            if p.exitcode is None:
                p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


@pytest.mark.parametrize("size,strategy", [(2, None), (3, None), (4, "RING"), (3, "CLIQUE"),
                                           (4, "BINARY_TREE")])
def test_session_async_any_order_host(size, strategy):
    _run_any_order(size, "host", strategy)


@pytest.mark.gpu
@pytest.mark.parametrize("size,strategy", [(3, None), (4, "RING"), (4, "BINARY_TREE"),
                                           (3, "CLIQUE")])
def test_session_async_any_order_device(size, strategy):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_any_order(size, "device", strategy)


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["CLIQUE", "BINARY_TREE"])
def test_lone_session_null_stream_with_torch_noise(strategy):
    """the streamed kernel of a process's only device
    session waits on the caller's (null) stream (kf_session.hip
    waiting_stream, g_device_sessions == 1). The invariant that makes this
    safe — nothing else the process queues there is needed for a body to
    arrive — is tested with other work in the process: np = 3, async calls
    started in opposite orders on even and odd ranks, and a second thread
    per rank issuing torch matmuls + syncs on the default stream throughout.
    Every result exact, every thread finished (profiles/r06/failures.md)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_any_order(3, "device", strategy, env={"KF_TEST_NOISE": "1", "KF_TEST_ORDER": "opposite"})


def _names_with_roots(n, want):
    """Bucket names whose single chunk a 2-peer CLIQUE roots at want[0],
    want[1], ... (strategy index = nameBasedHash % 2, shard.go:17-23)."""
    from oracle import schedule
    out = []
    for r in want:
        for j in range(1000):
            name = "g%d" % j
            if name not in out and schedule.chunk_roots(n, 4, 2, "CLIQUE", name)[0][2] == r:
                out.append(name)
                break
    return out


def _next_call_body(rank, sock_dir, mode, errq):
    """X is rooted at rank 1, Z at rank 0. Rank 0 queues
    X(0), Z(0), X(1), Z(1) at once; rank 1 queues X(0), X(1), waits for X(1)
    and only then queues Z(0), Z(1). Rank 0's X(0) completes on rank 1's
    bcast while Z(0) is still in flight; rank 1 then sends nothing until it
    has rank 0's X(1) chunk. So rank 0 must start X(1) as soon as X(0)
    completes, not after its next socket message (which never comes)."""
    sys.path[:0] = [ROOT, HERE]
    os.environ["KUNGFU_ALLREDUCE_STRATEGY"] = "CLIQUE"
    try:
        from kungfu_amd.session import Session
        n = 1000
        X, Z = _names_with_roots(n, (1, 0))
        if mode == "device":
            import torch
            dev = torch.device("cuda:0")
            s = Session(rank, 2, sock_dir, mode="device")
            mk = lambda v: torch.full((n,), float(v), device=dev)  # noqa: E731
        else:
            s = Session(rank, 2, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn())
            mk = lambda v: np.full(n, float(v), dtype=np.float32)  # noqa: E731
        want = {}
        hs = {}

        def go(name, step):
            x = mk((rank + 1) * (step + 1) + (name == Z))
            hs[(name, step)] = s.all_reduce_async(x, mk(0), name)
            want[(name, step)] = 3.0 * (step + 1) + 2 * (name == Z)

        if rank == 0:
            for step in (0, 1):
                go(X, step)
                go(Z, step)
        else:
            go(X, 0)
            go(X, 1)
            hs[(X, 1)].wait()
            go(Z, 0)
            go(Z, 1)
        s.wait_all()
        for key, h in hs.items():
            got = h.wait()
            got = got.cpu().numpy() if mode == "device" else got
            assert np.all(got == want[key]), (rank, key, got[:3])
        s.close()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def _run_next_call(mode):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_next_call_body, args=(r, d, mode, errq)) for r in range(2)]
        for p in ps:
            p.start()
        hung = join_all(ps, 60)
        for p in ps:
            if p.exitcode is None:
                p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not hung, "hung: a queued call was not started after its name freed"
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


def test_session_async_next_call_starts_on_completion_host():
    _run_next_call("host")


@pytest.mark.gpu
def test_session_async_next_call_starts_on_completion_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_next_call("device")


def _dead_peer_body(rank, sock_dir, errq):
    """Rank 1 connects and leaves without joining; rank 0's in-flight async
    all-reduces must fail (every peer connection closed), not hang."""
    sys.path[:0] = [ROOT, HERE]
    try:
        from kungfu_amd.session import Session
        s = Session(rank, 2, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn())
        if rank == 1:
            s.close()
            return
        xs = [inputs(0, n, "iota") for n in (9, 1 << 19)]
        got = []
        hs = [s.all_reduce_async(x, np.zeros_like(x), "dead/%d" % i,
                                 callback=lambda st: got.append(st))
              for i, x in enumerate(xs)]
        try:
            s.wait_all()
            raise AssertionError("wait_all succeeded with the peer gone")
        except RuntimeError as e:
            assert "closed" in str(e) or "KF_ERR_IO" in str(e), e
        assert len(got) == 2 and all(st != 0 for st in got), got
        assert all(h.done() for h in hs)
        # started after the peer was seen gone: fails at once too
        h = s.all_reduce_async(xs[0], np.zeros_like(xs[0]), "dead/late")
        try:
            s.wait_all()
            raise AssertionError("a call started after the peer left succeeded")
        except RuntimeError:
            pass
        assert h.done() and h.status != 0
        s.close()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def test_session_async_peer_gone():
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_dead_peer_body, args=(r, d, errq)) for r in range(2)]
        for p in ps:
            p.start()
        hung = join_all(ps, 60)
        for p in ps:
            if p.exitcode is None:
                p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


def test_session_async_arg_errors():
    import ctypes
    from kungfu_amd import _lib
    lib = _lib.load()
    cb = _lib.DONE_FN(lambda st, arg: None)
    assert lib.kf_session_all_reduce_async(None, None, None, 0, 0x20408, 0, b"x", None,
                                           cb, None) == 3
    assert lib.kf_session_wait_all(None) == 3
    with tempfile.TemporaryDirectory() as d:
        from kungfu_amd.session import Session
        s = Session(0, 1, d, mode="host", host_reduce_fn=oracle_reduce_fn())
        buf = np.zeros(4, dtype=np.int32)
        p = buf.ctypes.data
        assert lib.kf_session_all_reduce_async(s._h, p, p, 4, 0x12345, 0, b"x", None,
                                               cb, None) == 1  # unknown dtype: no exit
        assert lib.kf_session_all_reduce_async(s._h, p, p, 4, 0x30108, 0, b"x", None,
                                               cb, None) == 2  # BOOL
        assert lib.kf_session_all_reduce_async(s._h, p, p, 4, 0x10408, 7, b"x", None,
                                               cb, None) == 2  # unknown op
        s.close()
    del ctypes


def _rb_body(rank, size, sock_dir, mode, strategy, errq):
    """Session.Reduce / Session.Broadcast (session.go:159-167) against the
    schedule oracle's runGraphs over the first strategy's one graph: the
    root's reduction, inner nodes' partial folds, leaves' recv untouched (a
    sentinel), and the root's send everywhere after the broadcast. The c1
    values are exact in fp32, so every arrival order gives the same bits."""
    sys.path[:0] = [ROOT, HERE]
    try:
        from kungfu_amd.session import Session
        from oracle import schedule
        n = (3 << 20) // 4 + 5  # 4 chunks
        xs = [inputs(r, n, "c1") for r in range(size)]
        init = np.full(n, -7.0, np.float32)
        want_r = schedule.reduce(xs, "f32", "sum", strategy=strategy, initial=[init] * size)[rank]
        want_b = schedule.broadcast(xs, strategy=strategy)[rank]
        if mode == "device":
            import torch
            dev = torch.device("cuda:0")
            s = Session(rank, size, sock_dir, mode="device", strategy=strategy)
            x = torch.from_numpy(xs[rank]).to(dev)
            y = torch.from_numpy(init).to(dev)
            s.reduce(x, y, "red")
            z = torch.zeros_like(x)
            s.broadcast(x, z, "bc")
            y, z = y.cpu().numpy(), z.cpu().numpy()
        else:
            s = Session(rank, size, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn(),
                        strategy=strategy)
            y = init.copy()
            s.reduce(xs[rank], y, "red")
            z = np.zeros_like(xs[rank])
            s.broadcast(xs[rank], z, "bc")
        s.close()
        assert np.array_equal(y, want_r), ("reduce", strategy, rank)
        assert np.array_equal(z, want_b), ("broadcast", strategy, rank)
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def _run_rb(size, mode, strategy):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_rb_body, args=(r, size, d, mode, strategy, errq))
              for r in range(size)]
        for p in ps:
            p.start()
        hung = join_all(ps, 180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


@pytest.mark.parametrize("strategy", ["STAR", "BINARY_TREE", "RING", "CLIQUE"])
@pytest.mark.parametrize("size", [3, 4])
def test_session_reduce_broadcast_host(size, strategy):
    _run_rb(size, "host", strategy)


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["STAR", "BINARY_TREE", "RING"])
def test_session_reduce_broadcast_device(strategy):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_rb(4, "device", strategy)


def _subset_body(rank, size, sock_dir, mode, errq):
    """Session.SubsetAllReduce (allreduce.go:14-24) for several forests
    against the schedule oracle: two trees, a chain, all lone nodes; bad
    forests (cycle, out of range) are refused before any message moves."""
    sys.path[:0] = [ROOT, HERE]
    try:
        from kungfu_amd._lib import KungFuAMDError
        from kungfu_amd.session import Session
        from oracle import schedule
        n = (2 << 20) // 4 + 3
        xs = [inputs(r, n, "c1") for r in range(size)]
        forests = [[0, 0, 2, 2], [1, 1, 1, 2], [0, 1, 2, 3]]
        if mode == "device":
            import torch
            dev = torch.device("cuda:0")
            s = Session(rank, size, sock_dir, mode="device")
            x = torch.from_numpy(xs[rank]).to(dev)
        else:
            s = Session(rank, size, sock_dir, mode="host", host_reduce_fn=oracle_reduce_fn())
            x = xs[rank]
        for bad in ([1, 0, 2, 3], [0, 0, 9, 2]):
            try:
                s.subset_all_reduce(x, x, bad, "bad")
                raise AssertionError("bad forest accepted: %r" % bad)
            except KungFuAMDError as e:
                assert "KF_ERR_ARG" in str(e)
        s.barrier()
        for j, forest in enumerate(forests):
            want = schedule.subset_all_reduce(xs, "f32", "sum", forest, name="sub%d" % j)[rank]
            y = (torch.zeros_like(x) if mode == "device" else np.zeros_like(x))
            s.subset_all_reduce(x, y, forest, "sub%d" % j)
            got = y.cpu().numpy() if mode == "device" else y
            assert np.array_equal(got, want), (forest, rank)
        s.close()
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def _run_subset(mode):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_subset_body, args=(r, 4, d, mode, errq)) for r in range(4)]
        for p in ps:
            p.start()
        hung = join_all(ps, 180)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])


def test_session_subset_all_reduce_host():
    _run_subset("host")


@pytest.mark.gpu
def test_session_subset_all_reduce_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_subset("device")


def _barrier_body(rank, size, sock_dir, mode, q):
    """Session.Barrier (session.go:98-115): no peer leaves before the last one
    has entered; peers enter 0.3 s apart."""
    sys.path[:0] = [ROOT, HERE]
    try:
        import time
        from kungfu_amd.session import Session
        s = Session(rank, size, sock_dir, mode=mode,
                    **({} if mode == "device" else {"host_reduce_fn": oracle_reduce_fn()}))
        s.barrier()  # everyone connected
        for i in range(2):
            time.sleep(0.3 * ((rank + i) % size))
            t_in = time.time()
            s.barrier()
            q.put((i, rank, t_in, time.time()))
        s.close()
    except Exception:
        q.put(("err", rank, traceback.format_exc(), 0))


def _run_barrier(mode, size):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    with tempfile.TemporaryDirectory() as d:
        ps = [ctx.Process(target=_barrier_body, args=(r, size, d, mode, q)) for r in range(size)]
        for p in ps:
            p.start()
        hung = join_all(ps, 120)
    rows = []
    while not q.empty():
        rows.append(q.get())
    errs = [r[2] for r in rows if r[0] == "err"]
    assert not errs, "\n".join(errs)
    assert not hung and all(p.exitcode == 0 for p in ps), hung_msg(hung, [p.exitcode for p in ps])
    for i in range(2):
        mine = [r for r in rows if r[0] == i]
        assert len(mine) == size
        assert min(r[3] for r in mine) >= max(r[2] for r in mine)


@pytest.mark.parametrize("size", [2, 3])
def test_session_barrier_host(size):
    _run_barrier("host", size)


@pytest.mark.gpu
def test_session_barrier_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_barrier("device", 3)
