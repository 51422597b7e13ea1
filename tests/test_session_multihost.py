"""Multi-host Session: peers given as a KUNGFU_INIT_PEERS-style list. Hosts are
emulated with distinct loopback addresses (127.0.0.1, 127.0.0.2, ...), so
peers of one "host" talk over unix sockets and peers of different hosts over
TCP — connection.go:58-64's rule. Every multi-host strategy graph
(topology.go:17-136: TREE, MULTI_STAR, BINARY_TREE_STAR,
MULTI_BINARY_TREE_STAR, AUTO -> BINARY_TREE_STAR) is checked against the
oracle schedule (oracle/schedule.py) built on the same host layout."""
import itertools
import os
import sys
import tempfile
import time
import traceback

import numpy as np
import pytest
import multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from ports import draw_block, taken_port  # noqa: E402

NAME = "NegotiatedGrad_0/AllReduce"


def layout(hosts_sizes, base_port):
    peers = []
    for h, n in enumerate(hosts_sizes):
        peers += ["127.0.0.%d:%d" % (h + 1, base_port + i) for i in range(n)]
    return peers


def inputs(rank, n, kind):
    if kind == "iota":
        return (np.arange(n) + rank).astype(np.int32)
    return np.random.default_rng(70 + rank).standard_normal(n).astype(np.float32)


def _body(rank, peers, sock_dir, kind, n, strategy, errq, mode):
    sys.path[:0] = [ROOT, HERE]
    try:
        import ctypes
        from kungfu_amd.session import Session
        if strategy is not None:
            os.environ["KUNGFU_ALLREDUCE_STRATEGY"] = strategy
        os.environ["KUNGFU_INIT_PEERS"] = ",".join(peers)
        os.environ["KUNGFU_SELF_SPEC"] = peers[rank]
        x = inputs(rank, n, kind)
        if mode == "device":
            import torch
            dev = torch.device("cuda:0")
            xs = torch.from_numpy(x).to(dev)
            ys = torch.zeros_like(xs)
            s = Session.from_env(sock_dir=sock_dir, mode="device")
            s.all_reduce(xs, ys, NAME)
            got = ys.cpu().numpy()
        else:
            from oracle import oracle
            fn = ctypes.cast(oracle.lib().oracle_transform2, ctypes.c_void_p)
            y = np.zeros_like(x)
            s = Session.from_env(sock_dir=sock_dir, mode="host", host_reduce_fn=fn)
            assert (s.rank, s.size) == (rank, len(peers))
            s.all_reduce(x, y, NAME)
            got = y
        s.close()
        check(peers, kind, n, strategy or "BINARY_TREE_STAR", got)
    except Exception:
        errq.put("rank %d: %s" % (rank, traceback.format_exc()))


def check(peers, kind, n, strategy, got):
    from oracle import schedule
    k = len(peers)
    hosts = [p.split(":")[0] for p in peers]
    xs = [inputs(r, n, kind) for r in range(k)]
    dt = "i32" if kind == "iota" else "f32"
    if kind == "iota":  # order-free: one schedule run
        want = schedule.all_reduce(xs, dt, "sum", strategy=strategy, hosts=hosts, name=NAME)[0]
        assert np.array_equal(got, want)
        assert np.array_equal(got, sum(x.astype(np.int64) for x in xs).astype(np.int32))
        return
    # a node's reduce predecessors may arrive in any order; in a tree the
    # predecessor sets of different nodes are disjoint, so one global order of
    # the ranks per run covers every combination
    outs = []
    for order in itertools.permutations(range(k)):
        outs.append(schedule.all_reduce(
            xs, dt, "sum", strategy=strategy, hosts=hosts, name=NAME,
            arrival=lambda r, prevs, order=order: sorted(prevs, key=order.index))[0])
    nch = (n * 4 + (1 << 20) - 1) >> 20
    for b, e in schedule.even_partition(0, n, nch):
        assert any(np.array_equal(got[b:e], o[b:e]) for o in outs), (strategy, b, e)


def _addrs(peers):
    return [(p.rsplit(":", 1)[0], int(p.rsplit(":", 1)[1])) for p in peers]


def run(hosts_sizes, kind, n, strategy, mode="host", first=None, attempts=3):
    """The peers on a port block every address of which could be bound just
    before (tests/ports.py); if a rank still loses its port to another
    process ('Address already in use' at session creation), every rank is
    stopped and the run starts over on a new block. Returns the blocks used."""
    ctx = mp.get_context("spawn")
    used = []
    for attempt in range(attempts):
        if attempt == 0 and first is not None:
            base = first  # a test forces a taken block here
        else:
            base = draw_block(lambda b: _addrs(layout(hosts_sizes, b)))
        used.append(base)
        peers = layout(hosts_sizes, base)
        errq = ctx.SimpleQueue()
        with tempfile.TemporaryDirectory() as d:
            ps = [ctx.Process(target=_body, args=(r, peers, d, kind, n, strategy, errq, mode))
                  for r in range(len(peers))]
            for p in ps:
                p.start()
            errs, taken = [], False
            deadline = time.monotonic() + 300
            while any(p.is_alive() for p in ps) and time.monotonic() < deadline and not taken:
                while not errq.empty():
                    errs.append(errq.get())
                taken = any("Address already in use" in e for e in errs)
                time.sleep(0.05)
            for p in ps:
                if taken or p.is_alive():
                    p.kill()
                p.join()
        while not errq.empty():
            errs.append(errq.get())
        if any("Address already in use" in e for e in errs):
            continue  # the peers dialling it would wait for it: start over
        assert not errs, "\n".join(errs)
        assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
        return used
    raise AssertionError("every port block was taken: %r" % used)


STRATEGIES = ["STAR", "MULTI_STAR", "CLIQUE", "RING", "TREE", "BINARY_TREE",
              "BINARY_TREE_STAR", "MULTI_BINARY_TREE_STAR", "AUTO"]


@pytest.mark.parametrize("strategy", STRATEGIES)
def test_two_hosts_float(strategy):
    # 2 hosts x 2 peers, a 3-chunk bucket: each chunk picks its own graph
    run([2, 2], "rand", (3 << 20) // 4 + 11, strategy)


@pytest.mark.parametrize("strategy", ["TREE", "MULTI_STAR", "BINARY_TREE_STAR",
                                      "MULTI_BINARY_TREE_STAR", "RING"])
def test_three_uneven_hosts_iota(strategy):
    # hosts of 2, 1 and 3 peers: masters 0, 2, 3
    run([2, 1, 3], "iota", (5 << 20) // 4 + 3, strategy)


def test_default_strategy_is_binary_tree_star():
    # no KUNGFU_ALLREDUCE_STRATEGY: kungfu-run's default BINARY_TREE_STAR
    run([1, 2], "rand", 1 << 18, None)


def test_taken_port_restarts_on_a_new_block():
    """The first block's rank-0 port is held by another listener: that rank's
    session cannot bind ('Address already in use'), the run stops every rank
    and starts over on a new block, and passes."""
    s, p = taken_port()
    try:
        used = run([1, 1], "iota", 1000, "STAR", first=p)
    finally:
        s.close()
    assert used[0] == p and len(used) == 2, used


def test_bad_peer_specs():
    from kungfu_amd import _lib
    from kungfu_amd.session import Session
    lib = _lib.load()
    assert not lib.kf_session_create_peers(b"127.0.0.1:9", b"127.0.0.1:10", b"/tmp", 0, 0)
    assert b"not in the peer list" in lib.kf_session_last_error()
    assert not lib.kf_session_create_peers(b"127.0.0.1", b"127.0.0.1", b"/tmp", 0, 0)
    assert not lib.kf_session_create_peers(b"127.0.0.1:9,127.0.0.1:9", b"127.0.0.1:9",
                                           b"/tmp", 0, 0)
    assert not lib.kf_session_create_peers(b"300.0.0.1:9", b"300.0.0.1:9", b"/tmp", 0, 0)
    with pytest.raises(ValueError):
        Session(peers="127.0.0.1:9", self_spec="127.0.0.1:8", mode="host")


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["BINARY_TREE_STAR", "RING", "MULTI_STAR"])
def test_two_hosts_device(strategy):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    run([2, 2], "rand", (3 << 20) // 4 + 11, strategy, mode="device")
