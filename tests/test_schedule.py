"""Pins the all-reduce schedule restatement (oracle/schedule.py) with the
reference's own known-answer tests; the Go layer itself cannot run here."""
import numpy as np
import pytest

from oracle import schedule

STRATS = ["STAR", "RING", "CLIQUE", "TREE", "BINARY_TREE", "BINARY_TREE_STAR",
          "MULTI_BINARY_TREE_STAR", "MULTI_STAR", "AUTO"]


def test_even_partition():
    # interval.go:12-27
    assert schedule.even_partition(0, 10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert schedule.even_partition(0, 2, 4) == [(0, 1), (1, 2), (2, 2), (2, 2)]
    parts = schedule.even_partition(0, 25583592, 16)
    assert sum(e - b for b, e in parts) == 25583592
    assert max(e - b for b, e in parts) - min(e - b for b, e in parts) <= 1


def test_name_hash():
    # shard.go:17-23: sum of squared code points
    assert schedule.name_hash(0, "ab") == 97 * 97 + 98 * 98
    assert schedule.name_hash(0, "é") == 0xE9 * 0xE9  # rune, not byte


def test_chunking_is_1mib_by_bytes():
    # session.go:313-314: k = ceil(bytes / 1 MiB)
    roots = schedule.chunk_roots(1 << 20, 4, 2, strategy="RING")
    assert len(roots) == 4 and roots[0][:2] == (0, 262144)
    assert len(schedule.chunk_roots(262145, 4, 2)) == 2
    assert schedule.chunk_roots(0, 4, 2) == []


@pytest.mark.parametrize("strategy", STRATS)
@pytest.mark.parametrize("np_", [1, 2, 3, 4])
def test_fake_agent_iota(strategy, np_):
    # tests/cpp/integration/fake_agent.cpp:15-44: x = iota(4np), y[i] == i*np
    n = np_ * 4
    xs = [np.arange(n, dtype=np.int32) for _ in range(np_)]
    outs = schedule.all_reduce(xs, "i32", "sum", strategy=strategy, name="test-tensor")
    for y in outs:
        assert np.array_equal(y, np.arange(n, dtype=np.int32) * np_)


@pytest.mark.parametrize("strategy", ["STAR", "RING", "BINARY_TREE_STAR"])
@pytest.mark.parametrize("np_", [2, 4])
def test_public_apis_ones_2_20(strategy, np_):
    # kungfu-test-public-apis.go:87-104: int32 ones x 2^20 -> np everywhere
    xs = [np.ones(1 << 20, np.int32) for _ in range(np_)]
    for y in schedule.all_reduce(xs, "i32", "sum", strategy=strategy, name="0"):
        assert np.all(y == np_)


@pytest.mark.parametrize("np_", [1, 2, 4])
def test_in_proc_trainer_kat(np_):
    # fake_in_proc_trainer.cpp:28-48: node i holds i+1 -> np(np+1)/2, send bufs kept
    xs = [np.full(100003, i + 1, np.int32) for i in range(np_)]
    outs = schedule.all_reduce(xs, "i32", "sum", strategy="RING")
    for i, y in enumerate(outs):
        assert np.all(y == np_ * (np_ + 1) // 2)
        assert np.all(xs[i] == i + 1)


def test_np1_is_forward():
    # single peer: every graph isolated -> w.Forward() (session.go:235-238)
    x = np.arange(10, dtype=np.int32) + 1
    (y,) = schedule.all_reduce([x], "i32", "sum")
    assert np.array_equal(y, x)  # test_operations.cpp:3-26 (y[i] == i + 1)


def test_inplace():
    xs = [np.arange(50, dtype=np.float32) for _ in range(3)]
    outs = schedule.all_reduce(xs, "f32", "sum", strategy="RING", inplace=True)
    for y in outs:
        assert np.array_equal(y, np.arange(50, dtype=np.float32) * 3)


def _is_tree(bg, k):
    indeg = [len(bg.prevs[i]) for i in range(k)]
    return sorted(indeg).count(0) == 1 and all(d <= 1 for d in indeg) and \
        len(bg.edges()) == k - 1


def test_topology_tree_validity():
    # plan/topology_test.go:71-98 — 9 peers on 3 hosts
    hosts = ["h%d" % (i // 3) for i in range(9)]
    for strategy in ["TREE", "BINARY_TREE", "BINARY_TREE_STAR",
                     "MULTI_BINARY_TREE_STAR", "STAR", "CLIQUE"]:
        for rg, bg in schedule.strategy_list(strategy, hosts):
            assert _is_tree(bg, 9), strategy


def test_ring_fold_order_matches_schedule():
    # the ring root r computes x_r + (... (x_{r+2} + x_{r+1})); fp SUM is
    # commutative per hop, so a left fold over ring_order() is bit-identical
    from oracle import oracle
    rng = np.random.default_rng(0)
    k = 4
    n = 1 << 20  # 4 chunks of 1 MiB
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(k)]
    outs = schedule.all_reduce(xs, "f32", "sum", strategy="RING")
    for b, e, r in schedule.chunk_roots(n, 4, k, strategy="RING"):
        order = schedule.ring_order(k, r)
        want = oracle.reduce_k([xs[j][b:e].copy() for j in order], "f32", "sum")
        for y in outs:
            assert np.array_equal(y[b:e], want)


def test_star_arrival_order_changes_bits_within_bound():
    # star root folds peers in arrival order (session.go:255-264): results for
    # np > 2 depend on it, bounded by (np-1) * 2^-24 * sum|x|
    rng = np.random.default_rng(1)
    k, n = 4, 4096
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(k)]
    outs = []
    for perm in schedule.all_arrival_orders([1, 2, 3]):
        arrival = lambda r, prevs, perm=perm: [p for p in perm if p in prevs]  # noqa
        outs.append(schedule.all_reduce(xs, "f32", "sum", strategy="STAR",
                                        arrival=arrival)[0])
    exact = np.sum(np.array(xs, np.float64), axis=0)
    bound = (k - 1) * 2.0 ** -24 * np.sum(np.abs(np.array(xs, np.float64)), axis=0)
    for o in outs:
        assert np.all(np.abs(o - exact) <= bound)
