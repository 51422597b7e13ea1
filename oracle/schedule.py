"""TEST INFRASTRUCTURE ONLY — restatement of KungFu's all-reduce schedule.

Reproduces, in plain Python on top of the oracle's Transform2, WHO adds WHICH
peer chunk in WHAT order when KungFu all-reduces a bucket, so the HIP path's
multi-input reduce and the RCCL all-reduce can be compared against the
reference's accumulation order:

  chunking      srcs/go/kungfu/session/session.go:301-326  (1 MiB by bytes,
                EvenPartition by element count, one goroutine per chunk)
  chunk names   srcs/go/kungfu/base/workspace.go:18-25      "part::%s[%d:%d]"
  strategy pick srcs/go/kungfu/session/shard.go:13-31        Σ c² over runes
                srcs/go/kungfu/session/strategy.go:108-110   sl[h % len(sl)]
  strategies    srcs/go/kungfu/session/strategy.go:121-205
  graphs        srcs/go/plan/topology.go:17-160, srcs/go/plan/graph/graph.go:72-108
  execution     srcs/go/kungfu/session/session.go:231-299    (runGraphs)

The Go layer cannot be built here (no Go toolchain), so this
restatement is pinned by the reference's own known-answer tests instead
(tests/test_schedule.py): fake_agent.cpp:15-44, fake_in_proc_trainer.cpp:28-48,
kungfu-test-public-apis.go:49-104, test_operations.cpp:3-26 and the tree
validity checks of plan/topology_test.go:71-98.
"""
import itertools

import numpy as np

from . import oracle

CHUNK_SIZE = 1 << 20  # session.go:301-304

STRATEGIES = ("STAR", "MULTI_STAR", "CLIQUE", "RING", "TREE", "BINARY_TREE",
              "BINARY_TREE_STAR", "MULTI_BINARY_TREE_STAR", "AUTO")


def even_partition(begin, end, k):
    """interval.go:12-27"""
    n = end - begin
    quo, rem = n // k, n % k
    out, off = [], begin
    for i in range(k):
        c = quo + 1 if i < rem else quo
        out.append((off, off + c))
        off += c
    return out


def ceil_div(a, b):
    return a // b if a % b == 0 else a // b + 1


def name_hash(i, name):
    """nameBasedHash (shard.go:17-23): Σ c² over Unicode code points, uint64."""
    return sum(ord(c) * ord(c) for c in name) & 0xFFFFFFFFFFFFFFFF


def simple_hash(i, name):
    """shard.go:13-15"""
    return i


class Graph:
    """graph.go:18-108 — nodes with Prevs/Nexts lists and a self-loop flag."""

    def __init__(self, n):
        self.prevs = [[] for _ in range(n)]
        self.nexts = [[] for _ in range(n)]
        self.self_loop = [False] * n

    def __len__(self):
        return len(self.prevs)

    def add_edge(self, i, j):
        if i == j:
            self.self_loop[i] = True
            return
        self.nexts[i].append(j)
        self.prevs[j].append(i)

    def reverse(self):
        r = Graph(len(self))
        for i in range(len(self)):
            for j in self.nexts[i]:
                r.nexts[j].append(i)
            for j in self.prevs[i]:
                r.prevs[j].append(i)
        return r

    def is_isolated(self, i):
        return not self.prevs[i] and not self.nexts[i]

    def edges(self):
        return [(i, j) for i in range(len(self)) for j in self.nexts[i]]


def _masters(hosts):
    masters, host_master = [], {}
    for rank, h in enumerate(hosts):
        if h not in host_master:
            host_master[h] = rank
            masters.append(rank)
    return masters, host_master


def gen_tree(hosts):
    """topology.go:17-31"""
    g = Graph(len(hosts))
    masters, hm = _masters(hosts)
    for rank, h in enumerate(hosts):
        if hm[h] != rank:
            g.add_edge(hm[h], rank)
    for rank in masters[1:]:
        g.add_edge(masters[0], rank)
    return g


def gen_default_reduce_graph(bg):
    """topology.go:33-40"""
    g0 = bg.reverse()
    for i in range(len(bg)):
        g0.add_edge(i, i)
    return g0


def gen_binary_tree(k):
    """topology.go:42-53"""
    g = Graph(k)
    for i in range(k):
        for j in (2 * i + 1, 2 * i + 2):
            if j < k:
                g.add_edge(i, j)
    return g


def _gen_multi_star(hosts, root):
    """topology.go:55-74"""
    g = Graph(len(hosts))
    masters, hm = _masters(hosts)
    for rank, h in enumerate(hosts):
        if hm[h] != rank:
            g.add_edge(hm[h], rank)
    k = len(masters)
    if k > 1:
        for i in range(k):
            if i != root:
                g.add_edge(masters[root], masters[i])
    return g


def _gen_binary_tree_star(hosts, offset):
    """topology.go:76-101"""
    g = Graph(len(hosts))
    masters, hm = _masters(hosts)
    for rank, h in enumerate(hosts):
        if hm[h] != rank:
            g.add_edge(hm[h], rank)
    k = len(masters)
    if k > 1:
        idx = lambda i: (i + offset) % k  # noqa: E731
        for i in range(k):
            for j in (2 * i + 1, 2 * i + 2):
                if j < k:
                    g.add_edge(masters[idx(i)], masters[idx(j)])
    return g


def gen_star_bcast_graph(k, r):
    """topology.go:138-147"""
    g = Graph(k)
    for i in range(k):
        if i != r:
            g.add_edge(r, i)
    return g


def gen_circular_graph_pair(k, r):
    """topology.go:149-160 — returns (reduceGraph, bcastGraph)."""
    g = Graph(k)
    for i in range(k):
        g.add_edge(i, i)
    b = Graph(k)
    for i in range(1, k):
        g.add_edge((r + i) % k, (r + i + 1) % k)
        b.add_edge((r + i - 1) % k, (r + i) % k)
    return g, b


def _simple(bg):
    return (gen_default_reduce_graph(bg), bg)


def strategy_list(name, hosts):
    """strategy.go:121-205 -> list of (reduceGraph, bcastGraph)."""
    k = len(hosts)
    if name == "AUTO":  # strategy.go:196-205
        name = "STAR" if len(set(hosts)) == 1 else "BINARY_TREE_STAR"
    if name == "STAR":
        return [_simple(gen_star_bcast_graph(k, 0))]
    if name == "MULTI_STAR":
        m = len(_masters(hosts)[0])
        return [_simple(_gen_multi_star(hosts, i)) for i in range(m)]
    if name == "CLIQUE":
        return [_simple(gen_star_bcast_graph(k, r)) for r in range(k)]
    if name == "RING":
        return [gen_circular_graph_pair(k, r) for r in range(k)]
    if name == "TREE":
        return [_simple(gen_tree(hosts))]
    if name == "BINARY_TREE":
        return [_simple(gen_binary_tree(k))]
    if name == "BINARY_TREE_STAR":
        return [_simple(_gen_binary_tree_star(hosts, 0))]
    if name == "MULTI_BINARY_TREE_STAR":
        m = len(_masters(hosts)[0])
        return [_simple(_gen_binary_tree_star(hosts, i)) for i in range(m)]
    raise ValueError(name)


def _topo_order(g):
    """Order in which reduce-graph nodes finish (a node sends after all its
    predecessors arrived)."""
    n = len(g)
    indeg = [len(g.prevs[i]) for i in range(n)]
    ready = [i for i in range(n) if indeg[i] == 0]
    order = []
    while ready:
        i = ready.pop(0)
        order.append(i)
        for j in g.nexts[i]:
            indeg[j] -= 1
            if indeg[j] == 0:
                ready.append(j)
    if len(order) != n:
        raise ValueError("graph has a cycle")
    return order


def run_graphs(send, recv, dt, op, graphs, arrival=None):
    """Simulate Session.runGraphs (session.go:231-299) for ALL ranks at once.

    send[r], recv[r]: per-rank numpy arrays (recv[r] is overwritten; pass the
    same object as send[r] for the in-place case).
    arrival(rank, prevs) -> prevs in the order their messages are folded in
    (the reference folds them in arrival order under a lock; default = the
    order of the graph's Prevs list).
    """
    k = len(send)
    if all(all(g.is_isolated(r) for g in graphs) for r in range(k)):
        for r in range(k):  # w.Forward()
            if recv[r] is not send[r]:
                np.copyto(recv[r], send[r])
        return
    recv_count = [0] * k

    def effective(r):
        return recv[r] if (recv_count[r] > 0 or recv[r] is send[r]) else send[r]

    for g in graphs:
        # what each node sends in this graph, computed in dependency order
        sent = {}
        for r in _topo_order(g):
            prevs = list(g.prevs[r])
            if g.self_loop[r]:
                order = arrival(r, prevs) if arrival else prevs
                for p in order:  # recvOnto: RecvBuf = effective o peer
                    oracle.transform2(effective(r), sent[p], dt, op, out=recv[r])
                    recv_count[r] += 1
            else:
                if not prevs and recv_count[r] == 0:
                    if recv[r] is not send[r]:
                        np.copyto(recv[r], send[r])  # w.Forward()
                else:
                    for p in prevs:  # recvInto
                        np.copyto(recv[r], sent[p])
                        recv_count[r] += 1
            sent[r] = np.array(effective(r), copy=True)


def all_reduce(inputs, dt, op="sum", strategy="BINARY_TREE_STAR", hosts=None,
               name="NegotiatedGrad_0/AllReduce", hash_method="NAME",
               arrival=None, inplace=False):
    """Session.AllReduce (allreduce.go:10-12 -> session.go:313-326) on every
    rank; returns the list of per-rank outputs."""
    k = len(inputs)
    hosts = hosts if hosts is not None else ["127.0.0.1"] * k
    sl = strategy_list(strategy, hosts)
    h = name_hash if hash_method == "NAME" else simple_hash
    count = inputs[0].size
    send = [np.array(x, copy=True) for x in inputs]
    recv = send if inplace else [np.zeros_like(x) for x in inputs]
    nbytes = count * inputs[0].itemsize
    nchunks = ceil_div(nbytes, CHUNK_SIZE)
    for i, (b, e) in enumerate(even_partition(0, count, nchunks) if nchunks else []):
        cname = "part::%s[%d:%d]" % (name, b, e)
        rg, bg = sl[h(i, cname) % len(sl)]
        cs = [s[b:e] for s in send]
        cr = cs if inplace else [r[b:e] for r in recv]
        run_graphs(cs, cr, dt, op, [rg, bg], arrival=arrival)
    return recv


def from_forest_array(forest):
    """graph.go:46-62 FromForestArray: forest[i] is i's father (i itself for a
    root); returns (bcast graph, number of roots) or None if out of range."""
    n = len(forest)
    g, m = Graph(n), 0
    for i, father in enumerate(forest):
        if father < 0 or father >= n:
            return None
        if father == i:
            m += 1
        else:
            g.add_edge(father, i)
    return g, m


def subset_all_reduce(inputs, dt, op, forest, name="NegotiatedGrad_0/AllReduce",
                      hash_method="NAME", arrival=None):
    """Session.SubsetAllReduce (allreduce.go:14-24): every tree of the forest
    all-reduces within itself, chunked as AllReduce, one strategy
    (simpleSingleGraphStrategy, strategy.go:105-107)."""
    bg, _ = from_forest_array(forest)
    sl = [_simple(bg)]
    count = inputs[0].size
    send = [np.array(x, copy=True) for x in inputs]
    recv = [np.zeros_like(x) for x in inputs]
    nchunks = ceil_div(count * inputs[0].itemsize, CHUNK_SIZE)
    for b, e in (even_partition(0, count, nchunks) if nchunks else []):
        rg, g = sl[0]
        run_graphs([x[b:e] for x in send], [r[b:e] for r in recv], dt, op, [rg, g],
                   arrival=arrival)
    return recv


def reduce(inputs, dt, op="sum", strategy="BINARY_TREE_STAR", hosts=None, arrival=None,
           initial=None):
    """Session.Reduce (session.go:159-162): runGraphs(w, strategies[0].reduceGraph)
    on the whole workspace, every rank; recv starts as `initial` (per rank) so
    what runGraphs leaves untouched shows."""
    k = len(inputs)
    hosts = hosts if hosts is not None else ["127.0.0.1"] * k
    rg, _ = strategy_list(strategy, hosts)[0]
    send = [np.array(x, copy=True) for x in inputs]
    recv = [np.array(x, copy=True) for x in initial] if initial is not None else \
        [np.zeros_like(x) for x in inputs]
    run_graphs(send, recv, dt, op, [rg], arrival=arrival)
    return recv


def broadcast(inputs, strategy="BINARY_TREE_STAR", hosts=None):
    """Session.Broadcast (session.go:164-167): runGraphs(w, strategies[0].bcastGraph)."""
    k = len(inputs)
    hosts = hosts if hosts is not None else ["127.0.0.1"] * k
    _, bg = strategy_list(strategy, hosts)[0]
    send = [np.array(x, copy=True) for x in inputs]
    recv = [np.zeros_like(x) for x in inputs]
    run_graphs(send, recv, None, None, [bg])
    return recv


def chunk_roots(count, itemsize, k, strategy="RING", name="NegotiatedGrad_0/AllReduce",
                hash_method="NAME"):
    """Per-chunk (begin, end, strategy index) as runStrategiesWithHash picks."""
    hosts = ["127.0.0.1"] * k
    sl = strategy_list(strategy, hosts)
    h = name_hash if hash_method == "NAME" else simple_hash
    nchunks = ceil_div(count * itemsize, CHUNK_SIZE)
    out = []
    for i, (b, e) in enumerate(even_partition(0, count, nchunks) if nchunks else []):
        out.append((b, e, h(i, "part::%s[%d:%d]" % (name, b, e)) % len(sl)))
    return out


def ring_order(k, r):
    """Rank order in which a RING strategy rooted at r folds the chunk:
    node r+1 starts with its own buffer, each next node computes
    Transform2(own, received), ending at r (topology.go:149-160). Returns the
    operand list for a left fold with the same rounding: fold(x_{r+1}, x_{r+2},
    ..., x_r) — fp addition is commutative, so own+recv == recv+own."""
    return [(r + i) % k for i in range(1, k + 1)]


def all_arrival_orders(prevs):
    return list(itertools.permutations(prevs))
