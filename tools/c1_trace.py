#!/usr/bin/env python3
"""Where C1's time goes: bench.py's C1 peers (np = 2, one 4 MiB fp32 bucket,
4 x 1 MiB chunks, STAR at rank 0) with KUNGFU_AMD_SESSION_TRACE on, one run per
mode, and per-step timelines built from the peers' traces (CLOCK_MONOTONIC,
one clock for both processes).

    python tools/c1_trace.py [--modes device,cpu] [--steps 40] [--out f.json]

Per mode, medians over the timed steps (us from the leaf's op_start):
  leaf   rank 1: its chunks' D2H landed (tx_ready) and written (tx_done), the
         reduced chunks' headers in (rx_hdr) and bodies landed (rx_done),
         op_done;
  root   rank 0: each chunk's header in, body in + fold queued (rx_done),
         fold done (tx_ready: the mirror event / host fold), sent (tx_done).
"""
import argparse
import json
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def steps_of(recs):
    """Split one peer's records into all-reduce calls (op_start .. op_done)."""
    out, cur = [], None
    for r in recs:
        if r["ev"] == "op_start":
            cur = [r]
        elif cur is not None:
            cur.append(r)
            if r["ev"] == "op_done":
                out.append(cur)
                cur = None
    return out


def first(recs, ev, chunk=None, arg=None):
    for r in recs:
        if r["ev"] == ev and (chunk is None or r["chunk"] == chunk) and \
                (arg is None or r["arg"] == arg):
            return r["t_us"]
    return None


def timeline(root, leaf):
    t0 = leaf[0]["t_us"]
    rel = lambda t: None if t is None else round(t - t0, 2)  # noqa: E731
    d = {"leaf_op_done": rel(first(leaf, "op_done")),
         "root_op_done": rel(first(root, "op_done")),
         "root_op_start": rel(first(root, "op_start"))}
    for c in range(4):
        d["leaf_tx_ready_%d" % c] = rel(first(leaf, "tx_ready", c, 0))
        d["leaf_tx_done_%d" % c] = rel(first(leaf, "tx_done", c, 0))
        d["root_rx_hdr_%d" % c] = rel(first(root, "rx_hdr", c, 0))
        d["root_rx_done_%d" % c] = rel(first(root, "rx_done", c, 0))
        d["root_fold_end_%d" % c] = rel(first(root, "fold_end", c))
        d["root_tx_ready_%d" % c] = rel(first(root, "tx_ready", c, 1))
        d["root_tx_done_%d" % c] = rel(first(root, "tx_done", c, 1))
        d["leaf_rx_hdr_%d" % c] = rel(first(leaf, "rx_hdr", c, 1))
        d["leaf_rx_done_%d" % c] = rel(first(leaf, "rx_done", c, 1))
    return d


def run_mode(mode, steps, warmup):
    import bench
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "trace")
        os.environ["KUNGFU_AMD_SESSION_TRACE"] = path
        try:
            res = bench.c1_run(2, (mode,), steps, warmup, timeout=300, cpus=bench.gpu_local_cpus())
        finally:
            del os.environ["KUNGFU_AMD_SESSION_TRACE"]
        root, leaf = steps_of(load(path + ".0")), steps_of(load(path + ".1"))
    n = min(len(root), len(leaf))
    lines = [timeline(root[i], leaf[i]) for i in range(warmup, n)]
    med = {}
    for k in lines[0]:
        vals = [ln[k] for ln in lines if ln[k] is not None]
        med[k] = round(statistics.median(vals), 2) if vals else None
    return {"mode": mode, "record": res.get(mode), "steps": len(lines), "median_us": med}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="device,cpu")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    out = [run_mode(m, a.steps, a.warmup) for m in a.modes.split(",")]
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
