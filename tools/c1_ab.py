#!/usr/bin/env python3
"""A/B of C1 (np = 2, one 4 MiB fp32 bucket) session settings, interleaved:
each variant is a bench.py C1 mode plus environment for its peers, run in
turn `--repeats` times on the GPU's NUMA node; per variant the median of the
runs' medians and every run's median.

    python tools/c1_ab.py device device:KUNGFU_AMD_TX_AHEAD=4 cpu [--repeats 5]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--np", type=int, default=2)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import bench
    cpus = bench.gpu_local_cpus()
    runs = {v: [] for v in a.variants}
    for _ in range(a.repeats):
        for v in a.variants:
            mode, _, envs = v.partition(":")
            saved = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, _, val = kv.partition("=")
                os.environ[k] = val
            try:
                rec = bench.c1_run(a.np, (mode,), a.steps, a.warmup, timeout=300, cpus=cpus)[mode]
            finally:
                os.environ.clear()
                os.environ.update(saved)
            runs[v].append(rec)
    out = {}
    for v, recs in runs.items():
        ok = [r for r in recs if "error" not in r]
        meds = [r["latency_ms_median"] for r in ok]
        out[v] = {"median_ms": round(statistics.median(meds), 4) if meds else None,
                  "run_medians_ms": meds, "correct": all(r.get("correct") for r in ok),
                  "errors": [r["error"] for r in recs if "error" in r]}
    s = json.dumps({"np": a.np, "steps": a.steps, "repeats": a.repeats, "variants": out}, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
