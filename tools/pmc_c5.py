#!/usr/bin/env python3
"""C5's two HBM kernels on the exact shapes of bench.py's N = 1 line
(`kernels.sma_batch_c5_bf16`, `kernels.c5_a2a_fold_n8_bf16`): rocprofv3
kernel durations and PMC HBM bytes per launch.

  sma_batch  kf_sma_blend_batch over BERT-base's first 201 tensors in bf16,
             16 MiB buckets (GradBuckets, as bench.py / the exchange), in place
  a2a_fold   kf_bucket_reduce_batch k = 8, the 8 received bf16 shards of every
             bucket back to back in one workspace, /8 fused (C5 at N = 8)

Each launches LAUNCHES times over rotating sets (>= 0.75 GiB apart, cold
Infinity Cache), sma_batch first. Passes (MI355X_MICROARCH.md, HBM section;
FETCH_SIZE doubled for gfx950, both counters KiB):

  rocprofv3 --kernel-trace --stats -d D/t -o t --output-format csv -- python3 tools/pmc_c5.py run
  rocprofv3 --pmc FETCH_SIZE -d D/f -o pmc --output-format csv -- python3 tools/pmc_c5.py run
  rocprofv3 --pmc WRITE_SIZE -d D/w -o pmc --output-format csv -- python3 tools/pmc_c5.py run
  python3 tools/pmc_c5.py summarize D/t D/f D/w > profiles/r06/pmc_c5.jsonl
"""
import csv
import ctypes
import glob
import json
import os
import statistics
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

LAUNCHES = 12
# full names, or the short ones rocprofv3 -T (--truncate-kernels) writes
KERNELS = {"sma_batch": ("void kf::sma_batch_kernel", "sma_batch_kernel"),
           "a2a_fold": ("void kf::reduce_batch_kernel", "reduce_batch_kernel")}


def _is(name, prefix):
    return name.startswith(prefix[0]) or name == prefix[1]


def shapes():
    """(sma algorithmic bytes per launch, fold algorithmic bytes per launch)"""
    return json.load(open(os.path.join(ROOT, "profiles", "r06", "pmc_c5_shapes.json")))


def run():
    import torch
    from kungfu_amd import _lib
    from kungfu_amd.collective import GradBuckets
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(7)
    bert = json.load(open(os.path.join(ROOT, "tests", "golden", "models.json")))["bert"][:201]
    sets = []
    for _ in range(3):
        gbv = GradBuckets(bert, torch.bfloat16, dev, 8, bucket_bytes=16 << 20)
        for b in gbv.buckets:
            b.copy_(torch.randn(b.numel(), device=dev, generator=g).bfloat16())
        from kungfu_amd.collective import workspace_like
        sums = workspace_like(gbv.buckets)  # as the exchange lays them out (flat)
        for t in sums:
            t.copy_(torch.randn(t.numel(), device=dev, generator=g).bfloat16())
        sets.append((_lib.ptr_array([b.data_ptr() for b in gbv.buckets]),
                     _lib.ptr_array([t.data_ptr() for t in sums]),
                     (ctypes.c_size_t * len(sums))(*[t.numel() for t in sums]), gbv, sums))
    nbs = len(sets[0][4])
    sma_bytes = 3 * 2 * sum(t.numel() for t in sets[0][4])
    world = 8
    counts = [b.numel() for b in sets[0][3].buckets]
    qs = [c // world for c in counts]
    per_set = sum((world + 1) * q * 2 for q in qs)
    nsets = max(2, -(-(768 << 20) // per_set))
    fsets = []
    for _ in range(nsets):
        ws = [torch.randn(world * q, device=dev, generator=g).bfloat16() for q in qs]
        outs = [torch.empty(q, device=dev, dtype=torch.bfloat16) for q in qs]
        ins = _lib.ptr_array([w.data_ptr() + j * q * 2 for w, q in zip(ws, qs) for j in range(world)])
        fsets.append((ins, _lib.ptr_array([o.data_ptr() for o in outs]),
                      (ctypes.c_size_t * len(qs))(*qs), ws, outs))
    torch.cuda.synchronize()
    for i in range(LAUNCHES):
        st = sets[i % 3]
        _lib.check(lib.kf_sma_blend_batch(st[0], st[1], st[2], nbs, 0x20209, 8, 0.1, s), "sma")
    torch.cuda.synchronize()
    for i in range(LAUNCHES):
        st = fsets[i % nsets]
        _lib.check(lib.kf_bucket_reduce_batch(st[0], world, st[1], st[2], len(qs), 0x20209, 0,
                                              world, s), "fold")
    torch.cuda.synchronize()
    os.makedirs(os.path.join(ROOT, "profiles", "r06"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r06", "pmc_c5_shapes.json"), "w") as f:
        json.dump({"sma_batch": sma_bytes, "a2a_fold": per_set, "sma_buckets": nbs,
                   "fold_buckets": len(qs)}, f)
    print("launched sma_batch x %d (%d buckets), a2a_fold x %d (%d buckets)"
          % (LAUNCHES, nbs, LAUNCHES, len(qs)))


def _rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def per_dispatch(d, counter, prefix):
    rows = {}
    for r in _rows(d, "*counter_collection.csv"):
        if r["Counter_Name"] == counter and _is(r["Kernel_Name"], prefix):
            key = int(r["Dispatch_Id"])
            rows[key] = rows.get(key, 0.0) + float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def durations(d, prefix):
    ts = []
    for r in _rows(d, "*kernel_trace.csv"):
        if _is(r["Kernel_Name"], prefix):
            ts.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return [dt for _, dt in sorted(ts)]


def summarize(tdir, fdir, wdir):
    sh = shapes()
    for key, prefix in KERNELS.items():
        f = per_dispatch(fdir, "FETCH_SIZE", prefix)
        w = per_dispatch(wdir, "WRITE_SIZE", prefix)
        t = durations(tdir, prefix)
        if len(f) != LAUNCHES or len(w) != LAUNCHES or len(t) != LAUNCHES:
            raise SystemExit("%s: expected %d dispatches, got %d / %d / %d"
                             % (key, LAUNCHES, len(f), len(w), len(t)))
        rd = statistics.median(f[2:]) * 1024 * 2
        wr = statistics.median(w[2:]) * 1024
        us = statistics.mean(t[2:]) / 1e3
        algo = sh[key]
        print(json.dumps({
            "kernel": key, "rocprof_avg_us": round(us, 2), "algorithmic_bytes": algo,
            "achieved_GBps": round(algo / us / 1e3, 1), "frac": round(algo / us / 1e3 / 8000, 4),
            "read_bytes": int(rd), "write_bytes": int(wr),
            "traffic_ratio": round((rd + wr) / algo, 4),
            "source": "rocprofv3 --kernel-trace (mean of launches 3..%d) and --pmc FETCH_SIZE "
                      "(x2) / WRITE_SIZE in separate passes (median)" % LAUNCHES}))


if __name__ == "__main__":
    if sys.argv[1:2] == ["run"]:
        run()
    elif sys.argv[1:2] == ["summarize"]:
        summarize(*sys.argv[2:5])
    else:
        raise SystemExit(__doc__)
