#!/usr/bin/env python3
"""HBM traffic of the exchange's phase-2 launches at BASELINE's 8-GPU shapes
(bench.py exchange_phase2: C4's and C3's shard /np, C5's all-to-all fold),
from two rocprofv3 PMC passes, per dispatch of reduce_batch_kernel, grouped
by grid size (each shape has its own grid). Is the 2-D grid launch (equal
buckets, r05) still moving exactly its algorithmic bytes?

  rocprofv3 --pmc FETCH_SIZE -d D/f -o pmc --output-format csv -- python3 tools/pmc_phase2.py run
  rocprofv3 --pmc WRITE_SIZE -d D/w -o pmc --output-format csv -- python3 tools/pmc_phase2.py run
  python3 tools/pmc_phase2.py summarize D/f D/w > profiles/r05/pmc_phase2.json

FETCH_SIZE is doubled (gfx950 wide streaming reads, MI355X_MICROARCH.md
§HBM); both counters are KiB. Launches cycle over shard sets of >= 0.75 GiB
so none is served from the Infinity Cache.
"""
import csv
import ctypes
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

WORLD = 8
LAUNCHES = 8


def shapes():
    """(name, counts per bucket, k, dtype code, algorithmic bytes per launch)"""
    import json as _json
    import torch
    from kungfu_amd.collective import GradBuckets
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    with open(os.path.join(root, "tests", "golden", "models.json")) as f:
        models = _json.load(f)
    rn = GradBuckets(models["resnet50-imagenet"], torch.float32, torch.device("cpu"), WORLD,
                     n_buckets=16)
    c4 = [b.numel() // WORLD for b in rn.buckets]
    c3 = [(1 << 20) // WORLD] * 64
    return [("c4_shard_div_n8_f32", c4, 4), ("c3_shard_div_n8_f32", c3, 4)]


def run():
    import torch
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    sp = torch.cuda.current_stream().cuda_stream
    for name, qs, sz in shapes():
        per_set = sum(2 * q * sz for q in qs)
        nsets = max(2, -(-(768 << 20) // per_set))
        sets = []
        for _ in range(nsets):
            shards = [torch.randn(q, device=dev, generator=g) for q in qs]
            sets.append((_lib.ptr_array([s.data_ptr() for s in shards]),
                         (ctypes.c_size_t * len(qs))(*qs), shards))
        torch.cuda.synchronize()
        for i in range(LAUNCHES):
            s = sets[i % nsets]
            _lib.check(lib.kf_bucket_reduce_batch(s[0], 1, s[0], s[1], len(qs), 0x20408, 0,
                                                  WORLD, sp), name)
        torch.cuda.synchronize()
        print(json.dumps({"shape": name, "buckets": len(qs), "algorithmic_bytes": per_set}),
              flush=True)
        del sets
        torch.cuda.empty_cache()


def per_grid(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "reduce_batch_kernel" in r["Kernel_Name"]:
                vals.setdefault(int(r["Grid_Size"]), []).append(float(r["Counter_Value"]))
    return vals


def summarize(fdir, wdir):
    fv, wv = per_grid(fdir, "FETCH_SIZE"), per_grid(wdir, "WRITE_SIZE")
    algo = {}
    for name, qs, sz in shapes():
        algo[name] = sum(2 * q * sz for q in qs)
    out = []
    for grid in sorted(fv):
        fk = statistics.median(fv[grid])
        wk = statistics.median(wv.get(grid, [0.0]))
        hbm = 2 * fk * 1024 + wk * 1024
        out.append({"grid_threads": grid, "dispatches": len(fv[grid]),
                    "read_bytes": 2 * fk * 1024, "write_bytes": wk * 1024,
                    "hbm_bytes_per_launch": hbm})
    # match each grid to the shape whose algorithmic bytes it is closest to
    for o in out:
        name = min(algo, key=lambda n: abs(algo[n] - o["hbm_bytes_per_launch"]))
        o["shape"] = name
        o["algorithmic_bytes"] = algo[name]
        o["ratio_to_algorithmic"] = round(o["hbm_bytes_per_launch"] / algo[name], 4)
    print(json.dumps({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
                                "FETCH_SIZE x2 (gfx950)", "per_grid": out}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2], sys.argv[3])
