#!/usr/bin/env python3
"""HBM traffic of every kernel family behind the C ABI (not only C2's), from
rocprofv3 PMC passes: is any of them moving more bytes than its algorithm
needs (re-reads, partial-line writes)?

Run the workload once per counter, in separate passes (MI355X_MICROARCH.md
§HBM), then summarise:

  rocprofv3 --pmc FETCH_SIZE -d D/f -o pmc --output-format csv -- python3 tools/pmc_kernels.py run
  rocprofv3 --pmc WRITE_SIZE -d D/w -o pmc --output-format csv -- python3 tools/pmc_kernels.py run
  python3 tools/pmc_kernels.py summarize D/f D/w > profiles/r01/pmc_kernels.jsonl

`run` launches each variant LAUNCHES times, back to back, on 3 rotating
buffer sets of 256 MiB per input (cold Infinity Cache, as bench.py), after
every buffer is allocated and filled, so the variants' dispatches of our
kernels come in a known order. FETCH_SIZE is doubled (gfx950 wide streaming
reads), both counters are KiB.
"""
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

BYTES = 256 << 20
LAUNCHES = 6
OURS = ("void kf::reduce_kernel", "void kf::reduce_spread_kernel", "void kf::sma_kernel",
        "void kf::reduce_batch_kernel")

# (name, inputs read, outputs written) in units of BYTES
VARIANTS = [
    ("reduce SUM k=2 f32", 2, 1),
    ("reduce SUM k=4 f32", 4, 1),
    ("reduce SUM k=8 f32", 8, 1),
    ("reduce_peers avg k=4 f32 (P2P fold, local HBM)", 4, 1),
    ("reduce_peers avg k=8 f32 (P2P fold, local HBM)", 8, 1),
    ("div_ f32 (S-SGD shard epilogue)", 1, 1),
    ("sma_blend f32", 2, 1),
    ("reduce SUM k=2 bf16", 2, 1),
    ("reduce SUM k=2 i8 (packed 32-bit lanes)", 2, 1),
    ("reduce MAX k=8 i8 (packed 32-bit lanes)", 8, 1),
    ("batch: 16 buckets x 16 MiB, SUM k=2 f32 (one launch)", 2, 1),
    ("batch: 16 shards x 16 MiB, /np in place f32 (one launch)", 1, 1),
]


def run():
    import torch
    from kungfu_amd import _lib, ops
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    n = BYTES // 4

    def bufs(k, dtype=torch.float32):
        m = BYTES // torch.empty((), dtype=dtype).element_size()
        sets = []
        for _ in range(3):
            ins = [torch.randn(m, device=dev).to(dtype) if dtype.is_floating_point
                   else torch.randint(-128, 128, (m,), device=dev, dtype=dtype)
                   for _ in range(k)]
            sets.append((ins, torch.empty_like(ins[0])))
        return sets

    plan = []
    for k in (2, 4, 8):
        plan.append((lambda ins, out, k=k: lib.kf_bucket_reduce(
            _lib.ptr_array([t.data_ptr() for t in ins]), k, out.data_ptr(), n, 0x20408, 0, s),
            bufs(k)))
    for k in (4, 8):
        sets = bufs(k)
        plan.append((lambda ins, out, k=k: lib.kf_bucket_reduce_peers(
            _lib.ptr_array([t.data_ptr() for t in ins]), k, out.data_ptr(), n, 0x20408, 0, k, s),
            sets))
    plan.append((lambda ins, out: ops.bucket_div_(ins[0], 8), bufs(1)))
    plan.append((lambda ins, out: ops.sma_blend_(ins[0], ins[1], 8, 0.1), bufs(2)))
    sets = bufs(2, torch.bfloat16)
    plan.append((lambda ins, out: lib.kf_bucket_reduce(
        _lib.ptr_array([t.data_ptr() for t in ins]), 2, out.data_ptr(), out.numel(), 0x20209, 0,
        s), sets))
    for k, op in ((2, 0), (8, 2)):
        plan.append((lambda ins, out, k=k, op=op: lib.kf_bucket_reduce(
            _lib.ptr_array([t.data_ptr() for t in ins]), k, out.data_ptr(), out.numel(),
            0x10108, op, s), bufs(k, torch.int8)))
    import ctypes
    nb, m = 16, n // 16
    cnts = (ctypes.c_size_t * nb)(*([m] * nb))
    for k, np_ in ((2, 0), (1, 8)):
        def batch(ins, out, k=k, np_=np_):
            src = [ins[j][b * m:(b + 1) * m] for b in range(nb) for j in range(k)]
            dst = [(out if k > 1 else ins[0])[b * m:(b + 1) * m] for b in range(nb)]
            return lib.kf_bucket_reduce_batch(_lib.ptr_array([t.data_ptr() for t in src]), k,
                                              _lib.ptr_array([t.data_ptr() for t in dst]), cnts,
                                              nb, 0x20408, 0, np_, s)
        plan.append((batch, bufs(k)))
    assert len(plan) == len(VARIANTS)
    torch.cuda.synchronize()
    for fn, sets in plan:
        for i in range(LAUNCHES):
            ins, out = sets[i % len(sets)]
            fn(ins, out)
        torch.cuda.synchronize()
    print("launched %d variants x %d" % (len(plan), LAUNCHES))


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and r["Kernel_Name"].startswith(OURS):
                key = int(r["Dispatch_Id"])
                rows[key] = rows.get(key, 0.0) + float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def summarize(fdir, wdir):
    f = per_dispatch(fdir, "FETCH_SIZE")
    w = per_dispatch(wdir, "WRITE_SIZE")
    want = len(VARIANTS) * LAUNCHES
    if len(f) != want or len(w) != want:
        raise SystemExit("expected %d dispatches, got %d / %d" % (want, len(f), len(w)))
    for i, (name, nin, nout) in enumerate(VARIANTS):
        sl = slice(i * LAUNCHES + 1, (i + 1) * LAUNCHES)  # first launch of each: warm-up
        rd = statistics.median(f[sl]) * 1024 * 2
        wr = statistics.median(w[sl]) * 1024
        algo = (nin + nout) * BYTES
        print(json.dumps({"kernel": name, "read_bytes": int(rd), "write_bytes": int(wr),
                          "algorithmic_bytes": algo,
                          "ratio_to_algorithmic": round((rd + wr) / algo, 4),
                          "source": "rocprofv3 --pmc FETCH_SIZE (x2) / WRITE_SIZE, separate "
                                    "passes, median of %d launches" % (LAUNCHES - 1)}))


if __name__ == "__main__":
    if sys.argv[1:2] == ["run"]:
        run()
    elif sys.argv[1:2] == ["summarize"]:
        summarize(sys.argv[2], sys.argv[3])
    else:
        raise SystemExit(__doc__)
