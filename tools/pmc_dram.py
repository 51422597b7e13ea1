#!/usr/bin/env python3
"""Why the k-input fold runs below the two-input sum: the DRAM side, from
rocprofv3 PMC counters of the L2's memory-side (EA) interface.

For the fp32 fold at k = 2, 4, 8 (256 MiB per input, 3 rotating buffer sets
as bench.py) and the 16 x 4 MiB batched launch, per launch:
  * average read / write latency at the EA interface, in cycles:
    TCC_EA0_RDREQ_LEVEL_sum / TCC_EA0_RDREQ_sum (requests in flight integrated
    over time / requests: Little's law), same for WRREQ;
  * cycles the L2 could not send a request because the DRAM controller had
    no credits left: TCC_EA0_{RD,WR}REQ_DRAM_CREDIT_STALL_sum, as a fraction
    of the launch's GRBM_GUI_ACTIVE cycles (summed over the 16 L2 channels,
    so the fraction is per channel on average).

  D=gpurun_out/pmcd
  rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE -d $D/a -o pmc --output-format csv -- python3 tools/pmc_dram.py run
  rocprofv3 --pmc TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum -d $D/b -o pmc --output-format csv -- python3 tools/pmc_dram.py run
  rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum -d $D/c -o pmc --output-format csv -- python3 tools/pmc_dram.py run
  python3 tools/pmc_dram.py summarize $D/a $D/b $D/c
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
OURS = ("void kf::reduce_kernel", "void kf::reduce_batch_kernel")
VARIANTS = ["fold k=2 f32 (C2)", "fold k=4 f32", "fold k=8 f32",
            "batch 16 x 4 MiB SUM k=2 f32 (one launch)"]


def run():
    import ctypes
    import torch
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    n = BYTES // 4

    def sets(k):
        return [([torch.randn(n, device=dev) for _ in range(k)], torch.empty(n, device=dev))
                for _ in range(3)]

    plan = []
    for k in (2, 4, 8):
        plan.append((lambda ins, out, k=k: lib.kf_bucket_reduce(
            _lib.ptr_array([t.data_ptr() for t in ins]), k, out.data_ptr(), n, 0x20408, 0, s),
            sets(k)))
    nb, m = 16, (4 << 20) // 4
    cnts = (ctypes.c_size_t * nb)(*([m] * nb))

    def batch(ins, out):
        src = [ins[j][b * m:(b + 1) * m] for b in range(nb) for j in range(2)]
        dst = [out[b * m:(b + 1) * m] for b in range(nb)]
        return lib.kf_bucket_reduce_batch(_lib.ptr_array([t.data_ptr() for t in src]), 2,
                                          _lib.ptr_array([t.data_ptr() for t in dst]), cnts, nb,
                                          0x20408, 0, 0, s)
    plan.append((batch, sets(2)))
    torch.cuda.synchronize()
    for fn, ss in plan:
        for i in range(LAUNCHES):
            ins, out = ss[i % len(ss)]
            fn(ins, out)
        torch.cuda.synchronize()
    print("launched %d variants x %d" % (len(plan), LAUNCHES))


def per_dispatch(d):
    """{counter: [value per dispatch of our kernels, in dispatch order]}"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith(OURS):
                c = rows.setdefault(r["Counter_Name"], {})
                key = int(r["Dispatch_Id"])
                c[key] = c.get(key, 0.0) + float(r["Counter_Value"])
    return {c: [v[k] for k in sorted(v)] for c, v in rows.items()}


def summarize(*dirs):
    vals = {}
    for d in dirs:
        vals.update(per_dispatch(d))
    want = len(VARIANTS) * LAUNCHES
    for c, v in vals.items():
        if len(v) != want:
            raise SystemExit("%s: expected %d dispatches, got %d" % (c, want, len(v)))

    def med(c, i):
        return statistics.median(vals[c][i * LAUNCHES + 1:(i + 1) * LAUNCHES])

    for i, name in enumerate(VARIANTS):
        cyc = med("GRBM_GUI_ACTIVE", i)
        rec = {"kernel": name,
               "gui_active_cycles": int(cyc),
               "read_latency_cycles": round(med("TCC_EA0_RDREQ_LEVEL_sum", i) /
                                            med("TCC_EA0_RDREQ_sum", i), 1),
               "write_latency_cycles": round(med("TCC_EA0_WRREQ_LEVEL_sum", i) /
                                             med("TCC_EA0_WRREQ_sum", i), 1),
               "rd_credit_stall_per_channel": round(
                   med("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", i) / 16 / cyc, 4),
               "wr_credit_stall_per_channel": round(
                   med("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", i) / 16 / cyc, 4),
               "source": "rocprofv3 --pmc, 3 separate passes, median of %d launches"
                         % (LAUNCHES - 1)}
        print(json.dumps(rec))


if __name__ == "__main__":
    if sys.argv[1:2] == ["run"]:
        run()
    elif sys.argv[1:2] == ["summarize"]:
        summarize(*sys.argv[2:])
    else:
        raise SystemExit(__doc__)
