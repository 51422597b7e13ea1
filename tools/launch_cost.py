#!/usr/bin/env python3
"""Host-side cost of the calls a chunk's pieces would add to the session's
poll thread: one kf_bucket_reduce launch (2 inputs, a 256 KiB piece, one
input in page-locked host memory as the ingest slot is), one hipEventRecord,
one 256 KiB H2D hipMemcpyAsync — each issued back to back on one stream,
µs per call on the host (median of 5 batches of 200), then the stream
drained. Tells whether pieces can be queued from the thread that reads the
socket (DESIGN §4, C1 traced)."""
import ctypes
import json
import statistics
import sys
import time
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kungfu_amd import _lib
    lib = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so.7")
    dev = torch.device("cuda:0")
    n = (256 << 10) // 4
    own = torch.randn(n, device=dev)
    out = torch.empty(n, device=dev)
    host = torch.randn(n).pin_memory()
    s = torch.cuda.Stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    ev = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(ev), 2) == 0  # hipEventDisableTiming
    ins = _lib.ptr_array([own.data_ptr(), host.data_ptr()])

    def fold():
        return lib.kf_bucket_reduce(ins, 2, out.data_ptr(), n, 0x20408, 0, sp)

    def record():
        return hip.hipEventRecord(ev, sp)

    def h2d():
        return hip.hipMemcpyAsync(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(host.data_ptr()),
                                  ctypes.c_size_t(n * 4), 1, sp)  # hipMemcpyHostToDevice

    res = {}
    for name, fn in (("kf_bucket_reduce_256KiB_zero_copy", fold), ("hipEventRecord", record),
                     ("hipMemcpyAsync_H2D_256KiB", h2d)):
        batches = []
        for _ in range(6):
            t0 = time.perf_counter()
            for _ in range(200):
                assert fn() == 0
            batches.append((time.perf_counter() - t0) / 200 * 1e6)
            s.synchronize()
        res[name + "_host_us"] = round(statistics.median(batches[1:]), 2)
    # one piece end to end: launch, record, wait for the event
    lat = []
    for _ in range(200):
        t0 = time.perf_counter()
        fold()
        record()
        hip.hipEventSynchronize(ev)
        lat.append((time.perf_counter() - t0) * 1e6)
    res["fold_256KiB_launch_to_event_us"] = round(statistics.median(lat), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
