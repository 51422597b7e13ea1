#!/usr/bin/env python3
"""Rate of the element-at-a-time kernel (reduce_kernel_unaligned), taken when
the inputs' 16-B residues differ, against the vector kernel on the same
bytes: 256 MiB per input, launches cycling over 3 bucket sets, HIP events
around 20 launches, median of 5, for f32 / bf16 / u8 and a few offset pairs
(in elements) of (x, y, z).

  python tools/unaligned_rate.py > profiles/r02/unaligned_rate.jsonl
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

PEAK = 8000.0
BYTES = 256 << 20
CODES = {torch.float32: 0x20408, torch.bfloat16: 0x20209, torch.uint8: 0x00108}


def main():
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    for dtype in (torch.float32, torch.bfloat16, torch.uint8):
        isz = torch.empty((), dtype=dtype).element_size()
        n = BYTES // isz
        sets = []
        for _ in range(3):
            if dtype.is_floating_point:
                x, y = (torch.randn(n + 16, device=dev).to(dtype) for _ in range(2))
            else:
                x, y = (torch.randint(0, 256, (n + 16,), device=dev, dtype=dtype) for _ in range(2))
            sets.append((x, y, torch.empty(n + 16, device=dev, dtype=dtype)))
        for offs in ((0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 2, 3)):
            if isz * 1 >= 16 and offs != (0, 0, 0):
                continue
            args = []
            for x, y, z in sets:
                ox, oy, oz = offs
                args.append((_lib.ptr_array([x[ox:].data_ptr(), y[oy:].data_ptr()]),
                             z[oz:].data_ptr()))

            def launch(i):
                p, zp = args[i % 3]
                return lib.kf_bucket_reduce(p, 2, zp, n, CODES[dtype], 0, s)

            assert launch(0) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(5):
                e0.record()
                for i in range(20):
                    launch(i)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 20)
            us = statistics.median(ts)
            x, y, z = sets[0]
            ox, oy, oz = offs
            ok = bool(torch.equal(z[oz:oz + n], (x[ox:ox + n].float() + y[oy:oy + n].float())
                                  .to(dtype))) if dtype != torch.uint8 else bool(
                torch.equal(z[oz:oz + n], x[ox:ox + n] + y[oy:oy + n]))
            gbps = 3 * BYTES / us / 1e3
            print(json.dumps({"dtype": str(dtype).split(".")[-1], "offsets_xyz": offs,
                              "path": "vector" if offs == (0, 0, 0) else "unaligned",
                              "us": round(us, 2), "GBps": round(gbps, 1),
                              "frac": round(gbps / PEAK, 4), "correct": ok}), flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
