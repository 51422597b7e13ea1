#!/usr/bin/env python3
"""Stress of the k-input fold's two schedules (batched loads below 2048
blocks, inline-asm one-in-flight loads above): 400 launches over random k
(3..16), sizes across the 2048-block switch (up to 96 MiB per input), dtypes
f32 / bf16 / i32 and element offsets (so inputs sit at other 16-B residues),
every result checked against the in-order fold computed by torch (f32 adds in
input order are exact same IEEE ops; i32 wraps; bf16 through the oracle's
fp32-accumulate-once definition: compared against a float64-free fp32 chain
rounded once).

  python tools/fold_stress.py > profiles/r02/fold_stress.json
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(1234)
    codes = {torch.float32: 0x20408, torch.int32: 0x10408, torch.bfloat16: 0x20209}
    bad, runs, serial_runs = [], 0, 0
    for it in range(400):
        k = int(torch.randint(3, 17, (1,), generator=g))
        dt = [torch.float32, torch.int32, torch.bfloat16][it % 3]
        esz = torch.tensor([], dtype=dt).element_size()
        cap = (96 << 20) // esz if it % 5 == 0 else (8 << 20) // esz
        n = int(torch.randint(1, max(2, cap), (1,), generator=g))
        offs = [int(torch.randint(0, 8, (1,), generator=g)) for _ in range(k + 1)]
        if dt == torch.int32:
            bufs = [torch.randint(-2**31, 2**31 - 1, (n + 8,), dtype=torch.int32, device=dev)
                    for _ in range(k)]
        else:
            bufs = [torch.randn(n + 8, device=dev).to(dt) for _ in range(k)]
        ins = [b[o:o + n] for b, o in zip(bufs, offs)]
        out = torch.empty(n + 8, dtype=dt, device=dev)[offs[k]:offs[k] + n]
        rc = lib.kf_bucket_reduce(_lib.ptr_array([t.data_ptr() for t in ins]), k, out.data_ptr(), n,
                                  codes[dt], 0, s)
        assert rc == 0, lib.kf_last_error()
        if dt == torch.bfloat16:
            acc = ins[0].float()
            for t in ins[1:]:
                acc = acc + t.float()
            want = acc.to(torch.bfloat16)
        else:
            want = ins[0].clone()
            for t in ins[1:]:
                want = want + t
        torch.cuda.synchronize()
        ok = torch.equal(out.view(torch.int16) if dt == torch.bfloat16 else out,
                         want.view(torch.int16) if dt == torch.bfloat16 else want)
        runs += 1
        serial_runs += (n * esz + 16383) // 16384 >= 2048
        if not ok:
            bad.append({"it": it, "k": k, "n": n, "dtype": str(dt), "offs": offs})
    print(json.dumps({"launches": runs, "large_grid_launches": serial_runs, "mismatches": len(bad),
                      "first": bad[:3]}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
