"""The exchange's phase-2 kernels at BASELINE's 8-GPU shapes (bench.py
exchange_phase2: C5's all-to-all fold, C4's and C3's shard /np), on one GPU,
as one JSON line — the program `rocprofv3 --kernel-trace --stats` wraps for
profiles/r03/.

    python tools/phase2_rates.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from kungfu_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(11)
    print(json.dumps(bench.exchange_phase2(lib, dev, g)), flush=True)


if __name__ == "__main__":
    main()
