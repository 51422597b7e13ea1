"""bench.py's N > 1 code path, rehearsed on one GPU: two ranks under
torch.distributed.run on cuda:0 over gloo (RCCL refuses two ranks on one GPU,
so the native exchange is skipped by design and the torch path is primary).
Checks the driver's contract (exit 0, exactly one JSON line on stdout, the
whole-job value) and that the peer-to-peer sub-benchmarks, which run in one
child process per rank, come back into the line."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_n2_rehearsal_with_p2p_children():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--device-index", "0", "--steps", "3", "--warmup", "1", "--elems", str(4 << 20),
           "--extras", "c4_torch,c3_p2p,c5_p2p", "--extras-timeout", "100"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "weak"
    assert "error" not in d["c4_torch"], d["c4_torch"]
    for k in ("c3_p2p", "c5_p2p"):
        assert "error" not in d[k], d[k]
        assert d[k]["ms_per_step"] > 0
    assert d["p2p_children"]["all_ok"] is True
