"""bench.py's launch contract, checked without a GPU: a WORLD_SIZE that
disagrees with --gpus is an error (non-zero exit before anything touches the
GPU), and `--gpus N` with no launcher around it starts the N ranks itself
under torch.distributed.run (the reference's `kungfu-run -np N`,
srcs/go/kungfu/runner/flags.go:73) and relays their exit status."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.parametrize("gpus,world", [(2, "1"), (1, "2"), (8, "4")])
def test_world_size_mismatch_exits_nonzero(gpus, world):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--steps", "1"],
                       env=_env(WORLD_SIZE=world, RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr, r.stderr[-2000:]
    assert r.stdout.strip() == ""


def test_self_launch_starts_n_ranks_and_relays_status():
    """No GPU here: each of the 2 ranks the launcher starts fails at its
    first device call, so the parent must come back non-zero, having started
    torch.distributed.run with 2 ranks (its per-rank failure report names
    both local ranks)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check (the GPU variant is in test_bench_gpu.py)")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=_env(), capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode != 0
    assert "the 2 ranks ended with status" in r.stderr, r.stderr[-3000:]
    assert "(local_rank: 0)" in r.stderr and "(local_rank: 1)" in r.stderr, r.stderr[-3000:]


class _FakeNative:
    def __init__(self, count, ver):
        self.count, self.ver = count, ver

    def transport_info(self):
        return self.count, self.ver


def test_rccl_report_fails_loudly_on_a_short_communicator():
    """the N > 1 line names the exchange that ran and what
    RCCL reports (ncclCommCount, ncclGetVersion). A communicator that does not
    hold N ranks (each rank timing a world of its own) must end the run with
    an error, never print a number."""
    import bench
    with pytest.raises(SystemExit) as e:
        bench._rccl_report(_FakeNative(1, 22703), 8, None)
    assert "holds 1 ranks, not WORLD_SIZE 8" in str(e.value)
    rep = bench._rccl_report(_FakeNative(8, 22703), 8, None)
    assert rep == {"exchange_kind": "native C-ABI (kf_exchange)", "rccl_world": 8,
                   "rccl_version": "2.27.3", "rccl_version_code": 22703}
    # a host-provided transport is not RCCL: nothing to check
    assert bench._rccl_report(_FakeNative(-1, 0), 2, None)["rccl_world"] is None
    # the torch.distributed fallback says why
    rep = bench._rccl_report(None, 2, "not tried: ranks share a GPU (rehearsal)")
    assert rep["exchange_kind"] == "torch.distributed" and "share a GPU" in rep["why_not_native"]


def test_rccl_report_names_the_test_transport(monkeypatch):
    """--test-transport ipc (N processes on one GPU): the line says the
    exchange ran over the test transport and claims no RCCL world."""
    import bench
    monkeypatch.setitem(bench._OPTS, "test_transport", "ipc")
    rep = bench._rccl_report(_FakeNative(-1, 0), 2, None)
    assert rep["exchange_kind"] == "native (test transport)" and rep["rccl_world"] is None
    assert "not xGMI" in rep["transport"]


def test_rs_avg_verdict_records_the_transport(monkeypatch):
    """at N > 1, c4_rs_avg carries rs_avg_parity — ncclAvg
    against sum-then-/np on the same buckets, bit for bit, with the transport
    that produced it (the first real RCCL world's verdict lands here)."""
    import torch
    import bench
    a = [torch.tensor([1.0, 2.0, 3.0, 9.0]), torch.tensor([4.0, 5.0])]
    b = [torch.tensor([1.0, 2.0, 3.5, 7.0]), torch.tensor([4.0, 5.0])]
    v = bench._rs_avg_verdict(a, b, [3, 2], 8)  # element 3 of bucket 0 is padding
    assert v["bit_exact_vs_rs"] is False and v["mismatched_elements"] == 1
    assert v["elements"] == 5 and v["transport"] == "RCCL, 8 ranks"
    assert bench._rs_avg_verdict(a, a, [4, 2], 2)["bit_exact_vs_rs"] is True
    monkeypatch.setitem(bench._OPTS, "test_transport", "ipc")
    assert bench._rs_avg_verdict(a, a, [4, 2], 2)["transport"] == "test transport (ipc)"
