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
           "--extras", "c4_torch,c5_torch,c3_p2p,c5_p2p", "--extras-timeout", "100"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "weak"
    assert "error" not in d["c4_torch"], d["c4_torch"]
    # the N > 1 line says which exchange ran and splits C4's and C5's steps
    # into phases too; same-GPU gloo has no RCCL world
    c = d["collective"]
    assert c["exchange_kind"] == "torch.distributed" and c["rccl_world"] is None, c
    for k in ("c4_torch", "c5_torch"):
        ph = d[k]["phase_us"]
        assert ph and ph["step_us"] > 0 and ph["sum"] > 0, (k, ph)
    for k in ("c3_p2p", "c5_p2p"):
        assert "error" not in d[k], d[k]
        assert d[k]["ms_per_step"] > 0
    assert d["p2p_children"]["all_ok"] is True


def test_bench_gpus2_starts_its_own_ranks():
    """`bench.py --gpus 2` with no launcher: bench.py starts the two ranks
    itself (torch.distributed.run as a child) and relays rank 0's line."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--device-index", "0", "--steps", "3", "--warmup", "1", "--elems", str(4 << 20),
           "--extras", ""]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and "collective" in d and d["value"] > 0, d
    # which exchange ran and what RCCL says about it (same-GPU gloo: no RCCL)
    c = d["collective"]
    assert c["exchange_kind"] == "torch.distributed" and c["rccl_world"] is None, c
    assert "share a GPU" in c["why_not_native"], c
    # the per-phase split of the timed step (RS / epilogue / AG)
    ph = d["collective"]["phase_us"]
    total = sum(v for k, v in ph.items() if k in ("reduce_scatter", "epilogue", "all_gather"))
    assert abs(total - d["ms_per_step"] * 1e3) <= 0.1 * d["ms_per_step"] * 1e3, (ph, d["ms_per_step"])


_NATIVE_CHILD = r"""
import os, sys
sys.path[:0] = [%r, %r]
import torch
import torch.distributed as dist
import bench
from loopback import rccl1_exchange
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
bench._NATIVE["ex"] = rccl1_exchange("rs")
n = 16 << 20
x = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
res = {
    "c4": bench.bench_c4(1, 0, dev, 3, 1, exchange="native"),
    "c4_pipe": bench.bench_c4(1, 0, dev, 3, 1, exchange="native_pipe"),
    "c4_rs_avg": bench.bench_c4(1, 0, dev, 3, 1, exchange="native_rs_avg"),
    "c5": bench.bench_c5(1, 0, dev, 3, 1, exchange="native"),
    "c5_pipe": bench.bench_c5(1, 0, dev, 3, 1, exchange="native_pipe"),
    "c5_overlap": bench.bench_c5_overlap(1, 0, dev, 3, 1),
    "c4_overlap": bench.bench_c4_overlap(1, 0, dev, 3, 1),
    "c3_a2a": bench.bench_c3_native(1, 0, dev, 3, 1, n, x, "a2a", 64),
    "c3_fused": bench.bench_c3_native(1, 0, dev, 3, 1, n, x, "rs", 64, fused=True),
    "c3_pipe": bench.bench_c3_native(1, 0, dev, 3, 1, n, x, "rs", 64, pipe=True),
}
bad = {k: v for k, v in res.items() if "error" in v or not v.get("ms_per_step", 0) > 0}
bench._NATIVE.pop("ex").close()
dist.destroy_process_group()
print("NATIVE_SUB_OK" if not bad else "NATIVE_SUB_BAD %%r" %% bad)
"""


def test_bench_native_subbenchmarks_world1_rccl():
    """bench.py's native sub-benchmark bodies (c4, c5, c3_a2a, c3_fused, the
    pipelined c3/c4/c5 and C5 overlapped with compute) run end to end — parity check, timed loop — over a
    one-rank RCCL communicator bound through the test library's rccl1
    transport (librccl's collectives, no world-1 copy), so the code the
    driver's multi-GPU node runs first has run on real RCCL here."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    r = subprocess.run([sys.executable, "-c", _NATIVE_CHILD % (ROOT, os.path.join(ROOT, "tests"))],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0 and "NATIVE_SUB_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


_BRANCH_CHILD = r"""
import sys
sys.path[:0] = [%r, %r]
import bench
from kungfu_amd import exchange
from loopback import rccl1_exchange
# the primary exchange over librccl's own collectives (one rank, no world-1 copy)
exchange.NativeExchange = lambda *a, **kw: rccl1_exchange(kw.get("algo", "auto"))
exchange.NativeExchange.shared_id = staticmethod(lambda group=None: b"\0" * 128)
sys.argv = ["bench.py"] + %r
bench.main()
"""


def test_bench_exchange_branch_single_rank_rccl():
    """bench.py's whole N > 1 branch — the native exchange as the primary,
    its parity check, the timed C3 step, the agreed sub-benchmark loop and the
    JSON line — run by one rank on real RCCL (--rehearse-exchange, the
    primary's communicator bound through the test library's rccl1 transport,
    so librccl's collectives run): the primary must be the native exchange,
    not the fallback, and value is per GPU with value_aggregate beside it."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), RANK="0", LOCAL_RANK="0", WORLD_SIZE="1")
    extras = ("c4,c5,c5_pipe,c5_overlap,c4_overlap,c4_pipe,c4_rs_avg,c4_named,c3_pipe,c3_a2a,"
              "c3_fused,c4_torch,c5_torch")
    argv = ["--rehearse-exchange", "--steps", "3", "--warmup", "1", "--elems", str(4 << 20),
            "--extras", extras, "--extras-timeout", "200"]
    code = _BRANCH_CHILD % (ROOT, os.path.join(ROOT, "tests"), argv)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=260,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["collective"]["exchange"].startswith("native"), \
        json.dumps(d["collective"]) + r.stderr[-3000:]
    assert "native_exchange_error" not in d["collective"], d["collective"]
    assert d["value"] == d["collective"]["algbw_GiBps_per_gpu"]
    # the primary's schedule trial: every schedule parity-checked and timed
    trial = d["collective"]["schedule_trial_ms"]
    assert sorted(trial) == ["a2a", "fused", "grouped", "pipelined"], trial
    # the per-phase split of the timed step on the native exchange
    ph = d["collective"]["phase_us"]
    assert ph["timed_calls_per_step"] > 0 or ph.get("pipelined_calls_untimed"), ph
    assert all(v is not None and v > 0 for v in trial.values()), trial
    assert abs(d["value_aggregate"] - d["n_gpus"] * d["value"]) < 1e-2
    for k in extras.split(","):
        assert "error" not in d[k] and d[k]["ms_per_step"] > 0, (k, d[k])
    # the N > 1 line explains itself: the exchange kind, and the phase split of
    # C4 and C5 as well as C3's
    assert d["collective"]["exchange_kind"].startswith("native"), d["collective"]
    assert "rccl_world" in d["collective"] and "rccl_version" in d["collective"]
    for k in ("c4", "c5"):
        ph = d[k]["phase_us"]
        assert ph and ph["step_us"] > 0 and ph["sum"] > 0, (k, ph)


def test_rccl_report_on_real_rccl_world1():
    """kf_exchange_transport_info on a real one-rank RCCL communicator: the
    count is 1 and the version decodes (major.minor.patch)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    code = r"""
import sys
sys.path[:0] = [%r]
import torch
import bench
from kungfu_amd.exchange import NativeExchange
ex = NativeExchange(algo="rs", device=torch.device("cuda:0"), uid=NativeExchange.shared_id())
print("REPORT", bench._rccl_report(ex, 1, None))
ex.close()
""" % ROOT
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       cwd=ROOT, env=env)
    line = [l for l in r.stdout.splitlines() if l.startswith("REPORT")]
    assert r.returncode == 0 and line, r.stdout[-2000:] + r.stderr[-3000:]
    rep = eval(line[0][len("REPORT "):])
    assert rep["rccl_world"] == 1 and rep["exchange_kind"].startswith("native"), rep
    major = int(rep["rccl_version"].split(".")[0])
    assert major >= 2, rep


_IPC_EXTRAS = ("c4", "c5", "c5_pipe", "c4_pipe", "c4_rs_avg", "c3_pipe", "c4_named")


@pytest.mark.parametrize("world", [2, 4, pytest.param(
    8, marks=[pytest.mark.gpu_slow, pytest.mark.timeout(600)])])
def test_bench_native_branch_over_ipc_transport(world):
    """bench.py's NATIVE N > 1 branch with N ranks —
    the primary exchange's parity check and schedule trial, the timed C3 step
    with its phase windows, the agreed sub-benchmark loop, c4_named in its
    child process group, the line — run by N processes sharing cuda:0, the
    exchange's collectives moved by the test-only cross-process IPC transport
    (tests/c/kf_testing_ipc.hip through kf_exchange_create_transport) because
    RCCL refuses two ranks on one GPU. Every sub-benchmark must be parity-
    checked correct, the phases must account for the un-pipelined steps, and
    the line must say which transport ran (never an xGMI claim). World 8,
    the driver's BASELINE world size, is in the gpu_slow tier: eight
    processes' queues on one GPU are time-sliced, ~4 minutes a run
    (profiles/r06/bench_ipc_w8_r06f.json)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    # N processes' streams on one GPU: two hardware queues each, so the GPU
    # does not time-slice them (GPU_MAX_HW_QUEUES)
    env["GPU_MAX_HW_QUEUES"] = "2" if world <= 4 else "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(world), "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--dist-backend", "gloo",
           "--device-index", "0", "--test-transport", "ipc", "--steps", "3", "--warmup", "1",
           "--elems", str(4 << 20), "--extras", ",".join(_IPC_EXTRAS),
           "--extras-timeout", "150" if world <= 4 else "400"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240 if world <= 4 else 560,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    c = d["collective"]
    assert d["n_gpus"] == world and d["value"] > 0, d
    assert c["exchange_kind"] == "native (test transport)" and c["rccl_world"] is None, c
    assert "native_exchange_error" not in c and c["exchange"].startswith("native"), c
    assert c["correct"] is True, c
    assert sorted(c["schedule_trial_ms"]) == ["a2a", "fused", "grouped", "pipelined"], c
    why = "\n".join(l for l in r.stderr.splitlines() if "failed" in l)[-3000:]
    for k in _IPC_EXTRAS:
        assert "error" not in d[k] and d[k]["correct"] is True, (k, d[k], why)
        assert d[k]["ms_per_step"] > 0, (k, d[k])
    # the phase windows account for the un-pipelined timed steps: their sum
    # is the step minus the host's gaps between calls
    for ph in (c.get("phase_us"), d["c4"]["phase_us"], d["c5"]["phase_us"]):
        if ph is None or not ph["timed_calls_per_step"]:
            continue
        assert 0.3 * ph["step_us"] <= ph["sum"] <= 1.02 * ph["step_us"], ph
    # pipelined calls are counted, not split
    assert d["c5_pipe"]["phase_us"]["pipelined_calls_untimed"] > 0, d["c5_pipe"]
    assert d["c4_pipe"]["phase_us"]["pipelined_calls_untimed"] > 0, d["c4_pipe"]
    # rs_avg (ncclAvg) against rs on the same inputs, recorded with its transport
    par = d["c4_rs_avg"]["rs_avg_parity"]
    assert par["transport"] == "test transport (ipc)" and par["bit_exact_vs_rs"] is True, par
