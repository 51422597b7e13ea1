"""A plain C program built against include/kungfu_amd.h and linked with
-lkungfu_amd (tests/c/test_dropin.c): the drop-in works for C callers, as the
reference's C++ unit tests use it (tests/cpp/unit/test_kungfu.cpp:3-20)."""
import os
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.fixture(scope="module")
def binary(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("c") / "test_dropin")
    lib = os.path.join(ROOT, "kungfu_amd")
    subprocess.run(["gcc", "-Wall", "-Wextra", "-Werror", "-std=c99",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "test_dropin.c"),
                    "-L", lib, "-lkungfu_amd", "-Wl,-rpath," + lib, "-o", out],
                   check=True)
    return out


def test_c_consumer_builds_and_type_sizes(binary):
    r = subprocess.run([binary], capture_output=True, text=True, timeout=300)
    assert r.returncode in (0, 77), r.stderr  # 77: no device, host checks passed


@pytest.mark.gpu
def test_c_consumer_on_gpu(binary):
    r = subprocess.run([binary], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


@pytest.fixture(scope="module")
def exchange_binary(tmp_path_factory):
    """tests/c/test_exchange.cpp: a C++ host of kf_exchange_* through the C
    ABI alone (the reference's C++ side, gpu_collective.cpp / scheduler.cpp)."""
    out = str(tmp_path_factory.mktemp("cx") / "test_exchange")
    lib = os.path.join(ROOT, "kungfu_amd")
    tl = os.path.join(ROOT, "tests", "c")
    if not os.path.exists(os.path.join(tl, "libkf_testing.so")):
        subprocess.run(["make", "-s", "-C", tl], check=True)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", os.path.join(ROOT, "include"), "-I", tl, "-I", "/opt/rocm/include",
                    os.path.join(ROOT, "tests", "c", "test_exchange.cpp"),
                    "-L", lib, "-lkungfu_amd", "-Wl,-rpath," + lib,
                    "-L", tl, "-lkf_testing", "-Wl,-rpath," + tl,
                    "-L", "/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib",
                    "-lpthread", "-o", out], check=True)
    return out


def test_cpp_exchange_host_builds(exchange_binary):
    r = subprocess.run([exchange_binary], capture_output=True, text=True, timeout=300)
    assert r.returncode in (0, 77), r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_exchange_host_on_gpu(exchange_binary):
    r = subprocess.run([exchange_binary], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "exchange ok" in r.stdout


@pytest.fixture(scope="module")
def peer_binary(tmp_path_factory):
    """tests/c/test_peer.cpp: the reference's own C++ collective tests over
    include/kungfu_amd.hpp (the Peer facade on the C ABI)."""
    out = str(tmp_path_factory.mktemp("cp") / "test_peer")
    lib = os.path.join(ROOT, "kungfu_amd")
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    os.path.join(ROOT, "tests", "c", "test_peer.cpp"),
                    "-L", lib, "-lkungfu_amd", "-Wl,-rpath," + lib,
                    "-L", "/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib",
                    "-lpthread", "-o", out], check=True)
    return out


def test_cpp_peer_one_peer(peer_binary):
    # test_operations.cpp:3-26 with a single peer: no reduce, no GPU needed
    r = subprocess.run([peer_binary], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "peer ok" in r.stdout


def _peers(binary, np_, mode):
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        ps = [subprocess.Popen([binary, str(r), str(np_), d] + ([mode] if mode else []),
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
              for r in range(np_)]
        try:
            outs = [p.communicate(timeout=90) for p in ps]
        except subprocess.TimeoutExpired:
            for p in ps:
                p.kill()
            outs = [p.communicate() for p in ps]
            raise AssertionError("peers hung: %r" % (outs,))
    for p, (o, e) in zip(ps, outs):
        assert p.returncode == 0, o + e


@pytest.mark.gpu
@pytest.mark.parametrize("np_", [2, 3, 4])
@pytest.mark.parametrize("mode", ["", "dev"])
def test_cpp_peer_fake_agent(peer_binary, np_, mode):
    # fake_agent.cpp:15-44: iota summed over np peers == i * np, host buffers
    # (the drop-in's HIP fold) and HBM buffers (the device session)
    _peers(peer_binary, np_, mode)


@pytest.fixture(scope="module")
def hier_binary(tmp_path_factory):
    """tests/c/test_hier.cpp: the hierarchical all-reduce (kf_hier_all_reduce,
    kf_exchange_create_local, kf_session_info) from a C++ host, the C ABI
    alone: device-mode sessions across emulated hosts, the test library's
    loopback inside a host."""
    out = str(tmp_path_factory.mktemp("ch") / "test_hier")
    lib = os.path.join(ROOT, "kungfu_amd")
    tl = os.path.join(ROOT, "tests", "c")
    if not os.path.exists(os.path.join(tl, "libkf_testing.so")):
        subprocess.run(["make", "-s", "-C", tl], check=True)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", os.path.join(ROOT, "include"), "-I", tl, "-I", "/opt/rocm/include",
                    os.path.join(tl, "test_hier.cpp"),
                    "-L", lib, "-lkungfu_amd", "-Wl,-rpath," + lib,
                    "-L", tl, "-lkf_testing", "-Wl,-rpath," + tl,
                    "-L", "/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib",
                    "-lpthread", "-o", out], check=True)
    return out


def _hier_args():
    """test_hier's base port: every TCP address its three layouts bind
    (main(): base + rank, base + 10 + rank, base + 20 + rank on 127.0.0.1 /
    127.0.0.2) bindable now (tests/ports.py)."""
    import sys
    import tempfile
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from ports import draw_block

    def addrs(b):
        out = []
        for off, hosts in ((0, [[0, 1], [2, 3]]), (10, [[0, 1], [2]]), (20, [[0], [1]])):
            for h, ranks in enumerate(hosts):
                out += [("127.0.0.%d" % (h + 1), b + off + g) for g in ranks]
        return out
    return [str(draw_block(addrs)), tempfile.mkdtemp(prefix="kfh")]


def test_cpp_hier_host_builds(hier_binary):
    r = subprocess.run([hier_binary] + _hier_args(), capture_output=True, text=True, timeout=300)
    assert r.returncode in (0, 77), r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_hier_all_reduce_on_gpu(hier_binary):
    """2 emulated hosts x 2 ranks (sharded: local reduce-scatter or all-to-all
    fold -> cross-host session all-reduce of the shard -> / np -> local
    all-gather), 2 + 1 ranks (the reference's masters path) and 2 x 1 with
    kf_exchange_create_local: bit-exact against each host's rank-order fold
    combined across the hosts, / np."""
    r = subprocess.run([hier_binary] + _hier_args(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "hier ok" in r.stdout


@pytest.fixture(scope="module")
def session_async_binary(tmp_path_factory):
    """tests/c/test_session_async.cpp: host-mode sessions as threads of one C++
    process, async all-reduces started in a different order on every rank."""
    out = str(tmp_path_factory.mktemp("cs") / "test_session_async")
    lib = os.path.join(ROOT, "kungfu_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "test_session_async.cpp"),
                    "-L", lib, "-lkungfu_amd", "-Wl,-rpath," + lib, "-lpthread", "-o", out],
                   check=True)
    return out


@pytest.mark.parametrize("np_", [2, 3, 4])
def test_c_session_async_any_order(session_async_binary, tmp_path, np_):
    r = subprocess.run([session_async_binary, str(np_), "2", str(tmp_path)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("np_", [2, 3, 4])
def test_c_session_dead_peer_fails_calls(session_async_binary, tmp_path, np_):
    """The last rank destroys its session once every session is up; the
    others' async all-reduces must fail within 30 s (C++ host, threads)."""
    r = subprocess.run([session_async_binary, str(np_), "1", str(tmp_path), "dead"],
                       capture_output=True, text=True, timeout=90)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr
