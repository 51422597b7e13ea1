"""Test helper: the exchange's multi-rank logic on ONE GPU through the
test-only transports of tests/c/libkf_testing.so (tests/c/kf_testing.h),
plugged into the product library by kf_exchange_create_transport. Nothing
under kungfu_amd/ loads this library."""
import ctypes
import os
import subprocess
import threading
import traceback

from kungfu_amd.exchange import NativeExchange  # bound now: a test may stub the module's name

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "c", "libkf_testing.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        from kungfu_amd import _lib as kl
        kl.load()  # the product library first (the test library links it)
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-s", "-C", os.path.join(HERE, "c")], check=True)
        lib = ctypes.CDLL(LIB_PATH)
        lib.kf_loopback_create.argtypes = [ctypes.c_int]
        lib.kf_loopback_create.restype = ctypes.c_void_p
        lib.kf_loopback_destroy.argtypes = [ctypes.c_void_p]
        lib.kf_loopback_destroy.restype = None
        lib.kf_loopback_fail_at.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        lib.kf_loopback_fail_at.restype = None
        lib.kf_exchange_create_loopback.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        lib.kf_exchange_create_loopback.restype = ctypes.c_void_p
        lib.kf_exchange_create_rccl1.argtypes = [ctypes.c_int]
        lib.kf_exchange_create_rccl1.restype = ctypes.c_void_p
        lib.kf_testing_last_error.argtypes = []
        lib.kf_testing_last_error.restype = ctypes.c_char_p
        lib.kf_exchange_create_ipc.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int]
        lib.kf_exchange_create_ipc.restype = ctypes.c_void_p
        lib.kf_ipc_last_error.argtypes = []
        lib.kf_ipc_last_error.restype = ctypes.c_char_p
        _lib = lib
    return _lib


class LoopbackGroup:
    """kf_loopback_create: `world` ranks as threads of one process on one GPU."""

    def __init__(self, world):
        self.world = world
        self.lib = load()
        self._h = self.lib.kf_loopback_create(world)
        assert self._h, "kf_loopback_create(%d)" % world

    def exchange(self, rank, algo="auto", device=0):
        h = self.lib.kf_exchange_create_loopback(self._h, rank, device)
        assert h, self.lib.kf_testing_last_error().decode()
        return NativeExchange.from_handle(h, algo)

    def fail_at(self, call):
        """kf_loopback_fail_at: every rank's collective call #call fails."""
        self.lib.kf_loopback_fail_at(self._h, int(call))

    def close(self):
        if self._h:
            self.lib.kf_loopback_destroy(self._h)
            self._h = None


def rccl1_exchange(algo="auto", device=0):
    """A one-rank librccl communicator bound through the transport table: the
    exchange calls librccl's own entry points instead of the world-1 copy."""
    lib = load()
    h = lib.kf_exchange_create_rccl1(device)
    assert h, lib.kf_testing_last_error().decode()
    return NativeExchange.from_handle(h, algo)


def ipc_exchange(name, rank, world, algo="auto", device=0, timeout_s=120.0):
    """kf_exchange_create_ipc: this PROCESS as `rank` of `world` processes on
    one device, the exchange's collectives moved through HIP-IPC-mapped
    staging buffers and a shared-memory rendezvous named `name` (every rank
    passes the same "/name"). Collective: returns once every rank joined."""
    lib = load()
    h = lib.kf_exchange_create_ipc(name.encode(), int(rank), int(world), int(device),
                                   int(timeout_s * 1000))
    assert h, lib.kf_ipc_last_error().decode()
    return NativeExchange.from_handle(h, algo)


def loop_ranks(world, body, timeout=300, group=None):
    """Run body(rank, ex) on `world` threads, each with its own exchange of
    one loopback group (`group`, or a new one); re-raise the first failure."""
    import torch
    g = group if group is not None else LoopbackGroup(world)
    errs = []

    def run(r):
        try:
            torch.cuda.set_device(0)
            ex = g.exchange(r)
            body(r, ex)
            torch.cuda.synchronize()
            ex.close()
        except BaseException:  # pytest.raises failures are BaseException
            errs.append("rank %d: %s" % (r, traceback.format_exc()))

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=timeout)
    alive = any(t.is_alive() for t in ts)
    if not alive:
        g.close()
    assert not errs, "\n".join(errs)
    assert not alive, "a rank did not finish"
