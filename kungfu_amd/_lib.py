"""ctypes binding of libkungfu_amd.so (include/kungfu_amd.h).

The shared library is built in-tree by ``kungfu_amd/csrc/Makefile``
(``__graft_entry__.build()``). There is deliberately no fallback: if the
library is missing, or the process has no GPU, the product path raises.
"""
import atexit
import ctypes
import importlib.util
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkungfu_amd.so")

# Every symbol include/kungfu_amd.h declares (checked by tests/test_capi.py).
EXPORTED = (
    "std_transform_2",
    "kungfu_type_size",
    "float16_sum",
    "kf_bucket_reduce",
    "kf_bucket_reduce_avg",
    "kf_bucket_reduce_peers",
    "kf_bucket_div",
    "kf_sma_blend",
    "kf_device_count",
    "kf_version",
    "kf_last_error",
    "kf_shutdown",
    "kf_transform2_host",
    "kf_set_geometry",
    "kf_host_register",
    "kf_host_unregister",
    "kf_rch_client_handshake",
    "kf_rch_server_handshake",
    "kf_rch_send",
    "kf_rch_recv_header",
    "kf_rch_recv_body",
    "kf_ingest_create",
    "kf_ingest_destroy",
    "kf_ingest_recv_onto",
    "kf_ingest_recv_into",
    "kf_ingest_recv_onto_pieces",
    "kf_ingest_recv_into_pieces",
    "kf_ingest_send_from_device",
    "kf_ingest_fold_host",
    "kf_ingest_copy_host",
    "kf_ingest_sync",
    "kf_ingest_last_error",
    "kf_session_create",
    "kf_session_create_peers",
    "kf_session_set_strategy",
    "kf_session_set_host_reduce",
    "kf_session_all_reduce",
    "kf_session_all_reduce_async",
    "kf_session_subset_all_reduce",
    "kf_session_reduce",
    "kf_session_broadcast",
    "kf_session_wait_all",
    "kf_session_barrier",
    "kf_session_destroy",
    "kf_session_last_error",
    "kf_ipc_export",
    "kf_ipc_import",
    "kf_ipc_close",
    "kf_gather_segments",
    "kf_copy_segments",
    "kf_signal_alloc",
    "kf_signal_free",
    "kf_peer_barrier",
    "kf_p2p_last_error",
    "kf_bucket_reduce_batch",
    "kf_exchange_unique_id",
    "kf_exchange_share_id",
    "kf_exchange_create",
    "kf_exchange_create_timeout",
    "kf_exchange_create_session",
    "kf_exchange_all_reduce",
    "kf_exchange_all_reduce_batch",
    "kf_set_occupancy",
    "kf_sma_blend_batch",
    "kf_exchange_sma_batch",
    "kf_exchange_set_pipeline",
    "kf_exchange_set_timing",
    "kf_exchange_phase_times",
    "kf_exchange_begin_step",
    "kf_exchange_start",
    "kf_exchange_wait_all",
    "kf_exchange_check",
    "kf_exchange_info",
    "kf_exchange_transport_info",
    "kf_exchange_destroy",
    "kf_exchange_last_error",
    "kf_exchange_all_reduce_named",
    "kf_exchange_wait_named",
    "kf_exchange_create_transport",
    "kf_exchange_split",
    "kf_session_info",
    "kf_exchange_create_local",
    "kf_hier_all_reduce",
)

STATUS = {
    0: "KF_OK",
    1: "KF_ERR_DTYPE",
    2: "KF_ERR_OP",
    3: "KF_ERR_ARG",
    4: "KF_ERR_HIP",
    5: "KF_ERR_NO_DEVICE",
    6: "KF_ERR_IO",
    7: "KF_ERR_PROTO",
    8: "KF_ERR_TIMEOUT",
    9: "KF_ERR_RCCL",
}

MAX_INPUTS = 16

# kf_done_fn: void (*)(int status, void *arg)
DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_void_p)

_lib = None


class KungFuAMDError(RuntimeError):
    pass


def _preload_hip_runtime():
    """One HIP runtime per process: torch ships its own libamdhip64 (SONAME
    libamdhip64.so.7, like /opt/rocm's), which its libraries find by RPATH.
    Loading torch's file first makes the library's libamdhip64.so.7 resolve
    to it, and a later `import torch` finds it already mapped — without the
    2 s of importing torch in processes that never touch a tensor (host-mode
    peers). Without torch, /opt/rocm's runtime is used."""
    if "torch" in sys.modules:
        return
    spec = importlib.util.find_spec("torch")
    for d in (spec.submodule_search_locations or []) if spec else []:
        path = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(path):
            ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            return


def load():
    """Load (once) and return the ctypes handle of libkungfu_amd.so."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KungFuAMDError(
            "libkungfu_amd.so not built (%s); run __graft_entry__.build() or "
            "make -C kungfu_amd/csrc" % LIB_PATH)
    _preload_hip_runtime()
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    c_void_p, c_size_t, c_int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    lib.std_transform_2.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int]
    lib.std_transform_2.restype = None
    lib.kungfu_type_size.argtypes = [c_int]
    lib.kungfu_type_size.restype = ctypes.c_uint32
    lib.float16_sum.argtypes = [c_void_p, c_void_p, c_void_p, c_int]
    lib.float16_sum.restype = None
    lib.kf_bucket_reduce.argtypes = [ctypes.POINTER(c_void_p), c_int, c_void_p,
                                     c_size_t, c_int, c_int, c_void_p]
    lib.kf_bucket_reduce.restype = c_int
    lib.kf_bucket_reduce_avg.argtypes = [ctypes.POINTER(c_void_p), c_int, c_void_p,
                                         c_size_t, c_int, c_int, c_void_p]
    lib.kf_bucket_reduce_avg.restype = c_int
    lib.kf_bucket_reduce_peers.argtypes = [ctypes.POINTER(c_void_p), c_int, c_void_p,
                                           c_size_t, c_int, c_int, c_int, c_void_p]
    lib.kf_bucket_reduce_peers.restype = c_int
    lib.kf_bucket_div.argtypes = [c_void_p, c_size_t, c_int, c_int, c_void_p]
    lib.kf_bucket_div.restype = c_int
    lib.kf_sma_blend.argtypes = [c_void_p, c_void_p, c_size_t, c_int, c_int,
                                 ctypes.c_double, c_void_p]
    lib.kf_sma_blend.restype = c_int
    lib.kf_device_count.argtypes = []
    lib.kf_device_count.restype = c_int
    lib.kf_version.argtypes = []
    lib.kf_version.restype = ctypes.c_char_p
    lib.kf_last_error.argtypes = []
    lib.kf_last_error.restype = ctypes.c_char_p
    lib.kf_shutdown.argtypes = []
    lib.kf_shutdown.restype = c_int
    lib.kf_transform2_host.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t,
                                       c_int, c_int]
    lib.kf_transform2_host.restype = c_int
    lib.kf_set_geometry.argtypes = [c_int, c_int, c_int, c_int]
    lib.kf_sma_blend_batch.argtypes = [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p),
                                       ctypes.POINTER(c_size_t), c_int, c_int, c_int,
                                       ctypes.c_double, c_void_p]
    lib.kf_sma_blend_batch.restype = c_int
    lib.kf_set_occupancy.argtypes = [c_int, c_int]
    lib.kf_set_occupancy.restype = c_int
    lib.kf_set_geometry.restype = c_int
    lib.kf_host_register.argtypes = [c_void_p, c_size_t]
    lib.kf_host_register.restype = c_int
    lib.kf_host_unregister.argtypes = [c_void_p]
    lib.kf_host_unregister.restype = c_int
    u16, u32 = ctypes.c_uint16, ctypes.c_uint32
    lib.kf_rch_client_handshake.argtypes = [c_int, u16, u16, u32, u32]
    lib.kf_rch_client_handshake.restype = c_int
    lib.kf_rch_server_handshake.argtypes = [c_int, u32, ctypes.POINTER(u16),
                                            ctypes.POINTER(u16), ctypes.POINTER(u32)]
    lib.kf_rch_server_handshake.restype = c_int
    lib.kf_rch_send.argtypes = [c_int, ctypes.c_char_p, u32, c_void_p, u32]
    lib.kf_rch_send.restype = c_int
    lib.kf_rch_recv_header.argtypes = [c_int, ctypes.c_char_p, u32, ctypes.POINTER(u32),
                                       ctypes.POINTER(u32)]
    lib.kf_rch_recv_header.restype = c_int
    lib.kf_rch_recv_body.argtypes = [c_int, c_void_p, u32]
    lib.kf_rch_recv_body.restype = c_int
    lib.kf_ingest_create.argtypes = [c_size_t, c_int]
    lib.kf_ingest_create.restype = c_void_p
    lib.kf_ingest_destroy.argtypes = [c_void_p]
    lib.kf_ingest_destroy.restype = None
    lib.kf_ingest_recv_onto.argtypes = [c_void_p, c_int, u32, c_void_p, c_void_p,
                                        c_size_t, c_int, c_int, c_void_p]
    lib.kf_ingest_recv_onto.restype = c_int
    lib.kf_ingest_recv_into.argtypes = [c_void_p, c_int, u32, c_void_p, c_void_p]
    lib.kf_ingest_recv_into.restype = c_int
    lib.kf_ingest_send_from_device.argtypes = [c_void_p, c_int, ctypes.c_char_p, u32,
                                               c_void_p, c_size_t, c_void_p]
    lib.kf_ingest_send_from_device.restype = c_int
    lib.kf_ingest_sync.argtypes = [c_void_p]
    lib.kf_ingest_sync.restype = c_int
    lib.kf_ingest_last_error.argtypes = []
    lib.kf_ingest_last_error.restype = ctypes.c_char_p
    lib.kf_session_create.argtypes = [c_int, c_int, ctypes.c_char_p, u32, c_int]
    lib.kf_session_create.restype = c_void_p
    lib.kf_session_create_peers.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                            u32, c_int]
    lib.kf_session_create_peers.restype = c_void_p
    lib.kf_session_set_strategy.argtypes = [c_void_p, c_int, c_int]
    lib.kf_session_set_strategy.restype = c_int
    lib.kf_ingest_fold_host.argtypes = [c_void_p, c_void_p, u32, c_void_p, c_void_p,
                                        c_size_t, c_int, c_int, c_void_p]
    lib.kf_ingest_fold_host.restype = c_int
    lib.kf_ingest_copy_host.argtypes = [c_void_p, c_void_p, u32, c_void_p, c_void_p]
    lib.kf_ingest_copy_host.restype = c_int
    lib.kf_session_set_host_reduce.argtypes = [c_void_p, c_void_p]
    lib.kf_session_set_host_reduce.restype = c_int
    lib.kf_session_all_reduce.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_int,
                                          c_int, ctypes.c_char_p, c_void_p]
    lib.kf_session_all_reduce.restype = c_int
    lib.kf_session_destroy.argtypes = [c_void_p]
    lib.kf_session_destroy.restype = None
    lib.kf_session_all_reduce_async.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_int,
                                                c_int, ctypes.c_char_p, c_void_p, DONE_FN,
                                                c_void_p]
    lib.kf_session_all_reduce_async.restype = c_int
    lib.kf_session_subset_all_reduce.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_int,
                                                 c_int, ctypes.POINTER(ctypes.c_int32),
                                                 ctypes.c_char_p, c_void_p]
    lib.kf_session_subset_all_reduce.restype = c_int
    lib.kf_session_reduce.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int,
                                      ctypes.c_char_p, c_void_p]
    lib.kf_session_reduce.restype = c_int
    lib.kf_session_broadcast.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_int,
                                         ctypes.c_char_p, c_void_p]
    lib.kf_session_broadcast.restype = c_int
    lib.kf_session_wait_all.argtypes = [c_void_p]
    lib.kf_session_wait_all.restype = c_int
    lib.kf_session_barrier.argtypes = [c_void_p]
    lib.kf_session_barrier.restype = c_int
    lib.kf_session_last_error.argtypes = []
    lib.kf_session_last_error.restype = ctypes.c_char_p
    lib.kf_ipc_export.argtypes = [c_void_p, c_void_p, ctypes.POINTER(c_size_t)]
    lib.kf_ipc_export.restype = c_int
    lib.kf_ipc_import.argtypes = [c_void_p, ctypes.POINTER(c_void_p)]
    lib.kf_ipc_import.restype = c_int
    lib.kf_ipc_close.argtypes = [c_void_p]
    lib.kf_ipc_close.restype = c_int
    lib.kf_gather_segments.argtypes = [c_void_p, ctypes.POINTER(c_void_p),
                                       ctypes.POINTER(c_size_t), ctypes.POINTER(c_size_t),
                                       c_int, c_void_p]
    lib.kf_gather_segments.restype = c_int
    lib.kf_copy_segments.argtypes = [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p),
                                     ctypes.POINTER(c_size_t), c_int, c_void_p]
    lib.kf_copy_segments.restype = c_int
    lib.kf_signal_alloc.argtypes = [c_size_t, c_int, ctypes.POINTER(c_void_p)]
    lib.kf_signal_alloc.restype = c_int
    lib.kf_signal_free.argtypes = [c_void_p, c_int]
    lib.kf_signal_free.restype = c_int
    lib.kf_peer_barrier.argtypes = [ctypes.POINTER(c_void_p), c_int, c_int, ctypes.c_uint64,
                                    ctypes.c_uint32, c_void_p, c_void_p]
    lib.kf_peer_barrier.restype = c_int
    lib.kf_p2p_last_error.argtypes = []
    lib.kf_p2p_last_error.restype = ctypes.c_char_p
    P = ctypes.POINTER
    lib.kf_bucket_reduce_batch.argtypes = [P(c_void_p), c_int, P(c_void_p), P(c_size_t), c_int,
                                           c_int, c_int, c_int, c_void_p]
    lib.kf_bucket_reduce_batch.restype = c_int
    lib.kf_exchange_unique_id.argtypes = [c_void_p]
    lib.kf_exchange_unique_id.restype = c_int
    lib.kf_exchange_share_id.argtypes = [c_void_p, c_void_p]
    lib.kf_exchange_share_id.restype = c_int
    lib.kf_exchange_create.argtypes = [c_void_p, c_int, c_int, c_int]
    lib.kf_exchange_create.restype = c_void_p
    lib.kf_exchange_create_timeout.argtypes = [c_void_p, c_int, c_int, c_int, c_int]
    lib.kf_exchange_create_timeout.restype = c_void_p
    lib.kf_exchange_create_session.argtypes = [c_void_p, c_int, c_int, c_int]
    lib.kf_exchange_create_session.restype = c_void_p
    lib.kf_exchange_all_reduce.argtypes = [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int,
                                           c_int, c_int, c_void_p]
    lib.kf_exchange_all_reduce.restype = c_int
    lib.kf_exchange_all_reduce_batch.argtypes = [c_void_p, P(c_void_p), P(c_void_p), P(c_size_t),
                                                 c_int, c_int, c_int, c_int, c_int, c_void_p]
    lib.kf_exchange_all_reduce_batch.restype = c_int
    lib.kf_exchange_sma_batch.argtypes = [c_void_p, P(c_void_p), P(c_void_p), P(c_size_t), c_int,
                                          c_int, ctypes.c_double, c_int, c_void_p]
    lib.kf_exchange_sma_batch.restype = c_int
    lib.kf_exchange_begin_step.argtypes = [c_void_p, P(ctypes.c_char_p), c_int, c_int]
    lib.kf_exchange_begin_step.restype = c_int
    lib.kf_exchange_start.argtypes = [c_void_p, ctypes.c_char_p, c_void_p, c_void_p, c_size_t,
                                      c_int, c_int, c_int, c_int, c_void_p, DONE_FN, c_void_p]
    lib.kf_exchange_start.restype = c_int
    lib.kf_exchange_wait_all.argtypes = [c_void_p, P(ctypes.c_int32)]
    lib.kf_exchange_wait_all.restype = c_int
    lib.kf_exchange_check.argtypes = [c_void_p]
    lib.kf_exchange_check.restype = c_int
    lib.kf_exchange_set_pipeline.argtypes = [c_void_p, c_int]
    lib.kf_exchange_set_pipeline.restype = c_int
    lib.kf_exchange_set_timing.argtypes = [c_void_p, c_int]
    lib.kf_exchange_set_timing.restype = c_int
    lib.kf_exchange_phase_times.argtypes = [c_void_p, P(ctypes.c_double), P(ctypes.c_int64),
                                            P(ctypes.c_int64)]
    lib.kf_exchange_phase_times.restype = c_int
    lib.kf_exchange_info.argtypes = [c_void_p, P(c_int), P(c_int), P(c_int)]
    lib.kf_exchange_info.restype = c_int
    lib.kf_exchange_transport_info.argtypes = [c_void_p, P(c_int), P(c_int)]
    lib.kf_exchange_transport_info.restype = c_int
    lib.kf_exchange_destroy.argtypes = [c_void_p]
    lib.kf_exchange_destroy.restype = None
    lib.kf_exchange_last_error.argtypes = []
    lib.kf_exchange_last_error.restype = ctypes.c_char_p
    lib.kf_exchange_all_reduce_named.argtypes = [c_void_p, ctypes.c_char_p, c_void_p, c_void_p,
                                                 c_size_t, c_int, c_int, c_int, c_int, c_void_p,
                                                 DONE_FN, c_void_p]
    lib.kf_exchange_all_reduce_named.restype = c_int
    lib.kf_exchange_wait_named.argtypes = [c_void_p]
    lib.kf_exchange_wait_named.restype = c_int
    lib.kf_exchange_create_transport.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int]
    lib.kf_exchange_create_transport.restype = c_void_p
    lib.kf_exchange_split.argtypes = [c_void_p, c_int, c_int, P(c_int)]
    lib.kf_exchange_split.restype = c_void_p
    lib.kf_session_info.argtypes = [c_void_p, P(c_int), P(c_int), P(c_int), P(c_int), P(c_int)]
    lib.kf_session_info.restype = c_int
    lib.kf_exchange_create_local.argtypes = [c_void_p, c_int]
    lib.kf_exchange_create_local.restype = c_void_p
    lib.kf_hier_all_reduce.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int,
                                       c_int, c_int, c_int, ctypes.c_char_p, c_void_p]
    lib.kf_hier_all_reduce.restype = c_int
    _lib = lib
    # HIP resources go back while the runtime is alive, before the C exit
    # handlers run (include/kungfu_amd.h kf_shutdown)
    atexit.register(lib.kf_shutdown)
    return lib


def check(rc, what, source=None):
    """Raise KungFuAMDError for a non-zero status. The detail is the calling
    module's own last error first (`source`: e.g. "session" for a
    kf_session_* call), so a stale message another module left on this thread
    never stands in for it."""
    if rc != 0:
        lib = load()
        order = ["exchange", "session", "", "ingest", "p2p"]
        if source in order:
            order.remove(source)
            order.insert(0, source)
        detail = ""
        for m in order:
            detail = getattr(lib, "kf_%s_last_error" % m if m else "kf_last_error")().decode()
            if detail:
                break
        raise KungFuAMDError("%s failed: %s (%s)" % (what, STATUS.get(rc, rc), detail))


def ptr_array(ptrs):
    arr = (ctypes.c_void_p * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr
