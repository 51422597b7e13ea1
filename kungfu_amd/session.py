"""Single-host KungFu session over the reference's rchannel wire format, with
the reduce on the GPU.

Mirrors ``Session.AllReduce`` (srcs/go/kungfu/session/allreduce.go:10-12 ->
session.go:231-326) for the strategy KungFu uses when every peer is on one
host: AUTO selects STAR there (strategy.go:196-205) and BINARY_TREE_STAR
degenerates to the same star around rank 0 (topology.go:76-101). Per bucket:

* split into ceil(bytes / 1 MiB) chunks by EvenPartition, named
  ``part::<name>[b:e]`` (session.go:301-326, workspace.go:18-25);
* reduce graph: every peer sends its chunk to rank 0 (sendOnto, NoFlag);
  rank 0 folds the chunks **in arrival order** (select on the peer sockets),
  ``RecvBuf = effective o peer`` (recvOnto, session.go:255-264);
* bcast graph: rank 0 sends the result to every peer with WaitRecvBuf and the
  peers read it straight into RecvBuf (recvInto, session.go:266-270,
  handler/collective.go:43-61).

Peers are separate processes connected by unix sockets (same-host peers use
unix sockets in the reference too, connection.go:57-66), one simplex
connection per direction with the reference handshake.

Modes:
  "device": SendBuf/RecvBuf are GPU tensors. A peer chunk lands in a
            page-locked slot, is copied to HBM and folded by the HIP kernel
            (kf_ingest_recv_onto); results leave via page-locked slots.
  "host":   SendBuf/RecvBuf are host numpy arrays; the fold is
            std_transform_2 of libkungfu_amd.so (the drop-in, GPU offload) or
            a ``reduce_fn(x, y, out)`` the caller passes.
"""
import ctypes
import os
import select
import socket
import threading
import time

import numpy as np

from . import _lib
from .base import OP, OP_NAMES, EvenPartition

CHUNK_SIZE = 1 << 20          # session.go:301-304
PORT_BASE = 10000             # default peer ports (plan/hostspec.go:121-124)
LOCALHOST_IPV4 = 0x7F000001
CONN_RETRY = 500              # config.go:15-18: 500 x 200 ms
CONN_RETRY_PERIOD = 0.2


def sock_path(sock_dir, rank):
    return os.path.join(sock_dir, "kungfu-amd-%d.sock" % (PORT_BASE + rank))


class Session:
    def __init__(self, rank, size, sock_dir, mode="device", token=0,
                 reduce_fn=None, slot_bytes=CHUNK_SIZE + 4096, nslots=8):
        if mode not in ("device", "host"):
            raise ValueError(mode)
        self.rank, self.size, self.dir = rank, size, sock_dir
        self.mode, self.token = mode, token
        self.reduce_fn = reduce_fn
        self.lib = _lib.load()
        self.out, self.inc = {}, {}
        self._ingest = self._egress = None
        if mode == "device":
            # one landing ring for received chunks, one for outgoing chunks
            # (the sender thread and the receiver never share slots)
            self._ingest = self.lib.kf_ingest_create(slot_bytes, nslots)
            self._egress = self.lib.kf_ingest_create(slot_bytes, 2)
            if not self._ingest or not self._egress:
                raise _lib.KungFuAMDError("kf_ingest_create: " +
                                          self.lib.kf_ingest_last_error().decode())
        self._listener = None
        if size > 1:
            self._connect()

    # ---- connections (STAR: peers -> 0 for reduce, 0 -> peers for bcast) --
    def _senders_to_me(self):
        return list(range(1, self.size)) if self.rank == 0 else [0]

    def _connect(self):
        path = sock_path(self.dir, self.rank)
        if os.path.exists(path):
            os.unlink(path)
        self._listener = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self._listener.bind(path)
        self._listener.listen(self.size)
        expect = self._senders_to_me()
        errs = []

        def accept_all():
            try:
                for _ in expect:
                    c, _ = self._listener.accept()
                    t, p, ip = ctypes.c_uint16(), ctypes.c_uint16(), ctypes.c_uint32()
                    rc = self.lib.kf_rch_server_handshake(
                        c.fileno(), self.token, ctypes.byref(t), ctypes.byref(p),
                        ctypes.byref(ip))
                    _lib.check(rc, "kf_rch_server_handshake")
                    self.inc[p.value - PORT_BASE] = c
            except Exception as e:  # surfaced after join
                errs.append(e)

        th = threading.Thread(target=accept_all, daemon=True)
        th.start()
        for peer in expect:  # in the star, the send set equals the receive set
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            for attempt in range(CONN_RETRY):
                try:
                    s.connect(sock_path(self.dir, peer))
                    break
                except (FileNotFoundError, ConnectionRefusedError):
                    if attempt == CONN_RETRY - 1:
                        raise
                    time.sleep(CONN_RETRY_PERIOD)
            rc = self.lib.kf_rch_client_handshake(
                s.fileno(), 2, PORT_BASE + self.rank, LOCALHOST_IPV4, self.token)
            _lib.check(rc, "kf_rch_client_handshake")
            self.out[peer] = s
        th.join()
        if errs:
            raise errs[0]

    def close(self):
        for s in list(self.out.values()) + list(self.inc.values()):
            s.close()
        if self._listener is not None:
            self._listener.close()
            try:
                os.unlink(sock_path(self.dir, self.rank))
            except FileNotFoundError:
                pass
        for g in (self._ingest, self._egress):
            if g:
                self.lib.kf_ingest_destroy(g)
        self._ingest = self._egress = None

    # ---- buffers -------------------------------------------------------------
    def _meta(self, buf):
        if self.mode == "device":
            from .ops import kungfu_dtype
            return buf.numel(), buf.element_size(), int(kungfu_dtype(buf)), buf.data_ptr()
        from .base import dtype_of
        return buf.size, buf.itemsize, int(dtype_of(buf)), buf.ctypes.data

    def all_reduce(self, send, recv, name, op="sum"):
        """Session.AllReduce on one bucket; every rank returns with recv
        holding the reduction of all ranks' send (in place if send is recv)."""
        red = OP_NAMES[op] if isinstance(op, str) else OP(op)
        count, isz, dt, sp = self._meta(send)
        _, _, _, rp = self._meta(recv)
        inplace = sp == rp
        if count == 0:
            return recv
        if self.size == 1:  # isolated node: w.Forward() (session.go:235-238)
            if not inplace:
                self._copy(recv, send)
            return recv
        k = (count * isz + CHUNK_SIZE - 1) // CHUNK_SIZE
        parts = EvenPartition(0, count, k)
        names = ["part::%s[%d:%d]" % (name, b, e) for b, e in parts]
        index = {nm.encode(): i for i, nm in enumerate(names)}
        stream = self._stream(send)
        if self.rank == 0:
            self._root(parts, names, index, isz, dt, red, sp, rp, inplace, stream)
        else:
            self._leaf(parts, names, index, isz, sp, rp, stream)
        self._finish(stream)
        return recv

    def _stream(self, t):
        if self.mode != "device":
            return None
        import torch
        return torch.cuda.current_stream(t.device).cuda_stream

    def _finish(self, stream):
        if self.mode == "device":
            _lib.check(self.lib.kf_ingest_sync(self._ingest), "kf_ingest_sync")
            import torch
            torch.cuda.synchronize()

    def _copy(self, dst, src):
        if self.mode == "device":
            dst.copy_(src)
        else:
            np.copyto(dst, src)

    def _read_header(self, sock):
        name = ctypes.create_string_buffer(512)
        fl = ctypes.c_uint32()
        _lib.check(self.lib.kf_rch_recv_header(sock.fileno(), name, 512, None,
                                                ctypes.byref(fl)), "kf_rch_recv_header")
        return name.value, fl.value

    def _root(self, parts, names, index, isz, dt, red, sp, rp, inplace, stream):
        lib = self.lib
        peers = sorted(self.inc)
        folded = [0] * len(parts)
        remaining = len(parts) * len(peers)
        socks = {self.inc[p].fileno(): self.inc[p] for p in peers}
        scratch = None
        while remaining:
            ready, _, _ = select.select(list(socks), [], [])
            for fd in ready:  # arrival order
                nm, _ = self._read_header(socks[fd])
                c = index[nm]
                b, e = parts[c]
                n = e - b
                own = None if (folded[c] > 0 or inplace) else sp + b * isz
                dst = rp + b * isz
                if self.mode == "device":
                    rc = lib.kf_ingest_recv_onto(self._ingest, fd, n * isz, dst, own, n,
                                                 dt, int(red), stream)
                    _lib.check(rc, "kf_ingest_recv_onto")
                else:  # host: pooled receive buffer, then the fold
                    if scratch is None or scratch.nbytes < n * isz:
                        scratch = np.empty(CHUNK_SIZE + 64, np.uint8)
                    _lib.check(lib.kf_rch_recv_body(fd, scratch.ctypes.data, n * isz),
                               "kf_rch_recv_body")
                    self._host_fold(dst, own if own is not None else dst,
                                    scratch.ctypes.data, n, dt, red)
                folded[c] += 1
                remaining -= 1
                if folded[c] == len(peers):  # chunk complete: bcast it
                    for p in peers:
                        self._send(self.out[p], names[c], 1, dst, n * isz, stream)

    def _host_fold(self, out, x, y, n, dt, red):
        if self.reduce_fn is not None:
            self.reduce_fn(x, y, out, n, dt, int(red))
        else:
            self.lib.std_transform_2(x, y, out, n, dt, int(red))

    def _leaf(self, parts, names, index, isz, sp, rp, stream):
        root = self.out[0]
        errs = []

        def send_all():  # sendOnto the root, concurrently with the receives
            try:
                for (b, e), nm in zip(parts, names):
                    self._send(root, nm, 0, sp + b * isz, (e - b) * isz, stream)
            except Exception as ex:
                errs.append(ex)

        th = threading.Thread(target=send_all, daemon=True)
        th.start()
        src = self.inc[0]
        for _ in parts:  # recvInto from the root, straight into RecvBuf
            nm, flags = self._read_header(src)
            c = index[nm]
            b, e = parts[c]
            dst = rp + b * isz
            if self.mode == "device":
                _lib.check(self.lib.kf_ingest_recv_into(self._ingest, src.fileno(),
                                                        (e - b) * isz, dst, stream),
                           "kf_ingest_recv_into")
            else:
                _lib.check(self.lib.kf_rch_recv_body(src.fileno(), dst, (e - b) * isz),
                           "kf_rch_recv_body")
        th.join()
        if errs:
            raise errs[0]

    def _send(self, sock, name, flags, ptr, nbytes, stream):
        if self.mode == "device":
            rc = self.lib.kf_ingest_send_from_device(self._egress, sock.fileno(),
                                                     name.encode(), flags, ptr, nbytes,
                                                     stream)
            _lib.check(rc, "kf_ingest_send_from_device")
        else:
            _lib.check(self.lib.kf_rch_send(sock.fileno(), name.encode(), flags, ptr,
                                            nbytes), "kf_rch_send")
