"""rchannel wire format of libkungfu_amd.so (kf_rch_*), byte-exact against the
reference framing (srcs/go/rchannel/connection/message.go:44-198,
connection.go:28-101) and the reference's own round-trip tests
(message_test.go:8-79). Host-only: no GPU needed."""
import ctypes
import socket
import struct
import threading

import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib():
    from kungfu_amd import _lib
    return _lib.load()


def pair():
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
    return a, b


def recv_exact(s, n):
    buf = b""
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        assert chunk
        buf += chunk
    return buf


def test_send_bytes_are_reference_framing(lib):
    a, b = pair()
    data = np.frombuffer(b"123456", np.uint8).copy()
    assert lib.kf_rch_send(a.fileno(), b"part::g[0:6]", 1, data.ctypes.data, 6) == 0
    name = b"part::g[0:6]"
    want = struct.pack("<I", len(name)) + name + struct.pack("<I", 1) + \
        struct.pack("<I", 6) + b"123456"
    assert recv_exact(b, len(want)) == want


def test_handshake_roundtrip(lib):
    # Test_connectionHeader: type=ConnCollective, port 9999, ipv4 0x7f080808
    a, b = pair()
    out = {}

    def server():
        t, p, ip = ctypes.c_uint16(), ctypes.c_uint16(), ctypes.c_uint32()
        out["rc"] = lib.kf_rch_server_handshake(b.fileno(), 77, ctypes.byref(t),
                                                ctypes.byref(p), ctypes.byref(ip))
        out["hdr"] = (t.value, p.value, ip.value)

    th = threading.Thread(target=server)
    th.start()
    assert lib.kf_rch_client_handshake(a.fileno(), 2, 9999, 0x7F080808, 77) == 0
    th.join()
    assert out["rc"] == 0 and out["hdr"] == (2, 9999, 0x7F080808)


def test_handshake_bad_token_is_error(lib):
    a, b = pair()
    b.sendall(struct.pack("<I", 5))  # server token 5
    rc = lib.kf_rch_client_handshake(a.fileno(), 2, 1, 1, 6)
    assert rc == 7  # KF_ERR_PROTO: connection.go:93-99
    # header was still written: {u16 type, u16 port, u32 ipv4}
    assert recv_exact(b, 8) == struct.pack("<HHI", 2, 1, 1)


def test_message_roundtrip_16mib(lib):
    # Test_long_Message: 16 MiB payload of "01234567"*...
    a, b = pair()
    payload = np.frombuffer(b"01234567" * (2 * 1024 * 1024), np.uint8).copy()
    th = threading.Thread(target=lambda: lib.kf_rch_send(
        a.fileno(), b"123456", 0, payload.ctypes.data, payload.size))
    th.start()
    name = ctypes.create_string_buffer(64)
    nl, fl = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.kf_rch_recv_header(b.fileno(), name, 64, ctypes.byref(nl), ctypes.byref(fl)) == 0
    assert name.value == b"123456" and nl.value == 6 and fl.value == 0
    dst = np.zeros_like(payload)
    assert lib.kf_rch_recv_body(b.fileno(), dst.ctypes.data, dst.size) == 0
    th.join()
    assert np.array_equal(dst, payload)


def test_recv_body_length_mismatch(lib):
    # Message.ReadInto rejects a length different from the registered buffer
    a, b = pair()
    a.sendall(struct.pack("<I", 10) + b"x" * 10)
    dst = np.zeros(8, np.uint8)
    assert lib.kf_rch_recv_body(b.fileno(), dst.ctypes.data, 8) == 7


def test_short_stream_is_error(lib):
    a, b = pair()
    a.sendall(struct.pack("<I", 100) + b"abc")
    a.close()
    name = ctypes.create_string_buffer(256)
    assert lib.kf_rch_recv_header(b.fileno(), name, 256, None, None) == 7


def test_name_longer_than_buffer(lib):
    a, b = pair()
    a.sendall(struct.pack("<I", 300) + b"n" * 300 + struct.pack("<I", 0))
    name = ctypes.create_string_buffer(16)
    assert lib.kf_rch_recv_header(b.fileno(), name, 16, None, None) == 7
