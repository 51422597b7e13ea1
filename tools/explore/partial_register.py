"""Does std_transform_2 survive buffers that are only partly inside a
kf_host_register'd range (r06h: the parity test's process exited at that
case)? Prints the library's status and message per variant."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from kungfu_amd import _lib  # noqa: E402

lib = _lib.load()
n = (40 << 20) // 4 + 12345
rng = np.random.default_rng(1)
x = rng.standard_normal(n).astype(np.float32)
y = rng.standard_normal(n).astype(np.float32)
z = np.zeros_like(x)
case = sys.argv[1]
if case == "partial":
    assert lib.kf_host_register(x.ctypes.data, (n // 2) * 4) == 0
elif case == "whole":
    assert lib.kf_host_register(x.ctypes.data, n * 4) == 0
rc = lib.kf_transform2_host(x.ctypes.data, y.ctypes.data, z.ctypes.data, n, 0x20408, 0)
print(case, "rc", rc, lib.kf_last_error().decode(), "ok", bool(np.array_equal(z, x + y)), flush=True)
