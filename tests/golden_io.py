"""Access to the committed golden fixtures (tests/golden/, made by
tests/golden/gen_golden.py from the reference's own compiled reduce)."""
import hashlib
import json
import os
import sys

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import gen_golden  # noqa: E402  (pure-numpy input generators; no reference access)

_cache = {}


def index():
    if "index" not in _cache:
        with open(os.path.join(GOLDEN, "transform2.json")) as f:
            _cache["index"] = json.load(f)
    return _cache["index"]


def arrays():
    if "npz" not in _cache:
        _cache["npz"] = dict(np.load(os.path.join(GOLDEN, "transform2.npz")))
    return _cache["npz"]


def stored_cases():
    a = arrays()
    for c in index():
        if c["stored"]:
            yield c, a[c["id"] + "_x"], a[c["id"] + "_y"], a[c["id"] + "_z"]


def large_cases():
    for c in index():
        if not c["stored"]:
            x, y = gen_golden.gen_inputs(c["dtype"], c["n"], c["seed"], c["kind"])
            yield c, x, y


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def same_bits_or_nan(a, b):
    """Bit equality, except that two NaNs compare equal whatever their payload
    (x86 and gfx950 propagate NaN payloads differently; NaN-ness must match)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.dtype.kind != "f":
        return np.array_equal(a.view(np.uint8), b.view(np.uint8))
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    ua = a.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[a.itemsize])
    ub = b.view({2: np.uint16, 4: np.uint32, 8: np.uint64}[b.itemsize])
    return np.array_equal(ua[~na], ub[~nb])
