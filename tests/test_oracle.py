"""Pins the CPU oracle to the reference: every golden vector produced by the
reference's own std_transform_2 (compiled from srcs/go/kungfu/base) must be
reproduced bit for bit, plus the reference's unit-test known answers."""
import numpy as np
import pytest

import golden_io


def test_type_size_matches_reference(oracle_mod):
    # dtype.c:7-35 via tests/golden/type_size.json; test_kungfu.cpp:3-9
    for name, size in golden_io.load_json("type_size.json").items():
        assert oracle_mod.type_size(name) == size, name
    assert oracle_mod.type_size("i32") == 4
    assert oracle_mod.type_size("f16") == 2
    assert oracle_mod.type_size("f32") == 4
    assert oracle_mod.type_size("f64") == 8
    assert oracle_mod.type_size(0x12345) == 0  # reference: exit(1)


def test_transform_unit(oracle_mod):
    # test_kungfu.cpp:11-20: 1 + 2 = 3, in place into x
    x = np.array([1.0], np.float32)
    y = np.array([2.0], np.float32)
    oracle_mod.transform2(x, y, "f32", "sum", out=x)
    assert x[0] == 3.0


def test_stored_golden_bit_exact(oracle_mod):
    n = 0
    for c, x, y, z in golden_io.stored_cases():
        if c["kind"].startswith("alias"):
            continue
        got = oracle_mod.transform2(x, y, c["dtype"], c["op"])
        assert np.array_equal(got.view(np.uint8), z.view(np.uint8)), c
        n += 1
    assert n > 600


def test_alias_cases(oracle_mod):
    for c, x, y, z in golden_io.stored_cases():
        if not c["kind"].startswith("alias"):
            continue
        xx, yy = x.copy(), y.copy()
        out = xx if c["kind"] == "alias_x" else yy
        oracle_mod.transform2(xx, yy, c["dtype"], c["op"], out=out)
        assert np.array_equal(out.view(np.uint8), z.view(np.uint8))


def test_large_golden_sha(oracle_mod):
    for c, x, y in golden_io.large_cases():
        assert golden_io.sha(x) == c["sha_x"], "input generator drifted"
        assert golden_io.sha(y) == c["sha_y"], "input generator drifted"
        got = oracle_mod.transform2(x, y, c["dtype"], c["op"])
        assert golden_io.sha(got) == c["sha_z"], c


def test_rejects_match_reference(oracle_mod):
    for r in golden_io.load_json("rejects.json"):
        assert r["exit"] == 1
        x = np.zeros(8, np.uint8)
        op = {"sum": 0, "min": 1, "max": 2, "prod": 3}.get(r["op"], 7)
        with pytest.raises(ValueError):
            oracle_mod.transform2(x, x, r["code"], op)


def test_f16_sum_is_ieee_half_add(oracle_mod):
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(4097) * 300).astype(np.float16)
    y = (rng.standard_normal(4097) * 300).astype(np.float16)
    got = oracle_mod.transform2(x, y, "f16", "sum")
    with np.errstate(over="ignore"):
        assert np.array_equal(got.view(np.uint16), (x + y).view(np.uint16))


def test_reduce_k_is_chain_of_transform2(oracle_mod):
    rng = np.random.default_rng(6)
    xs = [rng.standard_normal(1000).astype(np.float32) for _ in range(5)]
    acc = xs[0].copy()
    for x in xs[1:]:
        acc = oracle_mod.transform2(acc, x, "f32", "sum")
    assert np.array_equal(oracle_mod.reduce_k(xs, "f32", "sum"), acc)
    # fp16 rounds per hop (f16.c per Transform2 call)
    hs = [(rng.standard_normal(1000) * 50).astype(np.float16) for _ in range(4)]
    acc = hs[0]
    for h in hs[1:]:
        acc = (acc + h).astype(np.float16)
    assert np.array_equal(oracle_mod.reduce_k(hs, "f16", "sum").view(np.uint16),
                          acc.view(np.uint16))


def test_avg_np2_exact(oracle_mod):
    # two-operand sum and /2 are exact => hand-computable
    x = np.array([1.5, -3.25, 1e-3, 7.0], np.float32)
    y = np.array([0.5, 1.25, 2e-3, -7.0], np.float32)
    got = oracle_mod.reduce_avg([x, y], "f32", 2)
    assert np.array_equal(got, ((x + y) / np.float32(2)).astype(np.float32))
    assert (got[0], got[1], got[3]) == (1.0, -1.0, 0.0)


@pytest.mark.parametrize("np_", [1, 2, 3, 5, 8])
def test_avg_is_true_division(oracle_mod, np_):
    rng = np.random.default_rng(np_)
    xs = [rng.standard_normal(777).astype(np.float32) for _ in range(np_)]
    s = oracle_mod.reduce_k(xs, "f32", "sum")
    want = (s / np.float32(np_)).astype(np.float32)
    assert np.array_equal(oracle_mod.reduce_avg(xs, "f32", np_), want)


def test_sma_blend_matches_tf_formula(oracle_mod):
    # sma_sgd.py:60-65 with float32 tensors and Python-float constants
    rng = np.random.default_rng(9)
    v = rng.standard_normal(1000).astype(np.float32)
    s = rng.standard_normal(1000).astype(np.float32)
    alpha = 0.1
    avg = (s / np.float32(4)).astype(np.float32)
    want = (np.float32(1 - alpha) * v).astype(np.float32) + \
        (np.float32(alpha) * avg).astype(np.float32)
    got = oracle_mod.sma_blend(v, s, "f32", 4, alpha)
    assert np.array_equal(got, want.astype(np.float32))


def test_bf16_build_semantics(oracle_mod):
    rng = np.random.default_rng(10)
    a = rng.standard_normal(5000).astype(np.float32)
    b = rng.standard_normal(5000).astype(np.float32)
    ab = oracle_mod.f32_to_bf16_bits(a)
    bb = oracle_mod.f32_to_bf16_bits(b)
    got = oracle_mod.transform2(ab, bb, "bf16", "sum")
    want = oracle_mod.f32_to_bf16_bits(oracle_mod.bf16_bits_to_f32(ab) +
                                       oracle_mod.bf16_bits_to_f32(bb))
    assert np.array_equal(got, want)
    # NaN stays NaN, quiet
    nanbits = np.array([0x7F81, 0xFFC1], np.uint16)
    f = oracle_mod.bf16_bits_to_f32(nanbits)
    assert np.all(np.isnan(oracle_mod.bf16_bits_to_f32(oracle_mod.f32_to_bf16_bits(f))))


def test_bf16_two_input_matches_torch(oracle_mod):
    """bf16 has no reference reduce (parity unpinned); its
    two-input SUM / MIN / MAX are cross-checked against an independent
    implementation, torch's CPU bfloat16 ops, on random values and every pair
    of specials (NaN compared by position)."""
    import torch
    rng = np.random.default_rng(11)
    vals = np.concatenate([rng.standard_normal(4000).astype(np.float32) * 10,
                           rng.standard_normal(1000).astype(np.float32) * 1e30,
                           rng.standard_normal(1000).astype(np.float32) * 1e-39])
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3.3895e38, 1.0],
                  np.float32)
    a = np.concatenate([vals, np.repeat(sp, len(sp))])
    b = np.concatenate([vals[::-1].copy(), np.tile(sp, len(sp))])
    ab, bb = oracle_mod.f32_to_bf16_bits(a), oracle_mod.f32_to_bf16_bits(b)
    ta = torch.from_numpy(ab.view(np.int16)).view(torch.bfloat16)
    tb = torch.from_numpy(bb.view(np.int16)).view(torch.bfloat16)
    for op, fn in (("sum", torch.add), ("min", torch.minimum), ("max", torch.maximum)):
        got = oracle_mod.transform2(ab, bb, "bf16", op)
        want = fn(ta, tb).view(torch.int16).numpy().view(np.uint16)
        gf = oracle_mod.bf16_bits_to_f32(got)
        wf = oracle_mod.bf16_bits_to_f32(want)
        nan = np.isnan(wf)
        if op == "sum":
            assert np.array_equal(np.isnan(gf), nan)
            assert np.array_equal(got[~nan], want[~nan])
        else:
            # torch propagates NaN from either side and orders -0 < +0; the
            # build selects an input like std::min/max (op.cpp:22-43), which
            # keeps the first of two equal zeros — the only other difference
            fa, fb = oracle_mod.bf16_bits_to_f32(ab), oracle_mod.bf16_bits_to_f32(bb)
            ok = ~(np.isnan(fa) | np.isnan(fb) | ((fa == 0) & (fb == 0)))
            assert np.array_equal(got[ok], want[ok]), op


@pytest.mark.parametrize("dt", ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64",
                                "f16", "f32", "f64"])
def test_oracle_vs_reference_build_random(oracle_mod, dt):
    # beyond the stored vectors: fresh random inputs (specials mixed in)
    # through the oracle and the reference's own compiled std_transform_2
    import ctypes
    import os
    import zlib
    if not os.path.exists(oracle_mod.REF_LIB):
        pytest.skip("reference build absent (make -C oracle ref)")
    ref = ctypes.CDLL(oracle_mod.REF_LIB)
    ref.std_transform_2.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3
    rng = np.random.default_rng(zlib.crc32(dt.encode()))
    npdt = oracle_mod.NP[dt]
    n = 100003
    if np.issubdtype(npdt, np.integer):
        info = np.iinfo(npdt)
        x = rng.integers(info.min, info.max, size=n, dtype=npdt, endpoint=True)
        y = rng.integers(info.min, info.max, size=n, dtype=npdt, endpoint=True)
    else:
        x = (rng.standard_normal(n) * 1e3).astype(npdt)
        y = (rng.standard_normal(n) * 1e3).astype(npdt)
        sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, np.finfo(npdt).max,
                       np.finfo(npdt).tiny / 2], dtype=npdt)
        idx = rng.integers(0, n, size=2000)
        x[idx] = sp[rng.integers(0, sp.size, size=idx.size)]
        y[idx[::-1]] = sp[rng.integers(0, sp.size, size=idx.size)]
    for op in (["sum"] if dt == "f16" else ["sum", "min", "max", "prod"]):
        want = np.empty_like(x)
        ref.std_transform_2(x.ctypes.data, y.ctypes.data, want.ctypes.data, n,
                            oracle_mod.DT[dt], oracle_mod.OPS[op])
        got = oracle_mod.transform2(x, y, dt, op)
        assert golden_io.same_bits_or_nan(got, want), (dt, op)
