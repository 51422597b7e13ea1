"""GPU parity: the HIP path (through the C-ABI) against the oracle and the
reference's golden vectors. Integers bit-exact; floats bit-exact where the
reference is deterministic (any 2-operand op, ring order, fixed fold order),
NaN-ness equal where payloads may differ (golden_io.same_bits_or_nan)."""
import os
import zlib

import numpy as np
import pytest

import golden_io

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def lib(dev):
    from kungfu_amd import _lib
    l = _lib.load()
    assert l.kf_device_count() > 0
    return l


@pytest.fixture(scope="module")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


def to_dev(a, dev):
    """numpy -> GPU tensor holding the same bytes (unsigned views for u16..)."""
    a = np.ascontiguousarray(a)
    t = torch.from_numpy(a.view(np.uint8).copy()).to(dev)
    return t


def from_dev(t, like):
    return t.cpu().numpy().view(like.dtype).reshape(like.shape)


def dev_reduce(lib, arrs, code, op, dev, out_alias=None):
    from kungfu_amd import _lib
    ts = [to_dev(a, dev) for a in arrs]
    out = ts[out_alias] if out_alias is not None else torch.empty_like(ts[0])
    rc = lib.kf_bucket_reduce(_lib.ptr_array([t.data_ptr() for t in ts]), len(ts),
                              out.data_ptr(), arrs[0].size, code, op,
                              torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.kf_last_error()
    torch.cuda.synchronize()
    return from_dev(out, arrs[0])


# ---- B1: std_transform_2 drop-in against every reference golden vector ----

def test_std_transform_2_golden(lib):
    n = 0
    for c, x, y, z in golden_io.stored_cases():
        xx, yy = x.copy(), y.copy()
        if c["kind"] == "alias_x":
            out = xx
        elif c["kind"] == "alias_y":
            out = yy
        else:
            out = np.empty_like(x)
        lib.std_transform_2(xx.ctypes.data, yy.ctypes.data, out.ctypes.data,
                            c["n"], c["code"], c["opcode"])
        assert golden_io.same_bits_or_nan(out, z), c
        n += 1
    assert n > 600


def test_std_transform_2_golden_large(lib):
    for c, x, y in golden_io.large_cases():
        z = np.empty_like(x)
        lib.std_transform_2(x.ctypes.data, y.ctypes.data, z.ctypes.data, c["n"],
                            c["code"], c["opcode"])
        assert golden_io.sha(z) == c["sha_z"], c


def test_float16_sum_entry(lib, orc):
    rng = np.random.default_rng(3)
    for n in (1, 5, 8, 13, 100003):
        x = (rng.standard_normal(n) * 100).astype(np.float16)
        y = (rng.standard_normal(n) * 100).astype(np.float16)
        z = np.empty_like(x)
        lib.float16_sum(z.ctypes.data, x.ctypes.data, y.ctypes.data, n)
        assert np.array_equal(z.view(np.uint16), orc.transform2(x, y, "f16", "sum").view(np.uint16))


def test_base_transform_mirror(lib):
    # kungfu_amd.base mirrors op.go: Transform2(z, x, y) / Transform(y, x)
    from kungfu_amd import base
    x = base.Vector.of(np.array([1.0, 2.0], np.float32))
    y = base.Vector.of(np.array([2.0, 5.0], np.float32))
    z = base.Vector.new(2, base.DataType.F32)
    base.Transform2(z, x, y, base.OP.SUM)
    assert list(z.Data) == [3.0, 7.0]
    base.Transform(y, x, base.OP.MAX)
    assert list(y.Data) == [2.0, 5.0]


# ---- B2: device bucket API ------------------------------------------------

INT_DTS = ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64"]


@pytest.mark.parametrize("dt", INT_DTS + ["f32", "f64", "bf16"])
@pytest.mark.parametrize("op", ["sum", "min", "max", "prod"])
def test_device_two_input_vs_oracle(lib, orc, dev, dt, op):
    from oracle.oracle import DT, NP, OPS
    rng = np.random.default_rng(zlib.crc32((dt + op).encode()))
    for n in (1, 3, 17, 4096 + 5, 1 << 20):
        if dt in INT_DTS:
            info = np.iinfo(NP[dt])
            x = rng.integers(info.min, info.max, size=n, dtype=NP[dt], endpoint=True)
            y = rng.integers(info.min, info.max, size=n, dtype=NP[dt], endpoint=True)
        elif dt == "bf16":
            x = orc.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32))
            y = orc.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32))
        else:
            x = rng.standard_normal(n).astype(NP[dt])
            y = rng.standard_normal(n).astype(NP[dt])
        got = dev_reduce(lib, [x, y], DT[dt], OPS[op], dev)
        want = orc.transform2(x, y, dt, op)
        assert golden_io.same_bits_or_nan(got, want), (dt, op, n)


def test_device_f16_sum_and_rejects(lib, orc, dev):
    from kungfu_amd import _lib
    rng = np.random.default_rng(4)
    x = (rng.standard_normal(333333) * 1000).astype(np.float16)  # overflows too
    y = (rng.standard_normal(333333) * 1000).astype(np.float16)
    got = dev_reduce(lib, [x, y], 0x20208, 0, dev)
    assert np.array_equal(got.view(np.uint16), orc.transform2(x, y, "f16", "sum").view(np.uint16))
    t = torch.zeros(16, dtype=torch.float16, device=dev)
    arr = _lib.ptr_array([t.data_ptr(), t.data_ptr()])
    for op in (1, 2, 3):  # op.cpp:45-54: fp16 is SUM only
        assert lib.kf_bucket_reduce(arr, 2, t.data_ptr(), 16, 0x20208, op, None) == 2


def test_specials_all_pairs(lib, orc, dev):
    # every ordered pair of specials, f32/f64 x all ops (NaN, +-0, inf, subnormal)
    for c, x, y, z in golden_io.stored_cases():
        if c["kind"] != "special" or c["dtype"] not in ("f32", "f64", "f16", "i32", "i64"):
            continue
        got = dev_reduce(lib, [x, y], c["code"], c["opcode"], dev)
        assert golden_io.same_bits_or_nan(got, z), c


def test_denormals_not_flushed(lib, dev):
    tiny = np.float32(np.finfo(np.float32).tiny)
    x = np.array([tiny / 4, tiny / 8, -tiny / 2] * 100, np.float32)
    y = np.array([tiny / 8, 0.0, tiny / 4] * 100, np.float32)
    got = dev_reduce(lib, [x, y], 0x20408, 0, dev)
    assert np.array_equal(got, x + y)
    assert np.all(got[:3] != 0)


@pytest.mark.parametrize("k", [3, 4, 5, 6, 7, 8, 16])
def test_k_input_ring_order_bit_exact(lib, orc, dev, k):
    # The k-input fused reduce, fed in the reference ring order, reproduces the
    # reference RING all-reduce of that chunk bit for bit (schedule.py).
    from oracle import schedule
    rng = np.random.default_rng(k)
    n = 262144 + 13
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(k)]
    for r in (0, k - 1):
        order = schedule.ring_order(k, r)
        got = dev_reduce(lib, [xs[j] for j in order], 0x20408, 0, dev)
        want = orc.reduce_k([xs[j] for j in order], "f32", "sum")
        assert np.array_equal(got, want)
    # int32 and fp16 (per-hop rounding) chains as well
    ints = [rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int32) for _ in range(k)]
    assert np.array_equal(dev_reduce(lib, ints, 0x10408, 0, dev), orc.reduce_k(ints, "i32"))
    hs = [(rng.standard_normal(n) * 30).astype(np.float16) for _ in range(k)]
    assert np.array_equal(dev_reduce(lib, hs, 0x20208, 0, dev).view(np.uint16),
                          orc.reduce_k(hs, "f16").view(np.uint16))
    bs = [orc.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32)) for _ in range(k)]
    assert np.array_equal(dev_reduce(lib, bs, 0x20209, 0, dev), orc.reduce_k(bs, "bf16"))


@pytest.mark.parametrize("k", [2, 3, 5, 8, 9, 16])
def test_peers_fold_bit_exact(lib, orc, dev, k):
    # kf_bucket_reduce_peers (all inputs' loads in flight, the P2P shard fold):
    # the same left fold in input order as the oracle, for plain ops and the
    # fused / np, with a ragged tail and a co-misaligned head
    from kungfu_amd import _lib
    from oracle.oracle import DT
    rng = np.random.default_rng(100 + k)
    n = 65536 * 3 + 7
    s = torch.cuda.current_stream().cuda_stream
    cases = [("f32", [rng.standard_normal(n + 1).astype(np.float32) for _ in range(k)]),
             ("i32", [rng.integers(-2**31, 2**31 - 1, size=n + 1, dtype=np.int32)
                      for _ in range(k)]),
             ("f16", [(rng.standard_normal(n + 1) * 30).astype(np.float16) for _ in range(k)]),
             ("bf16", [orc.f32_to_bf16_bits(rng.standard_normal(n + 1).astype(np.float32))
                       for _ in range(k)])]
    for dt, xs in cases:
        for head in (0, 1):
            ts = [to_dev(x, dev) for x in xs]
            isz = xs[0].itemsize
            out = torch.zeros_like(ts[0])
            ptrs = _lib.ptr_array([t.data_ptr() + head * isz for t in ts])
            ops = ["sum"] if dt == "f16" else ["sum", "max"]
            for op in ops:
                rc = lib.kf_bucket_reduce_peers(ptrs, k, out.data_ptr() + head * isz, n, DT[dt],
                                                {"sum": 0, "max": 2}[op], 0, s)
                assert rc == 0, lib.kf_last_error()
                torch.cuda.synchronize()
                got = from_dev(out, xs[0])[head:head + n]
                want = orc.reduce_k([x[head:head + n].copy() for x in xs], dt, op)
                assert golden_io.same_bits_or_nan(got, want), (dt, op, head)
            if dt != "i32":
                rc = lib.kf_bucket_reduce_peers(ptrs, k, out.data_ptr() + head * isz, n, DT[dt],
                                                0, k, s)
                assert rc == 0, lib.kf_last_error()
                torch.cuda.synchronize()
                got = from_dev(out, xs[0])[head:head + n]
                want = orc.reduce_avg([x[head:head + n].copy() for x in xs], dt, k)
                assert golden_io.same_bits_or_nan(got, want), (dt, "avg", head)


@pytest.mark.parametrize("dt", ["u8", "i8"])
def test_8bit_lanes_k_fold_and_peers(lib, orc, dev, dt):
    # The vector path carries 8-bit data as 32-bit words of 4 packed bytes
    # (Lane<T>: SWAR add, per-byte MIN/MAX/PROD). Runtime-k fold and the
    # peers fold, every op, heads 0..3 (byte offsets that leave the word
    # lanes at every alignment) and ragged tails, against the oracle chain.
    from kungfu_amd import _lib
    from oracle.oracle import DT, NP, OPS
    info = np.iinfo(NP[dt])
    rng = np.random.default_rng(zlib.crc32(dt.encode()))
    s = torch.cuda.current_stream().cuda_stream
    for k in (3, 8):
        n = 65536 * 4 + 11
        xs = [rng.integers(info.min, info.max, size=n + 3, dtype=NP[dt], endpoint=True)
              for _ in range(k)]
        ts = [to_dev(x, dev) for x in xs]
        out = torch.zeros_like(ts[0])
        for head in (0, 1, 2, 3):
            ptrs = _lib.ptr_array([t.data_ptr() + head for t in ts])
            m = n - head
            for op in ("sum", "min", "max", "prod"):
                want = orc.reduce_k([x[head:head + m].copy() for x in xs], dt, op)
                for fn in ("kf_bucket_reduce", "kf_bucket_reduce_peers"):
                    out.zero_()
                    if fn == "kf_bucket_reduce":
                        rc = lib.kf_bucket_reduce(ptrs, k, out.data_ptr() + head, m, DT[dt],
                                                  OPS[op], s)
                    else:
                        rc = lib.kf_bucket_reduce_peers(ptrs, k, out.data_ptr() + head, m,
                                                        DT[dt], OPS[op], 0, s)
                    assert rc == 0, lib.kf_last_error()
                    torch.cuda.synchronize()
                    got = from_dev(out, xs[0])[head:head + m]
                    assert np.array_equal(got, want), (k, head, op, fn)

def test_schedule_all_reduce_matches_device_fold(lib, orc, dev):
    # Whole reference schedule (RING, np=4, 4 MiB bucket = 4 chunks with
    # hash-chosen roots): per chunk, the device fold in that chunk's ring order
    # equals what every rank holds after the reference all-reduce.
    from oracle import schedule
    rng = np.random.default_rng(11)
    k, n = 4, 1 << 20
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(k)]
    ref = schedule.all_reduce(xs, "f32", "sum", strategy="RING")
    for b, e, r in schedule.chunk_roots(n, 4, k, strategy="RING"):
        order = schedule.ring_order(k, r)
        got = dev_reduce(lib, [xs[j][b:e].copy() for j in order], 0x20408, 0, dev)
        assert np.array_equal(got, ref[0][b:e])


def test_alignment_and_aliasing(lib, orc, dev):
    from kungfu_amd import _lib
    rng = np.random.default_rng(12)
    n = 100000
    x = rng.standard_normal(n + 8).astype(np.float32)
    y = rng.standard_normal(n + 8).astype(np.float32)
    tx, ty = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    s = torch.cuda.current_stream().cuda_stream
    for ox, oy, oz in ((1, 1, 1), (1, 2, 3), (3, 0, 0), (0, 0, 2), (2, 2, 2)):
        out = torch.zeros(n + 8, dtype=torch.float32, device=dev)
        ptrs = _lib.ptr_array([tx.data_ptr() + 4 * ox, ty.data_ptr() + 4 * oy])
        assert lib.kf_bucket_reduce(ptrs, 2, out.data_ptr() + 4 * oz, n, 0x20408, 0, s) == 0
        torch.cuda.synchronize()
        got = out.cpu().numpy()[oz:oz + n]
        assert np.array_equal(got, x[ox:ox + n] + y[oy:oy + n]), (ox, oy, oz)
        assert np.all(out.cpu().numpy()[:oz] == 0) and np.all(out.cpu().numpy()[oz + n:] == 0)
    # in place: out aliases input 0 and input 1
    for alias in (0, 1):
        got = dev_reduce(lib, [x[:n], y[:n]], 0x20408, 0, dev, out_alias=alias)
        assert np.array_equal(got, x[:n] + y[:n])


@pytest.mark.parametrize("dt,k", [("f32", 5), ("f32", 8), ("bf16", 4), ("f16", 3), ("u8", 6)])
def test_k_fold_inputs_at_other_residues(lib, orc, dev, dt, k):
    """The runtime-k fold with inputs at 16-B residues other than the
    output's: inputs 2..k-1 go through the one-in-flight inline-asm loads
    (ld_vec_serial) at unaligned addresses; the left fold in input order must
    equal the oracle's chain."""
    from kungfu_amd import _lib
    from oracle.oracle import DT, NP
    rng = np.random.default_rng(zlib.crc32(("res" + dt).encode()) + k)
    npdt = NP[dt]
    isz = np.dtype(npdt).itemsize
    n = 300007
    hs = [_rand(orc, rng, dt, n + 16) for _ in range(k)]
    ts = [torch.from_numpy(np.ascontiguousarray(h).view(np.uint8)).to(dev) for h in hs]
    s = torch.cuda.current_stream().cuda_stream
    offs = [(j * 3 + 1) % 7 for j in range(k)]  # element offsets, mixed residues
    oz = 2
    out = torch.zeros((n + 16) * isz, dtype=torch.uint8, device=dev)
    ptrs = _lib.ptr_array([t.data_ptr() + isz * o for t, o in zip(ts, offs)])
    assert lib.kf_bucket_reduce(ptrs, k, out.data_ptr() + isz * oz, n, DT[dt], 0, s) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(npdt)[oz:oz + n]
    want = orc.reduce_k([h[o:o + n] for h, o in zip(hs, offs)], dt, "sum")
    assert golden_io.same_bits_or_nan(got, want), (dt, k)


def test_k1_copy_and_empty(lib, dev):
    from kungfu_amd import _lib
    t = torch.arange(1000, dtype=torch.float32, device=dev)
    o = torch.zeros_like(t)
    s = torch.cuda.current_stream().cuda_stream
    assert lib.kf_bucket_reduce(_lib.ptr_array([t.data_ptr()]), 1, o.data_ptr(), 1000,
                                0x20408, 0, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(o, t)
    assert lib.kf_bucket_reduce(_lib.ptr_array([t.data_ptr()] * 2), 2, o.data_ptr(), 0,
                                0x20408, 0, s) == 0


# ---- fused S-SGD / SMA epilogues -------------------------------------------

@pytest.mark.parametrize("np_", [1, 2, 3, 4, 7, 8])
@pytest.mark.parametrize("dt", ["f32", "f64", "f16", "bf16"])
def test_avg_epilogue(orc, dev, np_, dt):
    from kungfu_amd import ops
    rng = np.random.default_rng(np_ * 7)
    n = 300001
    tdt = {"f32": torch.float32, "f64": torch.float64, "f16": torch.float16,
           "bf16": torch.bfloat16}[dt]
    if dt == "bf16":
        xs = [orc.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32)) for _ in range(np_)]
    else:
        xs = [rng.standard_normal(n).astype(orc.NP[dt]) for _ in range(np_)]
    ts = [torch.from_numpy(x.view(np.int16) if x.itemsize == 2 else x).to(dev).view(tdt) for x in xs]
    out = ops.bucket_reduce_avg(ts, np_)
    torch.cuda.synchronize()
    got = out.cpu().view(torch.int16 if out.element_size() == 2 else out.dtype).numpy()
    want = orc.reduce_avg(xs, dt, np_)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    # reduce-then-divide done in two steps (RS -> div -> AG) gives the same bits
    if dt in ("f32", "f64"):
        s = ops.bucket_reduce(ts, op="sum")
        ops.bucket_div_(s, np_)
        torch.cuda.synchronize()
        assert np.array_equal(s.cpu().numpy(), want)


@pytest.mark.parametrize("dt", ["f32", "f64", "f16", "bf16"])
def test_sma_blend(orc, dev, dt):
    from kungfu_amd import ops
    rng = np.random.default_rng(13)
    n = 250007
    tdt = {"f32": torch.float32, "f64": torch.float64, "f16": torch.float16,
           "bf16": torch.bfloat16}[dt]
    if dt == "bf16":
        v = orc.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32))
        s = orc.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32) * 4)
    else:
        v = rng.standard_normal(n).astype(orc.NP[dt])
        s = (rng.standard_normal(n) * 4).astype(orc.NP[dt])
    view = lambda a: a.view(np.int16) if a.itemsize == 2 else a  # noqa: E731
    tv = torch.from_numpy(view(v).copy()).to(dev).view(tdt)
    ts = torch.from_numpy(view(s).copy()).to(dev).view(tdt)
    for np_, alpha in ((4, 0.1), (3, 0.25), (8, 0.1)):
        want = orc.sma_blend(view(v).copy(), view(s), dt, np_, alpha)
        tv2 = tv.clone()
        ops.sma_blend_(tv2, ts, np_, alpha)
        torch.cuda.synchronize()
        got = tv2.cpu().view(torch.int16 if tv2.element_size() == 2 else tv2.dtype).numpy()
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (np_, alpha)


# ---- full BASELINE size (C2: 256 MiB fp32) ---------------------------------

def test_c2_full_size_bit_exact(lib, orc, dev):
    from kungfu_amd import ops
    n = 64 << 20  # 67,108,864 fp32 = 256 MiB per input
    g0 = torch.Generator(device=dev).manual_seed(0)
    g1 = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(n, device=dev, generator=g0)
    y = torch.randn(n, device=dev, generator=g1)
    z = ops.bucket_reduce([x, y])
    torch.cuda.synchronize()
    xh, yh, zh = x.cpu().numpy(), y.cpu().numpy(), z.cpu().numpy()
    assert np.array_equal(zh, orc.transform2(xh, yh, "f32", "sum"))
    # size-independent property: in-place repeat is idempotent on the copy
    z2 = ops.bucket_reduce([x, y], out=x)  # out aliases input 0
    torch.cuda.synchronize()
    assert torch.equal(z2, z)


# ---- optimizer surface on the GPU (world 1: default HIP epilogue) ---------

def test_optimizers_world1_on_gpu(orc, dev):
    from kungfu_amd.optimizers import (SynchronousAveragingOptimizer,
                                       SynchronousSGDOptimizer)
    torch.manual_seed(0)
    m = torch.nn.Linear(300, 70).to(dev)
    ref = torch.nn.Linear(300, 70).to(dev)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(16, 300, device=dev)
    opt = SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.05),
                                  named_parameters=m.named_parameters())
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05)
    for _ in range(3):
        for mm, oo in ((m, opt), (ref, ropt)):
            oo.zero_grad()
            (mm(x) ** 2).mean().backward()
            oo.step()
    for p, q in zip(m.parameters(), ref.parameters()):
        assert torch.equal(p, q)  # np = 1: g / 1 == g, identical updates
    # SMA at np = 1 still applies (1-a) v + a (v / 1), rounded per TF op order
    v_before = [p.detach().clone() for p in m.parameters()]
    sma = SynchronousAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.0), alpha=0.1)
    sma.zero_grad()
    (m(x) ** 2).mean().backward()
    sma.step()
    for p, v in zip(m.parameters(), v_before):
        vh = v.cpu().numpy().reshape(-1)
        want = orc.sma_blend(vh, vh, "f32", 1, 0.1)
        assert np.array_equal(p.detach().cpu().numpy().reshape(-1), want)


def test_host_paths_pageable_and_pinned(lib, orc):
    # kf_transform2_host: pageable (runtime staging) and page-locked (zero
    # copy: the kernel reads/writes host memory in place) give the oracle's bits
    rng = np.random.default_rng(21)
    n = (40 << 20) // 4 + 12345  # 40 MiB + ragged
    x = rng.standard_normal(n).astype(np.float32)
    y = rng.standard_normal(n).astype(np.float32)
    want = orc.transform2(x, y, "f32", "sum")
    z = np.empty_like(x)
    assert lib.kf_transform2_host(x.ctypes.data, y.ctypes.data, z.ctypes.data, n,
                                  0x20408, 0) == 0
    assert np.array_equal(z, want)
    tx = torch.from_numpy(x).pin_memory()
    ty = torch.from_numpy(y).pin_memory()
    tz = torch.empty_like(tx).pin_memory()
    assert lib.kf_transform2_host(tx.data_ptr(), ty.data_ptr(), tz.data_ptr(), n,
                                  0x20408, 0) == 0
    assert np.array_equal(tz.numpy(), want)
    # registered (not hipHostMalloc'ed) numpy memory also takes the DMA path
    z2 = np.zeros_like(x)
    for a in (x, y, z2):
        assert lib.kf_host_register(a.ctypes.data, a.nbytes) == 0
    try:
        lib.std_transform_2(x.ctypes.data, y.ctypes.data, z2.ctypes.data, n, 0x20408, 0)
        assert np.array_equal(z2, want)
        # 1 MiB chunks of the registered buffers at odd offsets, as a Go host's
        # receive pool hands them out: found in the library's registry
        z2[:] = 0
        for off in (0, 4099, n - (1 << 18)):
            m = 1 << 18
            lib.std_transform_2(x[off:].ctypes.data, y[off:].ctypes.data, z2[off:].ctypes.data, m,
                                0x20408, 0)
            assert np.array_equal(z2[off:off + m], want[off:off + m]), off
    finally:
        for a in (x, y, z2):
            lib.kf_host_unregister(a.ctypes.data)
    # buffers page-locked only in part (a chunk running past the end of a
    # registered pool): HIP's own copies refuse them, so the library bounces
    # them through page-locked memory of its own (profiles/r06/
    # partial_register_r06i.txt: "invalid argument" before)
    half = n // 2
    z3 = np.zeros_like(x)
    assert lib.kf_host_register(x.ctypes.data, half * 4) == 0
    assert lib.kf_host_register(z3.ctypes.data, half * 4) == 0
    try:
        assert lib.kf_transform2_host(x.ctypes.data, y.ctypes.data, z3.ctypes.data, n,
                                      0x20408, 0) == 0, lib.kf_last_error()
        assert np.array_equal(z3, want)
        z3[:] = 0
        lib.std_transform_2(x.ctypes.data, y.ctypes.data, z3.ctypes.data, n, 0x20408, 0)
        assert np.array_equal(z3, want)
    finally:
        lib.kf_host_unregister(x.ctypes.data)
        lib.kf_host_unregister(z3.ctypes.data)
    # x page-locked by two registrations that meet at a page boundary (two
    # pools back to back): no single device pointer need cover a call that
    # straddles them, so it is bounced too; and y page-locked only in its
    # middle (both ends pageable), found through the registry
    page = 4096
    cut = (-x.ctypes.data) % page + page * ((n * 4 // 2) // page)
    mid0 = (-y.ctypes.data) % page + page * 16
    mid1 = mid0 + page * ((n * 4 // 2) // page)
    z4 = np.zeros_like(x)
    assert lib.kf_host_register(x.ctypes.data, cut) == 0
    assert lib.kf_host_register(x.ctypes.data + cut, n * 4 - cut) == 0, lib.kf_last_error()
    assert lib.kf_host_register(y.ctypes.data + mid0, mid1 - mid0) == 0, lib.kf_last_error()
    try:
        lib.std_transform_2(x.ctypes.data, y.ctypes.data, z4.ctypes.data, n, 0x20408, 0)
        assert np.array_equal(z4, want)
    finally:
        lib.kf_host_unregister(x.ctypes.data)
        lib.kf_host_unregister(x.ctypes.data + cut)
        lib.kf_host_unregister(y.ctypes.data + mid0)


@pytest.mark.parametrize("dt", ["f32", "f16", "i32", "f64", "u8", "bf16"])
def test_host_zero_copy_shapes(lib, orc, dt):
    # zero-copy path (all three page-locked): every dtype, the reference's
    # 1 MiB chunk, tiny and ragged n, co-misaligned pointers (scalar head),
    # pointers with different 16-B residues (element kernel), out aliasing x,
    # and a mixed page-locked/pageable call (falls back to staging)
    from oracle.oracle import DT, NP
    code, npdt = DT[dt], NP[dt]
    rng = np.random.default_rng(zlib.crc32(dt.encode()))
    isz = np.dtype(npdt).itemsize
    for n in (1, 7, (1 << 20) // isz, (1 << 20) // isz + 3, 3 << 16):
        pool = [torch.empty(n * isz + 64, dtype=torch.uint8).pin_memory() for _ in range(3)]
        for offs in ((0, 0, 0), (isz, isz, isz), (0, isz, 2 * isz)):
            xs, ys, zs = (_host_view(b, o, n, npdt) for b, o in zip(pool, offs))
            xs[:] = _rand(orc, rng, dt, n)
            ys[:] = _rand(orc, rng, dt, n)
            want = orc.transform2(xs.copy(), ys.copy(), dt, "sum")
            assert lib.kf_transform2_host(xs.ctypes.data, ys.ctypes.data, zs.ctypes.data, n,
                                          code, 0) == 0, lib.kf_last_error()
            assert golden_io.same_bits_or_nan(zs, want), (dt, n, offs)
        xs, ys, zs = (_host_view(b, 0, n, npdt) for b in pool)
        x0 = xs.copy()
        want = orc.transform2(x0, ys.copy(), dt, "sum")
        lib.std_transform_2(xs.ctypes.data, ys.ctypes.data, xs.ctypes.data, n, code, 0)
        assert golden_io.same_bits_or_nan(xs, want), (dt, n, "out is x")
        xs[:] = x0
        yp = ys.copy()  # pageable
        lib.std_transform_2(xs.ctypes.data, yp.ctypes.data, zs.ctypes.data, n, code, 0)
        assert golden_io.same_bits_or_nan(zs, want), (dt, n, "mixed")


def test_host_api_on_device_pointers(lib, orc):
    # std_transform_2 handed HBM pointers runs the kernel on them directly
    rng = np.random.default_rng(9)
    n = 100003
    x = rng.standard_normal(n).astype(np.float32)
    y = rng.standard_normal(n).astype(np.float32)
    dx, dy = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    dz = torch.empty_like(dx)
    lib.std_transform_2(dx.data_ptr(), dy.data_ptr(), dz.data_ptr(), n, 0x20408, 0)
    torch.cuda.synchronize()
    assert np.array_equal(dz.cpu().numpy(), orc.transform2(x, y, "f32", "sum"))


def _host_view(buf, off, n, npdt):
    isz = np.dtype(npdt).itemsize
    return buf.numpy()[off:off + n * isz].view(npdt)


def _rand(orc, rng, dt, n):
    from oracle.oracle import NP
    if dt == "bf16":
        return orc.f32_to_bf16_bits(rng.standard_normal(n).astype(np.float32))
    if np.issubdtype(NP[dt], np.integer):
        info = np.iinfo(NP[dt])
        return rng.integers(info.min, info.max, size=n, dtype=NP[dt], endpoint=True)
    return (rng.standard_normal(n) * 10).astype(NP[dt])


# ---- straight against the reference's own compiled reduce ----------------

@pytest.mark.parametrize("dt", INT_DTS + ["f16", "f32", "f64"])
def test_dropin_vs_reference_build(lib, dt):
    # oracle/_ref/libkfbase_ref.so is KungFu's op.cpp/f16.c/dtype.c compiled
    # from /root/reference (make -C oracle ref; shipped with the tree). Same
    # random inputs (with specials mixed in for floats) through both
    # std_transform_2s, every op the reference accepts for the dtype.
    import ctypes
    from oracle import oracle
    from oracle.oracle import DT, NP
    if not os.path.exists(oracle.REF_LIB):
        pytest.skip("reference build absent (make -C oracle ref)")
    ref = ctypes.CDLL(oracle.REF_LIB)
    ref.std_transform_2.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3
    rng = np.random.default_rng(zlib.crc32(("ref" + dt).encode()))
    n = (1 << 20) + 5
    npdt = NP[dt]
    if dt in INT_DTS:
        info = np.iinfo(npdt)
        x = rng.integers(info.min, info.max, size=n, dtype=npdt, endpoint=True)
        y = rng.integers(info.min, info.max, size=n, dtype=npdt, endpoint=True)
    else:
        x = (rng.standard_normal(n) * 1e3).astype(npdt)
        y = (rng.standard_normal(n) * 1e3).astype(npdt)
        sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, np.finfo(npdt).max,
                       np.finfo(npdt).tiny / 2, 1.0], dtype=npdt)
        idx = rng.integers(0, n, size=4096)
        x[idx] = sp[rng.integers(0, sp.size, size=idx.size)]
        y[idx[::-1]] = sp[rng.integers(0, sp.size, size=idx.size)]
    ops = ["sum"] if dt == "f16" else ["sum", "min", "max", "prod"]
    for op in ops:
        code = {"sum": 0, "min": 1, "max": 2, "prod": 3}[op]
        want = np.empty_like(x)
        got = np.empty_like(x)
        ref.std_transform_2(x.ctypes.data, y.ctypes.data, want.ctypes.data, n, DT[dt], code)
        lib.std_transform_2(x.ctypes.data, y.ctypes.data, got.ctypes.data, n, DT[dt], code)
        assert golden_io.same_bits_or_nan(got, want), (dt, op)


# ---- maximum sizes: 64-bit element indices and the drop-in's int n limit ---

def _windows(n, w=4099):
    """Index windows that straddle the 2^31 / 2^32 element and byte edges."""
    edges = [0, (1 << 31) - w // 2, (1 << 32) - w // 2, n - w]
    return [(max(0, a), min(n, a + w)) for a in edges if a < n]


def test_device_u8_beyond_2pow32(lib, orc, dev):
    # 4 GiB + 37 per input: element (and byte) indices past 2^32 in the vector
    # body and the scalar tail; bit-exact vs the oracle on windows around
    # every 2^31/2^32 edge, and vs u8 wrap-around add over the whole bucket
    from kungfu_amd import _lib
    n = (1 << 32) + 37
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)
    y = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)
    z = torch.empty_like(x)
    rc = lib.kf_bucket_reduce(_lib.ptr_array([x.data_ptr(), y.data_ptr()]), 2,
                              z.data_ptr(), n, 0x00108, 0,
                              torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.kf_last_error()
    torch.cuda.synchronize()
    assert torch.equal(z, x + y)
    for a, b in _windows(n):
        xh, yh = x[a:b].cpu().numpy(), y[a:b].cpu().numpy()
        assert np.array_equal(z[a:b].cpu().numpy(), orc.transform2(xh, yh, "u8", "sum")), (a, b)
    del x, y, z
    torch.cuda.empty_cache()


def test_device_f32_beyond_2pow31_with_avg(lib, orc, dev):
    # 8 GiB + 20 B per input, k = 3 fold (byte offsets past 2^33): the SUM
    # over the whole bucket equals (x + y) + w added in order (each add
    # correctly rounded, so torch's adds are an exact check), and the fused
    # /np fold is bit-exact vs the oracle on windows around every edge
    from kungfu_amd import ops
    n = (1 << 31) + 5
    g = torch.Generator(device=dev).manual_seed(8)
    ins = [torch.randn(n, device=dev, generator=g) for _ in range(3)]
    z = ops.bucket_reduce(ins)
    torch.cuda.synchronize()
    assert torch.equal(z, (ins[0] + ins[1]) + ins[2])
    ops.bucket_reduce_avg(ins, 3, out=z)
    torch.cuda.synchronize()
    for a, b in _windows(n):
        hs = [t[a:b].cpu().numpy() for t in ins]
        assert np.array_equal(z[a:b].cpu().numpy(), orc.reduce_avg(hs, "f32", 3)), (a, b)
    del ins, z
    torch.cuda.empty_cache()


def test_dropin_int_max_n(lib, orc):
    # B1's n is a C int (op.h:17-19): the largest call the reference can make,
    # n = 2^31 - 1 u8 elements through pageable host buffers
    n = (1 << 31) - 1
    rng = np.random.default_rng(9)
    x = rng.integers(0, 256, size=n, dtype=np.uint8)
    y = rng.integers(0, 256, size=n, dtype=np.uint8)
    got = np.empty_like(x)
    lib.std_transform_2(x.ctypes.data, y.ctypes.data, got.ctypes.data, n, 0x00108, 0)
    assert np.array_equal(got, x + y)
    for a, b in _windows(n):
        assert np.array_equal(got[a:b], orc.transform2(x[a:b], y[a:b], "u8", "sum")), (a, b)


@pytest.mark.gpu
def test_bf16_two_input_sum_matches_torch_gpu(dev):
    """Independent cross-check of the bf16 definition (parity unpinned, no
    reference): the HIP two-input bf16 SUM equals torch's own bf16 add on the
    GPU bit for bit (fp32 add, one round to nearest even), incl. the 16-B
    vector path and a ragged tail."""
    from kungfu_amd import ops
    g = torch.Generator(device=dev).manual_seed(5)
    for n in (7, 65536 * 4 + 13):
        x = (torch.randn(n, device=dev, generator=g) * 100).bfloat16()
        y = torch.randn(n, device=dev, generator=g).bfloat16()
        got = ops.bucket_reduce([x, y])
        want = x + y
        assert torch.equal(got.view(torch.int16), want.view(torch.int16)), n


# ---- a15: the reference's TF dtype map on a bf16 tensor ----

def test_bf16_tensor_with_reference_tf_mapping(dev, lib, orc):
    """tensorflow/ops.h:14-33 maps DT_BFLOAT16 to KungFu_FLOAT16, so the
    reference reduces a bf16 tensor's bit patterns as fp16 numbers (per-hop
    fp16 rounding, f16.c:16-50). Asked for that code (ops.to_kungfu_type), the
    device op gives exactly those bits: the oracle's fp16 fold of the raw
    bf16 patterns, k = 2 and k = 4."""
    from kungfu_amd import ops
    g = torch.Generator(device=dev).manual_seed(15)
    for k in (2, 4):
        xs = [torch.randn(100003, device=dev, generator=g).bfloat16() for _ in range(k)]
        out = ops.bucket_reduce(xs, dtype=ops.to_kungfu_type("bfloat16"))
        torch.cuda.synchronize()
        bits = [x.view(torch.int16).cpu().numpy().view(np.uint16) for x in xs]
        want = orc.reduce_k(bits, "f16")
        assert np.array_equal(out.view(torch.int16).cpu().numpy().view(np.uint16), want)
        # the build's own map: fp32 accumulation, one rounding
        own = ops.bucket_reduce(xs)
        torch.cuda.synchronize()
        assert np.array_equal(own.view(torch.int16).cpu().numpy().view(np.uint16),
                              orc.reduce_k(bits, "bf16"))
    with pytest.raises(ValueError):
        ops.bucket_reduce(xs, dtype=ops.to_kungfu_type("float32"))  # 4-byte code, 2-byte data


# ---- B2 under stream capture: the device API is graph-safe ----

def test_b2_ops_capture_and_replay(dev, lib):
    """kf_bucket_reduce / _avg / kf_bucket_div / kf_sma_blend /
    kf_bucket_reduce_batch queued into a HIP graph (torch.cuda.CUDAGraph over
    hipStreamBeginCapture) and replayed give the eager results bit for bit:
    no allocation, no host sync and no pointer query inside the calls."""
    import ctypes
    from kungfu_amd import _lib
    g = torch.Generator(device=dev).manual_seed(11)
    n = 300007
    x, y, w = (torch.randn(n, device=dev, generator=g) for _ in range(3))
    v = torch.randn(n, device=dev, generator=g).bfloat16()
    sb = torch.randn(n, device=dev, generator=g).bfloat16()
    shards = [torch.randn(4099 + 17 * i, device=dev, generator=g) for i in range(8)]
    z, a = torch.empty_like(x), torch.empty_like(x)

    def work(s):
        sp = s.cuda_stream
        assert lib.kf_bucket_reduce(_lib.ptr_array([x.data_ptr(), y.data_ptr(), w.data_ptr()]), 3,
                                    z.data_ptr(), n, 0x20408, 0, sp) == 0
        assert lib.kf_bucket_reduce_avg(_lib.ptr_array([x.data_ptr(), y.data_ptr()]), 2,
                                        a.data_ptr(), n, 0x20408, 3, sp) == 0
        assert lib.kf_bucket_div(w.data_ptr(), n, 0x20408, 4, sp) == 0
        assert lib.kf_sma_blend(v.data_ptr(), sb.data_ptr(), n, 0x20209, 4, 0.1, sp) == 0
        ptrs = [t.data_ptr() for t in shards]
        assert lib.kf_bucket_reduce_batch(
            _lib.ptr_array(ptrs), 1, _lib.ptr_array(ptrs),
            (ctypes.c_size_t * len(shards))(*[t.numel() for t in shards]), len(shards),
            0x20408, 0, 8, sp) == 0

    keep = [t.clone() for t in (w, v, *shards)]
    work(torch.cuda.current_stream())  # eager
    torch.cuda.synchronize()
    want = [t.clone() for t in (z, a, w, v, *shards)]
    for t, k in zip((w, v, *shards), keep):  # restore the in-place inputs
        t.copy_(k)
    z.zero_()
    a.zero_()
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            work(s)
    torch.cuda.synchronize()
    for t, k in zip((w, v, *shards), keep):  # capture ran nothing; be sure
        t.copy_(k)
    graph.replay()
    torch.cuda.synchronize()
    got = (z, a, w, v, *shards)
    for i, (gt, wt) in enumerate(zip(got, want)):
        assert torch.equal(gt, wt), i
