"""gfx950 ISA of the shipped streaming kernels, read from the built library
(no GPU needed): every 16-B global load and store of a product instantiation
carries the non-temporal bit, and no kernel branches per element.

Both properties were lost once without any test failing: split into bytes,
the 8-bit kernels' loads were re-typed by the compiler and dropped `nt`, and
the bf16 narrow compiled to a divergent branch per element (DESIGN.md §3
notes 1 and 2; 0.72 and 0.79 of the roofline against 0.81 after the fix).
"""
import os
import re
import shutil
import subprocess
from collections import defaultdict

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB = os.path.join(ROOT, "kungfu_amd", "libkungfu_amd.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

# reduce_kernel<T, OP, EPI, KC, BLOCK, UNROLL, LOADNT, STPLAIN>: the product
# instantiations are LOADNT = 1, STPLAIN = 0; the other policy combinations,
# and unroll 1/2/8 of the fp32 SUM k = 2 kernel, exist only for
# tools/tune_reduce.py (kf_set_geometry). (At unroll 1 the compiler merges the
# full-tile and ragged-tile stores into one and drops its nt bit.)
PRODUCT_REDUCE = re.compile(r"^_ZN2kf13reduce_kernelI.*ELi256ELi\d+ELi1ELi0EEEv")
TUNING_ONLY = re.compile(r"^_ZN2kf13reduce_kernelIfLi0ELi0ELi2ELi256ELi[128]E")
STREAMING = ("_ZN2kf20reduce_spread_kernelI", "_ZN2kf10sma_kernelI",
             "_ZN2kf19reduce_batch_kernelI", "_ZN2kf16sma_batch_kernelI")
# the scalar head/tail and the ragged last tile are the only divergent code
MAX_EXEC_BRANCHES = 6
# kernels with the /np epilogue carry two bodies, chosen once on np.pow2
# (EPI_MUL / EPI_DIV, kf_reduce_kernels.hpp), each with its own edges
TWO_BODIES = re.compile(r"^_ZN2kf(\d+(reduce_kernel|reduce_batch_kernel|reduce_spread_kernel)"
                        r"I(f|d|NS_\d+\w+?_tE)Li0ELi1E|10sma_kernelI|16sma_batch_kernelI)")


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not found")
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "kungfu_amd", "csrc")],
                       check=True)
    d = tmp_path_factory.mktemp("isa")
    lib = d / "lib.so"
    shutil.copy(LIB, lib)
    # writes the bundled code objects next to its input: hence the copy
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True)
    objs = sorted(p for p in d.iterdir() if p.name.endswith("gfx950"))
    assert objs, "no gfx950 code object in the library"
    body = defaultdict(list)
    for o in objs:
        asm = subprocess.run([OBJDUMP, "-d", str(o)], check=True, capture_output=True,
                             text=True).stdout
        name = None
        for line in asm.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                name = m.group(1)
            elif name and line.strip():
                body[name].append(line.split("//")[0].strip())
            else:
                name = None
    return body


def product_kernels(kernels):
    return {k: v for k, v in kernels.items()
            if (PRODUCT_REDUCE.match(k) and not TUNING_ONLY.match(k)) or k.startswith(STREAMING)}


def test_product_kernels_found(kernels):
    ks = product_kernels(kernels)
    # 10 dtypes x ops x k forms, the peers fold and the SMA blend
    assert sum(1 for k in ks if k.startswith("_ZN2kf13reduce_kernel")) >= 100
    assert any(k.startswith("_ZN2kf13reduce_kernelIaLi0E") for k in ks)  # i8 SUM
    assert any(k.startswith("_ZN2kf13reduce_kernelINS_6bf16_t") for k in ks)
    assert any(k.startswith(STREAMING[0]) for k in ks)
    assert any(k.startswith(STREAMING[1]) for k in ks)
    # the multi-bucket launch: 12 dtypes plain (k = 1, 2, runtime) + 4 floats / np
    assert sum(1 for k in ks if k.startswith(STREAMING[2])) >= 40
    assert sum(1 for k in ks if k.startswith(STREAMING[3])) == 4  # f32 f64 f16 bf16


def test_streaming_loads_and_stores_are_nontemporal(kernels):
    bad = []
    for name, lines in product_kernels(kernels).items():
        for ins in lines:
            if ins.startswith(("global_load_dwordx4", "global_store_dwordx4")):
                if not re.search(r"\bnt\b", ins):
                    bad.append((name, ins))
                    break
    assert not bad, bad[:5]


def test_no_per_element_branches(kernels):
    bad = []
    for name, lines in product_kernels(kernels).items():
        n = sum(1 for ins in lines if ins.startswith("s_and_saveexec"))
        if n > MAX_EXEC_BRANCHES * (2 if TWO_BODIES.match(name) else 1):
            bad.append((name, n))
    assert not bad, bad[:5]


def test_div_epilogue_is_chosen_once(kernels):
    """The /np epilogue's power-of-two test is made once per kernel, not per
    element: the fp32 k = 2 fused-average kernel stays within a few dozen
    scalar branches (66 when it was made per element)."""
    ks = [k for k in product_kernels(kernels)
          if k.startswith("_ZN2kf13reduce_kernelIfLi0ELi1ELi2ELi256ELi4ELi1ELi0E")]
    assert ks
    for k in ks:
        assert TWO_BODIES.match(k)
        n = sum(1 for ins in kernels[k] if ins.startswith("s_cbranch"))
        assert n <= 24, (k, n)


RUNTIME_K = re.compile(r"^_ZN2kf(13reduce_kernel|19reduce_batch_kernel)I.*?ELi0ELi256ELi4E")


def _serial_loads(lines):
    """The longest run of 16-B loads each followed, before any other memory
    instruction, by `s_waitcnt vmcnt(0)` (load, wait, load, wait, ...)."""
    mem = []
    for ins in lines:  # memory instructions, repeated waits merged
        if ins.startswith(("global_", "s_waitcnt vmcnt")):
            if not (mem and ins.startswith("s_waitcnt") and mem[-1].startswith("s_waitcnt")):
                mem.append(ins)
    best = run = 0
    i = 0
    while i < len(mem):
        if (mem[i].startswith("global_load_dwordx4") and i + 1 < len(mem)
                and mem[i + 1].startswith("s_waitcnt vmcnt(0)")):
            run += 1
            best = max(best, run)
            i += 2
        else:
            run = 0
            i += 1
    return best


def test_runtime_k_fold_keeps_one_vector_in_flight(kernels):
    """The k-input fold reads inputs 2..k-1 one 16-B vector per lane at a time
    (ld_vec_serial: inline-asm load + wait), which measured 0.80 of 8 TB/s at
    k = 3..8 against 0.76-0.79 with an input's four vectors in flight (DESIGN.md
    §10 item 2). A compiler or refactor that reverts to the batched loads
    shows here: every runtime-k reduce / batch kernel has a run of four loads
    (the four vectors of one input) each followed directly by its wait."""
    ks = {k: v for k, v in product_kernels(kernels).items() if RUNTIME_K.match(k)}
    assert len(ks) >= 20, len(ks)
    bad = [(k, _serial_loads(v)) for k, v in ks.items() if _serial_loads(v) < 4]
    assert not bad, bad[:5]


READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


@pytest.fixture(scope="module")
def kernel_meta(tmp_path_factory):
    """name -> {vgpr_count, private_segment_fixed_size, vgpr_spill_count}
    from the code objects' amdhsa metadata notes."""
    if not (os.path.exists(OBJDUMP) and os.path.exists(READELF)):
        pytest.skip("llvm tools not found")
    d = tmp_path_factory.mktemp("meta")
    lib = d / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], check=True, capture_output=True)
    meta = {}
    for o in sorted(p for p in d.iterdir() if p.name.endswith("gfx950")):
        notes = subprocess.run([READELF, "--notes", str(o)], check=True, capture_output=True,
                               text=True).stdout
        cur = {}
        for line in notes.splitlines():
            m = re.match(r"^\s+-?\s*\.(\w+):\s+(\S+)\s*$", line)
            if not m:
                continue
            k, v = m.groups()
            if k == "agpr_count" and line.lstrip().startswith("-"):
                cur = {}
            if k == "name":
                meta[v] = cur
            elif k in ("vgpr_count", "private_segment_fixed_size", "vgpr_spill_count"):
                cur[k] = int(v)
    return meta


def test_streaming_kernels_never_spill(kernel_meta):
    """No product streaming kernel touches scratch: a spill would put private
    memory traffic beside the HBM streams every launch pays for."""
    ks = {k: v for k, v in kernel_meta.items()
          if (PRODUCT_REDUCE.match(k) and not TUNING_ONLY.match(k)) or k.startswith(STREAMING)}
    assert len(ks) >= 100, len(ks)
    bad = [(k, v) for k, v in ks.items()
           if v.get("private_segment_fixed_size", 0) or v.get("vgpr_spill_count", 0)]
    assert not bad, bad[:5]


def test_sma_kernels_keep_eight_waves(kernel_meta):
    """The SMA blends (C5's blend step) stay within 64 VGPRs — 8 waves per
    SIMD, two 256-thread blocks per SIMD of loads in flight. The packed-fp32
    bf16 blend took 68 (7 waves) in one formulation before it was rewritten
    on 32-bit words (DESIGN.md §3, C5's two kernels)."""
    ks = {k: v for k, v in kernel_meta.items() if k.startswith(STREAMING[1]) or
          k.startswith(STREAMING[3])}
    assert len(ks) == 8, sorted(ks)
    bad = [(k, v["vgpr_count"]) for k, v in ks.items() if v["vgpr_count"] > 64]
    assert not bad, bad


def test_bf16_sma_blend_is_packed(kernels):
    """The bf16 blend runs on pairs of lanes in packed fp32 (v_pk_mul_f32 /
    v_pk_add_f32): same IEEE operations as the scalar form, bit-identical
    (tests/test_gpu_parity.py), a quarter fewer VALU instructions."""
    ks = [k for k in kernels if k.startswith(("_ZN2kf10sma_kernelINS_6bf16_t",
                                              "_ZN2kf16sma_batch_kernelINS_6bf16_t"))]
    assert len(ks) == 2, ks
    for k in ks:
        assert sum(1 for ins in kernels[k] if ins.startswith("v_pk_mul_f32")) >= 48, k
        assert sum(1 for ins in kernels[k] if ins.startswith("v_pk_add_f32")) >= 16, k


def test_sma_full_tile_issues_all_loads_first(kernels):
    """Every SMA kernel's full tile (4 vectors of v and 4 of the sum per lane)
    issues its eight 16-B loads back to back, before the first wait on them:
    held to 64 VGPRs the compiler had split the bf16 and fp16 blends' loads
    3 + 5 around a wait, one wave then keeping fewer loads in flight
    (kf_reduce_kernels.hpp KF_SMA_SCHED; profiles/r06/ab_sma_sched_r06p.jsonl:
    0.793 -> 0.816 of 8 TB/s for bf16, same bits)."""
    ks = [k for k in kernels if k.startswith(("_ZN2kf10sma_kernelI", "_ZN2kf16sma_batch_kernelI"))]
    assert len(ks) == 8, ks  # f32 f64 f16 bf16, single and batch
    for k in ks:
        run, best = 0, 0
        for ins in kernels[k]:
            if ins.startswith("global_load_dwordx4"):
                run += 1
                best = max(best, run)
            elif ins.startswith("s_waitcnt") and "vmcnt" in ins:
                run = 0
        assert best >= 8, (k, best)


def test_two_input_reduce_issues_all_loads_first(kernels):
    """Every compile-time k = 2 product reduce (4 vectors of each input per
    lane) issues its eight 16-B loads before the first wait on them
    (kf_reduce_kernels.hpp KF_REDUCE_SCHED and KF_REDUCE_PIN, the latter for
    the 8-bit min/max, whose byte unpacking had split their loads 5 + 3;
    profiles/r06/ab_reduce_sched_r06s.jsonl, ab_reduce_pin_r06z5.jsonl)."""
    pat = re.compile(r"^_ZN2kf(13reduce_kernel|19reduce_batch_kernel)I(\w+?)Li(\d)ELi\d+ELi2ELi256ELi4E")
    checked = 0
    for name, lines in product_kernels(kernels).items():
        m = pat.match(name)
        if not m:
            continue
        run = best = 0
        for ins in lines:
            if ins.startswith("global_load_dwordx4"):
                run += 1
                best = max(best, run)
            elif ins.startswith("s_waitcnt") and "vmcnt" in ins:
                run = 0
        assert best >= 8, (name, best)
        checked += 1
    assert checked >= 40, checked
