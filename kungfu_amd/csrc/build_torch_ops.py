"""Build kungfu_amd/kungfu_amd_torch_ops<ext>.so (torch_ops.cpp) in-tree with
g++ against torch's headers and libraries, linked to libkungfu_amd.so — no
ninja, no JIT cache, so the built module travels with the tree.

    python kungfu_amd/csrc/build_torch_ops.py
"""
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
NAME = "kungfu_amd_torch_ops"


def target():
    return os.path.join(PKG, NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def build(force=False):
    import torch
    from torch.utils import cpp_extension
    src = os.path.join(HERE, "torch_ops.cpp")
    out = target()
    deps = [src, os.path.join(ROOT, "include", "kungfu_amd.h"), __file__]
    if not force and os.path.exists(out) and all(
            os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-w",
           "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM", "-DTORCH_API_INCLUDE_EXTENSION_H",
           "-DTORCH_EXTENSION_NAME=" + NAME, "-D_GLIBCXX_USE_CXX11_ABI=%d" % abi,
           "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
           "-I", sysconfig.get_paths()["include"]]
    for p in cpp_extension.include_paths():
        cmd += ["-I", p]
    cmd += [src, "-o", out,
            "-L", PKG, "-lkungfu_amd", "-Wl,-rpath,$ORIGIN",
            "-L", torch_lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch_python", "-Wl,-rpath," + torch_lib,
            "-L", "/opt/rocm/lib", "-lamdhip64"]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
