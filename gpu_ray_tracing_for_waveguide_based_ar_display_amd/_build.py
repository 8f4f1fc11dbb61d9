"""Build the in-tree HIP library ``libwgrt.so`` for gfx950 (hipcc, no JIT cache) and the
PyTorch-ROCm operator library ``_wgrt_torch.so`` over it (g++ against torch's headers).

Called by ``__graft_entry__.build()``; safe to call repeatedly (rebuilds only when a
source is newer than the library).
"""
from __future__ import annotations

import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
REPO = os.path.dirname(PKG)
LIB = os.path.join(PKG, "libwgrt.so")
OPS_LIB = os.path.join(PKG, "_wgrt_torch.so")
OPS_SOURCE = "wgrt_torch.cpp"
SOURCES = ["wgrt_trace.hip", "wgrt_shadow.hip", "wgrt_scene_build.cpp"]
HEADERS = ["wgrt_common.h", "wgrt_device.h", "wgrt_scene.h", "wgrt_scene_build.h"]
ARCH = os.environ.get("WGRT_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: the reference never fuses a*b+c (Python float semantics); keeping
# every product / sum separately rounded is what makes the results bit-reproducible.
# -mllvm -disable-machine-licm: machine-level LICM hoists the 64-bit constants of every
# polynomial in the Jones loop (sincos of the ray start, the RNG draw) into VGPRs held across the
# whole persistent loop -- about 20 VGPRs of the single-trace kernel, and what kept the fused
# kernels at 3 waves per SIMD; without it all four Jones kernels fit 4 waves per SIMD (<= 128
# VGPRs, no spills) and the fused C3 trace runs 11 % faster (single launches unchanged).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
         "-mllvm", "-disable-machine-licm",
         "-Wall", "-Wno-unused-function", f"--offload-arch={ARCH}"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(REPO, "include", h)
                                                                   for h in ("wgrt.h", "wgrt_debug.h")]
    deps.append(os.path.abspath(__file__))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    cmd = [_hipcc(), *FLAGS, "-I", os.path.join(REPO, "include"), "-o", LIB + ".tmp"] + \
          [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd))
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + out.stdout + out.stderr)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_ops(force: bool = False, verbose: bool = False) -> str:
    """``_wgrt_torch.so``: the ``torch.ops.wgrt`` operator library (csrc/wgrt_torch.cpp).  Host code
    only (no kernels), so the host compiler builds it against the installed torch's headers and
    libraries.  libwgrt.so is deliberately not linked: the operator calls the copy the Python layer
    loaded (RTLD_GLOBAL, _lib.load); -z now makes a load without it fail at once."""
    src = os.path.join(CSRC, OPS_SOURCE)
    deps = [src, os.path.join(REPO, "include", "wgrt.h"), os.path.abspath(__file__)]
    if not force and os.path.exists(OPS_LIB) and all(os.path.getmtime(d) <= os.path.getmtime(OPS_LIB) for d in deps):
        return OPS_LIB
    import torch
    from torch.utils import cpp_extension
    cxx = os.environ.get("CXX") or shutil.which("g++") or "c++"
    abi = int(bool(torch._C._GLIBCXX_USE_CXX11_ABI))
    # -isystem: torch's own headers never make the build warn (another torch / g++ version)
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           *[a for p in cpp_extension.include_paths() for a in ("-isystem", p)], "-I", os.path.join(REPO, "include"), src,
           *[f"-L{p}" for p in cpp_extension.library_paths()], "-lc10", "-ltorch", "-ltorch_cpu",
           *[f"-Wl,-rpath,{p}" for p in cpp_extension.library_paths()], "-Wl,-z,now", "-o", OPS_LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    out = subprocess.run(cmd, capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("torch operator library build failed:\n" + out.stdout + out.stderr)
    os.replace(OPS_LIB + ".tmp", OPS_LIB)
    return OPS_LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
    print(build_ops(force=True, verbose=True))
