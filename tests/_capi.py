"""The plain-C host of the C ABI (tests/capi_host.c): its build recipe and its input format.

``build_capi_host()`` compiles it with gcc against ``include/wgrt.h``, the in-tree
``libwgrt.so`` and the HIP runtime (``__graft_entry__.build()`` runs it, so the binary ships
with the tree like the library); ``write_input()`` writes the record file it reads."""
from __future__ import annotations

import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gpu_ray_tracing_for_waveguide_based_ar_display_amd")
SRC = os.path.join(REPO, "tests", "capi_host.c")
BIN = os.path.join(REPO, "tests", "bin", "capi_host")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

# the eight ray columns the kernel reads, in the order capi_host.c reads them
COLUMNS = ("x", "y", "m", "n", "lmd_num", "te", "tm", "delta_phase")


def build_capi_host(out: str = BIN) -> str:
    """gcc -std=c99 build of tests/capi_host.c into ``out``; returns ``out``."""
    os.makedirs(os.path.dirname(out), exist_ok=True)
    rpath = os.path.relpath(PKG, os.path.dirname(os.path.abspath(out)))
    # -isystem: warnings from the ROCm headers (another ROCm / gcc version) never fail the build; the
    # host program itself is held to -Werror
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
           "-I", os.path.join(REPO, "include"), "-isystem", os.path.join(ROCM, "include"), SRC, "-o", out,
           "-L", PKG, "-lwgrt", f"-Wl,-rpath,$ORIGIN/{rpath}",
           "-L", os.path.join(ROCM, "lib"), "-lamdhip64", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"capi_host build failed ({' '.join(cmd)}):\n{r.stdout}{r.stderr}")
    return out


def _record(f, a, dtype):
    a = np.ascontiguousarray(a, dtype=dtype).ravel()
    np.asarray([a.size], dtype=np.int64).tofile(f)
    a.tofile(f)


def write_input(path: str, geom, luts: dict, rays: dict, rng: np.ndarray, num_iter: int) -> None:
    """The record file capi_host reads: geometry, LUTs (complex128 as interleaved doubles),
    n_g, {ch5, ch3, num_lmd, nx, ny, num_iter}, the eight float32 ray columns, the RNG states."""
    c128 = lambda a: np.ascontiguousarray(a, dtype=np.complex128).view(np.float64)
    tir = np.asarray(geom.lut_TIR)
    nl, nx, ny = tir.shape[:3]
    with open(path, "wb") as f:
        for a in (geom.IC, geom.FC):
            _record(f, a, np.float64)
        _record(f, geom.FC_offset, np.int64)
        _record(f, geom.OC, np.float64)
        _record(f, geom.OC_offset, np.int64)
        for a in (geom.eff_reg1, geom.eff_reg2, geom.eff_reg_FOV, geom.eff_reg_FOV_range):
            _record(f, a, np.float64)
        for k in ("lut_ic1", "lut_ic2", "lut_ic3", "lut_fc1", "lut_fc2", "lut_oc1", "lut_oc2"):
            _record(f, c128(luts[k]), np.float64)
        _record(f, tir, np.float64)
        _record(f, geom.lut_gap, np.float64)
        _record(f, [geom.n_g], np.float64)
        ch5, ch3 = np.asarray(luts["lut_ic1"]).shape[-1], np.asarray(luts["lut_fc1"]).shape[-1]
        _record(f, [ch5, ch3, nl, nx, ny, num_iter], np.int64)
        for k in COLUMNS:
            _record(f, rays[k], np.float32)
        _record(f, rng, np.uint32)


def read_output(path: str, n_rays: int, eb_shape) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(rng_states, matrix_EB, wgrt_trace_stats as uint64[STATS_LEN]) from capi_host's output file."""
    raw = np.fromfile(path, dtype=np.uint8)
    n_eb = int(np.prod(eb_shape))
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd._lib import STATS_LEN
    want = 4 * n_rays + 4 * n_eb + 8 * STATS_LEN
    if raw.size != want:
        raise ValueError(f"capi_host output is {raw.size} bytes, expected {want}")
    rng = raw[:4 * n_rays].view(np.uint32)
    eb = raw[4 * n_rays:4 * n_rays + 4 * n_eb].view(np.float32).reshape(eb_shape)
    stats = raw[4 * n_rays + 4 * n_eb:].view(np.uint64)
    return rng, eb, stats
