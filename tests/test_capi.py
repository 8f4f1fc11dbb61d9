"""CPU-side checks of the C ABI (no kernel launches): the library loads, exports every
symbol include/wgrt.h declares, and rejects malformed scenes before touching the GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="wgrt.h"):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wgrt_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return _lib.load()


def test_header_declares_the_bound_symbols():
    assert declared_symbols() == sorted(_lib.EXPORTED)
    assert declared_symbols("wgrt_debug.h") == sorted(_lib.EXPORTED_DEBUG)


def test_library_exports_every_declared_symbol(lib):
    for name in declared_symbols() + declared_symbols("wgrt_debug.h"):
        assert hasattr(lib, name), name


def test_no_process_wide_debug_setters(lib):
    """The ABI-2 process-wide test setters are gone: every hook is per call (wgrt_debug_opts)."""
    for name in ("wgrt_debug_set_cert_tol", "wgrt_debug_set_cert_tol32", "wgrt_debug_set_timeline",
                 "wgrt_debug_set_chunk", "wgrt_debug_set_host_scene"):
        assert not hasattr(lib, name), name


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the ABI structs have the C compiler's sizes and field offsets (gcc on the
    headers themselves, x86-64 host ABI)."""
    structs = {"wgrt_trace_stats": _lib.TraceStats, "wgrt_launch_opts": _lib.LaunchOpts,
               "wgrt_debug_opts": _lib.DebugOpts, "wgrt_scene_opts": _lib.SceneOpts,
               "wgrt_scene_info": _lib.SceneInfo, "wgrt_scene_desc": _lib.SceneDesc, "wgrt_rays": _lib.Rays,
               "wgrt_shadow_stats": _lib.ShadowStats}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "wgrt_debug.h"', "int main(void) {"]
    for c, py in structs.items():
        lines.append(f'printf("{c} %zu\\n", sizeof({c}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{c}.{f} %zu\\n", offsetof({c}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n") if l)
    for c, py in structs.items():
        assert int(got[c]) == ctypes.sizeof(py), c
        for f, _ in py._fields_:
            assert int(got[f"{c}.{f}"]) == getattr(py, f).offset, f"{c}.{f}"


@pytest.fixture(scope="module")
def wgrt_ops(lib):
    torch = pytest.importorskip("torch")
    if not os.path.exists(_lib.OPS_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return torch, _lib.ops()


def test_torch_operator_schema(wgrt_ops):
    """The PyTorch-ROCm operator the trace launches go through (csrc/wgrt_torch.cpp) is registered
    with the reference kernel's in/out buffers marked as mutated."""
    torch, ops = wgrt_ops
    schema = str(ops.trace.default._schema)
    assert schema.startswith("wgrt::trace(int scene, Tensor x, Tensor y, Tensor m, Tensor n, Tensor? lmd_num")
    for arg in ("Tensor(a!) rng_states", "Tensor(b!) matrix_EB", "Tensor(c!)? stats", "Tensor(d!)? per_ray_bounces"):
        assert arg in schema, arg
    assert schema.endswith("-> int")


def test_torch_operator_calls_only_the_c_abi(wgrt_ops):
    """The operator library links no copy of the kernels: its only wgrt_ symbols are C-ABI entry
    points, resolved against the libwgrt.so the Python layer loaded."""
    out = subprocess.run(["nm", "-D", "--undefined-only", _lib.OPS_PATH], capture_output=True, text=True, check=True)
    used = sorted({l.split()[-1] for l in out.stdout.splitlines() if l.split() and l.split()[-1].startswith("wgrt_")})
    assert used == ["wgrt_scene_get_info", "wgrt_trace_opts"]
    assert set(used) <= set(_lib.EXPORTED)
    defined = subprocess.run(["nm", "-D", "--defined-only", _lib.OPS_PATH], capture_output=True, text=True, check=True)
    assert "wgrt_" not in defined.stdout


def test_torch_operator_rejects_null_scene(wgrt_ops):
    torch, ops = wgrt_ops
    t = torch.zeros(4)
    with pytest.raises(RuntimeError, match="NULL scene"):
        ops.trace(0, t, t, t, t, t, t, t, t, torch.zeros(4, dtype=torch.int32), torch.zeros(9600), None, None,
                  4, 0, 0, 0, 0, 0, None, 1, None, 0, 0, 0.0)


def test_abi_version_and_status_strings(lib):
    assert lib.wgrt_abi_version() == _lib.ABI_VERSION
    assert lib.wgrt_status_string(0) == b"ok"
    assert lib.wgrt_status_string(1) == b"invalid argument"


def _desc_from(geom, luts, **over):
    keep = []

    def p(a, t=np.float64, ct=ctypes.c_double):
        a = np.ascontiguousarray(a, dtype=t)
        keep.append(a)
        return a.ctypes.data_as(ctypes.POINTER(ct))
    d = _lib.SceneDesc(
        p(geom.IC), len(geom.IC), p(geom.FC), p(geom.FC_offset, np.int64, ctypes.c_int64),
        len(geom.FC_offset) - 1, p(geom.OC), p(geom.OC_offset, np.int64, ctypes.c_int64),
        len(geom.OC_offset) - 1, geom.n_g, p(geom.eff_reg1), len(geom.eff_reg1), p(geom.eff_reg2),
        len(geom.eff_reg2), p(geom.eff_reg_FOV), p(geom.eff_reg_FOV_range),
        *[p(luts[k], np.complex128) for k in ("lut_ic1", "lut_ic2", "lut_ic3", "lut_fc1", "lut_fc2",
                                              "lut_oc1", "lut_oc2")],
        42, 26, p(geom.lut_TIR), p(geom.lut_gap), 3, geom.eff_reg_FOV.shape[0], geom.eff_reg_FOV.shape[1])
    for k, v in over.items():
        setattr(d, k, v)
    return d, keep


@pytest.mark.parametrize("field,value,msg", [
    ("ch5", 30, b"channels"),
    ("ch3", 10, b"channels"),
    ("nx", 0, b"positive"),
    ("n_fc_slices", 40, b"too many"),
    ("lut_TIR", None, b"NULL"),
])
def test_scene_create_validates_before_gpu(lib, field, value, msg):
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
    g = design_geometry(3, 3)
    L = synthetic_luts(g)
    d, keep = _desc_from(g, L, **{field: value})
    h = ctypes.c_void_p()
    st = lib.wgrt_scene_create(ctypes.byref(d), 0, ctypes.byref(h))
    assert st == 1
    assert msg in lib.wgrt_last_error()
    assert not h.value


@pytest.mark.parametrize("mask", [0x01, 0x3f, 0x40, 0x80])
def test_scene_create_rejects_mixed_f32_luts(lib, mask):
    """lut_f32_angles must be 0 or 0x7f (wgrt_scene_opts): a mixed-precision LUT set would need numba's
    unified complex128 angle for the carried cosine and float32 for a table's own; it is
    refused before any GPU call."""
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
    g = design_geometry(3, 3)
    d, keep = _desc_from(g, synthetic_luts(g))
    opts = _lib.SceneOpts(0.0, 0, mask)
    h = ctypes.c_void_p()
    st = lib.wgrt_scene_create_ex(ctypes.byref(d), 0, ctypes.byref(opts), ctypes.byref(h))
    assert st == (1 if mask & ~0x7f else 4) and not h.value
    assert (b"beyond the 7" if mask & ~0x7f else b"mixed-precision") in lib.wgrt_last_error()


def test_trace_rejects_null_scene(lib):
    r = _lib.Rays()
    assert lib.wgrt_trace_fullcolor(None, ctypes.byref(r), 10, 0, None, None, None, None, None) == 1
    assert lib.wgrt_trace_single(None, ctypes.byref(r), 10, 0, None, None, None, None, None) == 1
    assert lib.wgrt_trace_single_ex(None, ctypes.byref(r), 10, 0, None, None, None, None, None, 0, 0) == 1


def test_single_wavelength_desc_matches_full_colour_slice():
    """Single-wavelength LUT shapes (process_rays_kernel_pro, GRTF:419-427) are described as a
    one-wavelength scene whose memory is exactly that wavelength's slice of the full set."""
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
    from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import single_wavelength, synthetic_luts
    g = design_geometry(4, 3)
    L = synthetic_luts(g, seed=1)
    S, tir, gap = single_wavelength(L, g.lut_TIR, g.lut_gap, 2)
    assert S["lut_ic1"].shape == (4, 3, 42) and S["lut_fc1"].shape == (g.num_fc_slices, 4, 3, 26)
    assert tir.shape == (4, 3, 4) and gap.shape == (4, 3, 8)
    args = (g.IC, g.FC, g.FC_offset, g.OC, g.OC_offset, g.n_g, g.eff_reg1, g.eff_reg2, g.eff_reg_FOV,
            g.eff_reg_FOV_range)
    d, keep, dims = _lib.make_desc(*args, S["lut_ic1"], S["lut_ic2"], S["lut_ic3"], S["lut_fc1"], S["lut_fc2"],
                                   S["lut_oc1"], S["lut_oc2"], tir, gap)
    assert dims == (1, 4, 3, g.num_fc_slices, g.num_oc_slices)
    np.testing.assert_array_equal(keep["fc1"][:, 0], L["lut_fc1"][:, 2])
    np.testing.assert_array_equal(keep["tir"][0], g.lut_TIR[2])
