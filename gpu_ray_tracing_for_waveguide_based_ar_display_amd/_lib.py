"""Bindings of the in-tree HIP library ``libwgrt.so`` (C ABI: ``include/wgrt.h``).

The scene, ray-setup and diagnostic entry points are bound with ctypes; the trace launch goes
through the PyTorch-ROCm operator ``torch.ops.wgrt.trace`` (``_wgrt_torch.so``, built from
csrc/wgrt_torch.cpp: ``ops()``), which forwards device tensors to ``wgrt_trace_opts`` of the same
loaded library.  There is no CPU fallback: if either library is missing or cannot be loaded,
every entry point raises ``WgrtError``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libwgrt.so")   # the in-tree build, the only one the product binds
OPS_PATH = os.path.join(PKG, "_wgrt_torch.so")   # the torch operator library (csrc/wgrt_torch.cpp)

ABI_VERSION = 7
# include/wgrt.h (the drop-in boundary) and include/wgrt_debug.h (test / profiling hooks)
EXPORTED = ("wgrt_scene_create", "wgrt_scene_create_ex", "wgrt_scene_destroy", "wgrt_scene_get_info",
            "wgrt_trace_fullcolor", "wgrt_trace_fullcolor_ex", "wgrt_trace_single", "wgrt_trace_single_ex",
            "wgrt_trace_opts", "wgrt_scene_reserve", "wgrt_rays_init", "wgrt_scene_classify",
            "wgrt_locator_classify_host", "wgrt_selftest_math", "wgrt_status_string", "wgrt_last_error",
            "wgrt_abi_version", "wgrt_eyebox_payload_floats", "wgrt_eyebox_pack", "wgrt_eyebox_assemble")
EXPORTED_DEBUG = ("wgrt_debug_shadow", "wgrt_debug_scene_copy")


class WgrtError(RuntimeError):
    pass


_d = ctypes.POINTER(ctypes.c_double)
_i64 = ctypes.POINTER(ctypes.c_int64)
_f = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p


class SceneDesc(ctypes.Structure):
    _fields_ = [
        ("IC", _d), ("n_ic", ctypes.c_int64),
        ("FC", _d), ("FC_offset", _i64), ("n_fc_slices", ctypes.c_int64),
        ("OC", _d), ("OC_offset", _i64), ("n_oc_slices", ctypes.c_int64),
        ("n_g", ctypes.c_double),
        ("eff_reg1", _d), ("n_eff_reg1", ctypes.c_int64),
        ("eff_reg2", _d), ("n_eff_reg2", ctypes.c_int64),
        ("eff_reg_FOV", _d), ("eff_reg_FOV_range", _d),
        ("lut_ic1", _d), ("lut_ic2", _d), ("lut_ic3", _d),
        ("lut_fc1", _d), ("lut_fc2", _d), ("lut_oc1", _d), ("lut_oc2", _d),
        ("ch5", ctypes.c_int32), ("ch3", ctypes.c_int32),
        ("lut_TIR", _d), ("lut_gap", _d),
        ("num_lmd", ctypes.c_int32), ("nx", ctypes.c_int32), ("ny", ctypes.c_int32),
    ]


class Rays(ctypes.Structure):
    _fields_ = [(k, _vp) for k in ("x", "y", "gap_x", "gap_y", "pol", "azi", "m", "n", "lmd_num", "te",
                                   "tm", "delta_phase")]


class TraceStats(ctypes.Structure):
    _fields_ = [("bounces", ctypes.c_uint64), ("bad_rays", ctypes.c_uint64),
                ("eyebox_hits", ctypes.c_uint64), ("replayed", ctypes.c_uint64),
                ("handoff_giveups", ctypes.c_uint64), ("interactions", ctypes.c_uint64),
                ("libm_rays", ctypes.c_uint64)]


STATS_LEN = len(TraceStats._fields_)   # int64 words of a wgrt_trace_stats (torch stats tensors)


class DebugOpts(ctypes.Structure):
    """wgrt_debug_opts (include/wgrt_debug.h): per-call test / profiling overrides."""
    _fields_ = [("cert_tol", ctypes.c_double), ("cert_tol32", ctypes.c_double), ("chunk_rays", ctypes.c_int),
                ("timeline", ctypes.c_void_p), ("timeline_waves", ctypes.c_int64),
                ("fail_after_trace", ctypes.c_int), ("handoff_wait_ticks", ctypes.c_uint64)]


class LaunchOpts(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_int), ("variant", ctypes.c_int), ("workgroups", ctypes.c_int),
                ("chunk_order", ctypes.c_void_p), ("n_chunk_order", ctypes.c_int64),
                ("num_iter", ctypes.c_int), ("gid_blocks", ctypes.c_void_p), ("gid_block_rays", ctypes.c_int64),
                ("debug", ctypes.POINTER(DebugOpts)), ("grid_sqrt_k", ctypes.c_double)]


LUT_ORDER = ("lut_ic1", "lut_ic2", "lut_ic3", "lut_fc1", "lut_fc2", "lut_oc1", "lut_oc2")   # lut_f32_angles bits


class SceneOpts(ctypes.Structure):
    _fields_ = [("cell_mm", ctypes.c_double), ("host_build", ctypes.c_int), ("lut_f32_angles", ctypes.c_int)]


class ShadowStats(ctypes.Structure):
    _fields_ = [("decisions", ctypes.c_uint64), ("uncertain", ctypes.c_uint64), ("silent_flips", ctypes.c_uint64),
                ("bounces", ctypes.c_uint64), ("fallbacks", ctypes.c_uint64), ("max_ratio", ctypes.c_double),
                ("max_ratio32", ctypes.c_double),
                ("max_ratio_by_depth", ctypes.c_double * 6), ("decisions_by_depth", ctypes.c_uint64 * 6),
                ("ratio_hist", ctypes.c_uint64 * 20), ("max_ener_ratio", ctypes.c_double), ("max_amp", ctypes.c_double)]


class SceneInfo(ctypes.Structure):
    _fields_ = [("tile_bytes", ctypes.c_int64), ("tiles", ctypes.c_int64),
                ("grid_cells_x", ctypes.c_int64), ("grid_cells_y", ctypes.c_int64),
                ("grid_cell_mm", ctypes.c_double), ("grid_edge_cells", ctypes.c_int64),
                ("n_polygons", ctypes.c_int32), ("device", ctypes.c_int32),
                ("jtile_bytes", ctypes.c_int64), ("nonunitary_blocks", ctypes.c_int64)]


_lib = None
_lib_path = LIB_PATH
_accept_abi = (ABI_VERSION,)


def use_library(path: str, accept_abi=(ABI_VERSION,)) -> None:
    """Tools only (tools/with_lib.py: A/B timing of build variants, tools/ab.py): bind another build of
    the library, optionally of an earlier ABI whose structs are prefixes of this one's, instead of the
    in-tree one.  Must run before anything loads the library; the product never calls it."""
    global _lib_path, _accept_abi
    if _lib is not None:
        raise WgrtError(f"libwgrt is already loaded from {_lib_path}")
    _lib_path, _accept_abi = os.path.abspath(path), tuple(accept_abi)


def loaded_path() -> str:
    """The library file load() binds (the in-tree build unless a tool chose another)."""
    return _lib_path


def load():
    """Load libwgrt.so (never builds implicitly: build with ``__graft_entry__.build()``)."""
    global _lib
    if _lib is not None:
        return _lib
    path = _lib_path
    if not os.path.exists(path):
        raise WgrtError(f"{path} not found: the HIP library is not built "
                        "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    try:
        # RTLD_GLOBAL: the torch operator library (ops()) resolves the C ABI against this copy
        L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:
        raise WgrtError(f"cannot load {path}: {e}") from e
    # the ABI first: an accepted earlier build (tools only, use_library) may lack later entry points
    L.wgrt_abi_version.restype = ctypes.c_int
    L.wgrt_abi_version.argtypes = []
    abi = L.wgrt_abi_version()
    if abi not in _accept_abi:
        raise WgrtError(f"libwgrt ABI {abi} not in the accepted {_accept_abi}")
    st = ctypes.c_int
    L.wgrt_scene_create.restype = st
    L.wgrt_scene_create.argtypes = [ctypes.POINTER(SceneDesc), ctypes.c_int, ctypes.POINTER(_vp)]
    L.wgrt_scene_create_ex.restype = st
    L.wgrt_scene_create_ex.argtypes = [ctypes.POINTER(SceneDesc), ctypes.c_int, ctypes.POINTER(SceneOpts),
                                       ctypes.POINTER(_vp)]
    L.wgrt_scene_destroy.restype = st
    L.wgrt_scene_destroy.argtypes = [_vp]
    L.wgrt_scene_get_info.restype = st
    L.wgrt_scene_get_info.argtypes = [_vp, ctypes.POINTER(SceneInfo)]
    L.wgrt_trace_fullcolor.restype = st
    L.wgrt_trace_fullcolor.argtypes = [_vp, ctypes.POINTER(Rays), ctypes.c_int64, ctypes.c_int64, _vp, _vp,
                                       _vp, _vp, _vp]
    L.wgrt_trace_fullcolor_ex.restype = st
    L.wgrt_trace_fullcolor_ex.argtypes = [_vp, ctypes.POINTER(Rays), ctypes.c_int64, ctypes.c_int64, _vp,
                                          _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int]
    L.wgrt_trace_single.restype = st
    L.wgrt_trace_single.argtypes = L.wgrt_trace_fullcolor.argtypes
    L.wgrt_trace_single_ex.restype = st
    L.wgrt_trace_single_ex.argtypes = L.wgrt_trace_fullcolor_ex.argtypes
    L.wgrt_trace_opts.restype = st
    L.wgrt_trace_opts.argtypes = [_vp, ctypes.POINTER(Rays), ctypes.c_int64, ctypes.c_int64, _vp, _vp, _vp, _vp,
                                  _vp, ctypes.POINTER(LaunchOpts)]
    L.wgrt_rays_init.restype = st
    L.wgrt_rays_init.argtypes = [_vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _vp, ctypes.c_int32,
                                 ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(Rays), _vp, _vp]
    L.wgrt_scene_classify.restype = st
    L.wgrt_scene_classify.argtypes = [_vp, _vp, ctypes.c_int64, _vp, _vp]
    L.wgrt_locator_classify_host.restype = st
    L.wgrt_locator_classify_host.argtypes = [ctypes.POINTER(SceneDesc), ctypes.c_double, _vp, ctypes.c_int64, _vp]
    L.wgrt_selftest_math.restype = st
    L.wgrt_selftest_math.argtypes = [_vp, _vp, ctypes.c_int64, _vp, _vp]
    L.wgrt_scene_reserve.restype = st
    L.wgrt_scene_reserve.argtypes = [_vp, ctypes.c_int64, ctypes.c_int, _vp]
    if abi >= 6:   # the strong-scaling gather's row-copy kernels (ABI 6)
        L.wgrt_eyebox_payload_floats.restype = ctypes.c_int64
        L.wgrt_eyebox_payload_floats.argtypes = [ctypes.c_int64]
        L.wgrt_eyebox_pack.restype = st
        L.wgrt_eyebox_pack.argtypes = [_vp, ctypes.c_int64, _vp, _vp, _vp, ctypes.c_int64, ctypes.c_int64, _vp, _vp]
        L.wgrt_eyebox_assemble.restype = st
        L.wgrt_eyebox_assemble.argtypes = [_vp, ctypes.c_int64, _vp, ctypes.c_int32, ctypes.c_int64, _vp, _vp, _vp]
    # test / profiling hooks (include/wgrt_debug.h)
    L.wgrt_debug_shadow.restype = st
    L.wgrt_debug_shadow.argtypes = [_vp, ctypes.POINTER(Rays), ctypes.c_int64, ctypes.c_int64, ctypes.c_int, _vp,
                                    _vp, _vp, _vp]
    L.wgrt_debug_scene_copy.restype = st
    L.wgrt_debug_scene_copy.argtypes = [_vp, ctypes.c_int, _vp, ctypes.c_int64]
    L.wgrt_status_string.restype = ctypes.c_char_p
    L.wgrt_status_string.argtypes = [ctypes.c_int]
    L.wgrt_last_error.restype = ctypes.c_char_p
    L.wgrt_last_error.argtypes = []
    _lib = L
    return L


_ops = None


def ops():
    """``torch.ops.wgrt``: the trace operator (``_wgrt_torch.so``), loaded after ``libwgrt.so``,
    whose C ABI it calls (never builds implicitly)."""
    global _ops
    if _ops is not None:
        return _ops
    load()
    if not os.path.exists(OPS_PATH):
        raise WgrtError(f"{OPS_PATH} not found: the torch operator library is not built "
                        "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    import torch
    try:
        torch.ops.load_library(OPS_PATH)
    except OSError as e:
        raise WgrtError(f"cannot load {OPS_PATH}: {e}") from e
    _ops = torch.ops.wgrt
    return _ops


def check(status: int, what: str):
    if status != 0:
        L = load()
        raise WgrtError(f"{what}: {L.wgrt_status_string(status).decode()} -- {L.wgrt_last_error().decode()}")


def _ptr(a: np.ndarray, t=_d):
    return a.ctypes.data_as(t)


def make_desc(IC, FC, FC_offset, OC, OC_offset, n_g, eff_reg1, eff_reg2, eff_reg_FOV, eff_reg_FOV_range,
          lut_ic1, lut_ic2, lut_ic3, lut_fc1, lut_fc2, lut_oc1, lut_oc2, lut_TIR, lut_gap):
    """Validate the reference's scene arrays and pack them into a ``wgrt_scene_desc``.

    Returns ``(desc, keepalive, (num_lmd, nx, ny, n_fc_slices, n_oc_slices))``; keep the
    second item alive while the descriptor is in use.  Single-wavelength LUTs (the
    ``process_rays_kernel_pro`` shapes: lut_TIR [NX, NY, 4], lut_fc1 [nFC, NX, NY, C], ...)
    are accepted and described as num_lmd = 1 (the same memory layout).  Raises ValueError on any shape
    mismatch (the reference would index out of bounds instead).
    """
    if np.ndim(lut_TIR) == 3:   # single-wavelength LUTs (GRTF:419-427): add a lambda axis of 1
        lut_ic1, lut_ic2, lut_ic3, lut_TIR, lut_gap = (np.asarray(a)[None] for a in
                                                       (lut_ic1, lut_ic2, lut_ic3, lut_TIR, lut_gap))
        lut_fc1, lut_fc2, lut_oc1, lut_oc2 = (np.asarray(a)[:, None] for a in (lut_fc1, lut_fc2, lut_oc1, lut_oc2))
    f64 = lambda a: np.ascontiguousarray(np.asarray(a), dtype=np.float64)
    c128 = lambda a: np.ascontiguousarray(np.asarray(a), dtype=np.complex128)
    i64 = lambda a: np.ascontiguousarray(np.asarray(a), dtype=np.int64)
    k = dict(IC=f64(IC), FC=f64(FC), FC_offset=i64(FC_offset), OC=f64(OC), OC_offset=i64(OC_offset),
             eff1=f64(eff_reg1), eff2=f64(eff_reg2), fov=f64(eff_reg_FOV), fovr=f64(eff_reg_FOV_range),
             ic1=c128(lut_ic1), ic2=c128(lut_ic2), ic3=c128(lut_ic3), fc1=c128(lut_fc1),
             fc2=c128(lut_fc2), oc1=c128(lut_oc1), oc2=c128(lut_oc2), tir=f64(lut_TIR), gap=f64(lut_gap))
    for name in ("IC", "FC", "OC", "eff1", "eff2"):
        a = k[name]
        if a.ndim != 2 or a.shape[1] != 2:
            raise ValueError(f"{name} must have shape (V, 2), got {a.shape}")
    if k["tir"].ndim != 4 or k["tir"].shape[-1] != 4:
        raise ValueError(f"lut_TIR must have shape (L, NX, NY, 4), got {k['tir'].shape}")
    nl, nx, ny = k["tir"].shape[:3]
    nfc, noc = k["FC_offset"].shape[0] - 1, k["OC_offset"].shape[0] - 1
    want = {"gap": (nl, nx, ny, 8), "fov": (nx, ny, 4, 2), "fovr": (nx, ny, 4)}
    for name, shp in want.items():
        if k[name].shape != shp:
            raise ValueError(f"{name}: shape {k[name].shape} != {shp}")
    for name in ("ic1", "ic2", "ic3"):
        if k[name].shape[:3] != (nl, nx, ny):
            raise ValueError(f"lut_{name}: shape {k[name].shape} does not match grid {(nl, nx, ny)}")
    for name, ns in (("fc1", nfc), ("fc2", nfc), ("oc1", noc), ("oc2", noc)):
        if k[name].shape[:4] != (ns, nl, nx, ny):
            raise ValueError(f"lut_{name}: shape {k[name].shape} does not match {(ns, nl, nx, ny)}")
    if k["FC_offset"][-1] > k["FC"].shape[0] or k["OC_offset"][-1] > k["OC"].shape[0]:
        raise ValueError("FC_offset / OC_offset point past the vertex arrays")
    ch5 = k["ic1"].shape[-1]
    if not (k["ic2"].shape[-1] == k["ic3"].shape[-1] == k["oc1"].shape[-1] == k["oc2"].shape[-1] == ch5):
        raise ValueError("ic*/oc* LUTs must share one channel count")
    ch3 = k["fc1"].shape[-1]
    if k["fc2"].shape[-1] != ch3:
        raise ValueError("fc1/fc2 LUTs must share one channel count")
    desc = SceneDesc(
        _ptr(k["IC"]), k["IC"].shape[0], _ptr(k["FC"]), _ptr(k["FC_offset"], _i64), nfc,
        _ptr(k["OC"]), _ptr(k["OC_offset"], _i64), noc, float(n_g),
        _ptr(k["eff1"]), k["eff1"].shape[0], _ptr(k["eff2"]), k["eff2"].shape[0],
        _ptr(k["fov"]), _ptr(k["fovr"]),
        _ptr(k["ic1"]), _ptr(k["ic2"]), _ptr(k["ic3"]), _ptr(k["fc1"]), _ptr(k["fc2"]),
        _ptr(k["oc1"]), _ptr(k["oc2"]), ch5, ch3, _ptr(k["tir"]), _ptr(k["gap"]), nl, nx, ny)
    return desc, k, (nl, nx, ny, nfc, noc)


class Scene:
    """Device-resident geometry + packed LUT tiles (``wgrt_scene_create``).

    Arguments are the reference's scene arrays (couplers_coor.py:740-750 and the
    seven LUTs of gpu_ray_tracing_pro_fullColor.py:28-34), as host numpy arrays.
    """

    def __init__(self, IC, FC, FC_offset, OC, OC_offset, n_g, eff_reg1, eff_reg2, eff_reg_FOV,
                 eff_reg_FOV_range, lut_ic1, lut_ic2, lut_ic3, lut_fc1, lut_fc2, lut_oc1, lut_oc2,
                 lut_TIR, lut_gap, device: int = 0, cell_mm: float = 0.0, host_build: bool = False,
                 lut_f32_angles: int | None = None):
        """``cell_mm`` / ``host_build`` / ``lut_f32_angles``: wgrt_scene_opts (0 / False: the defaults;
        ``lut_f32_angles=None``: bit k set for each LUT given in single precision, luts.lut_f32_mask)."""
        L = load()
        desc, _keep, (nl, nx, ny, nfc, noc) = make_desc(
            IC, FC, FC_offset, OC, OC_offset, n_g, eff_reg1, eff_reg2, eff_reg_FOV, eff_reg_FOV_range,
            lut_ic1, lut_ic2, lut_ic3, lut_fc1, lut_fc2, lut_oc1, lut_oc2, lut_TIR, lut_gap)
        h = _vp()
        if lut_f32_angles is None:
            from .luts import lut_f32_mask
            lut_f32_angles = lut_f32_mask(dict(zip(LUT_ORDER, (lut_ic1, lut_ic2, lut_ic3, lut_fc1, lut_fc2,
                                                               lut_oc1, lut_oc2))))
        opts = SceneOpts(float(cell_mm), 1 if host_build else 0, int(lut_f32_angles))
        self.lut_f32_angles = int(lut_f32_angles)
        check(L.wgrt_scene_create_ex(ctypes.byref(desc), int(device), ctypes.byref(opts), ctypes.byref(h)),
              "wgrt_scene_create")
        self._h = h
        self.single_lambda = np.ndim(lut_TIR) == 3
        self.device = int(device)
        self.num_lmd, self.nx, self.ny = nl, nx, ny
        self.n_fc_slices, self.n_oc_slices = nfc, noc
        self.n_g = float(n_g)

    @classmethod
    def from_geometry(cls, geom, luts: dict, device: int = 0, wavelength: int | None = None, **opts):
        """Scene of a geometry + LUT set.  ``wavelength=l`` builds the single-wavelength scene
        of wavelength l (the arrays process_rays_kernel_pro takes, luts.single_wavelength);
        ``opts``: ``cell_mm`` / ``host_build`` (wgrt_scene_opts)."""
        tir, gap = geom.lut_TIR, geom.lut_gap
        if wavelength is not None:
            from .luts import single_wavelength
            luts, tir, gap = single_wavelength(luts, tir, gap, wavelength)
        return cls(geom.IC, geom.FC, geom.FC_offset, geom.OC, geom.OC_offset, geom.n_g, geom.eff_reg1,
                   geom.eff_reg2, geom.eff_reg_FOV, geom.eff_reg_FOV_range, luts["lut_ic1"], luts["lut_ic2"],
                   luts["lut_ic3"], luts["lut_fc1"], luts["lut_fc2"], luts["lut_oc1"], luts["lut_oc2"],
                   tir, gap, device=device, **opts)

    @property
    def handle(self):
        if self._h is None:
            raise WgrtError("scene destroyed")
        return self._h

    def info(self) -> dict:
        inf = SceneInfo()
        check(load().wgrt_scene_get_info(self.handle, ctypes.byref(inf)), "wgrt_scene_get_info")
        return {f: getattr(inf, f) for f, _ in SceneInfo._fields_}

    def debug_copy(self, which: str) -> np.ndarray:
        """Host copy of a device structure (wgrt_debug_scene_copy): "cells" (uint64 [ncy, ncx]),
        "tiles" / "jtiles" (float64 [tiles, doubles per tile])."""
        inf = self.info()
        if which == "cells":
            out = np.empty((inf["grid_cells_y"], inf["grid_cells_x"]), np.uint64)
        else:
            per = inf["tile_bytes" if which == "tiles" else "jtile_bytes"] // 8
            out = np.empty((inf["tiles"], per), np.float64)
        k = {"cells": 0, "tiles": 1, "jtiles": 2}[which]
        check(load().wgrt_debug_scene_copy(self.handle, k, out.ctypes.data, out.nbytes), "wgrt_debug_scene_copy")
        return out

    def eb_shape(self):
        if self.single_lambda:   # process_rays_kernel_pro's matrix_EB [NY, NX, 80, 120]
            return (self.ny, self.nx, 80, 120)
        return (self.num_lmd, self.ny, self.nx, 80, 120)

    def close(self):
        if getattr(self, "_h", None) is not None:
            load().wgrt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def locator_classify_host(geom, luts, xy: np.ndarray, cell_mm: float = 0.125) -> np.ndarray:
    """Host replica of the kernels' polygon locator (``wgrt_locator_classify_host``): bit k of
    the result is is_inside_or_on_edge(point, polygon k) (0 eff_reg1, 1 eff_reg2, 2 IC,
    3.. FC slices, then OC slices).  Needs no GPU."""
    L = load()
    desc, keep, _ = make_desc(geom.IC, geom.FC, geom.FC_offset, geom.OC, geom.OC_offset, geom.n_g,
                              geom.eff_reg1, geom.eff_reg2, geom.eff_reg_FOV, geom.eff_reg_FOV_range,
                              luts["lut_ic1"], luts["lut_ic2"], luts["lut_ic3"], luts["lut_fc1"],
                              luts["lut_fc2"], luts["lut_oc1"], luts["lut_oc2"], geom.lut_TIR, geom.lut_gap)
    pts = np.ascontiguousarray(xy, dtype=np.float64)
    out = np.zeros(pts.shape[0], dtype=np.uint64)
    check(L.wgrt_locator_classify_host(ctypes.byref(desc), float(cell_mm), pts.ctypes.data_as(_vp), pts.shape[0],
                                       out.ctypes.data_as(_vp)),
          "wgrt_locator_classify_host")
    return out

