"""TEST INFRASTRUCTURE ONLY -- the CPU parity oracle.

``oracle/wgrt_oracle.c`` restates the reference kernels
``process_rays_kernel_pro_fullColor`` (GPU_ray_tracing_functions.py:833-1246) and
``process_rays_kernel_pro`` (GPU_ray_tracing_functions.py:419-831, the same FSM without
the wavelength axis and with threshold 1e-15) in plain float64 C; this module loads it with ctypes.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it -- as the checker / the timed CPU baseline, never as a product path.

Parity: pinned by the golden fixtures under ``tests/golden`` (generated from the
reference's own kernel code, see ``tests/golden/gen_golden.py``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libwgrt_oracle.so")

_f64p = ctypes.POINTER(ctypes.c_double)
_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u32p = ctypes.POINTER(ctypes.c_uint32)


class _Scene(ctypes.Structure):
    _fields_ = [
        ("ic", _f64p), ("n_ic", ctypes.c_int64),
        ("fc", _f64p), ("fc_offset", _i64p), ("n_fc_slices", ctypes.c_int64),
        ("oc", _f64p), ("oc_offset", _i64p), ("n_oc_slices", ctypes.c_int64),
        ("eff1", _f64p), ("n_eff1", ctypes.c_int64),
        ("eff2", _f64p), ("n_eff2", ctypes.c_int64),
        ("eff_reg_fov", _f64p), ("eff_reg_fov_range", _f64p),
        ("lut_tir", _f64p), ("lut_gap", _f64p),
        ("ic1", _f64p), ("ic2", _f64p), ("ic3", _f64p),
        ("fc1", _f64p), ("fc2", _f64p), ("oc1", _f64p), ("oc2", _f64p),
        ("num_lmd", ctypes.c_int32), ("nx", ctypes.c_int32), ("ny", ctypes.c_int32),
        ("ch5", ctypes.c_int32), ("ch3", ctypes.c_int32),
        ("n_g", ctypes.c_double), ("threshold", ctypes.c_double), ("f32_mask", ctypes.c_int32),
    ]


class _Rays(ctypes.Structure):
    _fields_ = [(k, _f32p) for k in ("x", "y", "m", "n", "lmd", "te", "tm", "dph")]


_lib = None
_lib_ev = None
LIB_EV_PATH = os.path.join(HERE, "build", "libwgrt_oracle_ev.so")


def build(quiet: bool = True) -> str:
    """Compile the oracle with the committed Makefile (gcc + OpenMP)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    return LIB_PATH


def lib(counting: bool = False):
    """The oracle library; ``counting``: its build with the interaction counter
    (oracle/wgrt_oracle_ev.c, ``wgrt_oracle_ev_interactions``)."""
    global _lib, _lib_ev
    if counting:
        if _lib_ev is None:
            if not os.path.exists(LIB_EV_PATH):
                build()
            _lib_ev = _declare(ctypes.CDLL(LIB_EV_PATH))
            _lib_ev.wgrt_oracle_ev_interactions.restype = ctypes.c_int64
            _lib_ev.wgrt_oracle_ev_interactions.argtypes = [ctypes.c_int]
            _lib_ev.wgrt_oracle_ev_set_flags.restype = None
            _lib_ev.wgrt_oracle_ev_set_flags.argtypes = [ctypes.POINTER(ctypes.c_uint8)]
        return _lib_ev
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = _declare(ctypes.CDLL(LIB_PATH))
    return _lib


def _declare(L):
    """ctypes signatures of the oracle library L."""
    L.wgrt_oracle_trace.restype = ctypes.c_int64
    L.wgrt_oracle_trace.argtypes = [ctypes.POINTER(_Scene), ctypes.POINTER(_Rays), ctypes.c_int64,
                                    ctypes.c_int64, _u32p, _f32p, _u32p, ctypes.POINTER(ctypes.c_uint8),
                                    ctypes.c_int]
    L.wgrt_oracle_hypot.restype = ctypes.c_double
    L.wgrt_oracle_hypot.argtypes = [ctypes.c_double, ctypes.c_double]
    L.wgrt_oracle_wrap.restype = ctypes.c_double
    L.wgrt_oracle_wrap.argtypes = [ctypes.c_double]
    L.wgrt_oracle_inside.restype = ctypes.c_int
    L.wgrt_oracle_inside.argtypes = [ctypes.c_double, ctypes.c_double, _f64p, ctypes.c_int64]
    L.wgrt_oracle_xorshift.restype = ctypes.c_uint32
    L.wgrt_oracle_xorshift.argtypes = [ctypes.c_uint32, ctypes.c_int64, _f64p]
    L.wgrt_oracle_inside_many.restype = None
    L.wgrt_oracle_inside_many.argtypes = [_f64p, ctypes.c_int64, _f64p, ctypes.c_int64,
                                          ctypes.POINTER(ctypes.c_int32)]
    return L


def inside_many(points: np.ndarray, poly: np.ndarray) -> np.ndarray:
    """Reference predicate is_inside_or_on_edge (GRTF:63-71) for many points."""
    pts = np.ascontiguousarray(points, dtype=np.float64)
    P = np.ascontiguousarray(poly, dtype=np.float64)
    out = np.zeros(pts.shape[0], dtype=np.int32)
    lib().wgrt_oracle_inside_many(pts.ctypes.data_as(_f64p), pts.shape[0], P.ctypes.data_as(_f64p),
                                  P.shape[0], out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def _p(a, t):
    return a.ctypes.data_as(t)


class OracleScene:
    """Geometry + LUT arrays in the reference's layout, held alive for the C side."""

    def __init__(self, IC, FC, FC_offset, OC, OC_offset, n_g, eff_reg1, eff_reg2, eff_reg_FOV,
                 eff_reg_FOV_range, luts: dict, lut_TIR, lut_gap, f32_mask: int = 0):
        """``f32_mask``: bit k set = LUT k (ic1, ic2, ic3, fc1, fc2, oc1, oc2) is complex64 in the
        reference's run, whose compiled kernel takes the cosine of its float32 angles in float32."""
        if f32_mask not in (0, 0x7F):
            # a mixed set: numba's unified complex128 theta would need a second cosine per table (the
            # carried cos(theta.real) in double, the numerator in float32); the product rejects it too
            raise ValueError("f32_mask must be 0 or 0x7f (a mixed-precision LUT set is not modelled)")
        c = lambda a, dt=np.float64: np.ascontiguousarray(a, dtype=dt)
        # single-wavelength LUT shapes (GRTF:419-427): lut_TIR [NX, NY, 4], ... -> lambda axis of 1
        self.single_lambda = np.ndim(lut_TIR) == 3
        if self.single_lambda:
            luts = dict(luts)
            for name in ("lut_ic1", "lut_ic2", "lut_ic3"):
                luts[name] = np.asarray(luts[name])[None]
            for name in ("lut_fc1", "lut_fc2", "lut_oc1", "lut_oc2"):
                luts[name] = np.asarray(luts[name])[:, None]
            lut_TIR, lut_gap = np.asarray(lut_TIR)[None], np.asarray(lut_gap)[None]
        self._keep = dict(
            IC=c(IC), FC=c(FC), FC_offset=c(FC_offset, np.int64), OC=c(OC), OC_offset=c(OC_offset, np.int64),
            eff1=c(eff_reg1), eff2=c(eff_reg2), fov=c(eff_reg_FOV), rng=c(eff_reg_FOV_range),
            tir=c(lut_TIR), gap=c(lut_gap),
            **{k: c(luts[k], np.complex128) for k in ("lut_ic1", "lut_ic2", "lut_ic3", "lut_fc1",
                                                       "lut_fc2", "lut_oc1", "lut_oc2")})
        k = self._keep
        L, NX, NY = k["tir"].shape[:3]
        self.num_lmd, self.nx, self.ny = L, NX, NY
        self._s = _Scene(
            _p(k["IC"], _f64p), k["IC"].shape[0],
            _p(k["FC"], _f64p), _p(k["FC_offset"], _i64p), k["FC_offset"].shape[0] - 1,
            _p(k["OC"], _f64p), _p(k["OC_offset"], _i64p), k["OC_offset"].shape[0] - 1,
            _p(k["eff1"], _f64p), k["eff1"].shape[0], _p(k["eff2"], _f64p), k["eff2"].shape[0],
            _p(k["fov"], _f64p), _p(k["rng"], _f64p), _p(k["tir"], _f64p), _p(k["gap"], _f64p),
            *[k[n].ctypes.data_as(_f64p) for n in ("lut_ic1", "lut_ic2", "lut_ic3", "lut_fc1",
                                                   "lut_fc2", "lut_oc1", "lut_oc2")],
            L, NX, NY, k["lut_ic1"].shape[-1], k["lut_fc1"].shape[-1], float(n_g),
            1e-15 if self.single_lambda else 0.0, int(f32_mask))

    @classmethod
    def from_geometry(cls, geom, luts, wavelength: int | None = None, f32_mask: int = 0):
        """``wavelength=l``: the single-wavelength scene of wavelength l (process_rays_kernel_pro)."""
        tir, gap = geom.lut_TIR, geom.lut_gap
        if wavelength is not None:
            luts = {k: (v[wavelength] if k in ("lut_ic1", "lut_ic2", "lut_ic3") else v[:, wavelength])
                    for k, v in luts.items() if k.startswith("lut_")}
            tir, gap = tir[wavelength], gap[wavelength]
        return cls(geom.IC, geom.FC, geom.FC_offset, geom.OC, geom.OC_offset, geom.n_g, geom.eff_reg1,
                   geom.eff_reg2, geom.eff_reg_FOV, geom.eff_reg_FOV_range, luts, tir, gap, f32_mask=f32_mask)

    def eb_shape(self):
        if self.single_lambda:
            return (self.ny, self.nx, 80, 120)
        return (self.num_lmd, self.ny, self.nx, 80, 120)

    def trace(self, rays: dict, rng: np.ndarray, eb: np.ndarray, gid_offset: int = 0,
              threads: int = 0, per_ray_bounces: bool = False, fate: bool = False,
              interactions: bool = False, underflow: bool = False):
        """One launch over the shard ``rays`` (mutates ``rng`` and ``eb``).

        Returns ``(total_bounces, per_ray_counts_or_None)``, plus the per-ray fate codes
        when ``fate`` is set, plus (last) the launch's coupler interactions -- the Monte-Carlo
        draws after the in-coupling event, counted by the oracle's event-hook build -- when
        ``interactions`` is set, plus (last) per-ray flags (uint8) of the rays whose trace entered the
        ener-underflow regime (a guard product ener * e below 2^-1000, oracle/wgrt_oracle_ev.c) when
        ``underflow`` is set."""
        cols = {k: np.ascontiguousarray(rays[src], dtype=np.float32) for k, src in
                (("x", "x"), ("y", "y"), ("m", "m"), ("n", "n"), ("lmd", "lmd_num"), ("te", "te"),
                 ("tm", "tm"), ("dph", "delta_phase")) if not (self.single_lambda and k == "lmd")}
        N = cols["x"].shape[0]
        assert rng.dtype == np.uint32 and rng.flags.c_contiguous and rng.shape == (N,)
        assert eb.dtype == np.float32 and eb.flags.c_contiguous and eb.shape == self.eb_shape()
        r = _Rays(*[_p(cols[k], _f32p) if k in cols else None
                    for k in ("x", "y", "m", "n", "lmd", "te", "tm", "dph")])
        counts = np.zeros(N, dtype=np.uint32) if per_ray_bounces else None
        fates = np.zeros(N, dtype=np.uint8) if fate else None
        L = lib(counting=interactions or underflow)
        if interactions:
            L.wgrt_oracle_ev_interactions(1)
        flags = np.zeros(N, dtype=np.uint8) if underflow else None
        if interactions or underflow:
            L.wgrt_oracle_ev_set_flags(flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if underflow else None)
        tot = L.wgrt_oracle_trace(ctypes.byref(self._s), ctypes.byref(r), N, int(gid_offset),
                                  _p(rng, _u32p), _p(eb, _f32p),
                                  _p(counts, _u32p) if counts is not None else None,
                                  fates.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if fate else None,
                                  int(threads))
        out = (int(tot), counts) + ((fates,) if fate else ())
        out = out + ((int(L.wgrt_oracle_ev_interactions(1)),) if interactions else ())
        if underflow:
            L.wgrt_oracle_ev_set_flags(None)
        return out + ((flags,) if underflow else ())
