"""Waveguide coupler geometry and per-FoV hop / TIR tables (host side, one-shot).

Restates ``couplers_coor_full_color`` (reference ``couplers_coor.py:122-750``)
without shapely: the only shapely operations on the path are

* ``Polygon.intersection(band)`` of a convex hull with a horizontal band
  (CC:431, CC:578) -> Sutherland-Hodgman clipping of a convex polygon by two
  half-planes (``_clip_convex_band``), returned as a *closed* ring like
  shapely's ``exterior.coords``;
* ``LineString.simplify(1e-3)`` of an open hull chain (CC:403, CC:553) ->
  Douglas-Peucker (``_douglas_peucker``);
* ``make_valid`` / ``polygon_to_xy`` (CC:393-394, CC:449) feed outputs that
  are never returned and are dropped here.

The arithmetic of every table that reaches the kernel without passing through
shapely (IC ring, ``lut_gap``, ``lut_TIR``, ``eff_reg_FOV``,
``eff_reg_FOV_range``) keeps the reference's per-element operation order, so
those arrays are bit-identical to the reference's.  Polygon vertices that go
through clipping / simplification are "parity unpinned" (no shapely anywhere in
this image); the golden fixtures therefore pin the kernel *given* this
geometry.

Public entry point: :func:`couplers_coor_full_color` returns the same 37-tuple
as the reference (CC:740-750).  :func:`design_geometry` returns the same data
as a :class:`CouplerGeometry` with named fields.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import math

import numpy as np
from scipy.spatial import ConvexHull

DEG = np.pi / 180


@dataclass(frozen=True)
class WaveguideDesign:
    """Design constants of the full-colour waveguide (CC:124-198)."""

    aspect: float = 4 / 3
    fov_x: float = 18 * DEG
    hull_fov_samples: int = 50          # FoV samples used to trace the FC hull (CC:128-129)
    wavelengths_nm: tuple = (465, 532, 630)
    n_glass: float = 1.9
    n_air: float = 1.0
    glass_x: float = 60.0               # half-width of the clipping band (CC:138, CC:421)
    thickness: float = 0.7
    num_fc: int = 7
    num_oc: int = 6
    ic_radius: float = 2.0
    ic_center: tuple = (-28.0, 15.0)
    ic_points: int = 100
    eyebox: tuple = (12.0, 8.0)
    eye_relief: float = -20.0
    eyebox_center: tuple = (0.0, 15.0)
    period_ic: float = 388.0
    azimuth_ic: float = -38 * DEG
    period_oc: float = 388.0
    azimuth_oc: float = -142 * DEG

    @property
    def fov_y(self) -> float:
        return self.fov_x / self.aspect


@dataclass
class CouplerGeometry:
    """Named view of the reference's 37-tuple (CC:740-750)."""

    IC: np.ndarray
    FC: np.ndarray
    FC_offset: np.ndarray
    OC: np.ndarray
    OC_offset: np.ndarray
    eff_reg1: np.ndarray
    eff_reg2: np.ndarray
    eff_reg_FOV: np.ndarray
    eff_reg_FOV_range: np.ndarray
    lut_TIR: np.ndarray
    lut_gap: np.ndarray
    lut_Fresnel: np.ndarray
    Lambda_ic: float
    phi_ic: float
    Lambda_fc: float
    phi_fc: float
    Lambda_oc: float
    phi_oc: float
    n_g: float
    lmd: np.ndarray
    angles: dict = field(default_factory=dict)   # th_in_ic ... th_out_oc_glow
    kvec: dict = field(default_factory=dict)     # kx0 ... ky_fc

    _ANGLE_KEYS = ("th_in_ic", "phi_in_ic", "th_out_ic", "phi_out_ic", "th_out_fc",
                   "phi_out_fc", "th_out_ic2", "phi_out_ic2", "th_out_oc", "phi_out_oc",
                   "th_out_oc_glow")
    _K_KEYS = ("kx0", "ky0", "kx_ic", "ky_ic", "kx_fc", "ky_fc")

    def as_tuple(self) -> tuple:
        head = (self.IC, self.FC, self.FC_offset, self.OC, self.OC_offset,
                self.eff_reg1, self.eff_reg2, self.eff_reg_FOV, self.eff_reg_FOV_range,
                self.lut_TIR, self.lut_gap, self.lut_Fresnel,
                self.Lambda_ic, self.phi_ic, self.Lambda_fc, self.phi_fc,
                self.Lambda_oc, self.phi_oc, self.n_g, self.lmd)
        return (head + tuple(self.angles[k] for k in self._ANGLE_KEYS)
                + tuple(self.kvec[k] for k in self._K_KEYS))

    @property
    def num_fc_slices(self) -> int:
        return len(self.FC_offset) - 1

    @property
    def num_oc_slices(self) -> int:
        return len(self.OC_offset) - 1


# ----------------------------------------------------------------------------
# planar helpers (shapely replacements)
# ----------------------------------------------------------------------------

def _rotate(px, py, angle, inverse=False):
    """Apply [[c, s], [-s, c]] (or its transpose) with explicit products (no BLAS/FMA)."""
    c, s = np.cos(angle), np.sin(angle)
    if inverse:
        return c * px - s * py, s * px + c * py
    return c * px + s * py, -s * px + c * py


def _clip_halfplane(poly, keep):
    """Sutherland-Hodgman step: keep the part of ``poly`` where ``keep(p) >= 0``.

    ``keep`` returns a signed distance-like value; intersection points are
    interpolated along the edge.
    """
    out = []
    n = len(poly)
    for k in range(n):
        cur, nxt = poly[k], poly[(k + 1) % n]
        dc, dn = keep(cur), keep(nxt)
        if dc >= 0:
            out.append(cur)
        if (dc >= 0) != (dn >= 0):
            t = dc / (dc - dn)
            out.append((cur[0] + t * (nxt[0] - cur[0]), cur[1] + t * (nxt[1] - cur[1])))
    return out


def _clip_convex_band(xs, ys, y_hi, y_lo, half_width):
    """Intersection of a convex ring with the box ``[-w, w] x [y_lo, y_hi]``.

    Returns a closed ring (first vertex repeated last) as shapely's
    ``exterior.coords`` does (CC:437), or ``None`` when the intersection has no
    area (shapely's empty / non-polygon results are skipped at CC:432-441).
    """
    poly = list(zip(xs.tolist(), ys.tolist()))
    for keep in (lambda p: y_hi - p[1], lambda p: p[1] - y_lo,
                 lambda p: half_width - p[0], lambda p: p[0] + half_width):
        poly = _clip_halfplane(poly, keep)
        if len(poly) < 3:
            return None
    # drop consecutive duplicates created when a vertex lies on a clip line
    ded = [poly[0]]
    for p in poly[1:]:
        if p != ded[-1]:
            ded.append(p)
    if len(ded) > 1 and ded[-1] == ded[0]:
        ded.pop()
    if len(ded) < 3:
        return None
    arr = np.asarray(ded + [ded[0]], dtype=np.float64)
    area = 0.5 * np.sum(arr[:-1, 0] * arr[1:, 1] - arr[1:, 0] * arr[:-1, 1])
    if abs(area) <= 0.0:
        return None
    return arr[:, 0].copy(), arr[:, 1].copy()


def _douglas_peucker(pts, tol):
    """Open-polyline Douglas-Peucker, endpoints kept (stands in for LineString.simplify)."""
    n = len(pts)
    if n < 3:
        return pts.copy()
    keep = np.zeros(n, dtype=bool)
    keep[0] = keep[-1] = True
    stack = [(0, n - 1)]
    while stack:
        a, b = stack.pop()
        if b <= a + 1:
            continue
        ax, ay = pts[a]
        bx, by = pts[b]
        seg = pts[a + 1:b]
        dx, dy = bx - ax, by - ay
        L2 = dx * dx + dy * dy
        if L2 == 0.0:
            d = np.hypot(seg[:, 0] - ax, seg[:, 1] - ay)
        else:
            t = np.clip(((seg[:, 0] - ax) * dx + (seg[:, 1] - ay) * dy) / L2, 0.0, 1.0)
            d = np.hypot(seg[:, 0] - (ax + t * dx), seg[:, 1] - (ay + t * dy))
        k = int(np.argmax(d))
        if d[k] > tol:
            idx = a + 1 + k
            keep[idx] = True
            stack.append((a, idx))
            stack.append((idx, b))
    return pts[keep].copy()


def _hull_vertices(x, y):
    return ConvexHull(np.column_stack((x, y))).vertices


def _slice_polygon(px, py, n_slices_design, half_width):
    """Cut a (rotated) convex polygon into bands of equal height along y (CC:313-320, CC:408-452)."""
    top, bottom = np.max(py), np.min(py)
    width = (top - bottom) / (n_slices_design + 0.001)
    count = int(np.ceil((top - bottom) / width))
    if (top - bottom) % width < width / 4:
        count -= 1
    bands = []
    for i in range(1, count + 1):
        hi = top - (i - 1) * width
        lo = bottom if i == count else top - i * width
        clipped = _clip_convex_band(px, py, hi, lo, half_width)
        if clipped is not None:
            bands.append(clipped)
    return bands


# ----------------------------------------------------------------------------
# the design
# ----------------------------------------------------------------------------

_pow = np.frompyfunc(math.pow, 2, 1)


def _sq(x):
    """``x ** 2`` as the reference evaluates it: on numpy float64 *scalars* inside its loops, which
    numpy computes with the C library's ``pow(x, 2.0)`` -- and this libm's pow rounds about 1 in
    1,200 squares differently from ``x * x``, the array path numpy takes for ``array ** 2``.
    Elementwise ``math.pow`` (the same libm call) keeps the tables bit-identical
    (tests/test_geometry_golden.py)."""
    return np.asarray(_pow(x, 2.0), dtype=np.float64)


def _field_angles(fx, fy):
    """Polar / azimuth angle of a field point (CC:226-227)."""
    tx, ty = np.tan(fx), np.tan(fy)
    return np.arctan(np.sqrt(_sq(tx) + _sq(ty))), np.arctan2(ty, tx)


def _pupil_tangents(d, k0, th, ph, kg):
    """Tangent-line intercepts of the input pupil and of the eyebox edges for
    one FoV direction (CC:228-266).  Everything broadcasts elementwise."""
    (kgx_ic, kgy_ic, kgx_fc, kgy_fc) = kg
    kx = d.n_air * k0 * np.sin(th) * np.cos(ph)
    ky = d.n_air * k0 * np.sin(th) * np.sin(ph)
    kx_ic = kx + kgx_ic
    ky_ic = ky + kgy_ic
    xc, yc = d.ic_center
    k1 = ky_ic / kx_ic
    root = d.ic_radius * np.sqrt(1 + _sq(k1))
    b11 = yc - k1 * xc + root
    b12 = yc - k1 * xc - root
    kx_fc = kx_ic + kgx_fc
    ky_fc = ky_ic + kgy_fc
    dx = d.eye_relief * np.tan(th) * np.cos(ph)
    dy = d.eye_relief * np.tan(th) * np.sin(ph)
    ex0, ey0 = d.eyebox_center
    hx, hy = d.eyebox[0] / 2, d.eyebox[1] / 2
    x_l, x_r = ex0 - hx + dx, ex0 + hx + dx
    y_t, y_b = ey0 + hy + dy, ey0 - hy + dy
    k2 = ky_fc / kx_fc
    neg = k2 <= 0
    b21 = np.where(neg, y_b - k2 * x_l, y_t - k2 * x_l)
    b22 = np.where(neg, y_t - k2 * x_r, y_b - k2 * x_r)
    return dict(kx=kx, ky=ky, kx_ic=kx_ic, ky_ic=ky_ic, kx_fc=kx_fc, ky_fc=ky_fc,
                k1=k1, k2=k2, b11=b11, b12=b12, b21=b21, b22=b22)


def _eyebox_rects(d, th, ph):
    """Eyebox footprint rectangles for field directions (CC:481-532): vertex
    order TL, BL, BR, TR."""
    dx = d.eye_relief * np.tan(th) * np.cos(ph)
    dy = d.eye_relief * np.tan(th) * np.sin(ph)
    ex0, ey0 = d.eyebox_center
    hx, hy = d.eyebox[0] / 2, d.eyebox[1] / 2
    xl, xr = ex0 - hx + dx, ex0 + hx + dx
    yt, yb = ey0 + hy + dy, ey0 - hy + dy
    xs = np.stack([xl, xl, xr, xr], axis=-1)
    ys = np.stack([yt, yb, yb, yt], axis=-1)
    return xs, ys, (xl, xr, yb, yt)


def _tir_phase(n_g, th):
    """delta_s - delta_p of a TIR bounce at polar angle ``th`` (CC:689-711)."""
    root = np.sqrt(n_g ** 2 * _sq(np.sin(th)) - 1)
    delta_s = 2 * np.arctan(root / (n_g * np.cos(th)))
    delta_p = 2 * np.arctan(n_g * root / np.cos(th))
    return delta_s - delta_p


def _polar_after(k0, n_g, kx, ky):
    kz = np.sqrt(_sq(k0) * n_g ** 2 - _sq(kx) - _sq(ky))
    return np.arctan(np.sqrt((_sq(kx) + _sq(ky)) / _sq(kz))), np.arctan2(ky, kx)


def design_geometry(num_FOV_x: int = 120, num_FOV_y: int = 80,
                    design: WaveguideDesign | None = None) -> CouplerGeometry:
    d = design or WaveguideDesign()
    lmd = np.array(d.wavelengths_nm)
    k0 = 2 * np.pi / lmd
    n_g = d.n_glass
    xc, yc = d.ic_center

    t_ic = np.linspace(0, 2 * np.pi, d.ic_points)
    X_ic = xc + d.ic_radius * np.sin(t_ic)
    Y_ic = yc + d.ic_radius * np.cos(t_ic)

    ex0, ey0 = d.eyebox_center
    ebx, eby = d.eyebox
    oc_w = np.tan(d.fov_x / 2) * abs(d.eye_relief) * 2 + ebx
    oc_h = np.tan(d.fov_y / 2) * abs(d.eye_relief) * 2 + eby
    X_oc = np.array([-oc_w / 2, -oc_w / 2, oc_w / 2, oc_w / 2]) + ex0
    Y_oc = np.array([-oc_h / 2, oc_h / 2, oc_h / 2, -oc_h / 2]) + ey0

    kg = 2 * np.pi / d.period_ic
    kgx_ic, kgy_ic = kg * np.cos(d.azimuth_ic), kg * np.sin(d.azimuth_ic)
    kg = 2 * np.pi / d.period_oc
    kgx_oc = kg * np.cos(d.azimuth_oc + 180 * DEG)
    kgy_oc = kg * np.sin(d.azimuth_oc + 180 * DEG)
    kgx_fc, kgy_fc = kgx_oc - kgx_ic, kgy_oc - kgy_ic
    Lambda_fc = 2 * np.pi / np.sqrt(kgx_fc ** 2 + kgy_fc ** 2)
    phi_fc = np.arctan2(kgy_fc, kgx_fc)
    kgs = (kgx_ic, kgy_ic, kgx_fc, kgy_fc)

    # --- folding-coupler hull from the dense FoV sweep (CC:222-304) -------------
    S = d.hull_fov_samples
    fxs = np.linspace(-d.fov_x / 2, d.fov_x / 2, S)
    fys = np.linspace(-d.fov_y / 2, d.fov_y / 2, S)
    FX, FY, K0 = np.meshgrid(fxs, fys, k0, indexing="ij")          # order (ii, jj, lambda)
    th, ph = _field_angles(FX, FY)
    tg = _pupil_tangents(d, K0, th, ph, kgs)
    den = tg["k1"] - tg["k2"]
    corners_x, corners_y = [], []
    for b1 in (tg["b11"], tg["b12"]):
        for b2 in (tg["b22"], tg["b21"]):
            xi = (b2 - b1) / den
            corners_x.append(xi)
            corners_y.append(tg["k1"] * xi + b1)
    x_f = np.stack(corners_x, axis=-1).reshape(-1)
    y_f = np.stack(corners_y, axis=-1).reshape(-1)
    kvec = {
        "kx0": np.moveaxis(tg["kx"], -1, 0).reshape(len(lmd), -1),
        "ky0": np.moveaxis(tg["ky"], -1, 0).reshape(len(lmd), -1),
        "kx_ic": np.moveaxis(tg["kx_ic"], -1, 0).reshape(len(lmd), -1),
        "ky_ic": np.moveaxis(tg["ky_ic"], -1, 0).reshape(len(lmd), -1),
        "kx_fc": np.moveaxis(tg["kx_fc"], -1, 0).reshape(len(lmd), -1),
        "ky_fc": np.moveaxis(tg["ky_fc"], -1, 0).reshape(len(lmd), -1),
    }

    bd = _hull_vertices(x_f, y_f)
    all_x, all_y = [x_f[bd]], [y_f[bd]]
    rot = np.pi / 2 + d.azimuth_ic
    rfx, rfy = _rotate(x_f[bd], y_f[bd], rot)

    # --- nine corner FoVs: FC footprints (CC:279-377) ---------------------------
    e = np.finfo(float).eps
    hx, hy = d.fov_x / 2, d.fov_y / 2
    f9x = np.array([-hx, e, hx, -hx, e, hx, hx, e, -hx])
    f9y = np.array([hy, hy, hy, e, e, e, -hy, -hy, -hy])
    F9X, K9 = np.meshgrid(f9x, k0, indexing="ij")
    F9Y, _ = np.meshgrid(f9y, k0, indexing="ij")
    th9, ph9 = _field_angles(F9X, F9Y)
    t9 = _pupil_tangents(d, K9, th9, ph9, kgs)
    den9 = t9["k1"] - t9["k2"]
    x_fc_fov = np.stack([(t9["b22"] - t9["b11"]) / den9, (t9["b21"] - t9["b11"]) / den9,
                         (t9["b21"] - t9["b12"]) / den9, (t9["b22"] - t9["b12"]) / den9],
                        axis=-1).reshape(-1, 4)
    inter = np.stack([t9["b11"], t9["b11"], t9["b12"], t9["b12"]], axis=-1).reshape(-1, 4)
    y_fc_fov = np.repeat(t9["k1"].reshape(-1, 1), 4, axis=1) * x_fc_fov + inter

    for i in range(x_fc_fov.shape[0]):
        cx = np.hstack((x_fc_fov[i], X_ic))
        cy = np.hstack((y_fc_fov[i], Y_ic))
        hb = _hull_vertices(cx, cy)
        all_x.append(cx[hb])
        all_y.append(cy[hb])

    ax_ = np.concatenate(all_x)
    ay_ = np.concatenate(all_y)
    hb = _hull_vertices(ax_, ay_)
    eff2 = _douglas_peucker(np.column_stack((ax_[hb], ay_[hb])), 1e-3)

    fc_rings = [_rotate(rx, ry, rot, inverse=True)
                for rx, ry in _slice_polygon(rfx, rfy, d.num_fc, d.glass_x)]

    # --- out-coupler slices (CC:454-475, CC:557-600) ---------------------------
    ob = _hull_vertices(X_oc, Y_oc)
    rot_oc = 3 * np.pi / 2 + d.azimuth_oc
    rox, roy = _rotate(X_oc[ob], Y_oc[ob], rot_oc)

    th9o, ph9o = _field_angles(f9x, f9y)
    x_oc_fov, y_oc_fov, _ = _eyebox_rects(d, th9o, ph9o)

    # --- per-FoV eyebox rectangles on the simulation grid (CC:502-532) ----------
    gx = np.linspace(-d.fov_x / 2, d.fov_x / 2, num_FOV_x)
    gy = np.linspace(-d.fov_y / 2, d.fov_y / 2, num_FOV_y)
    GX, GY = np.meshgrid(gx, gy, indexing="ij")
    thg, phg = _field_angles(GX, GY)
    rx, ry, (xl, xr, yb, yt) = _eyebox_rects(d, thg, phg)
    eff_reg_FOV = np.stack((rx, ry), axis=-1)
    eff_reg_FOV_range = np.stack((xl, xr, yb, yt), axis=-1)

    # --- whole effective region (CC:538-555) ----------------------------------
    nl = len(lmd)
    for i in range(len(f9x)):
        for l in range(nl):
            cx = np.concatenate([x_oc_fov[i], x_fc_fov[i * nl + l]])
            cy = np.concatenate([y_oc_fov[i], y_fc_fov[i * nl + l]])
            hb = _hull_vertices(cx, cy)
            all_x.append(cx[hb])
            all_y.append(cy[hb])
    ax_ = np.concatenate(all_x)
    ay_ = np.concatenate(all_y)
    hb = _hull_vertices(ax_, ay_)
    eff1 = _douglas_peucker(np.column_stack((ax_[hb], ay_[hb])), 1e-3)

    oc_rings = [_rotate(rx_, ry_, rot_oc, inverse=True)
                for rx_, ry_ in _slice_polygon(rox, roy, d.num_oc, d.glass_x)]

    # --- per-(lambda, FoV) propagation angles, hops and TIR phases (CC:614-711) --
    L3 = np.broadcast_to(k0[:, None, None], (nl, num_FOV_x, num_FOV_y))
    th_in = np.broadcast_to(thg, L3.shape).copy()
    ph_in = np.broadcast_to(phg, L3.shape).copy()
    kx = d.n_air * L3 * np.sin(th_in) * np.cos(ph_in)
    ky = d.n_air * L3 * np.sin(th_in) * np.sin(ph_in)
    th_glass = np.arcsin(np.sin(th_in) / n_g)
    cos_in = np.cos(th_in)
    r_te = (n_g * np.cos(th_glass) - cos_in) / (n_g * np.cos(th_glass) + cos_in)
    r_tm = (np.cos(th_glass) - n_g * cos_in) / (np.cos(th_glass) + n_g * cos_in)
    hop_glow = 2 * d.thickness * np.tan(th_glass) * np.cos(ph_in)
    lut_Fresnel = np.stack([r_te[-1], r_tm[-1], hop_glow[-1], hop_glow[-1]], axis=-1)

    th_ic2, ph_ic2 = _polar_after(L3, n_g, kx - kgx_ic, ky - kgy_ic)
    kxi, kyi = kx + kgx_ic, ky + kgy_ic
    th_ic, ph_ic = _polar_after(L3, n_g, kxi, kyi)
    kxf, kyf = kxi + kgx_fc, kyi + kgy_fc
    th_fc, ph_fc = _polar_after(L3, n_g, kxf, kyf)
    th_oc, ph_oc = _polar_after(L3, n_g, kxf - 2 * kgx_oc, kyf - 2 * kgy_oc)

    hop = 2 * d.thickness
    lut_gap = np.stack([
        hop * np.tan(th_ic) * np.cos(ph_ic), hop * np.tan(th_ic) * np.sin(ph_ic),
        hop * np.tan(th_fc) * np.cos(ph_fc), hop * np.tan(th_fc) * np.sin(ph_fc),
        hop * np.tan(th_ic2) * np.cos(ph_ic2), hop * np.tan(th_ic2) * np.sin(ph_ic2),
        hop * np.tan(th_oc) * np.cos(ph_oc), hop * np.tan(th_oc) * np.sin(ph_oc),
    ], axis=-1)
    lut_TIR = np.stack([_tir_phase(n_g, th_ic), _tir_phase(n_g, th_fc),
                        _tir_phase(n_g, th_ic2), _tir_phase(n_g, th_oc)], axis=-1)

    def _pack(rings):
        xs = np.concatenate([r[0] for r in rings])
        ys = np.concatenate([r[1] for r in rings])
        off = np.cumsum([0] + [len(r[0]) for r in rings])
        return np.stack((xs, ys), axis=1), off

    FC, FC_offset = _pack(fc_rings)
    OC, OC_offset = _pack(oc_rings)

    angles = dict(th_in_ic=th_in, phi_in_ic=ph_in, th_out_ic=th_ic, phi_out_ic=ph_ic,
                  th_out_fc=th_fc, phi_out_fc=ph_fc, th_out_ic2=th_ic2, phi_out_ic2=ph_ic2,
                  th_out_oc=th_oc, phi_out_oc=ph_oc, th_out_oc_glow=th_glass)
    return CouplerGeometry(
        IC=np.stack((X_ic, Y_ic), axis=1), FC=FC, FC_offset=FC_offset, OC=OC,
        OC_offset=OC_offset, eff_reg1=eff1, eff_reg2=eff2, eff_reg_FOV=eff_reg_FOV,
        eff_reg_FOV_range=eff_reg_FOV_range, lut_TIR=lut_TIR, lut_gap=lut_gap,
        lut_Fresnel=lut_Fresnel, Lambda_ic=d.period_ic, phi_ic=d.azimuth_ic,
        Lambda_fc=Lambda_fc, phi_fc=phi_fc, Lambda_oc=d.period_oc, phi_oc=d.azimuth_oc,
        n_g=n_g, lmd=lmd, angles=angles, kvec=kvec)


def couplers_coor_full_color(num_FOV_x: int = 120, num_FOV_y: int = 80):
    """Drop-in for reference ``couplers_coor_full_color`` (CC:122): same 37-tuple order."""
    return design_geometry(num_FOV_x, num_FOV_y).as_tuple()
