"""Host-side ray batch construction (reference ``gpu_ray_tracing_pro_fullColor.py:59-158``).

The reference fills twelve float32 structure-of-arrays columns in
``(FoV-x ii, FoV-y jj, wavelength)`` block order, ``R`` rays per block, the
first ``R/2`` TE-polarised and the last ``R/2`` TM-polarised, all blocks
sharing the same ``R/2`` in-coupler origin points (MAIN:82-115).  The RNG
state of global ray ``gid`` is seeded ``0x9E3779B9 * (gid + 1) mod 2**32``
(MAIN:158).

Ray layout used everywhere in this package::

    gid = ((ii * NY + jj) * n_lambda_used + l) * R + r

so a contiguous ``[gid0, gid1)`` range aligned to ``R`` is a set of whole
FoV x wavelength blocks -- the unit that multi-GPU sharding hands out.
"""
from __future__ import annotations

import numpy as np
from matplotlib.path import Path

RAY_FIELDS = ("x", "y", "gap_x", "gap_y", "pol", "azi", "m", "n", "lmd_num", "te", "tm",
              "delta_phase")
RNG_MULT = np.uint32(0x9E3779B9)


def generate_points_in_polygon(polygon_vertices, num_points, rng=None):
    """Uniform rejection sampling of ``num_points`` points inside a polygon (GRTF:12-23).

    Like the reference, it draws ``2 x`` the missing count per round from the
    polygon's bounding box and keeps the points ``matplotlib.path.Path``
    classifies as inside.  ``rng`` defaults to the global ``np.random`` state
    (the reference's unseeded behaviour); pass a Generator for reproducibility.
    """
    poly = np.asarray(polygon_vertices, dtype=np.float64)
    lo = poly.min(axis=0)
    hi = poly.max(axis=0)
    path = Path(poly)
    draw = (np.random.uniform if rng is None else rng.uniform)
    kept = np.empty((0, 2))
    while kept.shape[0] < num_points:
        want = (num_points - kept.shape[0]) * 2
        cand = draw(low=lo, high=hi, size=(want, 2))
        kept = np.concatenate([kept, cand[path.contains_points(cand)]])
    return kept[:num_points]


def rng_seeds(n_rays: int, gid_offset: int = 0) -> np.ndarray:
    """xorshift32 seeds ``0x9E3779B9 * (gid + 1)`` for gids ``[off, off + n)`` (MAIN:158)."""
    gid = np.arange(gid_offset, gid_offset + n_rays, dtype=np.uint64)
    return ((gid + 1) * np.uint64(0x9E3779B9) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def build_rays(points: np.ndarray, num_fov_x: int, num_fov_y: int, lambdas, rays_per_fov: int,
               blocks: tuple | None = None):
    """Twelve float32 SoA columns in the reference's block order (MAIN:65-115).

    ``points`` holds the ``rays_per_fov // 2`` origins shared by every block;
    ``lambdas`` lists the wavelength indices traced (``[0, 1, 2]`` full colour,
    ``[1]`` for the single-lambda 532 nm configs).  ``blocks = (lo, hi)`` builds only
    FoV x wavelength blocks ``[lo, hi)`` -- global rays ``[lo * R, hi * R)`` -- which
    is one rank's shard.
    """
    R = int(rays_per_fov)
    half = R // 2
    pts = np.asarray(points)
    if pts.shape != (half, 2):
        raise ValueError(f"points must have shape ({half}, 2), got {pts.shape}")
    lam = np.asarray(list(lambdas), dtype=np.float32)
    nl = len(lam)
    nblk_all = num_fov_x * num_fov_y * nl
    lo, hi = (0, nblk_all) if blocks is None else (int(blocks[0]), int(blocks[1]))
    if not 0 <= lo <= hi <= nblk_all:
        raise ValueError(f"block range {blocks} outside [0, {nblk_all}]")
    nblk = hi - lo
    N = nblk * R
    ii, jj, ll = np.meshgrid(np.arange(num_fov_x, dtype=np.float32),
                             np.arange(num_fov_y, dtype=np.float32), lam, indexing="ij")
    per_ray = lambda v: np.repeat(v.reshape(-1)[lo:hi], R)
    r = np.arange(N) % R
    te_half = r < half
    used = r < 2 * half   # odd R: MAIN's halves cover 2 * floor(R / 2) rays, the last stays all-zero
    block_pts = np.concatenate([pts, pts, np.zeros((R - 2 * half, 2))]).astype(np.float32)
    origin = np.tile(block_pts, (nblk, 1))
    zeros = np.zeros(N, dtype=np.float32)
    z = lambda v: np.where(used, v, np.float32(0)).astype(np.float32)
    return {
        "x": np.ascontiguousarray(origin[:, 0]),
        "y": np.ascontiguousarray(origin[:, 1]),
        "gap_x": zeros.copy(), "gap_y": zeros.copy(), "pol": zeros.copy(), "azi": zeros.copy(),
        "m": z(per_ray(ii)), "n": z(per_ray(jj)), "lmd_num": z(per_ray(ll)),
        "te": te_half.astype(np.float32), "tm": (used & ~te_half).astype(np.float32),
        "delta_phase": zeros.copy(),
    }
