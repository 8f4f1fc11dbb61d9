"""The five BASELINE.json workloads, shared by bench.py, the tests and the tools.

Each config is the reference driver's batch (gpu_ray_tracing_pro_fullColor.py:16-17, 60-115) on a
FoV grid, with a seeded synthetic LUT (luts.synthetic_luts) on the geometry of
``couplers_coor.design_geometry`` -- the real RCWA tables are not available offline,
so the LUT profile and seed are part of the workload definition.

C5, "deep-bounce stress", uses the ``stress`` LUT profile (higher 0th-order reflection, lower
out-coupling, a better in-coupler) on a waveguide 20x thinner than the design's (every hop of
``lut_gap`` = 2 t tan(theta), CC:656-687, scaled by 0.05): rays live 50 bounces on average
instead of C3's 6.4, and the batch's tail reaches past 1,000 bounces, so the certification's
depth term is exercised where it grows.  The short hops also make consecutive
locator lookups of a ray hit nearby cells, so C5's rate is not comparable with C3 / C4's; C5d is
the same stress batch on the design geometry (CC:140, t = 0.7 mm, hops unscaled).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class Workload:
    key: str
    name: str
    nx: int
    ny: int
    lambdas: tuple
    R: int
    profile: str = "default"
    gap_scale: float = 1.0

    @property
    def n_blocks(self) -> int:
        return self.nx * self.ny * len(self.lambdas)

    @property
    def n_rays(self) -> int:
        return self.n_blocks * self.R

    def metric(self) -> str:
        colour = "full-color" if len(self.lambdas) == 3 else "single-λ " + "/".join(
            str(WAVELENGTHS_NM[l]) + " nm" for l in self.lambdas)
        extra = "" if self.profile == "default" else f", {self.profile} LUT"
        if self.gap_scale != 1.0:
            extra += f", hops x{self.gap_scale:g}"
        return f"ray-bounces/sec, {colour} {self.nx}x{self.ny} FoV, num_rays_per_FoV={self.R}{extra}"


WAVELENGTHS_NM = (465, 532, 630)   # CC:132

CONFIGS = {
    "C1": Workload("C1", "BASELINE config 1: single-λ 532 nm, 3x3 FoV, num_rays_per_FoV=64 (CPU reference path)",
                   3, 3, (1,), 64),
    "C2": Workload("C2", "BASELINE config 2: single-λ 532 nm, 11x11 FoV, num_rays_per_FoV=1024", 11, 11, (1,), 1024),
    "C3": Workload("C3", "BASELINE config 3: full-colour 21x21 FoV x 3 λ, num_rays_per_FoV=1024", 21, 21, (0, 1, 2),
                   1024),
    "C4": Workload("C4", "BASELINE config 4: full-colour 21x21 FoV x 3 λ, num_rays_per_FoV=4096, FoV x λ sharded",
                   21, 21, (0, 1, 2), 4096),
    "C5": Workload("C5", "BASELINE config 5: full-colour 41x41 FoV x 3 λ, num_rays_per_FoV=16384, deep-bounce stress "
                         "(stress LUT, hops x0.05), FoV x λ sharded", 41, 41, (0, 1, 2), 16384, profile="stress",
                   gap_scale=0.05),
    "C5d": Workload("C5d", "BASELINE config 5 on the design geometry: full-colour 41x41 FoV x 3 λ, "
                           "num_rays_per_FoV=16384, stress LUT, unscaled hops (t = 0.7 mm, CC:140)", 41, 41, (0, 1, 2),
                    16384, profile="stress"),
}


def build_inputs(w: Workload, lut_seed: int = 0, point_seed: int = 1):
    """(geometry, LUT set, ray origin points) of a workload: the geometry restatement with
    ``lut_gap`` scaled by the workload's gap_scale, the seeded synthetic LUT, and the R/2 origins
    of the reference's sampler (GRTF:12-23) from ``np.random.default_rng(point_seed)``."""
    from .couplers_coor import design_geometry
    from .luts import synthetic_luts
    from .rays import generate_points_in_polygon
    geom = design_geometry(w.nx, w.ny)
    if w.gap_scale != 1.0:
        geom.lut_gap = geom.lut_gap * w.gap_scale
    luts = synthetic_luts(geom, seed=lut_seed, profile=w.profile)
    points = generate_points_in_polygon(geom.IC, w.R // 2, rng=np.random.default_rng(point_seed))
    return geom, luts, points


__all__ = ["Workload", "CONFIGS", "WAVELENGTHS_NM", "build_inputs"]
