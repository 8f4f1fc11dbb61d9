#!/usr/bin/env python3
"""Run the C3 launch N times with a given libwgrt build in this process (for rocprofv3).
Usage: run_lib.py LIB [variant] [launches]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
torch.cuda.init()
from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _lib  # noqa: E402
_lib.load(os.path.abspath(sys.argv[1]))
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, init_rays, trace_fullcolor  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts  # noqa: E402
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import generate_points_in_polygon  # noqa: E402

variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
launches = int(sys.argv[3]) if len(sys.argv) > 3 else 10
g = design_geometry(21, 21)
L = synthetic_luts(g, seed=0)
pts = generate_points_in_polygon(g.IC, 512, rng=np.random.default_rng(1))
dev = torch.device("cuda", 0)
sc = Scene.from_geometry(g, L)
rays, seeds = init_rays(pts, 21, 21, [0, 1, 2], 1024, device=dev)
eb = torch.zeros(sc.eb_shape(), dtype=torch.float32, device=dev)
for _ in range(launches):
    rng = seeds.clone()
    trace_fullcolor(sc, rays, rng, eb, variant=variant)
torch.cuda.synchronize()
print("ok", float(eb.sum()))
