#!/usr/bin/env python3
"""Ablation timing: builds libwgrt with one WGRT_ABL_* macro at a time (results are NOT
valid in those builds -- only time per bounce is read) and times the C3 workload in a
fresh process per build.  Usage: python tools/ablate.py [flags...]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
FLAGS = sys.argv[1:] or ["", "WGRT_ABL_RAYLOAD", "WGRT_ABL_TILE", "WGRT_ABL_SINCOS", "WGRT_ABL_ATAN2"]

RUN = r'''
import sys, json, numpy as np, torch
sys.path.insert(0, %r)
torch.cuda.init()
from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _lib
_lib.load(%r)
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.couplers_coor import design_geometry
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.engine import Scene, rays_to_device, trace_fullcolor
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.luts import synthetic_luts
from gpu_ray_tracing_for_waveguide_based_ar_display_amd.rays import build_rays, generate_points_in_polygon, rng_seeds
g = design_geometry(21, 21); L = synthetic_luts(g, seed=0)
pts = generate_points_in_polygon(g.IC, 512, rng=np.random.default_rng(1))
h = build_rays(pts, 21, 21, [0, 1, 2], 1024); dev = torch.device("cuda", 0)
sc = Scene.from_geometry(g, L); rays = rays_to_device(h, dev)
seeds = torch.from_numpy(rng_seeds(h["x"].shape[0]).view(np.int32)).to(dev)
eb = torch.zeros(sc.eb_shape(), dtype=torch.float32, device=dev)
ts = []; bs = []
for k in range(12):
    rng = seeds.clone(); st = torch.zeros(4, dtype=torch.int64, device=dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); trace_fullcolor(sc, rays, rng, eb, stats=st); b.record(); torch.cuda.synchronize()
    if k >= 2: ts.append(a.elapsed_time(b)); bs.append(int(st[0]))
print(json.dumps({"ms": float(np.median(ts)), "bounces": bs[0], "ns_per_bounce": float(np.median(ts)) * 1e6 / bs[0]}))
'''
from gpu_ray_tracing_for_waveguide_based_ar_display_amd import _build  # noqa: E402
for fl in FLAGS:
    out = f"/tmp/libwgrt_abl_{fl or 'base'}.so"
    cmd = [_build._hipcc(), *_build.FLAGS, "-I", os.path.join(REPO, "include"), "-o", out] + \
          ([f"-D{fl}=1"] if fl else []) + [os.path.join(_build.CSRC, f) for f in _build.SOURCES]
    subprocess.run(cmd, check=True, capture_output=True)
    r = subprocess.run([sys.executable, "-c", RUN % (REPO, out)], capture_output=True, text=True, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    print(fl or "baseline", line[-1] if line else r.stderr[-800:], flush=True)
